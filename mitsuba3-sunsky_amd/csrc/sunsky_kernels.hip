// sunsky_kernels.hip -- CDNA4 (gfx950) kernels of the sun/sky emitter.
//
// Compiled to a standalone code object (hipcc --genco --offload-arch=gfx950)
// and loaded by the C-ABI layer with hipModuleLoad / hipModuleGetFunction.
//
// Design (DESIGN.md "Kernels"; numbers from tools/kbench.cpp on MI355X):
//  * SoA fp32 rays in HBM (x[], y[], z[] planes) and SoA outputs (one plane per
//    channel / wavelength); VEC = 4 consecutive directions per lane so global
//    accesses are 16 B per lane (VEC = 1 kernels take tails / unaligned rays).
//    Plain loads + non-temporal stores measured fastest (RGB eval 68 us for
//    16M directions = 5.9 TB/s);
//  * every per-emitter constant arrives in the by-value SunskyKArgs kernarg
//    block (s_load -> SGPRs); tables that lanes index with DIFFERENT indices
//    (TGMM components, per-ray spectral channels, the sun polynomials in the
//    sampling kernels where ~(1 - w_sky) of the lanes hit the sun) are staged
//    in LDS once per workgroup;
//  * the sun disc (~1e-5 of random directions in eval) runs behind an
//    exec-masked branch that waves skip when no lane hits it, with rolled
//    loops so its registers do not lower the sky path's occupancy;
//  * FAST = true folds constants on the host (exp -> exp2 of log2(e)-scaled
//    coefficients, radiance x sky_scale (x CIE normalisation) into the
//    channel coefficients, pow(b, 1.5) -> rsq(b)^3, cos(unit_angle) ->
//    1 - 2 h^2, hardware sqrt); FAST = false follows the reference operation
//    order with full-precision libm.  Both are parity-tested against the oracle.
#include <hip/hip_runtime.h>

#include "sunsky_math.h"
#include "sunsky_staging.h"
#include "sunsky_types.h"

// fp contraction within a source expression only (C's FP_CONTRACT on), not across
// statements: hipcc's default lets the backend fuse a product into a later statement's
// add depending on the surrounding kernel, so the same inlined device function could
// round differently in two kernels.  With this, one sample / direction computes the
// same bits in every kernel that evaluates it (LEAN vs general vs wave-sorted sampling,
// eval vs eval_direction, sharded vs whole batches).  Instruction counts unchanged.
#pragma clang fp contract(on)

using namespace sunsky;

#define SS_BLOCK 256
#ifndef SS_NODES_ATTR       // tuning builds only (tools/gpu_ab2.sh): occupancy attributes
#define SS_NODES_ATTR
#endif
#ifndef SS_RAYS_ATTR         // tuning builds only: occupancy attribute of the per-ray spectral eval
#define SS_RAYS_ATTR
#endif
#ifndef SS_RGB_ATTR
#define SS_RGB_ATTR
#endif
#ifndef SS_SPEC_SAMPLE_ATTR
#define SS_SPEC_SAMPLE_ATTR
#endif
#ifndef SS_RGB_SORTED_ATTR   // probe builds (tools/build) set occupancy attributes here
#define SS_RGB_SORTED_ATTR
#endif
#ifndef SS_CONDUCTOR_ATTR    // occupancy of the FAST conductor caller (probe builds override it)
#define SS_CONDUCTOR_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#endif
#ifndef SS_SORT_R            // probe builds: the window of the wave-sorted RGB kernels
#define SS_SORT_R 4
#endif
constexpr float kLog2e = 1.44269504088896340736f;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

// safe_sqrt (sunsky.h / Dr.Jit): correctly rounded in the reference kernels, v_sqrt_f32
// (1 ulp) in FAST, which skips the ~16-instruction rounding fix-up sequence.
template <bool FAST>
__device__ __forceinline__ float safe_sqrt_sel(float x) {
    if constexpr (FAST) return __builtin_amdgcn_sqrtf(fmaxf(x, 0.f));
    else return sqrtf(x > 0.f ? x : 0.f);
}

// asin on [0, sqrt(0.5)]: the half chord h = |wo -/+ n| / 2 of unit_angle never
// exceeds sqrt(2) / 2, so one odd minimax polynomial x + x^3 P(x^2) (degree 7 in
// x^2; fitted by tools/fit_asin.py) replaces libm's two-range asin (select,
// sqrt, polynomial, fix-up).  Max error 0.71 ulp over [0, 0.7075] in fp32 (FAST only).
__device__ __forceinline__ float asin_half_chord(float x) {
    const float t = x * x;
    float p = 0.10696864128112793f;
    p = fmaf(p, t, -0.10311298817396164f);
    p = fmaf(p, t, 0.0816480815410614f);
    p = fmaf(p, t, 0.003488607471808791f);
    p = fmaf(p, t, 0.033441439270973206f);
    p = fmaf(p, t, 0.04438246041536331f);
    p = fmaf(p, t, 0.0750100240111351f);
    p = fmaf(p, t, 0.16666655242443085f);
    return fmaf(x * t, p, x);
}

// FAST sun elevation pi/2 - acos(z) for z = cos(theta) in [0, 1] (sun-disc lanes are above
// the horizon), as asin z: asin_half_chord(z) up to z = sqrt(1/2), above it
// pi/2 - 2 asin(sqrt((1 - z) / 2)) (argument <= sqrt(1/2); 0.5 - 0.5 z exact there).  One
// polynomial on a selected argument instead of libm's two-range acosf.  asin z does not
// cancel near the horizon, where pi/2 - acos z loses ~1e-7 absolute (measured 2x over
// the sun-disc bound at 0.1 degrees with a fast acos).
__device__ __forceinline__ float elevation_fast(float z) {
    const bool big = z > 0.70710678f;
    const float p = asin_half_chord(big ? fast_sqrt(fmaf(-0.5f, z, 0.5f)) : z);
    return big ? fmaf(-2.f, p, kHalfPi) : p;
}

// atan on [0, 1]: t + t^3 P(t^2), degree 7 in t^2 (tools/fit_atan.py; 1.07 ulp).
__device__ __forceinline__ float atan_unit(float t) {
    const float u = t * t;
    float p = 0.0025049929972738028f;
    p = fmaf(p, u, -0.014686254784464836f);
    p = fmaf(p, u, 0.040442489087581635f);
    p = fmaf(p, u, -0.07314199209213257f);
    p = fmaf(p, u, 0.1055244505405426f);
    p = fmaf(p, u, -0.14181630313396454f);
    p = fmaf(p, u, 0.19990065693855286f);
    p = fmaf(p, u, -0.3333298861980438f);
    return fmaf(t * u, p, t);
}

// FAST atan2 for the TGMM pdf's azimuth: octant reduction t = min / max with
// v_rcp_f32, atan_unit, then pi/2 - a and pi - a fix-ups (max error 4.4 ulp,
// 3.5e-7 absolute over the circle; tools/fit_atan.py).  atan2(0, 0) returns a
// finite value: the callers mask sin(theta) = 0 directions out (sunsky.cpp:717).
__device__ __forceinline__ float atan2_fast(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float t = fminf(fminf(ax, ay) * fast_rcp(fmaxf(ax, ay)), 1.f);
    float a = atan_unit(t);
    a = ay > ax ? kHalfPi - a : a;
    a = x < 0.f ? kPi - a : a;
    return copysignf(a, y);
}

// Correctly rounded a / b from rb = RN(1 / b) (Markstein's theorem: q = RN(a rb),
// r = a - q b exact by fma, RN(q + r rb) = RN(a / b)), valid while r does not
// underflow: |a| >= 2^-100 and rb normal; otherwise the plain division.  The FAST
// sampling transforms divide by the wave-uniform w_sky / 1 - w_sky and by the picked
// gaussian's pmf, whose reciprocals are computed once per wave / workgroup.  Exact,
// so the sample transform keeps the correctly rounded quotients it needs (one ulp in
// the reused sample moves sky directions by up to 2e-5).
__device__ __forceinline__ float div_by_rcp(float a, float b, float rb) {
    if (fabsf(a) >= 0x1p-100f && fabsf(rb) <= 0x1p100f) {
        const float q = a * rb;
        return fmaf(fmaf(-q, b, a), rb, q);
    }
    return a / b;
}

// (lambda - 320) / 40, the per-lane wavelength's channel coordinate (sunsky.cpp:326), as
// div_by_rcp by the correctly rounded 1/40: equal to the IEEE quotient for every float
// (checked exhaustively on the host for |a| in [2^-100, 2^100]; below, the division
// itself; inf / NaN give an invalid coordinate either way), without the division sequence.
__device__ __forceinline__ float wavelength_node(float lambda) {
    return div_by_rcp(lambda - kWavelength0, kWavelengthStep, 1.f / kWavelengthStep);
}

// A wave-uniform float the compiler may not re-derive per lane: the sampling loops
// select between the reciprocals 1 / w_sky and 1 / (1 - w_sky) (div_exact's rb), and
// without this InstCombine folds select(p, 1 / a, 1 / b) into 1 / select(p, a, b), a
// full per-lane division (13 VALU + v_rcp) in every sample.  Same value, bit for bit.
__device__ __forceinline__ float uniform_f(float x) {
    asm("" : "+v"(x));   // a value the optimiser cannot look through (no instruction)
    return x;
}

template <bool FAST>
__device__ __forceinline__ float div_exact(float a, float b, float rb) {
    if constexpr (FAST) return div_by_rcp(a, b, rb);
    else return a / b;
}

// FAST sincos for the sampling transforms (sphdir, the concentric disk): one
// Cody-Waite reduction by pi/2 (two fp32 constants, fma), then sin r = r + r^3 S(r^2)
// and cos r = 1 - r^2/2 + r^4 C(r^2) on [-pi/4, pi/4] (tools/fit_sincos.py: max
// 1.5 ulp, 9.2e-8 absolute for |x| <= 8 pi) and the quadrant swap / signs.  The
// arguments here stay within a few pi, far from where the two-constant reduction
// loses bits.
__device__ __forceinline__ void sincos_fast(float x, float* s, float* c) {
    const float k = rintf(x * 0.636619772f);
    float r = fmaf(-k, 1.57079637f, x);
    r = fmaf(-k, -4.37113883e-8f, r);
    const float r2 = r * r;
    float ps = 2.715222990445909e-06f;
    ps = fmaf(ps, r2, -0.00019838963635265827f);
    ps = fmaf(ps, r2, 0.008333328180015087f);
    ps = fmaf(ps, r2, -0.1666666716337204f);
    float pc = -2.7188141871192784e-07f;
    pc = fmaf(pc, r2, 2.4799224775051698e-05f);
    pc = fmaf(pc, r2, -0.001388888224028051f);
    pc = fmaf(pc, r2, 0.0416666679084301f);
    const float sn = fmaf(r * r2, ps, r);
    const float cs = fmaf(r2 * r2, pc, fmaf(-0.5f, r2, 1.f));
    const int q = (int)k;
    const float sv = (q & 1) ? cs : sn, cv = (q & 1) ? sn : cs;
    *s = (q & 2) ? -sv : sv;
    *c = ((q + 1) & 2) ? -cv : cv;
}

template <bool FAST>
__device__ __forceinline__ void sincos_sel(float x, float* s, float* c) {
    if constexpr (FAST) sincos_fast(x, s, c);
    else sincosf(x, s, c);
}

// FAST erfinv: Giles' single-precision polynomials (erfinvf_, sunsky_math.h) with
// w = -log(1 - x^2) from v_log_f32 (log2) times ln 2 instead of libm's logf.  The
// result's relative sensitivity to w is ~0.3 dw, so the hardware log's few-ulp
// error stays at the 1e-7 level.
__device__ __forceinline__ float erfinv_fast(float x) {
    float w = -0.693147180559945309f * __builtin_amdgcn_logf(fmaf(x, -x, 1.f)), p;
    if (w < 5.f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = fmaf(p, w, 3.43273939e-07f);
        p = fmaf(p, w, -3.5233877e-06f);
        p = fmaf(p, w, -4.39150654e-06f);
        p = fmaf(p, w, 0.00021858087f);
        p = fmaf(p, w, -0.00125372503f);
        p = fmaf(p, w, -0.00417768164f);
        p = fmaf(p, w, 0.246640727f);
        p = fmaf(p, w, 1.50140941f);
    } else {
        w = fast_sqrt(w) - 3.f;
        p = -0.000200214257f;
        p = fmaf(p, w, 0.000100950558f);
        p = fmaf(p, w, 0.00134934322f);
        p = fmaf(p, w, -0.00367342844f);
        p = fmaf(p, w, 0.00573950773f);
        p = fmaf(p, w, -0.0076224613f);
        p = fmaf(p, w, 0.00943887047f);
        p = fmaf(p, w, 1.00167406f);
        p = fmaf(p, w, 2.83297682f);
    }
    return p * x;
}

// Polar angle of an upper-hemisphere direction (unit_angle_z for z >= 0, sunsky.h:87):
// 2 asin(|v - e_z| / 2), whose half chord is <= sqrt(1/2), so asin_half_chord applies.
// Lanes with z < 0 get a meaningless finite angle: compute_pdfs masks them.
__device__ __forceinline__ float theta_upper_fast(float3_ v) {
    const float dz = v.z - 1.f;
    return 2.f * asin_half_chord(0.5f * fast_sqrt(fmaf(v.x, v.x, fmaf(v.y, v.y, dz * dz))));
}

// wo = -wi for eval(si), +d for eval_direction: a compile-time sign folds into
// the source modifiers of the first use instead of 3 multiplies per direction.
template <bool NEG>
__device__ __forceinline__ float3_ flip3(float x, float y, float z) {
    return NEG ? mk3(-x, -y, -z) : mk3(x, y, z);
}

template <bool FAST> struct ChanSel { using T = SkyChannel; };
template <> struct ChanSel<true> { using T = FastChannel; };

struct DirTerms {
    float cos_theta, gamma, cg, cg2, u;   // u = 1 + cos^2 gamma
    float r;        // 1 / (cos_theta + 0.01)
    float sq;       // safe_sqrt(cos_theta)
    float h;        // |wo -/+ n| / 2, so gamma = 2 asin(h) or pi - 2 asin(h)
    float wx, wy;   // wo.x, wo.y (wo.z = cos_theta): the FAST sun disc's cos psi
    bool active, hit_sun;
    // sun-disc terms, filled by add_sun_terms() for hit_sun lanes only
    int sun_pos;    // elevation segment (sunsky.cpp:579-587)
    float sun_x;    // elevation within the segment
    float sun_cpsi; // compute_cos_psi (sunsky.h:385-392)
};

// Shared per-direction terms of eval(), sunsky.cpp:309-314.
template <bool FAST>
__device__ __forceinline__ DirTerms dir_terms(const SunskyKArgs& K, float3_ wo, bool mask) {
    DirTerms t;
    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    t.cos_theta = wo.z;
    float d = dot3(sn, wo);
    // unit_angle(n, wo) = 2 asin(|wo -/+ n| / 2)
    // wo - mulsign(n, d) as fma(-s, n, wo) with s = +/-1: the product is exact, so this
    // is the reference's subtraction bit for bit, with one select instead of three
    const float sg = signbit(d) ? -1.f : 1.f;
    float3_ v = mk3(fmaf(-sg, sn.x, wo.x), fmaf(-sg, sn.y, wo.y), fmaf(-sg, sn.z, wo.z));
    float h = 0.5f * (FAST ? fast_sqrt(dot3(v, v)) : sqrtf(dot3(v, v)));
    t.h = h;
    t.wx = wo.x;
    t.wy = wo.y;
    float temp = 2.f * (FAST ? asin_half_chord(h) : asinf(h));
    t.gamma = d >= 0.f ? temp : kPi - temp;
    if (FAST) {
        float c = fmaf(h * h, -2.f, 1.f);   // cos(2 asin h) = 1 - 2 h^2 ; cos(pi - x) = -cos x
        t.cg = d >= 0.f ? c : -c;
        t.r = fast_rcp(t.cos_theta + 0.01f);
        t.sq = fast_sqrt(t.cos_theta);   // NaN below the horizon: those lanes are inactive, their output selected to 0
    } else {
        t.cg = cosf(t.gamma);
        t.r = 1.f / (t.cos_theta + 0.01f);
        t.sq = safe_sqrtf_(t.cos_theta);
    }
    t.cg2 = t.cg * t.cg;
    t.u = 1.f + t.cg2;
    t.active = mask && (t.cos_theta >= 0.f);
    t.hit_sun = t.active && (d >= K.cos_cutoff);
    t.sun_pos = 0;
    t.sun_x = t.sun_cpsi = 0.f;
    return t;
}

// render_sun's segment of a direction inside the sun disc (sunsky.cpp:579-584): the
// reference's fp32 floor(cbrt(2 elevation / pi) 45) decision, made exactly by counting the
// host-staged cos theta thresholds it passes (SunskyKArgs::sun_seg_z) over the disc's
// segments -- one compare each (wave-uniform bounds and table reads) instead of acos / cbrt,
// and no index flip within ulps of a segment start (tests/test_gpu_parity.py
// test_sun_segment_index_at_segment_starts).
__device__ __forceinline__ int sun_segment_index(const SunskyKArgs& K, float cos_theta) {
    int pos = K.sun_row_lo;
#pragma unroll 1
    for (int j = K.sun_row_lo + 1; j <= K.sun_row_hi; ++j) pos += cos_theta >= K.sun_seg_z[j] ? 1 : 0;
    return pos;
}

// The reference-precision kernels: the same index, x = elevation - pi/2 (pos / 45)^3 with the
// reference's elevation = pi/2 - acos(cos theta) (sunsky.cpp:580-587).
__device__ __forceinline__ int sun_segment_ref(const SunskyKArgs& K, float cos_theta, float* x) {
    const int pos = sun_segment_index(K, cos_theta);
    const float elevation = kHalfPi - acosf(cos_theta);
    const float frac = (float)pos / (float)kNbSunSegments;
    *x = elevation - kHalfPi * (frac * frac * frac);
    return pos;
}

// Sun-disc terms of a direction, once per ray and only on lanes inside the disc.
// Computed here rather than inside the per-wavelength loops: those calls are
// loop-invariant, and the compiler would otherwise hoist the acos / cbrt /
// divisions / sin out of both the loop and the hit_sun branch onto every lane.
//
// FAST: sin(gamma) from the half chord, sin(2 asin h) = sin(pi - 2 asin h) = 2h sqrt(1 - h^2),
// instead of sin() of the reconstructed angle; the segment fraction pos / 45 as a
// product with 1/45.
template <bool FAST>
__device__ __forceinline__ void add_sun_terms(const SunskyKArgs& K, DirTerms& t) {
    if (t.hit_sun) {
        if constexpr (FAST) {
            float elevation = elevation_fast(t.cos_theta);
            const int pos = sun_segment_index(K, t.cos_theta);
            float frac = (float)pos * (1.f / (float)kNbSunSegments);
            t.sun_pos = pos;
            t.sun_x = elevation - kHalfPi * (frac * frac * frac);
            // cos^2 psi = 1 - sin^2(gamma) / sin^2(half aperture) cancels towards the limb, where
            // d cos psi / d gamma is unbounded: its inputs in fp64.  With v = wo - n (exact in
            // fp32 next to the sun, the reference's subtraction) and |v|^2 = 4 h^2,
            // sin^2(gamma) = sin^2(2 asin h) = |v|^2 (1 - |v|^2 / 4); the fp32 products widen
            // exactly.  One rounding to fp32 before the square root (relative 3e-8 on cos psi).
            const double vx = (double)(t.wx - K.sun_n[0]), vy = (double)(t.wy - K.sun_n[1]),
                         vz = (double)(t.cos_theta - K.sun_n[2]);
            const double v2 = fma(vz, vz, fma(vy, vy, vx * vx));
            const double inv = (double)K.cpsi_inv_hi + (double)K.cpsi_inv_lo;
            const float c2 = (float)fma(-inv, v2 * fma(-0.25, v2, 1.0), 1.0);
            t.sun_cpsi = fast_sqrt(fmaxf(c2, 0.f));   // v_sqrt_f32, 1 ulp
        } else {
            t.sun_pos = sun_segment_ref(K, t.cos_theta, &t.sun_x);
            t.sun_cpsi = cos_psi(t.gamma, K.inv_sin2_half_ap);
        }
    }
}

// Division: correctly rounded in the reference kernels, v_rcp_f32 (1 ulp) in FAST.
template <bool FAST>
__device__ __forceinline__ float fdiv(float a, float b) {
    if constexpr (FAST) return a * fast_rcp(b);
    else return a / b;
}

// The emitter state as the disc branches read it: through a pointer the compiler cannot prove
// loop-invariant, so the branch's constant loads (segment thresholds, sun frame, ...) stay in
// the rare branch instead of being hoisted into SGPRs held across the whole ray loop (the
// headline kernel then spilled 19-28 SGPRs to VGPR lanes and ran 2-6 % slower).
__device__ __forceinline__ const SunskyKArgs& opaque_kargs(const SunskyKArgs& K) {
    int off = 0;   // a zero the compiler cannot see: the pointer stays based on K (no aliasing
    asm volatile("" : "+s"(off));   // doubts for the main loop's scalar loads) but cannot move
    return *(&K + off);
}

// ------------------------------------------------------------------ sun disc in fp64
// The FAST eval kernels (eval, eval_direction, the spectral broadcast / node / per-ray kernels,
// the lat-long bake) evaluate the sun-disc term of their rare disc lanes (~1e-5 of random
// directions) in fp64 on the fp32 inputs and staged fp32 tables: the exact value of
// render_sun x compute_sun_ld (sunsky.cpp:572-614, 631-650) up to the tables' own rounding.
// Near the limb cos psi = sqrt(1 - sin^2 gamma / sin^2(half aperture)) (sunsky.h:385-392)
// has an unbounded derivative and the limb-darkening sum nearly cancels, so an fp32 Horner
// there is off by up to 4.9e-5 (the reference's own fp32 by 1.5e-4); this branch holds the
// literal 1e-5 against the fp64 evaluation of the staged fp32 state
// (tests/test_gpu_disc_literal.py).  The samplers keep the
// fp32 form (65 % of their lanes are sun picks, already within 1e-5 of fp64).
struct SunDisc64 {
    int pos;     // render_sun's segment: the reference's fp32 decision (sun_segment_index)
    double x;    // elevation - pi/2 (pos / 45)^3: the fp32 elevation (elevation_fast, 0.7 ulp;
                 // x enters the polynomial smoothly), the segment start in fp64
    double cpsi; // compute_cos_psi from the chord v = wo - n formed in fp64 (exact)
};

__device__ __forceinline__ SunDisc64 sun_disc64(const SunskyKArgs& K, float wx, float wy, float cos_theta) {
    SunDisc64 d;
    d.pos = sun_segment_index(K, cos_theta);
    const double frac = (double)d.pos * (1.0 / (double)kNbSunSegments);
    d.x = (double)elevation_fast(cos_theta) - 1.5707963267948966 * (frac * frac * frac);
    // v = wo - n in fp64: exact for any aperture (in fp32 only next to the sun, where the
    // components' differences are exact; a 12 deg disc lost 1e-4 at its limb to the rounding)
    const double vx = (double)wx - (double)K.sun_n[0], vy = (double)wy - (double)K.sun_n[1],
                 vz = (double)cos_theta - (double)K.sun_n[2];
    const double v2 = fma(vz, vz, fma(vy, vy, vx * vx));
    const double inv = (double)K.cpsi_inv_hi + (double)K.cpsi_inv_lo;
    d.cpsi = sqrt(fmax(fma(-inv, v2 * fma(-0.25, v2, 1.0), 1.0), 0.0));
    return d;
}

// RGB: sum_k x^k sum_j cos psi^j S[pos][c][k][j] (sunsky.cpp:597-611), added to the fp32 sky
// value in fp64 and rounded once
__device__ __forceinline__ float add_sun_rgb64(const SunskyKArgs& K, const SunDisc64& d, int c, float sky) {
    const float* s = K.sun_table + d.pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
    double res = 0.0;
#pragma unroll 1
    for (int k = kNbSunCtrlPts - 1; k >= 0; --k) {
        const float* r = s + k * kNbSunLdParams;
        double inner = (double)r[kNbSunLdParams - 1];
#pragma unroll
        for (int j = kNbSunLdParams - 2; j >= 0; --j) inner = fma(inner, d.cpsi, (double)r[j]);
        res = fma(res, d.x, inner);
    }
    return (float)fma((double)K.sun_mul, res, (double)sky);
}

// Spectral: lerp of sum_k x^k S[pos][c][k] over the channel pair (lo, lo + 1, f) times the
// lerped limb darkening sum_j cos psi^j ld[c][j] (sunsky.cpp:341-347, 586-594, 631-650);
// channel 11 (720 nm, weight 0) contributes 0 as in the reference's masked gather
__device__ __forceinline__ float add_sun_spec64(const SunskyKArgs& K, const SunDisc64& d, int lo, float f, float sky) {
    const int hi = lo + 1;
    const double fd = (double)f;
    auto poly = [&](int c) {
        const float* q = K.sun_table + (d.pos * kNbWavelengths + c) * kNbSunCtrlPts;
        return fma(fma(fma((double)q[3], d.x, (double)q[2]), d.x, (double)q[1]), d.x, (double)q[0]);
    };
    double sun = poly(lo);
    if (f != 0.f) sun = fma(fd, (hi < kNbWavelengths ? poly(hi) : 0.0) - sun, sun);
    double ld = 0.0;
#pragma unroll 1
    for (int j = kNbSunLdParams - 1; j >= 0; --j) {
        double coef = (double)K.sun_ld[lo * kNbSunLdParams + j];
        if (f != 0.f) coef = fma(fd, (hi < kNbWavelengths ? (double)K.sun_ld[hi * kNbSunLdParams + j] : 0.0) - coef, coef);
        ld = fma(ld, d.cpsi, coef);
    }
    return (float)fma((double)K.sun_mul, sun * ld, (double)sky);
}

// render_sky (sunsky.cpp:538-555) with the output scale folded in (FastChannel)
__device__ __forceinline__ float sky_fast(const FastChannel& k, const DirTerms& t) {
    float c1 = fmaf(k.A, fast_exp2(k.Bl2 * t.r), 1.f);
    float rs = fast_rsq(fmaf(k.Q, t.cg, k.P));        // (1 + I^2 - 2 I cos g)^-1/2
    float w = rs * rs * rs;
    float c2 = fmaf(k.Ds, fast_exp2(k.El2 * t.gamma), k.Cs);
    c2 = fmaf(k.Fs, t.cg2, c2);
    c2 = fmaf(k.Gs, t.u * w, c2);
    c2 = fmaf(k.Hs, t.sq, c2);
    return c1 * c2;
}

// render_sky, reference operation order (sunsky.cpp:550-554), times sky_scale
__device__ __forceinline__ float sky_ref(const SkyChannel& k, const DirTerms& t, float sky_scale) {
    float c1 = 1.f + k.A * expf(k.B * t.r);
    float chi = t.u / powf(1.f + k.I * k.I - 2.f * k.I * t.cg, 1.5f);
    float c2 = k.C + k.D * expf(k.E * t.gamma) + k.F * t.cg2 + k.G * chi + k.H * t.sq;
    return sky_scale * (c1 * c2 * k.rad);
}

template <bool FAST>
__device__ __forceinline__ float sky_eval(const typename ChanSel<FAST>::T& k, const DirTerms& t, float sky_scale) {
    if constexpr (FAST) { (void)sky_scale; return sky_fast(k, t); }
    else return sky_ref(k, t, sky_scale);
}

// A channel gathered with a per-lane index: from an AoS table (eval kernels, sample_ray), or
// from the FAST spectral samplers' SoA table (FastChanSoA, below).
template <class T>
__device__ __forceinline__ T chan_get(const T* chans, int c) { return chans[c]; }

template <bool FAST>
__device__ __forceinline__ const typename ChanSel<FAST>::T* chan_table(const SunskyKArgs& K) {
    if constexpr (FAST) return K.fsky;
    else return K.sky;
}

// SS_XFORM_IDENTITY: the second code object, sunsky_kernels_ident.hsaco, which the C ABI
// launches only for emitters whose to_world is the identity (SunskyKArgs::identity_xform):
// the same v the runtime test returns there, without the test's branches and the SGPRs it
// holds (interleaved A/B, profiles/r04_v13_ab_identity_xform.log: headline eval 3.9 %,
// RGB sample_direction 2.9 %, pdf_direction 2.2 % faster).
#ifdef SS_XFORM_IDENTITY
// Marks the identity code object: the C ABI refuses it as the general module (and a general
// build as the identity module), so a rotated to_world is never silently dropped.
extern "C" __global__ void sunsky_xform_identity_marker() {}
#endif

__device__ __forceinline__ float3_ to_local(const SunskyKArgs& K, float3_ v) {
#ifdef SS_XFORM_IDENTITY
    (void)K;
    return v;
#else
    return K.identity_xform ? v : xform_vec(K.to_local, v);
#endif
}
__device__ __forceinline__ float3_ to_world(const SunskyKArgs& K, float3_ v) {
#ifdef SS_XFORM_IDENTITY
    (void)K;
    return v;
#else
    return K.identity_xform ? v : xform_vec(K.to_world, v);
#endif
}

// render_sun RGB branch (sunsky.cpp:597-611) as nested Horner forms:
// sum_k x^k (sum_j cos_psi^j S[k][j]) -- 6 table values live at a time.
__device__ __forceinline__ float render_sun_rgb_compact(const float* table, int pos, int c, float x, float cpsi) {
    const float* s = table + pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
    float res = 0.f;
#pragma unroll 1
    for (int k = kNbSunCtrlPts - 1; k >= 0; --k) {
        const float* r = s + k * kNbSunLdParams;
        float inner = r[kNbSunLdParams - 1];
#pragma unroll
        for (int j = kNbSunLdParams - 2; j >= 0; --j) inner = fmaf(inner, cpsi, r[j]);
        res = fmaf(res, x, inner);
    }
    return res;
}

// RGB sun-table segments [K.sun_row_lo, K.sun_row_lo + kSunRowsStaged) in LDS with
// per (row, k) the 18 values S[c][k][j] of render_sun's 45x3x4x6 table: channels 0 and 1
// interleaved at 2 j + c (the pairs a packed FMA takes), channel 2 at 12 + j, padded to
// 20 floats (five 16-byte slots).  One k step reads them as 4 ds_read_b128 + 1
// ds_read_b64 (18 LDS-array cycles) instead of 6 12-byte reads of padded (S0, S1, S2, 0)
// rows (48 cycles: ds_read_b96 services 8 lanes per cycle).  Same Horner order per
// channel as render_sun_rgb_compact (bitwise the same values).
constexpr int kSunRowFloats = 20;
#ifndef SS_SUN_ROWS_LDS   // probe builds: rows held in LDS (<= kSunRowsStaged; lanes past them read the table)
#define SS_SUN_ROWS_LDS kSunRowsStaged
#endif
constexpr int kSunRowsLds = SS_SUN_ROWS_LDS;
static_assert(kSunRowsLds <= kSunRowsStaged, "LDS rows");
struct SunRowsRgb {
    float4 r[kSunRowsLds][kNbSunCtrlPts][kSunRowFloats / 4];
};

__device__ __forceinline__ void stage_sun_rows(const SunskyKArgs& K, SunRowsRgb* s) {
    constexpr int per_row = kNbSunCtrlPts * kNbSunLdParams;
    constexpr int per_k = kSunRowFloats;
    float* dst = reinterpret_cast<float*>(s->r);
    for (int e = threadIdx.x; e < kSunRowsLds * kNbSunCtrlPts * per_k; e += blockDim.x) {
        const int row = e / (kNbSunCtrlPts * per_k), k = (e / per_k) % kNbSunCtrlPts, f = e % per_k;
        const int pos = min(K.sun_row_lo + row, kNbSunSegments - 1);
        const int j = f < 12 ? f >> 1 : f - 12, c = f < 12 ? f & 1 : 2;
        dst[e] = j < kNbSunLdParams ? K.sun_table[pos * 3 * per_row + c * per_row + k * kNbSunLdParams + j] : 0.f;
    }
}

// HOIST: the 4 control-point rows unrolled with no scheduling barrier, so their LDS reads
// can be issued ahead of the Horner steps (callers with VGPRs to spare: the sorted RGB
// sampler runs at 4 waves/SIMD, held there by its LDS, with ~35 VGPRs below the 4-wave cap).
template <bool HOIST = false>
__device__ __forceinline__ void render_sun_rgb_rows(const SunRowsRgb& R, int row, float x, float cpsi,
                                                    float out[3]) {
    static_assert(kNbSunLdParams == 6 && kSunRowFloats == 20, "row slots: 12 pair values, 6 channel-2 values, 2 pad");
    float r0 = 0.f, r1 = 0.f, r2 = 0.f;
    constexpr int kUnroll = HOIST ? 2 : 1;
#pragma unroll kUnroll
    for (int k = kNbSunCtrlPts - 1; k >= 0; --k) {
        const float4* q = R.r[row][k];
        float v[kSunRowFloats];
        constexpr int J = kNbSunLdParams - 1;
#pragma unroll
        for (int i = 3; i < kSunRowFloats / 4; ++i) {
            const float4 b = q[i];
            v[4 * i] = b.x; v[4 * i + 1] = b.y; v[4 * i + 2] = b.z; v[4 * i + 3] = b.w;
        }
        float i2 = v[12 + J];
#pragma unroll
        for (int j = J - 1; j >= 0; --j) i2 = fmaf(i2, cpsi, v[12 + j]);
        // Channel 2 first, then the pairs, with the scheduler held between them: without the
        // barrier it hoists all five reads (and more around them) and the callers' register
        // peaks rise (direct_conductor 0 -> 19 spilled VGPRs, the sorted sampler 96 -> 111).
        if constexpr (!HOIST) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float4 b = q[i];
            v[4 * i] = b.x; v[4 * i + 1] = b.y; v[4 * i + 2] = b.z; v[4 * i + 3] = b.w;
        }
        float i0 = v[2 * J], i1 = v[2 * J + 1];
#pragma unroll
        for (int j = J - 1; j >= 0; --j) {
            i0 = fmaf(i0, cpsi, v[2 * j]);
            i1 = fmaf(i1, cpsi, v[2 * j + 1]);
        }
        r0 = fmaf(r0, x, i0);
        r1 = fmaf(r1, x, i1);
        r2 = fmaf(r2, x, i2);
    }
    out[0] = r0;
    out[1] = r1;
    out[2] = r2;
}

// Full RGB eval for one local direction (sunsky.cpp:317-323).
// chans: the 3 channels (K.fsky / K.sky, or an LDS copy in the sampling kernels,
// whose other constants already fill the SGPR file).
// SUN (FAST only): kSunF32 the fp32 disc term (the samplers and callers), kSunF64 the fp64
// disc term (the eval kernels: eval, eval_direction, the bake), kSunNone none (*hit reports
// the disc test).
enum { kSunF32 = 0, kSunF64 = 1, kSunNone = 2 };

template <bool FAST, bool HOIST = false, int SUN = kSunF32>
__device__ __forceinline__ void eval_rgb_local(const SunskyKArgs& K, const typename ChanSel<FAST>::T* chans,
                                               const float* sun_tab, float3_ wo, bool mask, float out[3],
                                               const SunRowsRgb* rows = nullptr, bool* hit = nullptr) {
    DirTerms t = dir_terms<FAST>(K, wo, mask);
    if constexpr (FAST) {
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = sky_fast(chans[c], t);   // sky_scale and CIE folded
        if (hit) *hit = t.hit_sun;
        if constexpr (SUN == kSunNone) {
        } else if constexpr (SUN == kSunF64) {
            if (t.hit_sun) {
                const SunskyKArgs& Kf = opaque_kargs(K);   // the disc constants loaded in the branch
                const SunDisc64 d = sun_disc64(Kf, t.wx, t.wy, t.cos_theta);
#pragma unroll 1
                for (int c = 0; c < 3; ++c) out[c] = add_sun_rgb64(Kf, d, c, out[c]);
            }
        } else if (t.hit_sun) {
            add_sun_terms<true>(K, t);
            const int row = t.sun_pos - K.sun_row_lo;
            if (rows && row >= 0 && row < kSunRowsLds) {
                float sr[3];
                render_sun_rgb_rows<HOIST>(*rows, row, t.sun_x, t.sun_cpsi, sr);
#pragma unroll
                for (int c = 0; c < 3; ++c) out[c] += K.sun_mul * sr[c];
            } else {
#pragma unroll 1
                for (int c = 0; c < 3; ++c)
                    out[c] += K.sun_mul * render_sun_rgb_compact(sun_tab, t.sun_pos, c, t.sun_x, t.sun_cpsi);
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = t.active ? out[c] : 0.f;
    } else {
        const float cie = (float)kCieYNormalization;
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = sky_ref(chans[c], t, K.sky_scale);
        if (t.hit_sun) {
            float xs;
            int pos = sun_segment_ref(K, t.cos_theta, &xs);
            float cpsi = cos_psi(t.gamma, K.inv_sin2_half_ap);
            const float conv = (float)kSpecToRgbSunConv;
#pragma unroll 1
            for (int c = 0; c < 3; ++c)
                out[c] += K.sun_scale * render_sun_rgb(sun_tab, pos, c, xs, cpsi) * K.area_ratio * conv;
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = t.active ? out[c] * cie : 0.f;
    }
}

template <bool FAST, int SUN = kSunF32>
__device__ __forceinline__ void eval_rgb_local(const SunskyKArgs& K, const float* sun_tab, float3_ wo, bool mask,
                                               float out[3], bool* hit = nullptr) {
    eval_rgb_local<FAST, false, SUN>(K, chan_table<FAST>(K), sun_tab, wo, mask, out, nullptr, hit);
}

// Powers of the sun disc's polynomial variables, shared by every wavelength of a lane:
// x^k (render_sun, sunsky.cpp:586-594) and cos psi^j (compute_sun_ld, :631-650), each by
// repeated products as dr::pow(x, k) / powif_ form them.
struct SunPowers {
    float x1, x2, x3;
    float c[kNbSunLdParams];
};

__device__ __forceinline__ SunPowers sun_powers(float x, float cpsi) {
    SunPowers p;
    p.x1 = x;
    p.x2 = p.x1 * p.x1;
    p.x3 = p.x2 * p.x1;
    p.c[0] = 1.f;
    p.c[1] = cpsi;
#pragma unroll
    for (int j = 2; j < kNbSunLdParams; ++j) p.c[j] = p.c[j - 1] * cpsi;
    return p;
}

// render_sun, spectral branch (sunsky.cpp:586-594): sum_k x^k S[pos][c][k] in k order, the
// 4 control points of (pos, c) in one 16-byte read (the table is 16-byte aligned)
__device__ __forceinline__ float sun_spec_poly(const float* table, int pos, int c, const SunPowers& p) {
    const float4 s = *reinterpret_cast<const float4*>(table + (pos * kNbWavelengths + c) * kNbSunCtrlPts);
    return fmaf(p.x3, s.w, fmaf(p.x2, s.z, fmaf(p.x1, s.y, s.x)));
}

// Limb-darkening coefficients of channel c and of c + 1 (c itself for the last channel)
// interleaved, ldp[c][j] = (ld[c][j], ld[c + 1][j]): a channel pair's 12 coefficients in
// three 16-byte LDS reads instead of twelve 4-byte ones.
__device__ __forceinline__ void stage_ld_pairs(const float* ld, float* ldp) {
    for (int e = threadIdx.x; e < kNbWavelengths * 2 * kNbSunLdParams; e += blockDim.x) {
        const int c = e / (2 * kNbSunLdParams), j = (e / 2) % kNbSunLdParams, h = e & 1;
        const int cc = h && c + 1 < kNbWavelengths ? c + 1 : c;
        ldp[e] = ld[cc * kNbSunLdParams + j];
    }
}

// Spectral sun disc term for channel pair (lo, lo + 1, f): lerp(sun) x limb darkening
// (sunsky.cpp:341-347, compute_sun_ld :631-650).  At 720 nm (lo = 10, f = 0) the pair is
// (10, 10): lerpf_ returns its first operand at f = 0, so the reference's weight-0
// channel 11 never enters.
template <bool FAST>
__device__ __forceinline__ float sun_spec_pair(const SunskyKArgs& K, const float* sun_tab, const float* ldp,
                                               int pos, const SunPowers& p, int lo, float f) {
    const int hi = lo + 1 < kNbWavelengths ? lo + 1 : lo;
    const float sun = lerpf_(sun_spec_poly(sun_tab, pos, lo, p), sun_spec_poly(sun_tab, pos, hi, p), f);
    const float4* q = reinterpret_cast<const float4*>(ldp + lo * 2 * kNbSunLdParams);
    float ld = 0.f;
#pragma unroll
    for (int h = 0; h < kNbSunLdParams / 2; ++h) {
        const float4 v = q[h];   // (lo, hi) of coefficients 2h and 2h + 1
        ld = fmaf(p.c[2 * h], lerpf_(v.x, v.y, f), ld);
        ld = fmaf(p.c[2 * h + 1], lerpf_(v.z, v.w, f), ld);
    }
    return FAST ? K.sun_mul * (sun * ld) : K.sun_scale * sun * ld * K.area_ratio;
}

// One wavelength's term in the eval kernels, where the disc is rare (~1e-5 of random
// directions) and the VEC=4 bodies keep 4 directions in registers: the rolled render_sun_spec /
// sun_limb_darkening loops.  (sun_spec_pair there lets the compiler schedule the 4 directions'
// table reads together: 70 -> 94 VGPRs in the node kernel, measured statically.)
template <bool FAST>
__device__ __forceinline__ float sun_spec_term(const SunskyKArgs& K, const float* sun_tab, const float* ld_tab,
                                               const DirTerms& t, int lo, float f) {
    const int hi = lo + 1;
    float sa = render_sun_spec(sun_tab, t.sun_pos, lo, t.sun_x), sun = sa;
    if (f != 0.f) sun = lerpf_(sa, hi < kNbWavelengths ? render_sun_spec(sun_tab, t.sun_pos, hi, t.sun_x) : 0.f, f);
    float ld = sun_limb_darkening(ld_tab, lo, hi, f, t.sun_cpsi);
    return FAST ? K.sun_mul * (sun * ld) : K.sun_scale * sun * ld * K.area_ratio;
}

// The eval kernels' spectral disc term of one direction for channel pair (lo, lo + 1, f),
// added to its sky value o: FAST in fp64 (SunDisc64, its constants loaded in the branch),
// the reference kernels in fp32 from add_sun_terms().
template <bool FAST>
__device__ __forceinline__ float spec_disc_add(const SunskyKArgs& K, const DirTerms& t, int lo, float f, float o) {
    if constexpr (FAST) {
        const SunskyKArgs& Kf = opaque_kargs(K);
        return add_sun_spec64(Kf, sun_disc64(Kf, t.wx, t.wy, t.cos_theta), lo, f, o);
    } else {
        return o + sun_spec_term<false>(K, K.sun_table, K.sun_ld, t, lo, f);
    }
}

// Spectral eval of one per-lane wavelength (sunsky.cpp:325-348); `chans` is
// indexed by a per-lane channel, so it lives in LDS.  `t` carries add_sun_terms().
template <bool FAST>
__device__ __forceinline__ float eval_spec_one(const SunskyKArgs& K, const typename ChanSel<FAST>::T* chans,
                                               const float* sun_tab, const float* ld_tab, const DirTerms& t,
                                               float lambda) {
    float nw = wavelength_node(lambda);
    bool valid = (0.f <= nw) && (nw <= (float)(kNbWavelengths - 1));
    if (!(t.active && valid)) return 0.f;
    int lo = (int)floorf(nw), hi = lo + 1;
    float f = nw - (float)lo;
    float res = sky_eval<FAST>(chans[lo], t, K.sky_scale);
    if (f != 0.f) res = lerpf_(res, hi < kNbWavelengths ? sky_eval<FAST>(chans[hi], t, K.sky_scale) : 0.f, f);
    if (t.hit_sun) res += sun_spec_term<FAST>(K, sun_tab, ld_tab, t, lo, f);
    return res;
}

// eval_spec_one without per-wavelength branches on the sky side (the per-ray kernels, where
// random wavelengths almost never sit on a node): the channel pair clamped to (lo, lo + 1)
// with lo <= 9 and f in [0, 1], both sky evaluations always, as eval_spec4 does -- lerpf_
// returns its operands exactly at f = 0 and f = 1, so a node and 720 nm give eval_spec_one's
// bits -- and the sun term in the one rare branch with eval_spec_one's own (lo, f).
// SUN as eval_rgb_local's: kSunF32 (t carries add_sun_terms), kSunF64 (the eval kernels' fp64
// disc term, spec_disc_add), kSunNone (no disc term).
template <bool FAST, int SUN = kSunF32>
__device__ __forceinline__ float eval_spec_one_flat(const SunskyKArgs& K, const typename ChanSel<FAST>::T* chans,
                                                    const float* sun_tab, const float* ld_tab, const DirTerms& t,
                                                    float lambda) {
    const float nw = wavelength_node(lambda);
    const bool ok = t.active && (0.f <= nw) && (nw <= (float)(kNbWavelengths - 1));
    const int c = ok ? (int)floorf(nw) : 0;
    const int lo = c < kNbWavelengths - 2 ? c : kNbWavelengths - 2;
    const float f = ok ? nw - (float)lo : 0.f;
    float res = lerpf_(sky_eval<FAST>(chans[lo], t, K.sky_scale), sky_eval<FAST>(chans[lo + 1], t, K.sky_scale), f);
    if constexpr (SUN == kSunF64) {
        if (t.hit_sun && ok) res = spec_disc_add<true>(K, t, c, nw - (float)c, res);
    } else if constexpr (SUN == kSunF32) {
        if (t.hit_sun && ok) res += sun_spec_term<FAST>(K, sun_tab, ld_tab, t, c, nw - (float)c);
    }
    return ok ? res : 0.f;
}

// ------------------------------------------------------------ memory helpers
template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, size_t i, float v[VEC]) {
    if constexpr (VEC == 4) {
        f32x4 q = *reinterpret_cast<const f32x4*>(p + i);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else if constexpr (VEC == 2) {
        f32x2 q = *reinterpret_cast<const f32x2*>(p + i);
        v[0] = q.x; v[1] = q.y;
    } else {
        v[0] = p[i];
    }
}

// Work split of the per-ray spectral eval and the node kernel: workgroup b walks the contiguous
// span of `span_steps` steps of blockDim x VEC directions starting at step b x steps, instead of
// a grid-stride loop.  Beyond one step per lane (batches over ~16M directions at 64 workgroups
// per CU) each workgroup then writes contiguous 16 KB+ runs per plane: at 64M the per-ray
// spectral eval 1.09-1.11x and the node kernel 1.05-1.09x faster, equal at 16M (interleaved
// A/B, profiles/r05_v11_ab_span_split.log, r05_v12_ab_span_split_rays_nodes.log).  The headline
// RGB eval keeps its grid-stride loop: in this form it measured 4 % slower at 16M (one step per
// lane; tools/mk_probe.py rgb_span) and equal at 64M.  The step count
// is uniform: 1 without a 64-bit division for batches the grid covers in one step.  Two or
// more steps give the one-step split's bits (tests/test_gpu_span.py).
__device__ __forceinline__ size_t span_steps(size_t nvec) {
    const size_t lanes = (size_t)gridDim.x * blockDim.x;
    return nvec <= lanes ? 1 : (nvec + lanes - 1) / lanes;
}

// Outputs are written once and not re-read by this kernel: non-temporal.
template <int VEC>
__device__ __forceinline__ void store_vec(float* p, size_t i, const float v[VEC]) {
    if constexpr (VEC == 4) {
        f32x4 q = {v[0], v[1], v[2], v[3]};
        __builtin_nontemporal_store(q, reinterpret_cast<f32x4*>(p + i));
    } else if constexpr (VEC == 2) {
        f32x2 q = {v[0], v[1]};
        __builtin_nontemporal_store(q, reinterpret_cast<f32x2*>(p + i));
    } else {
        __builtin_nontemporal_store(v[0], p + i);
    }
}

// One non-temporal fp32 store (the per-sample kernels).
__device__ __forceinline__ void store_nt(float v, float* p) {
    __builtin_nontemporal_store(v, p);
}

template <int VEC>
__device__ __forceinline__ void load_mask(const uint8_t* m, size_t i, bool v[VEC]) {
    if (!m) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = true;
        return;
    }
    if constexpr (VEC == 4) {
        uint32_t q = *reinterpret_cast<const uint32_t*>(m + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = ((q >> (8 * j)) & 0xFF) != 0;
    } else if constexpr (VEC == 2) {
        uint16_t q = *reinterpret_cast<const uint16_t*>(m + i);
        v[0] = (q & 0xFF) != 0;
        v[1] = (q >> 8) != 0;
    } else {
        v[0] = m[i] != 0;
    }
}

template <int VEC>
__device__ __forceinline__ void load_dirs(const float* wx, const float* wy, const float* wz, const uint8_t* active,
                                          size_t i, float x[VEC], float y[VEC], float z[VEC], bool m[VEC]) {
    load_vec<VEC>(wx, i, x);
    load_vec<VEC>(wy, i, y);
    load_vec<VEC>(wz, i, z);
    load_mask<VEC>(active, i, m);
}

// ======================================================================
// eval(): RGB.  out plane c at out + c * ostride.  sign = -1 for eval(si)
// (local_wo = M^-1 (-si.wi)), +1 for eval_direction (wi = -ds.d).
// ======================================================================
template <int VEC, bool FAST, bool NEG>
__device__ __forceinline__ void eval_rgb_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                              const float* __restrict__ wy, const float* __restrict__ wz,
                                              const uint8_t* __restrict__ active, size_t n,
                                              float* __restrict__ out, size_t ostride) {
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC], r[VEC], g[VEC], b[VEC];
        bool m[VEC];
        load_dirs<VEC>(wx, wy, wz, active, i, x, y, z, m);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            float o[3];
            // FAST: the disc term in fp64 (SunDisc64)
            eval_rgb_local<FAST, FAST ? kSunF64 : kSunF32>(K, K.sun_table, to_local(K, flip3<NEG>(x[j], y[j], z[j])), m[j], o);
            r[j] = o[0]; g[j] = o[1]; b[j] = o[2];
        }
        store_vec<VEC>(out, i, r);
        store_vec<VEC>(out + ostride, i, g);
        store_vec<VEC>(out + 2 * ostride, i, b);
    }
}

// ======================================================================
// Tables staged in LDS once per workgroup.  Constants that every lane reads
// with the same index could live in SGPRs, but 11 spectral channels (110
// floats), 20 TGMM gaussians or a CDF exceed the SGPR file: the compiler then
// spills them through v_writelane / v_readlane + s_nop hazards inside the hot
// loop (measured: 696 readlanes in the first sample_direction kernel).  LDS
// reads with one address per wave are broadcasts, cheap and conflict-free.
// ======================================================================
template <typename T>
__device__ __forceinline__ void lds_copy(T* dst, const T* src, int count) {
    const int nwords = (int)(count * sizeof(T) / 4);
    const float* s = reinterpret_cast<const float*>(src);
    float* d = reinterpret_cast<float*>(dst);
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) d[w] = s[w];
}

template <bool FAST> struct ChanLds { typename ChanSel<FAST>::T c[kNbWavelengths]; };

template <bool FAST>
__device__ __forceinline__ const typename ChanSel<FAST>::T* stage_chans(const SunskyKArgs& K, ChanLds<FAST>* s) {
    lds_copy(s->c, chan_table<FAST>(K), kNbWavelengths);
    return s->c;
}

// ContinuousDistribution over [360, 720] (JIT: 10 nodes, scalar: 2)
struct SpecDistLds { float pdf[10]; float cdf[9]; float pad; };

__device__ __forceinline__ void stage_spec_dist(const SunskyKArgs& K, SpecDistLds* s) {
    lds_copy(s->pdf, K.spec_pdf, 10);
    lds_copy(s->cdf, K.spec_cdf, 9);
}

// ======================================================================
// eval(): spectral, one wavelength set broadcast to every direction (the
// test02/03 eval_full_spec layout and the C3 workload).  Wavelength k maps
// to channels (lo[k], lo[k] + 1, f[k]) computed on the host (wave-uniform).
// out plane k at out + k * ostride.
// ======================================================================
struct LambdaSet {
    int m;
    int lo[kMaxBroadcastLambda];
    float f[kMaxBroadcastLambda];   // < 0: invalid wavelength (output 0)
};

// The broadcast / node kernels' FAST disc lanes: in line in their channel loops the fp64 term
// (four copies, one per direction of a lane) held them to 5-6 waves/SIMD (86 / 80 VGPRs), so a
// lane that met a disc direction walks its steps again after the main loop instead: each
// direction re-read (with its mask byte), its terms and disc test recomputed by the same code
// (the main pass's bits), and for the disc ones each wavelength's sky value as the main pass
// computes it plus the fp64 term stored over the main pass's value (which had none).  The
// re-reads are issued after the main stores, so their waits order those before the overwrite.
// Broadcast list L (lerp factor f < 0: an invalid wavelength, left 0), or the 11 nodes (NODES:
// channel c, f = 0).  The constants come through opaque_kargs, so nothing of this is hoisted
// into registers held across the main loop.
template <int VEC, bool NEG, bool NODES>
__device__ __forceinline__ void fixup_spec_disc(const SunskyKArgs& K, const FastChannel* chans, const LambdaSet& L,
                                                const float* __restrict__ wx, const float* __restrict__ wy,
                                                const float* __restrict__ wz, const uint8_t* __restrict__ active,
                                                size_t i, float* __restrict__ out, size_t ostride) {
#pragma unroll 1
    for (int j = 0; j < VEC; ++j) {
        const SunskyKArgs& Kf = opaque_kargs(K);
        const size_t q = i + j;
        const bool mq = !active || active[q] != 0;
        const DirTerms tj = dir_terms<true>(Kf, to_local(Kf, flip3<NEG>(wx[q], wy[q], wz[q])), mq);
        if (!tj.hit_sun) continue;
        const SunDisc64 d = sun_disc64(Kf, tj.wx, tj.wy, tj.cos_theta);
        const int m = NODES ? kNbWavelengths : L.m;
#pragma unroll 1
        for (int k = 0; k < m; ++k) {
            const int lo = NODES ? k : L.lo[k];
            const float f = NODES ? 0.f : L.f[k];
            if (f < 0.f) continue;
            float o = sky_eval<true>(chans[lo], tj, Kf.sky_scale);
            if (f != 0.f) o = lerpf_(o, lo + 1 < kNbWavelengths ? sky_eval<true>(chans[lo + 1], tj, Kf.sky_scale) : 0.f, f);
            out[(size_t)k * ostride + q] = add_sun_spec64(Kf, d, lo, f, o);
        }
    }
}

template <int VEC, bool FAST, bool NEG>
__device__ __forceinline__ void eval_spec_bcast_body(const SunskyKArgs& K, const LambdaSet& L,
                                                     const float* __restrict__ wx, const float* __restrict__ wy,
                                                     const float* __restrict__ wz, const uint8_t* __restrict__ active,
                                                     size_t n, float* __restrict__ out, size_t ostride) {
    __shared__ ChanLds<FAST> S;
    const auto* chans = stage_chans<FAST>(K, &S);
    __syncthreads();
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    bool had_sun = false;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
        load_dirs<VEC>(wx, wy, wz, active, i, x, y, z, m);
        DirTerms t[VEC];
        bool any_sun = false;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(x[j], y[j], z[j])), m[j]);
            any_sun |= t[j].hit_sun;
        }
        if (!FAST && any_sun) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) add_sun_terms<FAST>(K, t[j]);
        }
        for (int k = 0; k < L.m; ++k) {
            const int lo = L.lo[k];
            const float f = L.f[k];
            float o[VEC];
            if (f < 0.f) {
#pragma unroll
                for (int j = 0; j < VEC; ++j) o[j] = 0.f;
            } else {
                const auto ca = chans[lo];
#pragma unroll
                for (int j = 0; j < VEC; ++j) o[j] = sky_eval<FAST>(ca, t[j], K.sky_scale);
                if (f != 0.f) {
                    if (lo + 1 < kNbWavelengths) {
                        const auto cb = chans[lo + 1];
#pragma unroll
                        for (int j = 0; j < VEC; ++j) o[j] = lerpf_(o[j], sky_eval<FAST>(cb, t[j], K.sky_scale), f);
                    } else {
#pragma unroll
                        for (int j = 0; j < VEC; ++j) o[j] = lerpf_(o[j], 0.f, f);
                    }
                }
                if (!FAST && any_sun) {
#pragma unroll
                    for (int j = 0; j < VEC; ++j)
                        if (t[j].hit_sun) o[j] = spec_disc_add<FAST>(K, t[j], lo, f, o[j]);
                }
#pragma unroll
                for (int j = 0; j < VEC; ++j) o[j] = t[j].active ? o[j] : 0.f;
            }
            store_vec<VEC>(out + (size_t)k * ostride, i, o);
        }
        had_sun |= any_sun;
    }
    if constexpr (FAST) {   // the disc lanes (fixup_spec_disc)
        if (had_sun) {
#pragma unroll 1
            for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride)
                fixup_spec_disc<VEC, NEG, false>(K, chans, L, wx, wy, wz, active, v * VEC, out, ostride);
        }
    }
}

// Broadcast at exactly the 11 model wavelengths 320:40:720 nm (lerp factor 0,
// sunsky.cpp:332-343): channel c -> plane c with compile-time channel indices.
// Work split: span_steps (contiguous spans per workgroup); at configs[4]'s 64M directions per
// GPU (4 steps) each workgroup writes 16 KB contiguous per plane (tools/c5_probe.hip: 3-read /
// 11-write shapes at 64M, cold).  Loading the next step's directions before this step's 11
// stores (through LDS with a counted vmcnt, so the wave does not wait for its own stores)
// measured 1.4 % faster at 64M and 3.6 % slower at 16M (one step per lane): not kept
// (DESIGN.md §3).
template <int VEC, bool FAST, bool NEG>
__device__ __forceinline__ void eval_spec_nodes_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                                     const float* __restrict__ wy, const float* __restrict__ wz,
                                                     const uint8_t* __restrict__ active, size_t n,
                                                     float* __restrict__ out, size_t ostride) {
    __shared__ ChanLds<FAST> S;
    const auto* chans = stage_chans<FAST>(K, &S);
    __syncthreads();
    const size_t nvec = n / VEC, G = span_steps(nvec);
    bool had_sun = false;
    {
#pragma unroll 1
      for (size_t g = 0; g < G; ++g) {
        const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;
        if (v >= nvec) break;
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
        load_dirs<VEC>(wx, wy, wz, active, i, x, y, z, m);
        DirTerms t[VEC];
        bool any_sun = false;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(x[j], y[j], z[j])), m[j]);
            any_sun |= t[j].hit_sun;
        }
        if (!FAST && any_sun) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) add_sun_terms<FAST>(K, t[j]);
        }
        // Rolled: one channel's constants (LDS broadcast reads) live at a time;
        // unrolling lets the compiler hoist all 110 out of the ray loop (184 VGPRs).
#pragma unroll 1
        for (int c = 0; c < kNbWavelengths; ++c) {
            const auto ch = chans[c];
            float o[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) o[j] = sky_eval<FAST>(ch, t[j], K.sky_scale);
            if (!FAST && any_sun) {
#pragma unroll
                for (int j = 0; j < VEC; ++j)
                    if (t[j].hit_sun) o[j] = spec_disc_add<FAST>(K, t[j], c, 0.f, o[j]);
            }
#pragma unroll
            for (int j = 0; j < VEC; ++j) o[j] = t[j].active ? o[j] : 0.f;
            store_vec<VEC>(out + (size_t)c * ostride, i, o);
        }
        had_sun |= any_sun;
      }
    }
    if constexpr (FAST) {   // the disc lanes (fixup_spec_disc)
        if (had_sun) {
            const LambdaSet none = {};
#pragma unroll 1
            for (size_t g = 0; g < G; ++g) {
                const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;
                if (v >= nvec) break;
                fixup_spec_disc<VEC, NEG, true>(K, chans, none, wx, wy, wz, active, v * VEC, out, ostride);
            }
        }
    }
}

// ======================================================================
// eval(): spectral with per-ray wavelengths (Mitsuba Spectrum<Float, k>):
// lambda plane k at lam + k * lstride, out plane k at out + k * ostride.
// ======================================================================
template <int VEC, bool FAST, bool NEG, int NL = 0>
__device__ __forceinline__ void eval_spec_rays_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                                    const float* __restrict__ wy, const float* __restrict__ wz,
                                                    const float* __restrict__ lam, size_t lstride, int nlam,
                                                    const uint8_t* __restrict__ active, size_t n,
                                                    float* __restrict__ out, size_t ostride) {
    __shared__ ChanLds<FAST> S;
    const auto* chans = stage_chans<FAST>(K, &S);
    __syncthreads();
    // NL > 0: the wavelength count as a compile-time constant (the rays4 kernels, Mitsuba's
    // Spectrum<Float, 4>): the chunk loop and its bounds fold away (4.4 % faster,
    // profiles/r04_v15_ab_rays_nl4.log)
    if constexpr (NL > 0) nlam = NL;
    const size_t nvec = n / VEC, G = span_steps(nvec);
    for (size_t gs = 0; gs < G; ++gs) {
        const size_t v = ((size_t)blockIdx.x * G + gs) * blockDim.x + threadIdx.x;
        if (v >= nvec) break;
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
        load_dirs<VEC>(wx, wy, wz, active, i, x, y, z, m);
        // wavelengths in chunks of 4 planes (Mitsuba's Spectrum<Float, 4> is one chunk):
        // every load of a chunk is issued before its first use
        float l4[4][VEC];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < nlam) load_vec<VEC>(lam + (size_t)k * lstride, i, l4[k]);
        DirTerms t[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(x[j], y[j], z[j])), m[j]);
            if constexpr (!FAST) add_sun_terms<FAST>(K, t[j]);
        }
        for (int k0 = 0; k0 < nlam; k0 += 4) {
            if (k0 > 0) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k0 + k < nlam) load_vec<VEC>(lam + (size_t)(k0 + k) * lstride, i, l4[k]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k0 + k >= nlam) break;
                float o[VEC];
#pragma unroll
                for (int j = 0; j < VEC; ++j)
                    o[j] = eval_spec_one_flat<FAST, FAST ? kSunF64 : kSunF32>(K, chans, K.sun_table, K.sun_ld, t[j], l4[k][j]);
                store_vec<VEC>(out + (size_t)(k0 + k) * ostride, i, o);
            }
        }
    }
}

// ======================================================================
// Sampling: TGMM sky + uniform-cone sun (sunsky.cpp:354-451, 661-763)
// ======================================================================
// TGMM tables in LDS.  tp holds the FAST form of tgmm_pdf's per-gaussian terms
// for PAIRS of gaussians (g, g + 1), so one 40-byte LDS read serves two terms:
//   sx = fma(phi, k_phi, m_phi),  sy = fma(theta, k_theta, m_theta),
//   pdf += c exp2(-(sx^2 + sy^2)),
// with k = sqrt(log2(e) / 2) / sigma, m = -RN(mu k) and c = weight / (volume * 2 pi), one
// fma per gaussian in mixture order.  The fma form (one instruction per coordinate instead
// of a subtraction and a product) is as accurate as the product form: over 2M directions
// at the C4 mixture both stay within 7.3e-7 of the fp64 sum (fma 4.8e-7, product 7.3e-7;
// they differ by at most 7.6e-7).  mphi / mth hold m.  An odd count is padded with a zero gaussian
// (k = 0, c = 0: fma(0, exp2(-0), pdf) = pdf exactly).  Scalar FP32 on purpose:
// on gfx950 v_fma_f32 issues in ~2.6 cycles per wave and v_pk_fma_f32 in ~4.7
// (tools/valu_probe.hip), so packing two lanes' work gains nothing.
// tp/tref hold only the K.tgmm_count gaussians with a non-zero coefficient
// (SunskyKArgs::tgmm_idx), so tgmm_pdf loops over those.
struct TgPair {
    f32x2 mphi, mth, kphi, kth, c;
};

template <bool FAST>
struct TgmmLds {
    Gaussian gauss[kNbMixture];                  // full mixture: sample_sky
    TgPair tp[kNbMixture / 2];
    Gaussian tref[FAST ? 1 : kNbMixture];        // compacted, reference-order tgmm_pdf (_ref kernels)
    float cdf[kNbMixture], pmf[kNbMixture];
    float inv_pmfn[kNbMixture];                  // 1 / RN(pmf * gauss_norm) (div_by_rcp)
    uint8_t guide[kGaussGuideSize];
};

template <bool FAST>
__device__ __forceinline__ void stage_tgmm(const SunskyKArgs& K, TgmmLds<FAST>* s) {
    lds_copy(s->gauss, K.gauss, kNbMixture);
    lds_copy(s->cdf, K.gauss_cdf, kNbMixture);
    lds_copy(s->pmf, K.gauss_pmf, kNbMixture);
    lds_copy(reinterpret_cast<uint32_t*>(s->guide), reinterpret_cast<const uint32_t*>(K.gauss_guide),
             kGaussGuideSize / 4);
    const int i = threadIdx.x;
    if (i < kNbMixture) s->inv_pmfn[i] = 1.f / (K.gauss_pmf[i] * K.gauss_norm);
    if (i < kNbMixture) {
        const float c = 0.84932180028801904272f;   // sqrt(log2(e) / 2)
        float* pair = reinterpret_cast<float*>(&s->tp[i >> 1]) + (i & 1);
        if (i < K.tgmm_count) {
            const Gaussian& g = K.gauss[K.tgmm_idx[i]];
            const float kp = g.inv_sigma_phi * c, kt = g.inv_sigma_theta * c;
            pair[0] = -(g.mu_phi * kp);
            pair[2] = -(g.mu_theta * kt);
            pair[4] = kp;
            pair[6] = kt;
            pair[8] = g.coef * kInvTwoPi;
            if constexpr (!FAST) s->tref[i] = g;
        } else {
            pair[0] = pair[2] = pair[4] = pair[6] = pair[8] = 0.f;
        }
    }
}

// Only what the variant reads: RGB keeps 3 sky channels and no spectral tables, the
// fast kernels no reference-order gaussians.
template <bool FAST, int N> struct ChanLdsN { typename ChanSel<FAST>::T c[N]; };

// The 11 FAST spectral channels as a structure of arrays for the samplers' per-lane gathers
// (4 wavelengths x 2 channels per sample).  Gathered from the 48-byte FastChannel records the
// compiler split each gather into ds_read_b128 + ds_read_b96 + ds_read2_b32 (or a
// ds_read2_b64 merging channels lo and lo + 1), whose banks are (a/4) mod 32: records 8
// channels apart share them, a bank conflict whenever a lane group holds channels c and c + 8
// (1.01e8 SQ_LDS_BANK_CONFLICT cycles per dispatch).  Here the parts are 16, 16
// and 8 bytes at strides of 4, 4 and 2 dwords: the 11 channels of a part span 44 (b128, banks
// mod 64) and 22 dwords (< 32), so every gather is conflict-free in any banking.
struct FastChanSoA {
    f32x4 q0[kNbWavelengths];   // A, Bl2, El2, P
    f32x4 q1[kNbWavelengths];   // Q, Cs, Ds, Fs
    f32x2 q2[kNbWavelengths];   // Gs, Hs
};

__device__ __forceinline__ FastChannel chan_get(const FastChanSoA* s, int c) {
    const f32x4 a = s->q0[c], b = s->q1[c];
    const f32x2 d = s->q2[c];
    FastChannel k;
    k.A = a.x; k.Bl2 = a.y; k.El2 = a.z; k.P = a.w;
    k.Q = b.x; k.Cs = b.y; k.Ds = b.z; k.Fs = b.w;
    k.Gs = d.x; k.Hs = d.y; k.pad[0] = k.pad[1] = 0.f;
    return k;
}

__device__ __forceinline__ void stage_chan_soa(const FastChannel* src, FastChanSoA* s) {
    for (int c = threadIdx.x; c < kNbWavelengths; c += blockDim.x) {
        const FastChannel& k = src[c];
        s->q0[c] = f32x4{k.A, k.Bl2, k.El2, k.P};
        s->q1[c] = f32x4{k.Q, k.Cs, k.Ds, k.Fs};
        s->q2[c] = f32x2{k.Gs, k.Hs};
    }
}

template <bool FAST, bool SPEC>
struct SamplerLds {
    TgmmLds<FAST> tgmm;
    ChanLdsN<FAST, SPEC ? kNbWavelengths : 3> chans;   // spectral: per-lane channel index
    FastChanSoA chsoa[FAST && SPEC ? 1 : 0];           // FAST spectral: the same channels, SoA (gathers)
    SpecDistLds sdist[SPEC ? 1 : 0];
    alignas(16) float sun[SPEC ? kSunSpecTableSize : 0];   // spectral: the whole turbidity-lerped table
    SunRowsRgb rows[SPEC ? 0 : 1];                 // RGB: the disc's segments, channels interleaved
    float ld[SPEC ? kNbWavelengths * kNbSunLdParams : 0];
    alignas(16) float ldp[SPEC ? kNbWavelengths * 2 * kNbSunLdParams : 0];   // spectral: LdPairs layout
};

template <bool FAST, bool SPEC>
__device__ __forceinline__ void stage_sampler_lds(const SunskyKArgs& K, SamplerLds<FAST, SPEC>* s) {
    stage_tgmm<FAST>(K, &s->tgmm);
    lds_copy(s->chans.c, chan_table<FAST>(K), SPEC ? kNbWavelengths : 3);
    if constexpr (FAST && SPEC) stage_chan_soa(K.fsky, s->chsoa);
    if constexpr (SPEC) {
        stage_spec_dist(K, &s->sdist[0]);
        lds_copy(s->ld, K.sun_ld, kNbWavelengths * kNbSunLdParams);
        stage_ld_pairs(K.sun_ld, s->ldp);
    }
    if constexpr (SPEC) lds_copy(s->sun, K.sun_table, kSunSpecTableSize);
    else stage_sun_rows(K, s->rows);
    __syncthreads();
}

// The channel table the spectral samplers gather from per lane: the SoA form in FAST.
template <bool FAST, bool SPEC>
__device__ __forceinline__ auto chan_src(const SamplerLds<FAST, SPEC>& S) {
    if constexpr (FAST && SPEC) return &S.chsoa[0];
    else return &S.chans.c[0];
}

// DiscreteDistribution::sample_reuse (distr_1d.h:173-183): JIT predicate
// ((cdf < s) || cdf == 0) && cdf != sum over [0, n-1) (:116-136), scalar
// variants search [first, last] with cdf < s.  Both predicates are true on a
// prefix of the entries and monotone in s, so the index is a prefix count that
// starts from the host's guide-table bound for the sample's bucket
// (SunskyKArgs::gauss_guide) and tests at most gauss_guide_span further entries:
// the same result as the full scan, ~1-2 LDS reads per lane instead of 19.
template <bool FAST>
__device__ __forceinline__ int discrete_sample_reuse(const SunskyKArgs& K, const TgmmLds<FAST>& T, float value,
                                                     float* reused) {
    const float s = value * K.gauss_sum;
    const bool jit = K.semantics == kJit;
    const int end = jit ? kNbMixture - 1 : K.gauss_last;
    auto pred = [&](int j) {
        const float c = T.cdf[j < kNbMixture ? j : kNbMixture - 1];
        return j < end && (jit ? (((c < s) || c == 0.f) && (c != K.gauss_sum)) : (c < s));
    };
    int idx;
    if (value >= 0.f && value < 1.f) {
        // the predicate (and j < end) holds on a prefix of the entries, and the answer lies
        // in [guide, guide + span]: the index is guide + the number of true tests among
        // the span entries.  A wave-uniform trip count with no early exit: no divergent
        // loop, no exec-mask bookkeeping.
        const int g = T.guide[(int)(value * (float)kGaussGuideSize)];
        int add = 0;
#pragma unroll 1
        for (int k = 0; k < K.gauss_guide_span; ++k) add += pred(g + k) ? 1 : 0;
        idx = g + add;
    } else {   // outside [0, 1) (or NaN): the full search
        idx = jit ? 0 : K.gauss_first;
#pragma unroll 1
        for (int k = 0; k < kNbMixture; ++k) {
            if (!pred(idx)) break;
            ++idx;
        }
    }
    const float pmf = T.pmf[idx];
    const float cdf_prev = idx > 0 ? T.cdf[idx - 1] : 0.f;
    // eval_cdf_normalized / eval_pmf_normalized are rounded products of their own in the
    // reference (distr_1d.h:179-182): no fma contraction of the numerator, whose
    // rounding the near-pole erfinv of the reused sample amplifies
    float num;
    {
#pragma clang fp contract(off)
        num = value - cdf_prev * K.gauss_norm;
    }
    *reused = div_exact<FAST>(num, pmf * K.gauss_norm, T.inv_pmfn[idx]);
    return idx;
}

// sphdir(theta, phi) with shared sin/cos reductions
template <bool FAST>
__device__ __forceinline__ float3_ sphdir_dev(float theta, float phi) {
    float st, ct, sp, cp;
    sincos_sel<FAST>(theta, &st, &ct);
    sincos_sel<FAST>(phi, &sp, &cp);
    return mk3(cp * st, sp * st, ct);
}

// sample_sky, sunsky.cpp:661-689
template <bool FAST>
__device__ __forceinline__ float3_ sample_sky(const SunskyKArgs& K, const TgmmLds<FAST>& T, float ux, float uy) {
    float temp;
    int idx = discrete_sample_reuse<FAST>(K, T, ux, &temp);
    const Gaussian& g = T.gauss[idx];
    float sx = lerpf_(g.cdf_a_phi, g.cdf_b_phi, temp);
    float sy = lerpf_(g.cdf_a_theta, g.cdf_b_theta, uy);
    sx = fminf(fmaxf(sx, kEpsilon), kOneMinusEpsilon);
    sy = fminf(fmaxf(sy, kEpsilon), kOneMinusEpsilon);
    const float ex = FAST ? erfinv_fast(2.f * sx - 1.f) : erfinvf_(2.f * sx - 1.f);
    const float ey = FAST ? erfinv_fast(2.f * sy - 1.f) : erfinvf_(2.f * sy - 1.f);
    float phi = kSqrtTwo * ex * g.sigma_phi + g.mu_phi;
    float theta = kSqrtTwo * ey * g.sigma_theta + g.mu_theta;
    phi += K.sun_phi - 0.5f * kPi;
    theta = fminf(theta, 0.5f * kPi - kEpsilon);
    return sphdir_dev<FAST>(theta, phi);
}

// square_to_uniform_disk_concentric (warp.h:54-90) with one shared sin/cos
// reduction (FAST: v_rcp_f32 division and sincos_fast).
template <bool FAST>
__device__ __forceinline__ void disk_concentric_dev(float sx, float sy, float* px, float* py) {
    float x = fmaf(2.f, sx, -1.f), y = fmaf(2.f, sy, -1.f);
    bool is_zero = (x == 0.f) && (y == 0.f);
    bool q13 = fabsf(x) < fabsf(y);
    float r = q13 ? y : x, rp = q13 ? x : y;
    float phi = fdiv<FAST>(0.25f * kPi * rp, r);
    if (q13) phi = 0.5f * kPi - phi;
    if (is_zero) phi = 0.f;
    float s, c;
    sincos_sel<FAST>(phi, &s, &c);
    *px = r * c;
    *py = r * s;
}

// square_to_uniform_cone (warp.h:533-551)
template <bool FAST>
__device__ __forceinline__ float3_ uniform_cone_dev(float sx, float sy, float cos_cutoff) {
    float px, py;
    disk_concentric_dev<FAST>(sx, sy, &px, &py);
    float omc = 1.f - cos_cutoff;
    float pn = fmaf(px, px, py * py);
    float z = cos_cutoff + omc * (1.f - pn);
    float sc = safe_sqrt_sel<FAST>(omc * (2.f - omc * pn));
    return mk3(px * sc, py * sc, z);
}

// sample_sun, sunsky.cpp:697-701
template <bool FAST>
__device__ __forceinline__ float3_ sample_sun(const SunskyKArgs& K, float ux, float uy) {
    return frame_to_world(mk3(K.sun_s[0], K.sun_s[1], K.sun_s[2]), mk3(K.sun_t[0], K.sun_t[1], K.sun_t[2]),
                          mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]), uniform_cone_dev<FAST>(ux, uy, K.cos_cutoff));
}

// sample_sky (sunsky.cpp:661-689) or sample_sun (:697-701) per lane, with the
// sky's sincos(theta) and the concentric disk's sincos(phi) (warp.h:54-90) as ONE
// call on a per-lane argument: a wave holding both kinds of lanes (nearly every
// wave, ~1 - w_sky of them are sun picks) runs two sincos instead of three.  The
// quotient u.x / w_sky or (u.x - w_sky) / (1 - w_sky) is one div_exact on selected
// operands.  Same functions on the same arguments as sample_sky / sample_sun: bitwise
// the same directions.
template <bool FAST>
__device__ __forceinline__ float3_ sample_sky_or_sun(const SunskyKArgs& K, const TgmmLds<FAST>& T, bool pick_sky,
                                                     float ux, float uy, float inv_w, float inv_w_sun,
                                                     float* sun_a, float* sun_b) {
    const float a = div_exact<FAST>(pick_sky ? ux : ux - K.w_sky, pick_sky ? K.w_sky : 1.f - K.w_sky,
                                    pick_sky ? inv_w : inv_w_sun);
    float arg, phi = 0.f, r = 0.f;
    if (pick_sky) {
        float temp;
        const int idx = discrete_sample_reuse<FAST>(K, T, a, &temp);
        const Gaussian& g = T.gauss[idx];
        float sx = lerpf_(g.cdf_a_phi, g.cdf_b_phi, temp);
        float sy = lerpf_(g.cdf_a_theta, g.cdf_b_theta, uy);
        sx = fminf(fmaxf(sx, kEpsilon), kOneMinusEpsilon);
        sy = fminf(fmaxf(sy, kEpsilon), kOneMinusEpsilon);
        const float ex = FAST ? erfinv_fast(2.f * sx - 1.f) : erfinvf_(2.f * sx - 1.f);
        const float ey = FAST ? erfinv_fast(2.f * sy - 1.f) : erfinvf_(2.f * sy - 1.f);
        phi = kSqrtTwo * ex * g.sigma_phi + g.mu_phi;
        float theta = kSqrtTwo * ey * g.sigma_theta + g.mu_theta;
        phi += K.sun_phi - 0.5f * kPi;
        arg = fminf(theta, 0.5f * kPi - kEpsilon);
    } else {
        const float x = fmaf(2.f, a, -1.f), y = fmaf(2.f, uy, -1.f);
        const bool is_zero = (x == 0.f) && (y == 0.f);
        const bool q13 = fabsf(x) < fabsf(y);
        r = q13 ? y : x;
        const float rp = q13 ? x : y;
        float pd = fdiv<FAST>(0.25f * kPi * rp, r);
        if (q13) pd = 0.5f * kPi - pd;
        arg = is_zero ? 0.f : pd;
    }
    float s1, c1;
    sincos_sel<FAST>(arg, &s1, &c1);
    if (pick_sky) {
        float sp, cp;
        sincos_sel<FAST>(phi, &sp, &cp);
        return mk3(cp * s1, sp * s1, c1);
    }
    // square_to_uniform_cone (warp.h:533-551) of the disk point, then Frame(sun).to_world
    const float px = r * c1, py = r * s1;
    const float omc = 1.f - K.cos_cutoff;
    const float pn = fmaf(px, px, py * py);
    const float z = K.cos_cutoff + omc * (1.f - pn);
    const float sc = safe_sqrt_sel<FAST>(omc * (2.f - omc * pn));
    *sun_a = px * sc;
    *sun_b = py * sc;
    return frame_to_world(mk3(K.sun_s[0], K.sun_s[1], K.sun_s[2]), mk3(K.sun_t[0], K.sun_t[1], K.sun_t[2]),
                          mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]), mk3(*sun_a, *sun_b, z));
}

// The FAST mixture sum of tgmm_pdf at a wrapped (phi, theta), one pair of
// gaussians per iteration, one fma per gaussian in mixture order.
__device__ __forceinline__ float tgmm_sum_fast(const SunskyKArgs& K, const TgmmLds<true>& T, float phi, float theta) {
    float pdf = 0.f;
    const int np = (K.tgmm_count + 1) >> 1;
#pragma unroll 2
    for (int p = 0; p < np; ++p) {
        const TgPair P = T.tp[p];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float sx = fmaf(phi, P.kphi[h], P.mphi[h]), sy = fmaf(theta, P.kth[h], P.mth[h]);
            pdf = fmaf(P.c[h], fast_exp2(-fmaf(sy, sy, sx * sx)), pdf);
        }
    }
    return pdf;
}

// tgmm_pdf, sunsky.cpp:732-763, with the per-gaussian truncation volume hoisted
// to the host (coef = weight / volume); same summation order as the reference.
template <bool FAST>
__device__ __forceinline__ float tgmm_pdf(const SunskyKArgs& K, const TgmmLds<FAST>& T, float phi, float theta,
                                          bool active) {
    phi -= K.sun_phi - 0.5f * kPi;
    phi = phi < 0.f ? phi + kTwoPi : phi;
    phi = phi > kTwoPi ? phi - kTwoPi : phi;
    active = active && (theta >= 0.f) && (theta <= 0.5f * kPi);
    float pdf = 0.f;
    // Partially unrolled so the 20 gaussians' LDS reads are not hoisted out of
    // the ray loop into ~100 VGPRs.
    if constexpr (FAST) {
        pdf = tgmm_sum_fast(K, T, phi, theta);
    } else {
#pragma unroll 4
        for (int i = 0; i < K.tgmm_count; ++i) {
            const Gaussian& g = T.tref[i];
            float sx = (phi - g.mu_phi) * g.inv_sigma_phi, sy = (theta - g.mu_theta) * g.inv_sigma_theta;
            float q = fmaf(sy, sy, sx * sx);
            pdf = fmaf(g.coef, kInvTwoPi * expf(-0.5f * q), pdf);
        }
    }
    return active ? pdf : 0.f;
}

// compute_pdfs, sunsky.cpp:711-723
template <bool FAST>
__device__ __forceinline__ void compute_pdfs(const SunskyKArgs& K, const TgmmLds<FAST>& T, float3_ d, bool check_sun,
                                             bool active, float* sky_pdf, float* sun_pdf) {
    float sin_theta = safe_sqrt_sel<FAST>(fmaf(d.x, d.x, d.y * d.y));
    active = active && (d.z >= 0.f) && (sin_theta != 0.f);
    sin_theta = fmaxf(sin_theta, kEpsilon);
    float phi, theta;
    if constexpr (FAST) {
        phi = atan2_fast(d.y, d.x);
        theta = theta_upper_fast(d);
    } else {
        phi = atan2f(d.y, d.x);
        theta = unit_angle_z(d);
    }
    *sky_pdf = fdiv<FAST>(tgmm_pdf<FAST>(K, T, phi, theta, active), sin_theta);
    float cosg = dot3(mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]), d);
    *sun_pdf = (!check_sun || cosg >= K.cos_cutoff) ? K.sun_pdf : 0.f;
}

// compute_pdfs of a sampled direction (check_sun = pick_sky, sunsky.cpp:415).  FAST sun
// picks take the sky pdf from the host's quadratic fit over the disc at their disc
// coordinates (a, b) when the staging turned it on (SunskyKArgs::sun_sky_fit_on): a sun
// pick's pdf is dominated by (1 - w) sun_pdf, and the fit moves it by < kSunSkyFitTol =
// 1e-7 relative (the host's bound), while the exact path costs the TGMM sum (one exp2 per
// gaussian), atan2, the polar angle and a division per sample.
template <bool FAST>
__device__ __forceinline__ void sample_pdfs(const SunskyKArgs& K, const TgmmLds<FAST>& T, float3_ sd, bool pick_sky,
                                            float sun_a, float sun_b, bool active, float* sky_pdf, float* sun_pdf) {
    if (FAST && !pick_sky && K.sun_sky_fit_on) {
        const float* c = K.sun_sky_fit;
        const float f = fmaf(sun_a, fmaf(c[3], sun_a, fmaf(c[4], sun_b, c[1])), fmaf(sun_b, fmaf(c[5], sun_b, c[2]), c[0]));
        *sky_pdf = active ? f : 0.f;
        *sun_pdf = K.sun_pdf;
        return;
    }
    compute_pdfs<FAST>(K, T, sd, pick_sky, active, sky_pdf, sun_pdf);
}

// ContinuousDistribution::sample_pdf (distr_1d.h:468-499) over [360, 720]
__device__ __forceinline__ float spectral_sample_pdf(const SunskyKArgs& K, const SpecDistLds& D, float sample,
                                                     float* pdf_out) {
    sample *= K.spec_integral;
    const int nint = K.spec_size - 1;
    int idx = 0;
    if (K.semantics == kJit) {
        bool run = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < nint - 1) {
                const float c = D.cdf[i];
                run = run && ((c < sample) || c == 0.f) && (c != K.spec_integral);
                idx += run ? 1 : 0;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i < nint - 1 && D.cdf[i] < sample) idx = i + 1;
    }
    const float y0 = D.pdf[idx], y1 = D.pdf[idx + 1];
    const float c0 = idx > 0 ? D.cdf[idx - 1] : 0.f;
    sample = (sample - c0) * K.spec_inv_interval;
    float t_linear = (y0 - safe_sqrtf_(fmaf(y0, y0, 2.f * sample * (y1 - y0)))) * (1.f / (y0 - y1));
    float t_const = sample * (1.f / y0);
    float t = (y0 == y1) ? t_const : t_linear;
    *pdf_out = fmaf(t, y1 - y0, y0) * K.spec_norm;
    return fmaf((float)idx + t, K.spec_interval, 360.f);
}

// sample_wavelengths, sunsky.cpp:463-480 (spectral: 4 shifted samples, Spectrum<Float, 4>):
// the 4 wavelengths drawn, then the eval at all 4 and the weights eval / pdf (FAST: times
// v_rcp_f32 of the pdf).  EVAL4: one branchless eval (eval_spec4, bitwise eval_spec_one per
// wavelength; ldp in the LdPairs layout), taken by sample_ray (1.26x faster there, interleaved
// A/B); the standalone sample_wavelengths kernel keeps the rolled eval_spec_one (ld_tab plain),
// whose 67 VGPRs hold 7 waves/SIMD (eval_spec4: 121 VGPRs, 7 % slower).
template <bool FAST, class CH>
__device__ __forceinline__ void eval_spec4(const SunskyKArgs& K, const CH* chans, const float* sun_tab,
                                           const float* ldp, const DirTerms& t, const float lam[4], float e[4]);
template <bool FAST, bool EVAL4>
__device__ __forceinline__ void sample_wavelengths_one(const SunskyKArgs& K, const typename ChanSel<FAST>::T* chans,
                                                       const SpecDistLds& D, const float* sun_tab,
                                                       const float* ld, const DirTerms& t, float sample,
                                                       float lam[4], float w[4]) {
    if constexpr (EVAL4) {
        float lpdf[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float s = sample + (float)k / 4.f;   // math::sample_shifted, math.h:408-431
            s = s > 1.f ? s - 1.f : s;
            lam[k] = spectral_sample_pdf(K, D, s, &lpdf[k]);
        }
        float e[4];
        eval_spec4<FAST>(K, chans, sun_tab, ld, t, lam, e);
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = fdiv<FAST>(e[k], lpdf[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float s = sample + (float)k / 4.f;
            s = s > 1.f ? s - 1.f : s;
            float lpdf;
            lam[k] = spectral_sample_pdf(K, D, s, &lpdf);
            w[k] = fdiv<FAST>(eval_spec_one<FAST>(K, chans, sun_tab, ld, t, lam[k]), lpdf);
        }
    }
}

// sample_direction, sunsky.cpp:399-441.  Weight planes: 3 (RGB) or nlam (spectral).
// LEAN: the host found it_p, ds.dist, ds.p and the active mask all NULL (the common
// call, u -> d, pdf, weight); the optional pointers and their branches are compiled
// out, which frees the SGPRs the kernel otherwise spills through v_writelane/v_readlane.
template <bool FAST, class CH>
__device__ __forceinline__ void eval_spec4(const SunskyKArgs& K, const CH* chans, const float* sun_tab,
                                           const float* ldp, const DirTerms& t, const float lam[4], float e[4]);
template <bool FAST, bool SPEC, bool LEAN = false>
__device__ __forceinline__ void sample_direction_body(
    const SunskyKArgs& K, const float* __restrict__ ux, const float* __restrict__ uy,
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ pz,
    const float* __restrict__ lam, size_t lstride, int nlam, const uint8_t* __restrict__ active, size_t n,
    float* __restrict__ dx, float* __restrict__ dy, float* __restrict__ dz, float* __restrict__ pdf,
    float* __restrict__ dist, float* __restrict__ opx, float* __restrict__ opy, float* __restrict__ opz,
    float* __restrict__ weight, size_t wstride) {
    if constexpr (LEAN) {
        px = py = pz = nullptr;
        active = nullptr;
        dist = opx = opy = opz = nullptr;
    }
    __shared__ SamplerLds<FAST, SPEC> S;
    stage_sampler_lds<FAST, SPEC>(K, &S);
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    // the next sample's u is loaded before this one's work, so its HBM latency overlaps the
    // ~500 VALU instructions of a sample: 4.4 % faster, bitwise the same (interleaved A/B,
    // profiles/r02_v6_ab_sample_prefetch.log).  Prefetching pdf_direction's directions
    // measured 3.7 % slower (70 VGPRs: 7 waves/SIMD instead of 8).
    // A sorted form (a workgroup ranks 256-1024 samples sky-first through LDS so only
    // one 64-lane pass per tile runs both branches, outputs staged in LDS) was 5-25 %
    // slower: profiles/r02_v6_ab_sample_prefetch_sorted.log.
    // (the general call's it.p and mask are prefetched the same way: they feed ds.p / ds.dist
    // and the weight after the sample's work)
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    float nx = 0.f, ny = 0.f, npx = 0.f, npy = 0.f, npz = 0.f;
    bool nact = true;
    auto load = [&](size_t j) {
        nx = ux[j];
        ny = uy[j];
        if (active) nact = active[j] != 0;
        if (px) npx = px[j];
        if (py) npy = py[j];
        if (pz) npz = pz[j];
    };
    if (i < n) load(i);
    for (; i < n; i += stride) {
        bool act = nact;
        const float sx = nx, sy = ny;
        const float3_ itp = mk3(npx, npy, npz);
        if (i + stride < n) load(i + stride);
        const bool pick_sky = sx < K.w_sky;
        // sx / w and the reused sample stay correctly rounded even in FAST: the
        // discrete-distribution reuse divides by the picked gaussian's pmf, so one
        // ulp here moves sky directions by up to ~1e-5 (measured).
        float sun_a = 0.f, sun_b = 0.f;
        const float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, sx, sy, inv_w, inv_w_sun, &sun_a, &sun_b);
        act = act && (sd.z >= 0.f);
        float3_ d = to_world(K, sd);
        float skyp, sunp;
        sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
        float pd = lerpf_(sunp, skyp, K.w_sky);
        store_nt(d.x, dx + i);
        store_nt(d.y, dy + i);
        store_nt(d.z, dz + i);
        store_nt(pd, pdf + i);
        if (dist || opx) {
            float3_ rel = mk3(itp.x - K.bs_center[0], itp.y - K.bs_center[1], itp.z - K.bs_center[2]);
            float dd = 2.f * fmaxf(K.bs_radius, sqrtf(dot3(rel, rel)));
            if (dist) store_nt(dd, dist + i);
            if (opx) { store_nt(fmaf(d.x, dd, itp.x), opx + i); store_nt(fmaf(d.y, dd, itp.y), opy + i); store_nt(fmaf(d.z, dd, itp.z), opz + i); }
        }
        // weight = eval(si{wi = -d}) / pdf, zeroed when not finite (sunsky.cpp:430-439)
        float3_ wo = to_local(K, d);
        if constexpr (!SPEC) {
            float e[3];
            eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, wo, act, e, S.rows);
            const float inv_pd = fdiv<FAST>(1.f, pd);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float w = FAST ? e[c] * inv_pd : e[c] / pd;
                store_nt(isfinite(w) ? w : 0.f, weight + (size_t)c * wstride + i);
            }
        } else {
            DirTerms t = dir_terms<FAST>(K, wo, act);
            add_sun_terms<FAST>(K, t);
            const float inv_pd = fdiv<FAST>(1.f, pd);
            if (nlam == 4) {   // Mitsuba's Spectrum<Float, 4>: the LEAN kernel's eval, same bits
                const float l4[4] = {lam[i], lam[lstride + i], lam[2 * lstride + i], lam[3 * lstride + i]};
                float e[4];
                eval_spec4<FAST>(K, chan_src(S), S.sun, S.ldp, t, l4, e);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float w = FAST ? e[k] * inv_pd : e[k] / pd;
                    store_nt(isfinite(w) ? w : 0.f, weight + (size_t)k * wstride + i);
                }
                continue;
            }
            for (int k = 0; k < nlam; ++k) {
                float e = eval_spec_one<FAST>(K, S.chans.c, S.sun, S.ld, t, lam[(size_t)k * lstride + i]);
                float w = FAST ? e * inv_pd : e / pd;
                store_nt(isfinite(w) ? w : 0.f, weight + (size_t)k * wstride + i);
            }
        }
    }
}

// Spectral eval at Mitsuba's 4 per-lane wavelengths (Spectrum<Float, 4>, sunsky.cpp:325-348)
// without per-wavelength branches: the channel pair is clamped to (lo, lo + 1) with lo <= 9
// and f in [0, 1].  lerpf_ (dr::lerp's fma(b, t, fnmadd(a, t, a))) returns a at t = 0 and
// b at t = 1 exactly, so a node (f = 0, where eval_spec_one skips the lerp) and 720 nm
// (lo = 10, f = 0 there; lo = 9, f = 1 here) give eval_spec_one's bits; the sun-disc
// terms of the 4 wavelengths run in one branch per lane.
template <bool FAST, class CH>
__device__ __forceinline__ void eval_spec4(const SunskyKArgs& K, const CH* chans, const float* sun_tab,
                                           const float* ldp, const DirTerms& t, const float lam[4], float e[4]) {
    int lo[4];
    float f[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float nw = wavelength_node(lam[k]);
        ok[k] = t.active && (0.f <= nw) && (nw <= (float)(kNbWavelengths - 1));
        const int c = ok[k] ? (int)floorf(nw) : 0;
        lo[k] = c < kNbWavelengths - 2 ? c : kNbWavelengths - 2;
        f[k] = ok[k] ? nw - (float)lo[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        e[k] = lerpf_(sky_eval<FAST>(chan_get(chans, lo[k]), t, K.sky_scale),
                      sky_eval<FAST>(chan_get(chans, lo[k] + 1), t, K.sky_scale),
                      f[k]);
    if (t.hit_sun) {
        const SunPowers p = sun_powers(t.sun_x, t.sun_cpsi);
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] += sun_spec_pair<FAST>(K, sun_tab, ldp, t.sun_pos, p, lo[k], f[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = ok[k] ? e[k] : 0.f;
}

// LEAN spectral sample_direction with 4 wavelengths per sample (sunsky.cpp:399-441 in the
// spectral variants, Spectrum<Float, 4>): the per-sample work of
// sample_direction_body<FAST, true, true> with the wavelength loop unrolled and branchless
// (eval_spec4), the next sample's u and 4 wavelengths loaded before this one's work, and
// non-temporal stores.  Bitwise the general kernel's outputs.
template <bool FAST>
__device__ __forceinline__ void sample_direction_spec4_body(
    const SunskyKArgs& K, const float* __restrict__ ux, const float* __restrict__ uy, const float* __restrict__ lam,
    size_t lstride, size_t n, float* __restrict__ dx, float* __restrict__ dy, float* __restrict__ dz,
    float* __restrict__ pdf, float* __restrict__ weight, size_t wstride) {
    __shared__ SamplerLds<FAST, true> S;
    stage_sampler_lds<FAST, true>(K, &S);
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    float nx = 0.f, ny = 0.f, nl[4] = {0.f, 0.f, 0.f, 0.f};
    auto load = [&](size_t j) {
        nx = ux[j];
        ny = uy[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) nl[k] = lam[(size_t)k * lstride + j];
    };
    if (i < n) load(i);
    for (; i < n; i += stride) {
        const float sx = nx, sy = ny;
        float l[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) l[k] = nl[k];
        if (i + stride < n) load(i + stride);
        const bool pick_sky = sx < K.w_sky;
        float sun_a = 0.f, sun_b = 0.f;
        const float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, sx, sy, inv_w, inv_w_sun, &sun_a, &sun_b);
        const bool act = sd.z >= 0.f;
        const float3_ d = to_world(K, sd);
        float skyp, sunp;
        sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
        const float pd = lerpf_(sunp, skyp, K.w_sky);
        store_nt(d.x, dx + i);
        store_nt(d.y, dy + i);
        store_nt(d.z, dz + i);
        store_nt(pd, pdf + i);
        DirTerms t = dir_terms<FAST>(K, to_local(K, d), act);
        add_sun_terms<FAST>(K, t);
        float e[4];
        eval_spec4<FAST>(K, chan_src(S), S.sun, S.ldp, t, l, e);
        const float inv_pd = fdiv<FAST>(1.f, pd);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float w = FAST ? e[k] * inv_pd : e[k] / pd;
            store_nt(isfinite(w) ? w : 0.f, weight + (size_t)k * wstride + i);
        }
    }
}

// Orders a wave's own LDS accesses across the phases of a sorted window: an IR-level
// wavefront-scope fence (no instruction on gfx950: a wave's LDS operations execute in
// issue order) plus the scheduling barrier.
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Window storage of the wave-sorted kernels: sky picks at ascending addresses from 0, sun picks
// at descending addresses from W - 1.  A 32-lane group's sky run and sun run then cover
// complementary banks of the 32-bank rows ((a/4) mod 32; W a multiple of 32), so the ranked
// writes, the passes' reads and writes and the un-sort reads are all conflict-free (with both
// classes at ascending addresses the two runs overlapped: up to 2-way conflicts on every row
// access, 2.9e7 SQ_LDS_BANK_CONFLICT cycles per 64M-sample spectral dispatch).  Combined rank
// q (sky picks first) -> address.
__device__ __forceinline__ int win_addr(int q, int nsky, int W) { return q < nsky ? q : (W - 1 + nsky) - q; }

__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// One spectral sample at 4 wavelengths (u, lambda -> d, pdf, 4 weights): the per-sample
// work of sample_direction_spec4_body in the same operation order (bitwise its outputs).
template <bool FAST, int KIND = 0>
__device__ __forceinline__ void sample_one_spec4(const SunskyKArgs& K, const SamplerLds<FAST, true>& S, float sx,
                                                 float sy, const float l[4], float inv_w, float inv_w_sun, float o[8]) {
    const bool pick_sky = KIND == 1 ? true : KIND == 2 ? false : sx < K.w_sky;   // KIND: sample_one_rgb
    float sun_a = 0.f, sun_b = 0.f;
    const float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, sx, sy, inv_w, inv_w_sun, &sun_a, &sun_b);
    const bool act = sd.z >= 0.f;
    const float3_ d = to_world(K, sd);
    float skyp, sunp;
    sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
    const float pd = lerpf_(sunp, skyp, K.w_sky);
    o[0] = d.x; o[1] = d.y; o[2] = d.z; o[3] = pd;
    // scheduler held between the pdf and the eval: 127 -> 124 VGPRs, no spills, 1.7 % faster
    // (profiles/r03_v22_ab_sched_barriers.log)
    __builtin_amdgcn_sched_barrier(0);
    DirTerms t = dir_terms<FAST>(K, to_local(K, d), act);
    add_sun_terms<FAST>(K, t);
    float e[4];
    eval_spec4<FAST>(K, chan_src(S), S.sun, S.ldp, t, l, e);
    const float inv_pd = fdiv<FAST>(1.f, pd);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float w = FAST ? e[k] * inv_pd : e[k] / pd;
        o[4 + k] = isfinite(w) ? w : 0.f;
    }
}

// Wave-sorted spectral LEAN sample_direction at Mitsuba's 4 wavelengths per sample, the
// RGB kernel's windows (sample_direction_sorted_body) for the spectral body: a wave ranks a
// window of 64 R samples sky picks first, runs R passes over the ranked order (only the
// pass holding the sky/sun boundary runs both the TGMM sampling branch and the sun-disc
// terms of 4 wavelengths), and un-sorts the 8 outputs through its LDS rows so the global
// loads and non-temporal stores stay coalesced in sample order.  The 6 inputs (u, 4 lambda)
// and the 8 outputs share the rows: pass p reads its columns' inputs, then writes their
// outputs.  Each sample goes through sample_one_spec4: bitwise the unsorted kernel.
// POS: Mitsuba's unmasked DirectionSample call in the spectral variants (it.p in, ds.dist and ds.p
// out, sunsky.cpp:416-428): ds.dist and ds.p are functions of d and it.p, computed at the store
// stage from it.p read there (the windows' VGPRs and LDS are full: no prefetch); bitwise the
// unsorted general kernel, which takes the same eval_spec4 for 4 wavelengths.
template <bool FAST, int R, bool POS = false>
__device__ __forceinline__ void sample_direction_spec4_sorted_body(
    const SunskyKArgs& K, const float* __restrict__ ux, const float* __restrict__ uy, const float* __restrict__ lam,
    size_t lstride, size_t n, float* __restrict__ dx, float* __restrict__ dy, float* __restrict__ dz,
    float* __restrict__ pdf, float* __restrict__ weight, size_t wstride, const float* __restrict__ px = nullptr,
    const float* __restrict__ py = nullptr, const float* __restrict__ pz = nullptr, float* __restrict__ dist = nullptr,
    float* __restrict__ opx = nullptr, float* __restrict__ opy = nullptr, float* __restrict__ opz = nullptr) {
    constexpr int W = 64 * R;
    __shared__ SamplerLds<FAST, true> S;
    __shared__ float X[SS_BLOCK / 64][8][W];
    stage_sampler_lds<FAST, true>(K, &S);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*Y)[W] = X[wv];
    const float inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / (1.f - K.w_sky));
    const size_t nwin = (n + W - 1) / W;
    const size_t wstep = (size_t)gridDim.x * (SS_BLOCK / 64);
    float na[R], nb[R], nl[4][R];
    auto load_window = [&](size_t w) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = w * W + (size_t)(r * 64 + lane);
            na[r] = i < n ? ux[i] : 1.f;   // past the end: a sun pick, computed and not stored
            nb[r] = i < n ? uy[i] : 0.5f;
#pragma unroll
            for (int k = 0; k < 4; ++k) nl[k][r] = i < n ? lam[(size_t)k * lstride + i] : 500.f;
        }
    };
    size_t w = (size_t)blockIdx.x * (SS_BLOCK / 64) + wv;
    if (w < nwin) load_window(w);
    for (; w < nwin; w += wstep) {
        const size_t base = w * W;
        int slot[R], nsky = 0;
        {
            float a[R], b[R], l[4][R];
            uint64_t m[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                a[r] = na[r];
                b[r] = nb[r];
#pragma unroll
                for (int k = 0; k < 4; ++k) l[k][r] = nl[k][r];
            }
            if (w + wstep < nwin) load_window(w + wstep);
#pragma unroll
            for (int r = 0; r < R; ++r) m[r] = __ballot(a[r] < K.w_sky);
            int psky = 0, psun = 0;   // sky / sun picks of the rows before this one
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool sky = (m[r] >> lane) & 1;
                slot[r] = sky ? psky + lanes_below(m[r]) : (W - 1) - (psun + lanes_below(~m[r]));   // win_addr
                Y[0][slot[r]] = a[r];
                Y[1][slot[r]] = b[r];
#pragma unroll
                for (int k = 0; k < 4; ++k) Y[2 + k][slot[r]] = l[k][r];
                const int c = __popcll(m[r]);
                psky += c;
                psun += 64 - c;
            }
            nsky = psky;
        }
        wave_lds_order();
#pragma unroll 1
        for (int p = 0; p < R; ++p) {
            const int q = win_addr(p * 64 + lane, nsky, W);
            const float l4[4] = {Y[2][q], Y[3][q], Y[4][q], Y[5][q]};
            float o[8];
            sample_one_spec4<FAST>(K, S, Y[0][q], Y[1][q], l4, inv_w, inv_w_sun, o);
#pragma unroll
            for (int k = 0; k < 8; ++k) Y[k][q] = o[k];
        }
        wave_lds_order();
        float* const planes[8] = {dx, dy, dz, pdf, weight, weight + wstride, weight + 2 * wstride, weight + 3 * wstride};
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = base + (size_t)(r * 64 + lane);
            if (i < n) {
#pragma unroll
                for (int k = 0; k < 8; ++k) store_nt(Y[k][slot[r]], planes[k] + i);
                if (POS && (dist || opx)) {   // as sample_direction_body: ds.dist, ds.p
                    const float3_ d = mk3(Y[0][slot[r]], Y[1][slot[r]], Y[2][slot[r]]);
                    const float3_ itp = px ? mk3(px[i], py[i], pz[i]) : mk3(0.f, 0.f, 0.f);
                    const float3_ rel = mk3(itp.x - K.bs_center[0], itp.y - K.bs_center[1], itp.z - K.bs_center[2]);
                    const float dd = 2.f * fmaxf(K.bs_radius, sqrtf(dot3(rel, rel)));
                    if (dist) store_nt(dd, dist + i);
                    if (opx) { store_nt(fmaf(d.x, dd, itp.x), opx + i); store_nt(fmaf(d.y, dd, itp.y), opy + i); store_nt(fmaf(d.z, dd, itp.z), opz + i); }
                }
            }
        }
        wave_lds_order();
    }
}

// One RGB sample (u -> d, pdf, weight), the per-sample work of
// sample_direction_body<FAST, false, LEAN> in the same operation order; `act` is the
// caller's mask (true in the LEAN form).
// KIND: 0 = each lane's own pick (u.x < w_sky); 1 / 2 = a sorted pass known to hold sky /
// sun picks only (the same pick on every lane, so the other branch is compiled out).
template <bool FAST, int KIND = 0, bool HOIST = false>
__device__ __forceinline__ void sample_one_rgb(const SunskyKArgs& K, const SamplerLds<FAST, false>& S, float sx,
                                               float sy, bool act, float inv_w, float inv_w_sun, float o[7]) {
    const bool pick_sky = KIND == 1 ? true : KIND == 2 ? false : sx < K.w_sky;
    float sun_a = 0.f, sun_b = 0.f;
    const float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, sx, sy, inv_w, inv_w_sun, &sun_a, &sun_b);
    act = act && (sd.z >= 0.f);
    const float3_ d = to_world(K, sd);
    float skyp, sunp;
    sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
    const float pd = lerpf_(sunp, skyp, K.w_sky);
    o[0] = d.x; o[1] = d.y; o[2] = d.z; o[3] = pd;
    float e[3];
    eval_rgb_local<FAST, HOIST>(K, S.chans.c, K.sun_table, to_local(K, d), act, e, S.rows);
    const float inv_pd = fdiv<FAST>(1.f, pd);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float w = FAST ? e[c] * inv_pd : e[c] / pd;
        o[4 + c] = isfinite(w) ? w : 0.f;
    }
}

// Wave-sorted RGB sample_direction (sunsky.cpp:399-441).  A wave takes a window of
// 64 R consecutive samples, ranks them sky picks first (ballot + mbcnt, stable), and runs
// R 64-lane passes over the ranked order: only the pass holding the sky/sun boundary runs
// both the TGMM sampling branch and the sun-disc polynomial, the others run one of them.
// The window goes through a wave-private LDS block (no workgroup barrier): each lane
// writes its samples' u (and, FULL, the caller's mask) at their ranks, pass p reads ranks
// [64p, 64p + 64) and writes its 7 outputs back at the same ranks (the rows it just
// consumed), and each lane then reads its own samples' outputs from their ranks, so the
// global loads and the non-temporal stores stay coalesced in sample order.  FULL adds
// the optional it.p / ds.dist / ds.p / mask of the general kernel: ds.dist and ds.p are
// functions of d and it.p, computed after the un-sort from each lane's own it.p.  Each
// sample is computed by sample_one_rgb from its own u: bitwise the outputs of
// sample_direction_body<FAST, false, !FULL>.
// MODE: kSortLean (u -> d, pdf, weight), kSortFull (+ it.p, mask, ds.dist, ds.p; it.p loaded
// before the passes) or kSortPos (Mitsuba's unmasked DirectionSample call: it.p in, ds.dist and
// ds.p out).  kSortPos loads the next window's it.p with its u (its HBM latency overlaps this
// window's passes) and gives up the hoisted sun-row reads for the 12 VGPRs (119 VGPRs, 10 SGPR
// spills): interleaved A/B per 64M samples (profiles/r05_v4_ab_general_call_itp_prefetch.log)
// 946 us against 1011 us with it.p read at the store stage, 1044 us with it.p read before the
// last pass (154 VGPRs), 1028 us for the unsorted general kernel.
constexpr int kSortLean = 0, kSortFull = 1, kSortPos = 2;
template <bool FAST, int R, int MODE>
__device__ __forceinline__ void sample_direction_sorted_body(
    const SunskyKArgs& K, const float* __restrict__ ux, const float* __restrict__ uy,
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ pz,
    const uint8_t* __restrict__ active, size_t n, float* __restrict__ dx, float* __restrict__ dy,
    float* __restrict__ dz, float* __restrict__ pdf, float* __restrict__ dist, float* __restrict__ opx,
    float* __restrict__ opy, float* __restrict__ opz, float* __restrict__ weight, size_t wstride) {
    constexpr bool FULL = MODE == kSortFull;
    constexpr bool POS = MODE == kSortPos;
    if constexpr (MODE == kSortLean) {
        px = py = pz = nullptr;
        dist = opx = opy = opz = nullptr;
    }
    if constexpr (!FULL) active = nullptr;
    constexpr int W = 64 * R;
    // the LEAN form has VGPRs to spare below the 4-wave cap its LDS sets: hoist the sun-row reads
    constexpr bool kHoist = MODE == kSortLean;
    __shared__ SamplerLds<FAST, false> S;
    __shared__ float X[SS_BLOCK / 64][7][W];
    stage_sampler_lds<FAST, false>(K, &S);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*Y)[W] = X[wv];
    const float inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / (1.f - K.w_sky));
    const size_t nwin = (n + W - 1) / W;
    const size_t wstep = (size_t)gridDim.x * (SS_BLOCK / 64);
    // the next window's u (FULL: and mask) is loaded before this window's passes (its HBM
    // latency overlaps them)
    float na[R], nb[R], nm[R];
    float npx[POS ? R : 1], npy[POS ? R : 1], npz[POS ? R : 1];   // POS: the next window's it.p, loaded with its u
    auto load_window = [&](size_t w) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = w * W + (size_t)(r * 64 + lane);
            na[r] = i < n ? ux[i] : 1.f;   // past the end: a sun pick, computed and not stored
            nb[r] = i < n ? uy[i] : 0.5f;
            if (FULL && active) nm[r] = (i < n && active[i] != 0) ? 1.f : 0.f;
            if constexpr (POS) {
                const bool in = (dist || opx) && px && i < n;
                npx[r] = in ? px[i] : 0.f;
                npy[r] = in ? py[i] : 0.f;
                npz[r] = in ? pz[i] : 0.f;
            }
        }
    };
    size_t w = (size_t)blockIdx.x * (SS_BLOCK / 64) + wv;
    if (w < nwin) load_window(w);
    for (; w < nwin; w += wstep) {
        const size_t base = w * W;
        int slot[R], nsky = 0;
        float qpx[POS ? R : 1], qpy[POS ? R : 1], qpz[POS ? R : 1];   // POS: this window's it.p
        {
            float a[R], b[R];
            uint64_t m[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                a[r] = na[r];
                b[r] = nb[r];
                if constexpr (POS) {
                    qpx[r] = npx[r];
                    qpy[r] = npy[r];
                    qpz[r] = npz[r];
                }
            }
            if (w + wstep < nwin) load_window(w + wstep);
#pragma unroll
            for (int r = 0; r < R; ++r) m[r] = __ballot(a[r] < K.w_sky);
            int psky = 0, psun = 0;   // sky / sun picks of the rows before this one
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool sky = (m[r] >> lane) & 1;
                slot[r] = sky ? psky + lanes_below(m[r]) : (W - 1) - (psun + lanes_below(~m[r]));   // win_addr
                Y[0][slot[r]] = a[r];
                Y[1][slot[r]] = b[r];
                if (FULL && active) Y[2][slot[r]] = nm[r];
                const int c = __popcll(m[r]);
                psky += c;
                psun += 64 - c;
            }
            nsky = psky;
        }
        // FULL: this window's it.p, loaded before the passes and consumed after them
        float ipx[FULL ? R : 1], ipy[FULL ? R : 1], ipz[FULL ? R : 1];
        if constexpr (FULL) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const size_t i = base + (size_t)(r * 64 + lane);
                const bool in = (dist || opx) && i < n;
                ipx[r] = in && px ? px[i] : 0.f;
                ipy[r] = in && py ? py[i] : 0.f;
                ipz[r] = in && pz ? pz[i] : 0.f;
            }
        }
        wave_lds_order();
#pragma unroll 1
        for (int p = 0; p < R; ++p) {
            const int q = win_addr(p * 64 + lane, nsky, W);
            const bool act = FULL && active ? Y[2][q] != 0.f : true;
            float o[7];
            // ranks [0, nsky) are the window's sky picks: a pass wholly on one side takes the
            // specialised body (wave-uniform branch)
            if (p * 64 + 64 <= nsky) sample_one_rgb<FAST, 1, kHoist>(K, S, Y[0][q], Y[1][q], act, inv_w, inv_w_sun, o);
            else if (p * 64 >= nsky) sample_one_rgb<FAST, 2, kHoist>(K, S, Y[0][q], Y[1][q], act, inv_w, inv_w_sun, o);
            else
            sample_one_rgb<FAST, 0, kHoist>(K, S, Y[0][q], Y[1][q], act, inv_w, inv_w_sun, o);
#pragma unroll
            for (int k = 0; k < 7; ++k) Y[k][q] = o[k];
        }
        wave_lds_order();
        float* const planes[7] = {dx, dy, dz, pdf, weight, weight + wstride, weight + 2 * wstride};
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = base + (size_t)(r * 64 + lane);
            if (i < n) {
#pragma unroll
                for (int k = 0; k < 7; ++k) store_nt(Y[k][slot[r]], planes[k] + i);
                if (MODE != kSortLean && (dist || opx)) {   // as sample_direction_body: ds.dist, ds.p (sunsky.cpp:417-420)
                    const float3_ d = mk3(Y[0][slot[r]], Y[1][slot[r]], Y[2][slot[r]]);
                    float3_ itp = POS ? mk3(qpx[POS ? r : 0], qpy[POS ? r : 0], qpz[POS ? r : 0])
                                      : mk3(ipx[FULL ? r : 0], ipy[FULL ? r : 0], ipz[FULL ? r : 0]);
                    float3_ rel = mk3(itp.x - K.bs_center[0], itp.y - K.bs_center[1], itp.z - K.bs_center[2]);
                    float dd = 2.f * fmaxf(K.bs_radius, sqrtf(dot3(rel, rel)));
                    if (dist) store_nt(dd, dist + i);
                    if (opx) { store_nt(fmaf(d.x, dd, itp.x), opx + i); store_nt(fmaf(d.y, dd, itp.y), opy + i); store_nt(fmaf(d.z, dd, itp.z), opz + i); }
                }
            }
        }
        wave_lds_order();
    }
}

// pdf_direction, sunsky.cpp:443-451.  VEC directions per lane: each gaussian's
// LDS-broadcast parameters are read once for VEC directions; 16-byte loads/stores.
template <int VEC, bool FAST>
__device__ __forceinline__ void pdf_direction_body(const SunskyKArgs& K, const float* __restrict__ dx,
                                                   const float* __restrict__ dy, const float* __restrict__ dz,
                                                   const uint8_t* __restrict__ active, size_t n,
                                                   float* __restrict__ pdf) {
    __shared__ TgmmLds<FAST> T;
    stage_tgmm<FAST>(K, &T);
    __syncthreads();
    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
        load_dirs<VEC>(dx, dy, dz, active, i, x, y, z, m);
        // compute_pdfs (sunsky.cpp:711-723) per direction, tgmm_pdf (:732-763) vectorised
        float phi[VEC], theta[VEC], sin_theta[VEC], sunp[VEC], acc[VEC];
        bool ok[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            float3_ d = to_local(K, mk3(x[j], y[j], z[j]));
            float st = safe_sqrt_sel<FAST>(fmaf(d.x, d.x, d.y * d.y));
            bool a = (d.z >= 0.f) && (st != 0.f);
            sin_theta[j] = fmaxf(st, kEpsilon);
            float ph = (FAST ? atan2_fast(d.y, d.x) : atan2f(d.y, d.x)) - (K.sun_phi - 0.5f * kPi);
            ph = ph < 0.f ? ph + kTwoPi : ph;
            phi[j] = ph > kTwoPi ? ph - kTwoPi : ph;
            theta[j] = FAST ? theta_upper_fast(d) : unit_angle_z(d);
            ok[j] = a && (theta[j] >= 0.f) && (theta[j] <= 0.5f * kPi);
            sunp[j] = dot3(sn, d) >= K.cos_cutoff ? K.sun_pdf : 0.f;
            acc[j] = 0.f;
        }
        if constexpr (FAST) {
            static_assert(VEC % 2 == 0 || VEC == 1, "direction pairs");
            if constexpr (VEC == 1) {
                acc[0] = tgmm_sum_fast(K, T, phi[0], theta[0]);
            } else {
                // directions in pairs: each gaussian's sx, sy, q and the accumulation run as
                // packed FP32 over two directions (bitwise the scalar loop).  Measured 2.6 %
                // faster than the scalar form here (interleaved A/B, tools/gpu_ab2.sh), unlike
                // the per-lane sums and the spectral channels, where packing lost.
                constexpr int NP = VEC / 2;
                f32x2 ph2[NP], th2[NP], ac2[NP];
#pragma unroll
                for (int j = 0; j < NP; ++j) {
                    ph2[j] = f32x2{phi[2 * j], phi[2 * j + 1]};
                    th2[j] = f32x2{theta[2 * j], theta[2 * j + 1]};
                    ac2[j] = f32x2{0.f, 0.f};
                }
                const int np = (K.tgmm_count + 1) >> 1;
#pragma unroll 1
                for (int p = 0; p < np; ++p) {
                    const TgPair P = T.tp[p];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float mphi = P.mphi[h], mth = P.mth[h], kphi = P.kphi[h], kth = P.kth[h], c = P.c[h];
#pragma unroll
                        for (int j = 0; j < NP; ++j) {
                            const f32x2 sx = __builtin_elementwise_fma(ph2[j], f32x2{kphi, kphi}, f32x2{mphi, mphi});
                            const f32x2 sy = __builtin_elementwise_fma(th2[j], f32x2{kth, kth}, f32x2{mth, mth});
                            const f32x2 q = __builtin_elementwise_fma(sy, sy, sx * sx);
                            const f32x2 e = f32x2{fast_exp2(-q.x), fast_exp2(-q.y)};
                            ac2[j] = __builtin_elementwise_fma(f32x2{c, c}, e, ac2[j]);
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < NP; ++j) { acc[2 * j] = ac2[j].x; acc[2 * j + 1] = ac2[j].y; }
            }
        } else {
#pragma unroll 2
            for (int g = 0; g < K.tgmm_count; ++g) {
                const Gaussian& G = T.tref[g];
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    float sx = (phi[j] - G.mu_phi) * G.inv_sigma_phi, sy = (theta[j] - G.mu_theta) * G.inv_sigma_theta;
                    float q = fmaf(sy, sy, sx * sx);
                    acc[j] = fmaf(G.coef, kInvTwoPi * expf(-0.5f * q), acc[j]);
                }
            }
        }
        float pd[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            float skyp = fdiv<FAST>(ok[j] ? acc[j] : 0.f, sin_theta[j]);
            pd[j] = m[j] ? lerpf_(sunp[j], skyp, K.w_sky) : 0.f;
        }
        store_vec<VEC>(pdf, i, pd);
    }
}

template <bool FAST, bool SPEC>
__device__ __forceinline__ void sample_wavelengths_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                                        const float* __restrict__ wy, const float* __restrict__ wz,
                                                        const float* __restrict__ sample, const uint8_t* __restrict__ active,
                                                        size_t n, float* __restrict__ lam_out, size_t lstride,
                                                        float* __restrict__ weight, size_t wstride) {
    __shared__ ChanLds<FAST> S;
    __shared__ SpecDistLds D;
    if (SPEC) {
        stage_chans<FAST>(K, &S);
        stage_spec_dist(K, &D);
    }
    __syncthreads();
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool act = active ? active[i] != 0 : true;
        float3_ wo = to_local(K, mk3(-wx[i], -wy[i], -wz[i]));
        if constexpr (!SPEC) {
            float e[3];
            eval_rgb_local<FAST>(K, K.sun_table, wo, act, e);
            for (int c = 0; c < 3; ++c) store_nt(e[c], weight + (size_t)c * wstride + i);
            for (int k = 0; k < 4; ++k) store_nt(0.f, lam_out + (size_t)k * lstride + i);
        } else {
            DirTerms t = dir_terms<FAST>(K, wo, act);
            add_sun_terms<FAST>(K, t);
            __builtin_amdgcn_sched_barrier(0);   // 44 -> 0 spilled SGPRs, 0.7 % faster (r03_v22_ab_sched_barriers.log)
            float lam[4], w[4];
            sample_wavelengths_one<FAST, false>(K, S.c, D, K.sun_table, K.sun_ld, t, sample[i], lam, w);
            for (int k = 0; k < 4; ++k) {
                lam_out[(size_t)k * lstride + i] = lam[k];
                weight[(size_t)k * wstride + i] = w[k];
            }
        }
    }
}

// sample_ray, sunsky.cpp:354-397
template <bool FAST, bool SPEC>
__device__ __forceinline__ void sample_ray_body(const SunskyKArgs& K, const float* __restrict__ wls,
                                                const float* __restrict__ s2x, const float* __restrict__ s2y,
                                                const float* __restrict__ s3x, const float* __restrict__ s3y,
                                                const uint8_t* __restrict__ active, size_t n,
                                                float* __restrict__ ox, float* __restrict__ oy, float* __restrict__ oz,
                                                float* __restrict__ dxo, float* __restrict__ dyo, float* __restrict__ dzo,
                                                float* __restrict__ lam_out, size_t lstride,
                                                float* __restrict__ weight, size_t wstride) {
    __shared__ SamplerLds<FAST, SPEC> S;
    stage_sampler_lds<FAST, SPEC>(K, &S);
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool act = active ? active[i] != 0 : true;
        float offx, offy;
        disk_concentric_dev<FAST>(s2x[i], s2y[i], &offx, &offy);
        const float sx = s3x[i], sy = s3y[i];
        const bool pick_sky = sx < K.w_sky;
        float sun_a = 0.f, sun_b = 0.f;
        const float3_ d = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, sx, sy, inv_w, inv_w_sun, &sun_a, &sun_b);
        float3_ dw = to_world(K, mk3(-d.x, -d.y, -d.z));
        act = act && (d.z >= 0.f);
        float skyp, sunp;
        sample_pdfs<FAST>(K, S.tgmm, d, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
        float pd = lerpf_(sunp, skyp, K.w_sky);
        pd *= kInvPi * (1.f / (K.bs_radius * K.bs_radius));
        act = act && pd > 0.f;
        // spectral: the scheduler held between the pdf and the wavelength sampling: 121 -> 27
        // spilled SGPRs, 4.3 % faster (profiles/r03_v22_ab_sched_barriers.log)
        if constexpr (SPEC) __builtin_amdgcn_sched_barrier(0);
        float3_ wo = to_local(K, mk3(-dw.x, -dw.y, -dw.z));
        float w[4];
        int nw;
        if constexpr (!SPEC) {
            eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, wo, act, w, S.rows);
            nw = 3;
            for (int k = 0; k < 4; ++k) store_nt(0.f, lam_out + (size_t)k * lstride + i);
        } else {
            DirTerms t = dir_terms<FAST>(K, wo, act);
            add_sun_terms<FAST>(K, t);
            float lam[4];
            sample_wavelengths_one<FAST, true>(K, S.chans.c, S.sdist[0], S.sun, S.ldp, t, wls[i], lam, w);
            for (int k = 0; k < 4; ++k) store_nt(lam[k], lam_out + (size_t)k * lstride + i);
            nw = 4;
        }
        float3_ fs, ft;
        coordinate_system(dw, &fs, &ft);
        float3_ po = frame_to_world(fs, ft, dw, mk3(offx, offy, 0.f));
        store_nt(K.bs_center[0] + (po.x - dw.x) * K.bs_radius, ox + i);
        store_nt(K.bs_center[1] + (po.y - dw.y) * K.bs_radius, oy + i);
        store_nt(K.bs_center[2] + (po.z - dw.z) * K.bs_radius, oz + i);
        store_nt(dw.x, dxo + i); store_nt(dw.y, dyo + i); store_nt(dw.z, dzo + i);
        const float inv_pd = fdiv<FAST>(1.f, pd);
        for (int k = 0; k < nw; ++k) {
            float v = FAST ? w[k] * inv_pd : w[k] / pd;
            store_nt(isfinite(v) ? v : 0.f, weight + (size_t)k * wstride + i);
        }
    }
}

// RGB sample_ray without a mask in wave-sorted windows (the RGB sample_direction kernel's
// windows, sample_direction_sorted_body): a wave ranks 64 R rays by their direction sample
// (sky picks first), runs R passes computing direction, pdf and weight (sample_ray_body's
// operations in its order) into 6 LDS rows, and un-sorts them; each lane then forms its
// rays' origins from its own sample2 (prefetched with sample3) and stores everything in ray
// order.  Bitwise sample_ray_body<FAST, false>.
template <bool FAST, int R>
__device__ __forceinline__ void sample_ray_rgb_sorted_body(
    const SunskyKArgs& K, const float* __restrict__ s2x, const float* __restrict__ s2y,
    const float* __restrict__ s3x, const float* __restrict__ s3y, size_t n, float* __restrict__ ox,
    float* __restrict__ oy, float* __restrict__ oz, float* __restrict__ dxo, float* __restrict__ dyo,
    float* __restrict__ dzo, float* __restrict__ lam_out, size_t lstride, float* __restrict__ weight,
    size_t wstride) {
    constexpr int W = 64 * R;
    __shared__ SamplerLds<FAST, false> S;
    __shared__ float X[SS_BLOCK / 64][6][W];
    stage_sampler_lds<FAST, false>(K, &S);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float(*Y)[W] = X[wv];
    const float inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / (1.f - K.w_sky));
    const size_t nwin = (n + W - 1) / W;
    const size_t wstep = (size_t)gridDim.x * (SS_BLOCK / 64);
    float na[R], nb[R], nc[R], nd[R];
    auto load_window = [&](size_t w) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = w * W + (size_t)(r * 64 + lane);
            na[r] = i < n ? s3x[i] : 1.f;   // past the end: a sun pick, computed and not stored
            nb[r] = i < n ? s3y[i] : 0.5f;
            nc[r] = i < n ? s2x[i] : 0.5f;
            nd[r] = i < n ? s2y[i] : 0.5f;
        }
    };
    size_t w = (size_t)blockIdx.x * (SS_BLOCK / 64) + wv;
    if (w < nwin) load_window(w);
    for (; w < nwin; w += wstep) {
        const size_t base = w * W;
        int slot[R], nsky = 0;
        float c2[R], d2[R];
        {
            float a[R], b[R];
            uint64_t m[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                a[r] = na[r];
                b[r] = nb[r];
                c2[r] = nc[r];
                d2[r] = nd[r];
            }
            if (w + wstep < nwin) load_window(w + wstep);
#pragma unroll
            for (int r = 0; r < R; ++r) m[r] = __ballot(a[r] < K.w_sky);
            int psky = 0, psun = 0;   // sky / sun picks of the rows before this one
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool sky = (m[r] >> lane) & 1;
                slot[r] = sky ? psky + lanes_below(m[r]) : (W - 1) - (psun + lanes_below(~m[r]));   // win_addr
                Y[0][slot[r]] = a[r];
                Y[1][slot[r]] = b[r];
                const int c = __popcll(m[r]);
                psky += c;
                psun += 64 - c;
            }
            nsky = psky;
        }
        wave_lds_order();
#pragma unroll 1
        for (int p = 0; p < R; ++p) {
            const int q = win_addr(p * 64 + lane, nsky, W);
            const float sx = Y[0][q], sy = Y[1][q];
            const bool pick_sky = sx < K.w_sky;
            float sun_a = 0.f, sun_b = 0.f;
            const float3_ d = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, sx, sy, inv_w, inv_w_sun, &sun_a, &sun_b);
            const float3_ dw = to_world(K, mk3(-d.x, -d.y, -d.z));
            bool act = d.z >= 0.f;
            float skyp, sunp;
            sample_pdfs<FAST>(K, S.tgmm, d, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
            float pd = lerpf_(sunp, skyp, K.w_sky);
            pd *= kInvPi * (1.f / (K.bs_radius * K.bs_radius));
            act = act && pd > 0.f;
            float e[3];
            eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, to_local(K, mk3(-dw.x, -dw.y, -dw.z)), act, e, S.rows);
            const float inv_pd = fdiv<FAST>(1.f, pd);
            Y[0][q] = dw.x; Y[1][q] = dw.y; Y[2][q] = dw.z;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float v = FAST ? e[k] * inv_pd : e[k] / pd;
                Y[3 + k][q] = isfinite(v) ? v : 0.f;
            }
        }
        wave_lds_order();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = base + (size_t)(r * 64 + lane);
            if (i < n) {
                const float3_ dw = mk3(Y[0][slot[r]], Y[1][slot[r]], Y[2][slot[r]]);
                float offx, offy;
                disk_concentric_dev<FAST>(c2[r], d2[r], &offx, &offy);
                float3_ fs, ft;
                coordinate_system(dw, &fs, &ft);
                const float3_ po = frame_to_world(fs, ft, dw, mk3(offx, offy, 0.f));
                store_nt(K.bs_center[0] + (po.x - dw.x) * K.bs_radius, ox + i);
                store_nt(K.bs_center[1] + (po.y - dw.y) * K.bs_radius, oy + i);
                store_nt(K.bs_center[2] + (po.z - dw.z) * K.bs_radius, oz + i);
                store_nt(dw.x, dxo + i); store_nt(dw.y, dyo + i); store_nt(dw.z, dzo + i);
#pragma unroll
                for (int k = 0; k < 4; ++k) store_nt(0.f, lam_out + (size_t)k * lstride + i);
#pragma unroll
                for (int k = 0; k < 3; ++k) store_nt(Y[3 + k][slot[r]], weight + (size_t)k * wstride + i);
            }
        }
        wave_lds_order();
    }
}

// ======================================================================
// Lat-long bake (a caller of eval: sky -> environment map, as the reference's
// sunsky-testing/sky_data_test.py:58-79 builds an envmap from eval() over
// helpers.py get_spherical_rays): pixel (x, y) of a W x H image looks along
// d = sphdir(theta_y, phi_x), theta_y = linspace(theta0, theta1, H)[y],
// phi_x = linspace(phi0, phi1, W)[x] (dr::linspace: fma(i, step, start)), and
// holds eval(si.wi = -d).  Directions are generated in-kernel: the bake only
// writes HBM (12 B per RGB pixel).  Planes [c][H * W], row-major.
// ======================================================================
// The sines and cosines of the W column and H row angles are tabulated once per
// bake by sunsky_latlong_tables (tab = [cos phi (W), sin phi (W), sin theta (H),
// cos theta (H)]); each pixel then reads 4 L2-resident table entries instead of
// two sincosf.
// ------------------------------------------------ caller: direct light at diffuse points
// mis_weight (power heuristic, src/integrators/path.cpp:315-321)
template <bool FAST>
__device__ __forceinline__ float mis_power(float a, float b) {
    a *= a;
    b *= b;
    const float w = fdiv<FAST>(a, a + b);
    return isfinite(w) ? w : 0.f;
}

// The emitter-sampling half of one direct_diffuse sample, RGB (path.cpp:204-228): the
// factor and the weight of `acc += scale * w`; scale = w = 0 where the reference adds
// nothing (occluded, pdf 0, below the surface): fma(0, 0, acc) is acc.
template <bool FAST>
__device__ __forceinline__ void dd_emitter_rgb(const SunskyKArgs& K, const SamplerLds<FAST, false>& S, float3_ nrm,
                                               float u0, float u1, unsigned v, float inv_w, float inv_w_sun,
                                               float* scale, float w[3]) {
    const bool pick_sky = u0 < K.w_sky;
    float sun_a = 0.f, sun_b = 0.f;
    const float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, u0, u1, inv_w, inv_w_sun, &sun_a, &sun_b);
    const bool act = sd.z >= 0.f;
    const float3_ d = to_world(K, sd);
    float skyp, sunp;
    sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
    const float pd = lerpf_(sunp, skyp, K.w_sky);
    const float cos_em = dot3(nrm, d);
    *scale = 0.f;
    w[0] = w[1] = w[2] = 0.f;
    if ((v & 1u) && pd != 0.f && cos_em > 0.f) {
        const float bpdf = kInvPi * cos_em;     // diffuse eval / pdf: rho / pi cos, cos / pi
        *scale = bpdf * mis_power<FAST>(pd, bpdf);
        float e[3];
        eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, to_local(K, d), act, e, S.rows);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float x = e[c] / pd;
            w[c] = isfinite(x) ? x : 0.f;
        }
    }
}

// The BSDF-sampling half, RGB (path.cpp:176-196): square_to_cosine_hemisphere, the miss,
// pdf_direction of the escaped ray and the power-heuristic MIS, accumulated into acc.
template <bool FAST>
__device__ __forceinline__ void dd_bsdf_rgb(const SunskyKArgs& K, const SamplerLds<FAST, false>& S, float3_ nrm,
                                            float3_ fs, float3_ ft, float u2, float u3, unsigned v, float acc[3]) {
    float px, py;
    disk_concentric_dev<FAST>(u2, u3, &px, &py);
    const float lz = safe_sqrt_sel<FAST>(1.f - fmaf(px, px, py * py));
    const float bpdf = kInvPi * lz;
    if ((v & 2u) && bpdf > 0.f) {
        const float3_ dw = frame_to_world(fs, ft, nrm, mk3(px, py, lz));
        const float3_ wo = to_local(K, dw);
        float bskyp, bsunp;
        compute_pdfs<FAST>(K, S.tgmm, wo, true, true, &bskyp, &bsunp);
        const float mis = mis_power<FAST>(bpdf, lerpf_(bsunp, bskyp, K.w_sky));
        float e[3];
        eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, wo, wo.z >= 0.f, e, S.rows);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] = fmaf(e[c], mis, acc[c]);
    }
}

// The sky-and-sun lighting of an unoccluded diffuse point, as the path
// integrator gathers it in one vertex (src/integrators/path.cpp:176-250 with
// the smooth diffuse BSDF of src/bsdfs/diffuse.cpp:100-180, the sun/sky the
// scene's only emitter, nothing occluding):
//   emitter sampling: (ds, w) = sample_direction(u_em); f = rho/pi max(0, n.d);
//     result += f * w * mis(ds.pdf, pdf_bsdf(d))           (when ds.pdf != 0)
//   BSDF sampling: wo = Frame(n).to_world(square_to_cosine_hemisphere(u_bsdf)),
//     pdf_bsdf = cos/pi, weight = rho; the ray escapes, so
//     result += rho * eval(-wo) * mis(pdf_bsdf, pdf_direction(wo))
// averaged over spp samples drawn from PCG32Sampler-seeded streams
// (next_2d for u_em, then next_2d for u_bsdf).  Out: 3 planes (RGB) or one per
// per-point wavelength (spectral, si.wavelengths).  Everything between the
// normal and the accumulated radiance stays in VGPRs: per point the kernel
// reads 12 B (+ rho, + wavelengths) and writes 4 B per channel, whatever spp.
// Occlusion (optional): vis[s * vstride + i] holds the caller's ray-tracer
// verdicts for sample s of point i -- bit 0 the shadow ray along the emitter
// sample is unoccluded (path.cpp:216-219, scene->ray_test), bit 1 the BSDF ray
// escapes to the environment (path.cpp:176-196, no surface hit).  The rays are
// the ones sunsky_direct_diffuse_rays writes from the same streams; vis = null
// is the unoccluded point (every bit set).
// Spectral eval at a point's nlam <= 4 wavelengths for the callers: Mitsuba's 4 (nlam == 4)
// through the branchless eval_spec4, fewer through eval_spec_one each (the same bits).
template <bool FAST, int C>
__device__ __forceinline__ void eval_spec_point(const SunskyKArgs& K, const SamplerLds<FAST, true>& S,
                                                const DirTerms& t, const float wl[C], int nlam, float e[C]) {
    static_assert(C == 4, "up to 4 wavelengths per point");
    if (nlam == 4) {
        eval_spec4<FAST>(K, chan_src(S), S.sun, S.ldp, t, wl, e);
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) e[c] = c < nlam ? eval_spec_one<FAST>(K, S.chans.c, S.sun, S.ld, t, wl[c]) : 0.f;
    }
}

template <bool FAST, bool SPEC>
__device__ __forceinline__ void direct_diffuse_body(
    const SunskyKArgs& K, const float* __restrict__ nx, const float* __restrict__ ny, const float* __restrict__ nz,
    const float* __restrict__ rho, const float* __restrict__ lam, size_t lstride, int nlam, uint32_t seed,
    uint32_t spp, const uint8_t* __restrict__ vis, size_t vstride, size_t n, float* __restrict__ out,
    size_t ostride) {
    __shared__ SamplerLds<FAST, SPEC> S;
    stage_sampler_lds<FAST, SPEC>(K, &S);
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    constexpr int C = SPEC ? 4 : 3;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float3_ nrm = mk3(nx[i], ny[i], nz[i]);
        float3_ fs, ft;
        coordinate_system(nrm, &fs, &ft);
        uint32_t v0 = seed, v1 = (uint32_t)i;
        sample_tea_32(&v0, &v1);
        Pcg32 rng;
        rng.seed(v0, v1);
        float wl[C];
        if constexpr (SPEC) {
#pragma unroll
            for (int k = 0; k < C; ++k) wl[k] = k < nlam ? lam[(size_t)k * lstride + i] : 0.f;
        }
        float acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.f;
        for (uint32_t smp = 0; smp < spp; ++smp) {
            const float u0 = rng.next_float(), u1 = rng.next_float();
            (void)rng.next_float();   // sample_1 (path.cpp:233), unused by the diffuse BSDF
            const float u2 = rng.next_float(), u3 = rng.next_float();
            const unsigned v = vis ? (unsigned)vis[(size_t)smp * vstride + i] : 3u;
            if constexpr (!SPEC) {
                float scale, w[3];
                dd_emitter_rgb<FAST>(K, S, nrm, u0, u1, v, inv_w, inv_w_sun, &scale, w);
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[c] = fmaf(scale, w[c], acc[c]);
                __builtin_amdgcn_sched_barrier(0);   // between the halves, as in the spectral path below
                dd_bsdf_rgb<FAST>(K, S, nrm, fs, ft, u2, u3, v, acc);
                continue;
            }
            // ---- emitter sampling: sample_direction (sunsky.cpp:399-441)
            const bool pick_sky = u0 < K.w_sky;
            float sun_a = 0.f, sun_b = 0.f;
            float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, u0, u1, inv_w, inv_w_sun, &sun_a, &sun_b);
            bool act = sd.z >= 0.f;
            const float3_ d = to_world(K, sd);
            float skyp, sunp;
            sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
            const float pd = lerpf_(sunp, skyp, K.w_sky);
            const float cos_em = dot3(nrm, d);
            if ((v & 1u) && pd != 0.f && cos_em > 0.f) {
                const float bpdf = kInvPi * cos_em;     // diffuse eval / pdf: rho / pi cos, cos / pi
                const float scale = bpdf * mis_power<FAST>(pd, bpdf);
                const float3_ wo = to_local(K, d);
                {
                    DirTerms t = dir_terms<FAST>(K, wo, act);
                    add_sun_terms<FAST>(K, t);
                    float e[C];
                    if constexpr (SPEC) eval_spec_point<FAST, C>(K, S, t, wl, nlam, e);
#pragma unroll
                    for (int c = 0; c < C; ++c)
                        if (c < nlam) {
                            const float w = e[c] / pd;
                            acc[c] = fmaf(scale, isfinite(w) ? w : 0.f, acc[c]);
                        }
                }
            }
            // the scheduler held between the emitter and BSDF halves: spectral diffuse 1.9 %, spectral
            // conductor 1.0 % faster, RGB neutral (profiles/r03_v22_ab_sched_barriers.log)
            __builtin_amdgcn_sched_barrier(0);
            // ---- BSDF sampling: square_to_cosine_hemisphere (warp.h:412-420), then the miss
            float px, py;
            disk_concentric_dev<FAST>(u2, u3, &px, &py);
            const float lz = safe_sqrt_sel<FAST>(1.f - fmaf(px, px, py * py));
            const float bpdf = kInvPi * lz;
            if ((v & 2u) && bpdf > 0.f) {
                const float3_ dw = frame_to_world(fs, ft, nrm, mk3(px, py, lz));
                const float3_ wo = to_local(K, dw);
                // pdf_direction (sunsky.cpp:443-451) of the escaped ray
                float bskyp, bsunp;
                compute_pdfs<FAST>(K, S.tgmm, wo, true, true, &bskyp, &bsunp);
                const float mis = mis_power<FAST>(bpdf, lerpf_(bsunp, bskyp, K.w_sky));
                const bool up = wo.z >= 0.f;
                if constexpr (!SPEC) {
                    float e[3];
                    eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, wo, up, e, S.rows);
#pragma unroll
                    for (int c = 0; c < 3; ++c) acc[c] = fmaf(e[c], mis, acc[c]);
                } else {
                    DirTerms t = dir_terms<FAST>(K, wo, up);
                    add_sun_terms<FAST>(K, t);
                    float e[C];
                    eval_spec_point<FAST, C>(K, S, t, wl, nlam, e);
#pragma unroll
                    for (int c = 0; c < C; ++c)
                        if (c < nlam) acc[c] = fmaf(e[c], mis, acc[c]);
                }
            }
        }
        const float r = (rho ? rho[i] : 1.f) / (float)spp;
        const int nc = SPEC ? nlam : 3;
#pragma unroll
        for (int c = 0; c < C; ++c)
            if (c < nc) __builtin_nontemporal_store(acc[c] * r, out + (size_t)c * ostride + i);
    }
}

// ======================================================================
// Caller with a glossy vertex: the rough conductor (src/bsdfs/roughconductor.cpp) with a
// Beckmann or GGX microfacet distribution, isotropic or anisotropic (alpha_u along the shading
// frame's s, alpha_v along t), and visible-normal sampling (include/mitsuba/render/microfacet.h),
// Mitsuba's default sampling.  All in the point's shading frame Frame3f(n) (coordinate_system),
// fp32 with the libm functions.
// ======================================================================
struct ConductorArgs {
    int type;            // 0 Beckmann, 1 GGX (MicrofacetType)
    float alpha_u;       // roughness along the frame's s (microfacet.h m_alpha_u)
    float eta[4], k[4];  // complex IOR per RGB channel (spectral: eta[0], k[0] for every wavelength)
    float alpha_v;       // roughness along t (= alpha_u: isotropic)
};

// MicrofacetDistribution::eval (microfacet.h:186-207).  FAST: products with 1 / alpha_u,
// 1 / alpha_v and v_rcp_f32 / v_exp_f32 in place of the divisions and expf.
template <bool FAST>
__device__ __forceinline__ float mf_eval(const ConductorArgs& c, float3_ m) {
    const float ct2 = m.z * m.z, a2 = c.alpha_u * c.alpha_v;
    float r;
    if constexpr (FAST) {
        const float mx = m.x * fast_rcp(c.alpha_u), my = m.y * fast_rcp(c.alpha_v);
        if (c.type == 0) {
            const float ict2 = fast_rcp(ct2);
            r = fast_exp2(-(mx * mx + my * my) * ict2 * kLog2e) * (fast_rcp(kPi * a2) * (ict2 * ict2));
        } else {
            const float q = mx * mx + my * my + ct2;
            r = fast_rcp(kPi * a2 * (q * q));
        }
    } else {
        if (c.type == 0) {
            const float mx = m.x / c.alpha_u, my = m.y / c.alpha_v;
            r = expf(-(mx * mx + my * my) / ct2) / (kPi * a2 * (ct2 * ct2));
        } else {
            const float mx = m.x / c.alpha_u, my = m.y / c.alpha_v, q = mx * mx + my * my + m.z * m.z;
            r = 1.f / (kPi * a2 * (q * q));
        }
    }
    return r * m.z > 1e-20f ? r : 0.f;
}

// MicrofacetDistribution::smith_g1 (microfacet.h:330-354)
template <bool FAST>
__device__ __forceinline__ float mf_smith_g1(const ConductorArgs& c, float3_ v, float3_ m) {
    const float xy = (c.alpha_u * v.x) * (c.alpha_u * v.x) + (c.alpha_v * v.y) * (c.alpha_v * v.y);
    const float t2 = fdiv<FAST>(xy, v.z * v.z);
    float r;
    if (c.type == 0) {
        const float a = FAST ? fast_rsq(t2) : 1.f / sqrtf(t2), a2 = a * a;
        r = a >= 1.6f ? 1.f : fdiv<FAST>(3.535f * a + 2.181f * a2, 1.f + 2.276f * a + 2.577f * a2);
    } else {
        r = fdiv<FAST>(2.f, 1.f + (FAST ? fast_sqrt(1.f + t2) : sqrtf(1.f + t2)));
    }
    if (xy == 0.f) r = 1.f;
    if (dot3(v, m) * v.z <= 0.f) r = 0.f;
    return r;
}

// The part of MicrofacetDistribution::sample (microfacet.h:293-320, 357-410) that depends only
// on wi, computed once per point for its spp samples: the stretched wi's azimuth (sin, cos;
// (0, 1) at the pole, Frame3f::sincos_phi) and cos theta, and per distribution the
// sample-independent terms of sample_visible_11.
struct MfView {
    float sp, cp, ct;
    float tan_i, maxval, ktan, kexp;   // Beckmann: tan theta, erf(cot), tan / sqrt(pi), tan exp(-cot^2) / sqrt(pi)
    float sin_i;                       // GGX
};

template <bool FAST>
__device__ __forceinline__ MfView mf_view(const ConductorArgs& c, float3_ wi) {
    MfView V;
    float3_ wp = mk3(c.alpha_u * wi.x, c.alpha_v * wi.y, wi.z);
    const float inv = FAST ? fast_rsq(dot3(wp, wp)) : 1.f / sqrtf(dot3(wp, wp));
    wp = mk3(wp.x * inv, wp.y * inv, wp.z * inv);
    const float st2 = fmaxf(1.f - wp.z * wp.z, 0.f);
    const float inv_st = FAST ? fast_rsq(st2) : 1.f / sqrtf(st2);
    float sp = wp.y * inv_st, cp = wp.x * inv_st;
    if (!(st2 > 0.f) || !isfinite(inv_st)) { sp = 0.f; cp = 1.f; }
    V.sp = fminf(fmaxf(sp, -1.f), 1.f);
    V.cp = fminf(fmaxf(cp, -1.f), 1.f);
    V.ct = wp.z;
    V.tan_i = V.maxval = V.ktan = V.kexp = V.sin_i = 0.f;
    if (c.type == 0) {
        V.tan_i = fdiv<FAST>(sqrtf(fmaxf(fmaf(-V.ct, V.ct, 1.f), 0.f)), V.ct);
        const float cot_i = fdiv<FAST>(1.f, V.tan_i);
        V.maxval = erff(cot_i);
        V.ktan = 0.56418958354775628695f * V.tan_i;
        V.kexp = V.ktan * (FAST ? fast_exp2(-cot_i * cot_i * kLog2e) : expf(-cot_i * cot_i));
    } else {
        V.sin_i = sqrtf(fmaxf(1.f - V.ct * V.ct, 0.f));
    }
    return V;
}

// MicrofacetDistribution::sample_visible_11 (microfacet.h:357-410) from the view's terms
template <bool FAST>
__device__ __forceinline__ void mf_sample_visible_11(const ConductorArgs& c, const MfView& V, float ux, float uy,
                                                     float* sx, float* sy) {
    if (c.type == 0) {
        ux = fmaxf(fminf(ux, 1.f - 1e-6f), 1e-6f);
        uy = fmaxf(fminf(uy, 1.f - 1e-6f), 1e-6f);
        const float lg = FAST ? -0.693147180559945309f * __builtin_amdgcn_logf(ux) : -logf(ux);
        float x = V.maxval - (V.maxval + 1.f) * erff(FAST ? fast_sqrt(lg) : sqrtf(lg));
        ux *= 1.f + V.maxval + V.kexp;
#pragma unroll 1
        for (int it = 0; it < 3; ++it) {
            const float slope = FAST ? erfinv_fast(x) : erfinvf_(x);
            const float value = 1.f + x + V.ktan * (FAST ? fast_exp2(-slope * slope * kLog2e) : expf(-slope * slope)) - ux;
            const float deriv = 1.f - slope * V.tan_i;
            x -= fdiv<FAST>(value, deriv);
        }
        *sx = FAST ? erfinv_fast(x) : erfinvf_(x);
        *sy = FAST ? erfinv_fast(fmaf(2.f, uy, -1.f)) : erfinvf_(fmaf(2.f, uy, -1.f));
    } else {
        float px, py;
        disk_concentric_dev<FAST>(ux, uy, &px, &py);
        const float sl = 0.5f * (1.f + V.ct);
        py = lerpf_(sqrtf(fmaxf(1.f - px * px, 0.f)), py, sl);
        const float pz = sqrtf(fmaxf(1.f - (px * px + py * py), 0.f));
        const float norm = fdiv<FAST>(1.f, fmaf(V.sin_i, py, V.ct * pz));
        *sx = fmaf(V.ct, py, -(V.sin_i * pz)) * norm;
        *sy = px * norm;
    }
}

// MicrofacetDistribution::sample, visible normals (microfacet.h:293-320): m and its pdf
template <bool FAST>
__device__ __forceinline__ float3_ mf_sample(const ConductorArgs& c, const MfView& V, float3_ wi, float ux, float uy,
                                             float* pdf) {
    float slx, sly;
    mf_sample_visible_11<FAST>(c, V, ux, uy, &slx, &sly);
    const float tx = fmaf(V.cp, slx, -(V.sp * sly)) * c.alpha_u, ty = fmaf(V.sp, slx, V.cp * sly) * c.alpha_v;
    float3_ m = mk3(-tx, -ty, 1.f);
    const float mi = FAST ? fast_rsq(dot3(m, m)) : 1.f / sqrtf(dot3(m, m));
    m = mk3(m.x * mi, m.y * mi, m.z * mi);
    *pdf = fdiv<FAST>(mf_eval<FAST>(c, m) * mf_smith_g1<FAST>(c, wi, m) * fabsf(dot3(wi, m)), wi.z);
    return m;
}

// fresnel_conductor (fresnel.h:93-117)
template <bool FAST>
__device__ __forceinline__ float fresnel_conductor_dev(float cos_i, float eta, float k) {
    const float c2 = cos_i * cos_i, s2 = 1.f - c2, s4 = s2 * s2;
    const float t1 = eta * eta - k * k - s2;
    const float ab = safe_sqrt_sel<FAST>(t1 * t1 + 4.f * k * k * eta * eta);
    const float a = safe_sqrt_sel<FAST>(0.5f * (ab + t1));
    const float term1 = ab + c2, term2 = 2.f * cos_i * a;
    const float rs = fdiv<FAST>(term1 - term2, term1 + term2);
    const float term3 = ab * c2 + s4, term4 = term2 * s2;
    const float rp = rs * fdiv<FAST>(term3 - term4, term3 + term4);
    return 0.5f * (rs + rp);
}

// RoughConductor::eval and ::pdf (roughconductor.cpp:308-420) for wi, wo in the shading
// frame: f cos(theta_o) per channel without the Fresnel factor (returned as D G / (4 cos_i),
// the caller multiplies F(dot(wi, H)) per channel) and the pdf.
template <bool FAST>
__device__ __forceinline__ float conductor_eval_pdf(const ConductorArgs& c, float3_ wi, float3_ wo, float* pdf,
                                                    float* cos_ih) {
    *pdf = 0.f;
    *cos_ih = 0.f;
    if (!(wi.z > 0.f && wo.z > 0.f)) return 0.f;
    float3_ h = mk3(wo.x + wi.x, wo.y + wi.y, wo.z + wi.z);
    const float hi = FAST ? fast_rsq(dot3(h, h)) : 1.f / sqrtf(dot3(h, h));
    h = mk3(h.x * hi, h.y * hi, h.z * hi);
    const float D = mf_eval<FAST>(c, h);
    const float g1i = mf_smith_g1<FAST>(c, wi, h);
    *cos_ih = dot3(wi, h);
    if (dot3(wi, h) > 0.f && dot3(wo, h) > 0.f) *pdf = fdiv<FAST>(D * g1i, 4.f * wi.z);
    if (D == 0.f) return 0.f;
    return fdiv<FAST>(D * (g1i * mf_smith_g1<FAST>(c, wo, h)), 4.f * wi.z);
}

// The sky-and-sun lighting a rough-conductor point reflects towards wi (one path vertex,
// src/integrators/path.cpp:176-250 with src/bsdfs/roughconductor.cpp): per sample the
// emitter sample (next_2d) weighted by f cos / pdf x MIS, then sample_1 (next_1d, unused by
// the conductor) and the BSDF sample (next_2d: visible normal, reflection, weight
// G1(wo) F) whose escaped ray meets eval() x MIS; power heuristic; PCG32Sampler streams.
// wi: world unit directions towards the viewer (si.wi); visibility as direct_diffuse.
template <bool FAST, bool SPEC>
__device__ __forceinline__ void direct_conductor_body(
    const SunskyKArgs& K, const ConductorArgs C, const float* __restrict__ nx, const float* __restrict__ ny,
    const float* __restrict__ nz, const float* __restrict__ vx, const float* __restrict__ vy,
    const float* __restrict__ vz, const float* __restrict__ lam, size_t lstride, int nlam, uint32_t seed,
    uint32_t spp, const uint8_t* __restrict__ vis, size_t vstride, size_t n, float* __restrict__ out,
    size_t ostride) {
    __shared__ SamplerLds<FAST, SPEC> S;
    stage_sampler_lds<FAST, SPEC>(K, &S);
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    constexpr int CH = SPEC ? 4 : 3;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float3_ nrm = mk3(nx[i], ny[i], nz[i]);
        float3_ fs, ft;
        coordinate_system(nrm, &fs, &ft);
        const float3_ vw = mk3(vx[i], vy[i], vz[i]);
        const float3_ wi = mk3(dot3(vw, fs), dot3(vw, ft), dot3(vw, nrm));   // si.to_local(si.wi)
        const MfView V = mf_view<FAST>(C, wi);
        uint32_t v0 = seed, v1 = (uint32_t)i;
        sample_tea_32(&v0, &v1);
        Pcg32 rng;
        rng.seed(v0, v1);
        float wl[CH], eta[CH], kk[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            wl[c] = (SPEC && c < nlam) ? lam[(size_t)c * lstride + i] : 0.f;
            eta[c] = SPEC ? C.eta[0] : C.eta[c];
            kk[c] = SPEC ? C.k[0] : C.k[c];
        }
        float acc[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = 0.f;
        for (uint32_t smp = 0; smp < spp; ++smp) {
            const float u0 = rng.next_float(), u1 = rng.next_float();
            (void)rng.next_float();   // sample_1 (path.cpp:233), unused by the conductor
            const float u2 = rng.next_float(), u3 = rng.next_float();
            const unsigned v = vis ? (unsigned)vis[(size_t)smp * vstride + i] : 3u;
            // ---- emitter sampling
            {
                const bool pick_sky = u0 < K.w_sky;
                float sun_a = 0.f, sun_b = 0.f;
                const float3_ sd = sample_sky_or_sun<FAST>(K, S.tgmm, pick_sky, u0, u1, inv_w, inv_w_sun, &sun_a, &sun_b);
                const bool act = sd.z >= 0.f;
                const float3_ d = to_world(K, sd);
                float skyp, sunp;
                sample_pdfs<FAST>(K, S.tgmm, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
                const float pd = lerpf_(sunp, skyp, K.w_sky);
                const float3_ wo = mk3(dot3(d, fs), dot3(d, ft), dot3(d, nrm));
                float bpdf, cih;
                const float dg = conductor_eval_pdf<FAST>(C, wi, wo, &bpdf, &cih);
                if ((v & 1u) && pd != 0.f && dg != 0.f) {
                    const float mis = mis_power<FAST>(pd, bpdf);
                    const float3_ lw = to_local(K, d);
                    float e[CH];
                    if constexpr (!SPEC) {
                        eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, lw, act, e, S.rows);
                    } else {
                        DirTerms t = dir_terms<FAST>(K, lw, act);
                        add_sun_terms<FAST>(K, t);
#pragma unroll   // per wavelength (eval_spec4 here: 65 VGPRs spilled at 4 waves, 7 % slower)
                        for (int c = 0; c < CH; ++c) e[c] = c < nlam ? eval_spec_one<FAST>(K, S.chans.c, S.sun, S.ld, t, wl[c]) : 0.f;
                    }
                    const float inv_pd = fdiv<FAST>(1.f, pd);
#pragma unroll
                    for (int c = 0; c < CH; ++c) {
                        float w = FAST ? e[c] * inv_pd : e[c] / pd;
                        w = isfinite(w) ? w : 0.f;
                        acc[c] = fmaf(dg * fresnel_conductor_dev<FAST>(cih, eta[c], kk[c]) * w, mis, acc[c]);
                    }
                }
            }
            // the scheduler held between the emitter and BSDF halves: spectral diffuse 1.9 %, spectral
            // conductor 1.0 % faster, RGB neutral (profiles/r03_v22_ab_sched_barriers.log)
            __builtin_amdgcn_sched_barrier(0);
            // ---- BSDF sampling
            if (wi.z > 0.f) {
                float mpdf;
                const float3_ m = mf_sample<FAST>(C, V, wi, u2, u3, &mpdf);
                const float dwm = dot3(wi, m);
                const float3_ wo = mk3(fmaf(2.f * dwm, m.x, -wi.x), fmaf(2.f * dwm, m.y, -wi.y), fmaf(2.f * dwm, m.z, -wi.z));
                const float bpdf = fdiv<FAST>(mpdf, 4.f * dot3(wo, m));
                if ((v & 2u) && bpdf != 0.f && wo.z > 0.f) {
                    const float g1 = mf_smith_g1<FAST>(C, wo, m);
                    const float3_ dw = frame_to_world(fs, ft, nrm, wo);
                    const float3_ lw = to_local(K, dw);
                    float bskyp, bsunp;
                    compute_pdfs<FAST>(K, S.tgmm, lw, true, true, &bskyp, &bsunp);
                    const float mis = mis_power<FAST>(bpdf, lerpf_(bsunp, bskyp, K.w_sky));
                    const bool up = lw.z >= 0.f;
                    float e[CH];
                    if constexpr (!SPEC) {
                        eval_rgb_local<FAST>(K, S.chans.c, K.sun_table, lw, up, e, S.rows);
                    } else {
                        DirTerms t = dir_terms<FAST>(K, lw, up);
                        add_sun_terms<FAST>(K, t);
#pragma unroll   // per wavelength (eval_spec4 here: 65 VGPRs spilled at 4 waves, 7 % slower)
                        for (int c = 0; c < CH; ++c) e[c] = c < nlam ? eval_spec_one<FAST>(K, S.chans.c, S.sun, S.ld, t, wl[c]) : 0.f;
                    }
#pragma unroll
                    for (int c = 0; c < CH; ++c)   // throughput (F G1) x eval x MIS (path.cpp:184-190)
                        acc[c] = fmaf(fresnel_conductor_dev<FAST>(dwm, eta[c], kk[c]) * g1, e[c] * mis, acc[c]);
                }
            }
        }
        const float r = 1.f / (float)spp;
        const int nc = SPEC ? nlam : 3;
#pragma unroll
        for (int c = 0; c < CH; ++c)
            if (c < nc) __builtin_nontemporal_store(acc[c] * r, out + (size_t)c * ostride + i);
    }
}

// The rays of direct_conductor_body's samples, from the same streams and arithmetic (the
// directions bit for bit): em[s * rstride + i] the emitter sample's world direction, (0, 0,
// 0) where it contributes nothing (pdf 0, or f cos 0: below either hemisphere or outside
// the lobe), bs[...] the BSDF sample's reflected world direction, (0, 0, 0) where invalid;
// bw (if not null) the BSDF sample's weight F(wi.m) G1(wo, m) (roughconductor.cpp:250-262,
// the caller's path throughput factor) at bw[(c * spp + s) * rstride + i], c < nw, 0 where
// invalid.
template <bool FAST>
__device__ __forceinline__ void direct_conductor_rays_body(
    const SunskyKArgs& K, const ConductorArgs C, const float* __restrict__ nx, const float* __restrict__ ny,
    const float* __restrict__ nz, const float* __restrict__ vx, const float* __restrict__ vy,
    const float* __restrict__ vz, uint32_t seed, uint32_t spp, size_t n, float* __restrict__ ex,
    float* __restrict__ ey, float* __restrict__ ez, float* __restrict__ bx, float* __restrict__ by,
    float* __restrict__ bz, size_t rstride, float* __restrict__ bw, int nw) {
    __shared__ TgmmLds<FAST> T;
    stage_tgmm<FAST>(K, &T);
    __syncthreads();
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float3_ nrm = mk3(nx[i], ny[i], nz[i]);
        float3_ fs, ft;
        coordinate_system(nrm, &fs, &ft);
        const float3_ vw = mk3(vx[i], vy[i], vz[i]);
        const float3_ wi = mk3(dot3(vw, fs), dot3(vw, ft), dot3(vw, nrm));
        const MfView V = mf_view<FAST>(C, wi);
        uint32_t v0 = seed, v1 = (uint32_t)i;
        sample_tea_32(&v0, &v1);
        Pcg32 rng;
        rng.seed(v0, v1);
        for (uint32_t smp = 0; smp < spp; ++smp) {
            const float u0 = rng.next_float(), u1 = rng.next_float();
            (void)rng.next_float();
            const float u2 = rng.next_float(), u3 = rng.next_float();
            const bool pick_sky = u0 < K.w_sky;
            float sun_a = 0.f, sun_b = 0.f;
            const float3_ sd = sample_sky_or_sun<FAST>(K, T, pick_sky, u0, u1, inv_w, inv_w_sun, &sun_a, &sun_b);
            const bool act = sd.z >= 0.f;
            const float3_ d = to_world(K, sd);
            float skyp, sunp;
            sample_pdfs<FAST>(K, T, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
            const float pd = lerpf_(sunp, skyp, K.w_sky);
            const float3_ wo = mk3(dot3(d, fs), dot3(d, ft), dot3(d, nrm));
            float bpdf, cih;
            const bool em_ok = pd != 0.f && conductor_eval_pdf<FAST>(C, wi, wo, &bpdf, &cih) != 0.f;
            const size_t o = (size_t)smp * rstride + i;
            ex[o] = em_ok ? d.x : 0.f;
            ey[o] = em_ok ? d.y : 0.f;
            ez[o] = em_ok ? d.z : 0.f;
            float3_ dw = mk3(0.f, 0.f, 0.f);
            float g1 = 0.f, dwm = 0.f;
            if (wi.z > 0.f) {
                float mpdf;
                const float3_ m = mf_sample<FAST>(C, V, wi, u2, u3, &mpdf);
                dwm = dot3(wi, m);
                const float3_ r = mk3(fmaf(2.f * dwm, m.x, -wi.x), fmaf(2.f * dwm, m.y, -wi.y), fmaf(2.f * dwm, m.z, -wi.z));
                const float p = fdiv<FAST>(mpdf, 4.f * dot3(r, m));
                if (p != 0.f && r.z > 0.f) {
                    dw = frame_to_world(fs, ft, nrm, r);
                    g1 = mf_smith_g1<FAST>(C, r, m);
                }
            }
            bx[o] = dw.x;
            by[o] = dw.y;
            bz[o] = dw.z;
            if (bw) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    if (c < nw)
                        bw[((size_t)c * spp + smp) * rstride + i] =
                            g1 != 0.f ? fresnel_conductor_dev<FAST>(dwm, C.eta[c], C.k[c]) * g1 : 0.f;
            }
        }
    }
}

// The rays a caller's tracer tests between the two halves of direct_diffuse_body,
// from the same PCG32 streams and the same arithmetic: for sample s of point i,
// em[s * rstride + i] is the world direction of the emitter sample (the shadow ray
// of path.cpp:216-219), (0, 0, 0) where that sample contributes nothing anyway
// (pdf 0 or below the point's horizon), and bs[s * rstride + i] the cosine-sampled
// BSDF direction (path.cpp:176-196), (0, 0, 0) where its pdf is 0.  Directions
// are the same values direct_diffuse_body computes, so a caller's verdicts about
// them (vis) apply bit for bit.  Only the mixture tables are needed (LDS).
template <bool FAST>
__device__ __forceinline__ void direct_diffuse_rays_body(
    const SunskyKArgs& K, const float* __restrict__ nx, const float* __restrict__ ny, const float* __restrict__ nz,
    uint32_t seed, uint32_t spp, size_t n, float* __restrict__ ex, float* __restrict__ ey, float* __restrict__ ez,
    float* __restrict__ bx, float* __restrict__ by, float* __restrict__ bz, size_t rstride) {
    __shared__ TgmmLds<FAST> T;
    stage_tgmm<FAST>(K, &T);
    __syncthreads();
    const float w_sun = 1.f - K.w_sky, inv_w = uniform_f(1.f / K.w_sky), inv_w_sun = uniform_f(1.f / w_sun);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float3_ nrm = mk3(nx[i], ny[i], nz[i]);
        float3_ fs, ft;
        coordinate_system(nrm, &fs, &ft);
        uint32_t v0 = seed, v1 = (uint32_t)i;
        sample_tea_32(&v0, &v1);
        Pcg32 rng;
        rng.seed(v0, v1);
        for (uint32_t smp = 0; smp < spp; ++smp) {
            const float u0 = rng.next_float(), u1 = rng.next_float();
            (void)rng.next_float();   // sample_1 (path.cpp:233), unused by the diffuse BSDF
            const float u2 = rng.next_float(), u3 = rng.next_float();
            const bool pick_sky = u0 < K.w_sky;
            float sun_a = 0.f, sun_b = 0.f;
            const float3_ sd = sample_sky_or_sun<FAST>(K, T, pick_sky, u0, u1, inv_w, inv_w_sun, &sun_a, &sun_b);
            const bool act = sd.z >= 0.f;
            const float3_ d = to_world(K, sd);
            float skyp, sunp;
            sample_pdfs<FAST>(K, T, sd, pick_sky, sun_a, sun_b, act, &skyp, &sunp);
            const float pd = lerpf_(sunp, skyp, K.w_sky);
            const bool em_ok = pd != 0.f && dot3(nrm, d) > 0.f;
            float px, py;
            disk_concentric_dev<FAST>(u2, u3, &px, &py);
            const float lz = safe_sqrt_sel<FAST>(1.f - fmaf(px, px, py * py));
            const bool bs_ok = kInvPi * lz > 0.f;
            const float3_ dw = frame_to_world(fs, ft, nrm, mk3(px, py, lz));
            const size_t o = (size_t)smp * rstride + i;
            __builtin_nontemporal_store(em_ok ? d.x : 0.f, ex + o);
            __builtin_nontemporal_store(em_ok ? d.y : 0.f, ey + o);
            __builtin_nontemporal_store(em_ok ? d.z : 0.f, ez + o);
            __builtin_nontemporal_store(bs_ok ? dw.x : 0.f, bx + o);
            __builtin_nontemporal_store(bs_ok ? dw.y : 0.f, by + o);
            __builtin_nontemporal_store(bs_ok ? dw.z : 0.f, bz + o);
        }
    }
}

struct LatLong { int w, h; float theta0, dtheta, phi0, dphi; const float* tab; };

__device__ __forceinline__ float3_ latlong_dir(const LatLong& G, size_t i) {
    const unsigned y = (unsigned)i / (unsigned)G.w, x = (unsigned)i - y * (unsigned)G.w;   // W * H < 2^31
    const float cp = G.tab[x], sp = G.tab[G.w + x], st = G.tab[2 * G.w + y], ct = G.tab[2 * G.w + G.h + y];
    return mk3(cp * st, sp * st, ct);
}

extern "C" __global__ __launch_bounds__(SS_BLOCK) void sunsky_latlong_tables(LatLong G, float* tab) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < G.w) {
        float sp, cp;
        sincosf(fmaf((float)i, G.dphi, G.phi0), &sp, &cp);
        tab[i] = cp;
        tab[G.w + i] = sp;
    }
    if (i < G.h) {
        float st, ct;
        sincosf(fmaf((float)i, G.dtheta, G.theta0), &st, &ct);
        tab[2 * G.w + i] = st;
        tab[2 * G.w + G.h + i] = ct;
    }
}

// One lane = 4 consecutive pixels of one row: (row, column group) from one 32-bit
// division per group; 16-byte stores when the row width is a multiple of 4.
template <bool FAST>
__device__ __forceinline__ void bake_rgb_body(const SunskyKArgs& K, LatLong G, float* __restrict__ out,
                                              size_t ostride) {
    const unsigned gpr = ((unsigned)G.w + 3u) / 4u, ngroups = gpr * (unsigned)G.h;
    const bool vec_ok = ((uintptr_t)out & 15u) == 0 && (ostride & 3u) == 0 && (G.w & 3) == 0;
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned v = blockIdx.x * blockDim.x + threadIdx.x; v < ngroups; v += stride) {
        const unsigned y = v / gpr, x0 = (v - y * gpr) * 4u;
        const float st = G.tab[2 * G.w + y], ct = G.tab[2 * G.w + G.h + y];
        const size_t i0 = (size_t)y * (unsigned)G.w + x0;
        float r[4] = {0, 0, 0, 0}, g[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
        // rows below the horizon are 0 (eval's cos_theta >= 0 mask) without evaluating
        // them when no to_world rotation maps them back up
        const bool below = K.identity_xform && ct < 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (below) break;
            const unsigned x = x0 + j < (unsigned)G.w ? x0 + j : (unsigned)G.w - 1;
            float3_ d = mk3(G.tab[x] * st, G.tab[G.w + x] * st, ct);
            float o[3];
            eval_rgb_local<FAST, FAST ? kSunF64 : kSunF32>(K, K.sun_table, to_local(K, d), true, o);
            r[j] = o[0]; g[j] = o[1]; b[j] = o[2];
        }
        if (vec_ok) {
            store_vec<4>(out, i0, r);
            store_vec<4>(out + ostride, i0, g);
            store_vec<4>(out + 2 * ostride, i0, b);
        } else {
            for (unsigned j = 0; j < 4 && x0 + j < (unsigned)G.w; ++j) {
                out[i0 + j] = r[j];
                out[ostride + i0 + j] = g[j];
                out[2 * ostride + i0 + j] = b[j];
            }
        }
    }
}

template <bool FAST>
__device__ __forceinline__ void bake_spec_body(const SunskyKArgs& K, LatLong G, const LambdaSet& L,
                                               float* __restrict__ out, size_t ostride) {
    __shared__ ChanLds<FAST> S;
    const auto* chans = stage_chans<FAST>(K, &S);
    __syncthreads();
    const size_t n = (size_t)G.w * G.h;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        DirTerms t = dir_terms<FAST>(K, to_local(K, latlong_dir(G, i)), true);
        if constexpr (!FAST) add_sun_terms<FAST>(K, t);
        for (int k = 0; k < L.m; ++k) {
            const int lo = L.lo[k];
            const float f = L.f[k];
            float o = 0.f;
            if (f >= 0.f && t.active) {
                o = sky_eval<FAST>(chans[lo], t, K.sky_scale);
                if (f != 0.f) o = lerpf_(o, lo + 1 < kNbWavelengths ? sky_eval<FAST>(chans[lo + 1], t, K.sky_scale) : 0.f, f);
                if (t.hit_sun) o = spec_disc_add<FAST>(K, t, lo, f, o);
            }
            __builtin_nontemporal_store(o, out + (size_t)k * ostride + i);
        }
    }
}

// ======================================================================
// eval_jvp: forward-mode derivative of eval() with respect to one
// differentiable parameter (turbidity / albedo / sun_direction, sunsky.cpp:
// 220-240) -- what dr::forward_from(param) + dr::grad(eval(si)) give in the
// reference.  sunsky_stage_tangent stages the tangent of the tables on the device
// (sunsky_staging.h, the same code as SunskyModel::eval_tangent); this kernel carries
// value and tangent through the reference operation order of eval (sunsky.cpp:303-352,
// 538-614, 631-650).
// jvp buffer: [0, 110) d{A..I, rad} x 11 channels, [110, 113) d local sun
// direction, [128, 128 + sun table size) d sun radiance table (kJvpSunOffset).
// ======================================================================

// sky: the channel constants, indexed per lane by the spectral AD kernels (a per-lane
// index into the kernarg block would gather from memory, 13 loads per channel).
struct JvpLds { float dsky[kNbWavelengths * 10]; float dsun_local[4]; SkyChannel sky[kNbWavelengths]; };

// d unit_angle(a, b) along da (sunsky.cpp:311): gamma = 2 asin(h) or pi - 2 asin(h),
// h = |b -/+ a| / 2.
__device__ __forceinline__ float unit_angle_tangent(float3_ a, float3_ b, float3_ da) {
    float d = dot3(a, b);
    float3_ v = mk3(b.x - mulsignf_(a.x, d), b.y - mulsignf_(a.y, d), b.z - mulsignf_(a.z, d));
    float3_ dv = mk3(-mulsignf_(da.x, d), -mulsignf_(da.y, d), -mulsignf_(da.z, d));
    float h = 0.5f * sqrtf(dot3(v, v));
    if (!(h > 0.f)) return 0.f;
    float dtemp = 2.f * (dot3(v, dv) / (4.f * h)) / sqrtf(1.f - h * h);
    return d >= 0.f ? dtemp : -dtemp;
}

// Value terms of render_sky (sunsky.cpp:550-554) for one channel and direction: they do
// not depend on the tangent, so the reverse-mode kernels, which differentiate along 5
// basis tangents per channel, evaluate the exps and the pow once instead of 5 times.
struct SkyVal { float e1, c1, e2, b, pb, chi, c2, inv_pb, inv_b; };

__device__ __forceinline__ SkyVal sky_val(const SkyChannel& k, const DirTerms& t) {
    SkyVal s;
    s.e1 = expf(k.B * t.r);
    s.c1 = 1.f + k.A * s.e1;
    s.e2 = expf(k.E * t.gamma);
    s.b = 1.f + k.I * k.I - 2.f * k.I * t.cg;
    s.pb = s.b * sqrtf(s.b);   // b^1.5 (b > 0): within 2 ulp of powf, without its log/exp registers
    s.chi = t.u / s.pb;
    s.c2 = k.C + k.D * s.e2 + k.F * t.cg2 + k.G * s.chi + k.H * t.sq;
    s.inv_pb = 1.f / s.pb;   // the tangents multiply: 2 divisions per tangent and channel fewer
    s.inv_b = 1.f / s.b;
    return s;
}

// Tangent of render_sky (dk = d{A..I, rad}, dgamma), unscaled, from its value terms
__device__ __forceinline__ float sky_tan(const SkyChannel& k, const float* dk, const DirTerms& t, const SkyVal& s,
                                         float dgamma, float sg) {
    const float cg = t.cg, dcg = -sg * dgamma;
    const float dc1 = dk[0] * s.e1 + k.A * s.e1 * t.r * dk[1];
    const float db = 2.f * k.I * dk[8] - 2.f * dk[8] * cg - 2.f * k.I * dcg;
    const float dchi = 2.f * cg * dcg * s.inv_pb - 1.5f * s.chi * db * s.inv_b;
    const float dc2 = dk[2] + dk[3] * s.e2 + k.D * s.e2 * (dk[4] * t.gamma + k.E * dgamma) + dk[5] * t.cg2 +
                      k.F * 2.f * cg * dcg + dk[6] * s.chi + k.G * dchi + dk[7] * t.sq;
    return (dc1 * s.c2 + s.c1 * dc2) * k.rad + s.c1 * s.c2 * dk[9];
}

// sky_tan along d gamma = 1 with d params = 0 (the gamma part of a sun-axis tangent)
__device__ __forceinline__ float sky_tan_gamma(const SkyChannel& k, const DirTerms& t, const SkyVal& s, float sg) {
    const float cg = t.cg, dcg = -sg;
    const float db = -2.f * k.I * dcg;
    const float dchi = 2.f * cg * dcg * s.inv_pb - 1.5f * s.chi * db * s.inv_b;
    const float dc2 = k.D * s.e2 * k.E + k.F * 2.f * cg * dcg + k.G * dchi;
    return s.c1 * dc2 * k.rad;
}

// unit_angle_tangent split for several tangents da of one (a, b): the per-direction part
// (the chord v and 1 / (2 h sqrt(1 - h^2)) with the branch sign) once, then one dot per tangent.
struct UnitAngleTan { float3_ v; float f, sd; };

__device__ __forceinline__ UnitAngleTan unit_angle_tan_setup(float3_ a, float3_ b) {
    UnitAngleTan u;
    const float d = dot3(a, b);
    u.v = mk3(b.x - mulsignf_(a.x, d), b.y - mulsignf_(a.y, d), b.z - mulsignf_(a.z, d));
    u.sd = d;
    const float h = 0.5f * sqrtf(dot3(u.v, u.v));
    u.f = h > 0.f ? (d >= 0.f ? 1.f : -1.f) / (2.f * h * sqrtf(1.f - h * h)) : 0.f;
    return u;
}

__device__ __forceinline__ float unit_angle_tan_apply(const UnitAngleTan& u, float3_ da) {
    const float3_ dv = mk3(-mulsignf_(da.x, u.sd), -mulsignf_(da.y, u.sd), -mulsignf_(da.z, u.sd));
    return dot3(u.v, dv) * u.f;
}

// render_sky and its tangent (dk = d{A..I, rad}), unscaled
__device__ __forceinline__ void sky_jvp(const SkyChannel& k, const float* dk, const DirTerms& t, float dgamma,
                                        float sg, float* L, float* dL) {
    const SkyVal s = sky_val(k, t);
    *L = s.c1 * s.c2 * k.rad;
    *dL = sky_tan(k, dk, t, s, dgamma, sg);
}

// cos_psi (sunsky.h:385-392) and its tangent
__device__ __forceinline__ void cos_psi_jvp(const SunskyKArgs& K, const DirTerms& t, float sg, float dgamma,
                                            float* cp, float* dcp) {
    *cp = cos_psi(t.gamma, K.inv_sin2_half_ap);
    *dcp = *cp > 0.f ? -K.inv_sin2_half_ap * sg * t.cg * dgamma / *cp : 0.f;
}

// sin(gamma) for gamma = 2 asin(h) or pi - 2 asin(h): 2 h sqrt(1 - h^2), a few ulp from
// sinf(gamma) without libm's large-argument reduction (whose registers set the AD
// kernels' VGPR count).  Only the tangents use it.
__device__ __forceinline__ float sin_gamma(const DirTerms& t) {
    return 2.f * t.h * sqrtf(fmaxf(1.f - t.h * t.h, 0.f));
}

// Shared per-direction setup: reference-order DirTerms (cg = cos(gamma)), sin(gamma), d gamma.
__device__ __forceinline__ DirTerms jvp_dir(const SunskyKArgs& K, const JvpLds& J, float3_ wo, bool m, float* sg,
                                            float* dgamma) {
    DirTerms t = dir_terms<false>(K, wo, m);
    *sg = sin_gamma(t);
    *dgamma = unit_angle_tangent(mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]), wo,
                                 mk3(J.dsun_local[0], J.dsun_local[1], J.dsun_local[2]));
    return t;
}

__device__ __forceinline__ void stage_jvp(const SunskyKArgs& K, const float* jvp, JvpLds* J, int nch) {
    lds_copy(J->sky, K.sky, kNbWavelengths);
    for (int i = threadIdx.x; i < nch * 10; i += blockDim.x) J->dsky[i] = jvp[i];
    if (threadIdx.x < 3) J->dsun_local[threadIdx.x] = jvp[kNbWavelengths * 10 + threadIdx.x];
    __syncthreads();
}

__device__ __forceinline__ void eval_jvp_rgb_body(const SunskyKArgs& K, const float* __restrict__ jvp,
                                                  const float* __restrict__ wx, const float* __restrict__ wy,
                                                  const float* __restrict__ wz, const uint8_t* __restrict__ active,
                                                  size_t n, float* __restrict__ out, float* __restrict__ dout,
                                                  size_t ostride, float sign) {
    __shared__ JvpLds J;
    stage_jvp(K, jvp, &J, 3);
    const float* dsun_tab = jvp + kJvpSunOffset;
    const float cie = (float)kCieYNormalization, conv = (float)kSpecToRgbSunConv;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool m = active ? active[i] != 0 : true;
        float3_ wo = to_local(K, mk3(sign * wx[i], sign * wy[i], sign * wz[i]));
        float sg, dg;
        DirTerms t = jvp_dir(K, J, wo, m, &sg, &dg);
        float v[3], dv[3];
#pragma unroll 1
        for (int c = 0; c < 3; ++c) {
            sky_jvp(K.sky[c], J.dsky + c * 10, t, dg, sg, &v[c], &dv[c]);
            v[c] *= K.sky_scale;
            dv[c] *= K.sky_scale;
        }
        if (t.hit_sun) {
            float xs, cp, dcp;
            int pos = sun_segment_ref(K, t.cos_theta, &xs);
            cos_psi_jvp(K, t, sg, dg, &cp, &dcp);
            const float sc = K.sun_scale * K.area_ratio * conv;
#pragma unroll 1
            for (int c = 0; c < 3; ++c) {
                const float* S = K.sun_table + pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
                const float* dS = dsun_tab + pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
                float sv = 0.f, dsv = 0.f;
                for (int k = 0; k < kNbSunCtrlPts; ++k)
                    for (int j = 0; j < kNbSunLdParams; ++j) {
                        const float xk = powif_(xs, k), cj = powif_(cp, j);
                        sv += xk * cj * S[k * kNbSunLdParams + j];
                        dsv += xk * cj * dS[k * kNbSunLdParams + j];
                        if (j > 0) dsv += xk * (float)j * powif_(cp, j - 1) * S[k * kNbSunLdParams + j] * dcp;
                    }
                v[c] += sc * sv;
                dv[c] += sc * dsv;
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            out[(size_t)c * ostride + i] = t.active ? v[c] * cie : 0.f;
            dout[(size_t)c * ostride + i] = t.active ? dv[c] * cie : 0.f;
        }
    }
}

__device__ __forceinline__ void eval_jvp_spec_body(const SunskyKArgs& K, const float* __restrict__ jvp,
                                                   const float* __restrict__ wx, const float* __restrict__ wy,
                                                   const float* __restrict__ wz, const float* __restrict__ lam,
                                                   size_t lstride, int nlam, const uint8_t* __restrict__ active,
                                                   size_t n, float* __restrict__ out, float* __restrict__ dout,
                                                   size_t ostride, float sign) {
    __shared__ JvpLds J;
    stage_jvp(K, jvp, &J, kNbWavelengths);
    const float* dsun_tab = jvp + kJvpSunOffset;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool m = active ? active[i] != 0 : true;
        float3_ wo = to_local(K, mk3(sign * wx[i], sign * wy[i], sign * wz[i]));
        float sg, dg;
        DirTerms t = jvp_dir(K, J, wo, m, &sg, &dg);
        float xs = 0.f, cp = 0.f, dcp = 0.f;
        int pos = 0;
        if (t.hit_sun) {
            pos = sun_segment_ref(K, t.cos_theta, &xs);
            cos_psi_jvp(K, t, sg, dg, &cp, &dcp);
        }
        for (int q = 0; q < nlam; ++q) {
            const float lambda = lam[(size_t)q * lstride + i];
            float nw = (lambda - kWavelength0) / kWavelengthStep;
            bool valid = (0.f <= nw) && (nw <= (float)(kNbWavelengths - 1));
            float res = 0.f, dres = 0.f;
            if (t.active && valid) {
                int lo = (int)floorf(nw), hi = lo + 1;
                float f = nw - (float)lo;
                float la, dla, lb = 0.f, dlb = 0.f;
                sky_jvp(J.sky[lo], J.dsky + lo * 10, t, dg, sg, &la, &dla);
                if (hi < kNbWavelengths) sky_jvp(J.sky[hi], J.dsky + hi * 10, t, dg, sg, &lb, &dlb);
                res = K.sky_scale * (f != 0.f ? lerpf_(la, lb, f) : la);
                dres = K.sky_scale * (f != 0.f ? lerpf_(dla, dlb, f) : dla);
                if (t.hit_sun) {
                    float sa = render_sun_spec(K.sun_table, pos, lo, xs), dsa = render_sun_spec(dsun_tab, pos, lo, xs);
                    float sun = sa, dsun = dsa;
                    if (f != 0.f) {
                        float sb = hi < kNbWavelengths ? render_sun_spec(K.sun_table, pos, hi, xs) : 0.f;
                        float dsb = hi < kNbWavelengths ? render_sun_spec(dsun_tab, pos, hi, xs) : 0.f;
                        sun = lerpf_(sa, sb, f);
                        dsun = lerpf_(dsa, dsb, f);
                    }
                    float ld = sun_limb_darkening(K.sun_ld, lo, hi, f, cp), dld = 0.f;
                    for (int j = 1; j < kNbSunLdParams; ++j) {
                        float a = K.sun_ld[lo * kNbSunLdParams + j], coef = a;
                        if (f != 0.f) coef = lerpf_(a, hi < kNbWavelengths ? K.sun_ld[hi * kNbSunLdParams + j] : 0.f, f);
                        dld += (float)j * powif_(cp, j - 1) * coef * dcp;
                    }
                    res += K.sun_scale * sun * ld * K.area_ratio;
                    dres += K.sun_scale * K.area_ratio * (dsun * ld + sun * dld);
                }
            }
            out[(size_t)q * ostride + i] = res;
            dout[(size_t)q * ostride + i] = dres;
        }
    }
}

// ======================================================================
// eval_vjp: reverse mode.  grad[p] += sum_rays sum_channels d_out * d eval / d p
// for p = turbidity (0), albedo per channel (1 + c), sun_direction x/y/z (12..14),
// the gradient dr.backward(dot(d_out, eval(si))) accumulates in the reference.
// Each ray evaluates the derivative along the 5 basis tangents (T, albedo
// diagonal, 3 sun axes) with the JVP kernels' device code; the sums are reduced
// per workgroup in a fixed order (wave shuffles, then LDS) into per-block
// partials, which sunsky_grad_reduce adds to grad in block order --
// deterministic, no float atomics.
// vjp buffer: [0, 330) dsky for T / albedo-diagonal / unit sun elevation (3 x 110; 330..549
// the per-axis tables, not read), [550, 559) d local sun direction of the 3 sun axes,
// [559, 562) d eta of the 3 sun axes, [576, ...) d sun table (T).
// The sky parameters depend on the sun only through its elevation eta, and the sky tangent
// is linear in (d params, d gamma): along sun axis k it is d eta_k x (unit-eta tangent at
// d gamma = 0) + d gamma_k x (the gamma part).  Each ray accumulates the first, summed over
// rays, in g[15] (scaled by d eta_k per lane before the reduction) and the second per axis.
// ======================================================================
constexpr int kGradCount = 16;           // 0: T, 1..11: albedo channel, 12..14: sun_direction, 15: per-lane unit-elevation sum (0 in the partials)

struct VjpLds {
    SkyChannel sky[kNbWavelengths];   // per-lane channel index in the spectral kernel (see JvpLds)
    float dsky[3][kNbWavelengths * 10];
    float dlocal[3][3];
    float deta[3];
    float red[SS_BLOCK / 64][kGradCount];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;   // lane 0 holds the wave's sum
}

// Per-workgroup reduction of the per-lane gradient accumulators -> partials[block][16]
__device__ __forceinline__ void block_reduce_grad(VjpLds& L, float g[kGradCount], float* partials) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) g[12 + k] += L.deta[k] * g[15];   // the unit-elevation sums
    g[15] = 0.f;
#pragma unroll
    for (int p = 0; p < kGradCount; ++p) {
        float w = wave_sum(g[p]);
        if (lane == 0) L.red[wave][p] = w;
    }
    __syncthreads();
    if (threadIdx.x < kGradCount) {
        float acc = 0.f;
        for (int w = 0; w < SS_BLOCK / 64; ++w) acc += L.red[w][threadIdx.x];
        partials[(size_t)blockIdx.x * kGradCount + threadIdx.x] = acc;
    }
}

__device__ __forceinline__ void stage_vjp(const SunskyKArgs& K, const float* vjp, VjpLds* L) {
    lds_copy(L->sky, K.sky, kNbWavelengths);
    for (int i = threadIdx.x; i < 3 * kNbWavelengths * 10; i += blockDim.x) (&L->dsky[0][0])[i] = vjp[i];
    if (threadIdx.x < 9) (&L->dlocal[0][0])[threadIdx.x] = vjp[kVjpSunLocal + threadIdx.x];
    if (threadIdx.x < 3) L->deta[threadIdx.x] = vjp[kVjpSunEta + threadIdx.x];
    __syncthreads();
}

// The d gamma = 0 sky tangent is linear in d{A..I, rad}: sky_tan(dk) = sum_p W_p dk_p with
// weights that depend on the ray and the channel only.  The reverse-mode kernels form W once
// per channel and take the turbidity, albedo and unit-elevation tangents as 10-term dot
// products (the same sums as sky_tan, reassociated).
struct SkyTanW { float w[10]; };

__device__ __forceinline__ SkyTanW sky_tan_weights(const SkyChannel& k, const DirTerms& t, const SkyVal& s) {
    SkyTanW W;
    const float c2r = s.c2 * k.rad, q = s.c1 * k.rad;
    W.w[0] = c2r * s.e1;
    W.w[1] = c2r * (k.A * s.e1 * t.r);
    W.w[2] = q;
    W.w[3] = q * s.e2;
    W.w[4] = q * (k.D * s.e2 * t.gamma);
    W.w[5] = q * t.cg2;
    W.w[6] = q * s.chi;
    W.w[7] = q * t.sq;
    W.w[8] = q * (k.G * (-1.5f * s.chi * s.inv_b) * (2.f * k.I - 2.f * t.cg));   // d chi through d I
    W.w[9] = s.c1 * s.c2;
    return W;
}

__device__ __forceinline__ float sky_dot(const SkyTanW& W, const float* dk) {
    float acc = W.w[0] * dk[0];
#pragma unroll
    for (int p = 1; p < 10; ++p) acc = fmaf(W.w[p], dk[p], acc);
    return acc;
}

// One sky channel's reverse-mode terms: the tangents along turbidity, albedo and the unit
// elevation (d gamma = 0), and the gamma part of the sun axes
struct SkySide { float t, a, e, gm; };

__device__ __forceinline__ SkySide sky_side(const SkyChannel& k, const VjpLds& L, int ch, const DirTerms& t, float sg) {
    const SkyVal s = sky_val(k, t);
    const SkyTanW W = sky_tan_weights(k, t, s);
    SkySide r;
    r.t = sky_dot(W, L.dsky[0] + ch * 10);
    r.a = sky_dot(W, L.dsky[1] + ch * 10);
    r.e = sky_dot(W, L.dsky[2] + ch * 10);
    r.gm = sky_tan_gamma(k, t, s, sg);
    return r;
}

__device__ __forceinline__ void eval_vjp_rgb_body(const SunskyKArgs& K, const float* __restrict__ vjp,
                                                  const float* __restrict__ wx, const float* __restrict__ wy,
                                                  const float* __restrict__ wz, const uint8_t* __restrict__ active,
                                                  size_t n, const float* __restrict__ dout, size_t ostride,
                                                  float sign, float* __restrict__ partials) {
    __shared__ VjpLds L;
    stage_vjp(K, vjp, &L);
    const float* dsun_tab = vjp + kVjpSunOffset;
    const float cie = (float)kCieYNormalization, conv = (float)kSpecToRgbSunConv;
    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    float g[kGradCount];
#pragma unroll
    for (int p = 0; p < kGradCount; ++p) g[p] = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool m = active ? active[i] != 0 : true;
        float3_ wo = to_local(K, mk3(sign * wx[i], sign * wy[i], sign * wz[i]));
        DirTerms t = dir_terms<false>(K, wo, m);
        if (!t.active) continue;
        const float sg = sin_gamma(t);
        float dgs[3];
        const UnitAngleTan ua = unit_angle_tan_setup(sn, wo);
#pragma unroll
        for (int k = 0; k < 3; ++k) dgs[k] = unit_angle_tan_apply(ua, mk3(L.dlocal[k][0], L.dlocal[k][1], L.dlocal[k][2]));
        int pos = 0;
        float xs = 0.f, cp = 0.f, dcps[3] = {0.f, 0.f, 0.f};
        if (t.hit_sun) {
            pos = sun_segment_ref(K, t.cos_theta, &xs);
#pragma unroll
            for (int k = 0; k < 3; ++k) cos_psi_jvp(K, t, sg, dgs[k], &cp, &dcps[k]);
        }
        const float sc = K.sun_scale * K.area_ratio * conv;
#pragma unroll 1
        for (int c = 0; c < 3; ++c) {
            const float cot = dout[(size_t)c * ostride + i] * cie;
            const SkySide S = sky_side(K.sky[c], L, c, t, sg);   // value terms once for the 5 tangents
            const float cs = cot * K.sky_scale;
            g[0] += cs * S.t;
            g[1 + c] += cs * S.a;
            g[15] += cs * S.e;   // unit elevation
            const float gam = S.gm;
#pragma unroll
            for (int k = 0; k < 3; ++k) g[12 + k] += cs * gam * dgs[k];
            if (t.hit_sun) {
                const float* S = K.sun_table + pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
                const float* dS = dsun_tab + pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
                float dT = 0.f, dC = 0.f;   // d/dT, d/d cos_psi
#pragma unroll 1
                for (int kk = 0; kk < kNbSunCtrlPts; ++kk)
#pragma unroll 1
                    for (int j = 0; j < kNbSunLdParams; ++j) {
                        const float xk = powif_(xs, kk);
                        dT += xk * powif_(cp, j) * dS[kk * kNbSunLdParams + j];
                        if (j > 0) dC += xk * (float)j * powif_(cp, j - 1) * S[kk * kNbSunLdParams + j];
                    }
                g[0] += cot * sc * dT;
#pragma unroll
                for (int k = 0; k < 3; ++k) g[12 + k] += cot * sc * dC * dcps[k];
            }
        }
    }
    block_reduce_grad(L, g, partials);
}

__device__ __forceinline__ void eval_vjp_spec_body(const SunskyKArgs& K, const float* __restrict__ vjp,
                                                   const float* __restrict__ wx, const float* __restrict__ wy,
                                                   const float* __restrict__ wz, const float* __restrict__ lam,
                                                   size_t lstride, int nlam, const uint8_t* __restrict__ active,
                                                   size_t n, const float* __restrict__ dout, size_t ostride,
                                                   float sign, float* __restrict__ partials) {
    __shared__ VjpLds L;
    stage_vjp(K, vjp, &L);
    const float* dsun_tab = vjp + kVjpSunOffset;
    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    float g[kGradCount];
#pragma unroll
    for (int p = 0; p < kGradCount; ++p) g[p] = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool m = active ? active[i] != 0 : true;
        float3_ wo = to_local(K, mk3(sign * wx[i], sign * wy[i], sign * wz[i]));
        DirTerms t = dir_terms<false>(K, wo, m);
        if (!t.active) continue;
        const float sg = sin_gamma(t);
        float dgs[3];
        const UnitAngleTan ua = unit_angle_tan_setup(sn, wo);
#pragma unroll
        for (int k = 0; k < 3; ++k) dgs[k] = unit_angle_tan_apply(ua, mk3(L.dlocal[k][0], L.dlocal[k][1], L.dlocal[k][2]));
        int pos = 0;
        float xs = 0.f, cp = 0.f, dcps[3] = {0.f, 0.f, 0.f};
        if (t.hit_sun) {
            pos = sun_segment_ref(K, t.cos_theta, &xs);
#pragma unroll
            for (int k = 0; k < 3; ++k) cos_psi_jvp(K, t, sg, dgs[k], &cp, &dcps[k]);
        }
#pragma unroll 1
        for (int q = 0; q < nlam; ++q) {
            const float cot = dout[(size_t)q * ostride + i];
            const float lambda = lam[(size_t)q * lstride + i];
            float nw = (lambda - kWavelength0) / kWavelengthStep;
            if (!((0.f <= nw) && (nw <= (float)(kNbWavelengths - 1)))) continue;
            int lo = (int)floorf(nw), hi = lo + 1;
            float f = nw - (float)lo;
            const bool has_hi = f != 0.f && hi < kNbWavelengths;
            const float wlo = f != 0.f ? 1.f - f : 1.f, whi = f;   // lerp weights (f = 0: low channel only)
            // turbidity, albedo (diagonal), sun axes: each lerped over the two channels; the
            // value terms of each channel once for its 5 tangents
            const SkySide A = sky_side(L.sky[lo], L, lo, t, sg);
            // the two sides one after the other: hoisting the second side's table reads over
            // the first holds both sets of weights and reads live (164 VGPRs, 3 waves/SIMD)
            __builtin_amdgcn_sched_barrier(0);
            SkySide B = {0.f, 0.f, 0.f, 0.f};
            if (has_hi) B = sky_side(L.sky[hi], L, hi, t, sg);
            const float cs = cot * K.sky_scale;
            g[0] += cs * (wlo * A.t + whi * B.t);
            g[1 + lo] += cs * wlo * A.a;
            if (has_hi) g[1 + hi] += cs * whi * B.a;
            g[15] += cs * (wlo * A.e + whi * B.e);   // unit elevation
            const float gam = cs * (wlo * A.gm + whi * B.gm);
#pragma unroll
            for (int k = 0; k < 3; ++k) g[12 + k] += gam * dgs[k];
            if (t.hit_sun) {
                float sa = render_sun_spec(K.sun_table, pos, lo, xs), dsa = render_sun_spec(dsun_tab, pos, lo, xs);
                float sun = sa, dsun = dsa;
                if (f != 0.f) {
                    float sb = hi < kNbWavelengths ? render_sun_spec(K.sun_table, pos, hi, xs) : 0.f;
                    float dsb = hi < kNbWavelengths ? render_sun_spec(dsun_tab, pos, hi, xs) : 0.f;
                    sun = lerpf_(sa, sb, f);
                    dsun = lerpf_(dsa, dsb, f);
                }
                float ld = sun_limb_darkening(K.sun_ld, lo, hi, f, cp), dldc = 0.f;
#pragma unroll 1
                for (int j = 1; j < kNbSunLdParams; ++j) {
                    float a = K.sun_ld[lo * kNbSunLdParams + j], coef = a;
                    if (f != 0.f) coef = lerpf_(a, hi < kNbWavelengths ? K.sun_ld[hi * kNbSunLdParams + j] : 0.f, f);
                    dldc += (float)j * powif_(cp, j - 1) * coef;
                }
                const float sc = K.sun_scale * K.area_ratio;
                g[0] += cot * sc * dsun * ld;
#pragma unroll
                for (int k = 0; k < 3; ++k) g[12 + k] += cot * sc * sun * dldc * dcps[k];
            }
        }
    }
    block_reduce_grad(L, g, partials);
}

// ======================================================================
// extern "C" entry points (hipModuleGetFunction names)
// ======================================================================
#define SS_EVAL_RGB(NAME, VEC, FAST, NEG)                                                                          \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_RGB_ATTR void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, const float* wx, const float* wy, const float* wz, const uint8_t* active, size_t n,     \
        float* out, size_t ostride, float sign) {                                                              \
        (void)sign;                                                                                            \
        eval_rgb_body<VEC, FAST, NEG>(*Kp, wx, wy, wz, active, n, out, ostride);                                 \
    }
// eval(si): wo = -wi (NEG); eval_direction(ds): wo = ds.d (the _dir kernels)
SS_EVAL_RGB(sunsky_eval_rgb_v4_fast, 4, true, true)
SS_EVAL_RGB(sunsky_eval_rgb_v1_fast, 1, true, true)
SS_EVAL_RGB(sunsky_eval_rgb_v4_ref, 4, false, true)
SS_EVAL_RGB(sunsky_eval_rgb_v1_ref, 1, false, true)
SS_EVAL_RGB(sunsky_eval_rgb_v4_dir_fast, 4, true, false)
SS_EVAL_RGB(sunsky_eval_rgb_v1_dir_fast, 1, true, false)
SS_EVAL_RGB(sunsky_eval_rgb_v4_dir_ref, 4, false, false)
SS_EVAL_RGB(sunsky_eval_rgb_v1_dir_ref, 1, false, false)

#define SS_EVAL_SPEC_BCAST(NAME, VEC, FAST)                                                                   \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_NODES_ATTR void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, LambdaSet L, const float* wx, const float* wy, const float* wz, const uint8_t* active,  \
        size_t n, float* out, size_t ostride, float sign) {                                                    \
        (void)sign;   /* always eval(si): wo = -wi */                                                         \
        eval_spec_bcast_body<VEC, FAST, true>(*Kp, L, wx, wy, wz, active, n, out, ostride);                      \
    }
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v4_fast, 4, true)
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v1_fast, 1, true)
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v4_ref, 4, false)
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v1_ref, 1, false)

#define SS_EVAL_SPEC_NODES(NAME, VEC, FAST)                                                                   \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_NODES_ATTR void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, LambdaSet L, const float* wx, const float* wy, const float* wz, const uint8_t* active,  \
        size_t n, float* out, size_t ostride, float sign) {                                                    \
        (void)L;                                                                                               \
        (void)sign;                                                                                            \
        eval_spec_nodes_body<VEC, FAST, true>(*Kp, wx, wy, wz, active, n, out, ostride);                         \
    }
SS_EVAL_SPEC_NODES(sunsky_eval_spec_nodes_v4_fast, 4, true)
SS_EVAL_SPEC_NODES(sunsky_eval_spec_nodes_v4_ref, 4, false)

#define SS_EVAL_SPEC_RAYS(NAME, VEC, FAST, NEG, NL)                                                                \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_RAYS_ATTR void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, const float* wx, const float* wy, const float* wz, const float* lam, size_t lstride,    \
        int nlam, const uint8_t* active, size_t n, float* out, size_t ostride, float sign) {                   \
        (void)sign;                                                                                            \
        eval_spec_rays_body<VEC, FAST, NEG, NL>(*Kp, wx, wy, wz, lam, lstride, nlam, active, n, out, ostride);   \
    }
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v4_fast, 4, true, true, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v1_fast, 1, true, true, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v4_ref, 4, false, true, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v1_ref, 1, false, true, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v4_dir_fast, 4, true, false, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v1_dir_fast, 1, true, false, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v4_dir_ref, 4, false, false, 0)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_v1_dir_ref, 1, false, false, 0)
// exactly 4 wavelengths per ray (Mitsuba's Spectrum<Float, 4>), VEC = 4 over rays
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays4_v4_fast, 4, true, true, 4)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays4_v4_ref, 4, false, true, 4)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays4_v4_dir_fast, 4, true, false, 4)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays4_v4_dir_ref, 4, false, false, 4)


#define SS_SAMPLE_DIRECTION(NAME, FAST, SPEC, LEAN)                                                           \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, const float* ux, const float* uy, const float* px, const float* py, const float* pz,   \
        const float* lam, size_t lstride, int nlam, const uint8_t* active, size_t n, float* dx, float* dy,     \
        float* dz, float* pdf, float* dist, float* opx, float* opy, float* opz, float* weight, size_t wstride) { \
        sample_direction_body<FAST, SPEC, LEAN>(*Kp, ux, uy, px, py, pz, lam, lstride, nlam, active, n, dx, dy,  \
                                                dz, pdf, dist, opx, opy, opz, weight, wstride);                \
    }
SS_SAMPLE_DIRECTION(sunsky_sample_direction_rgb_fast, true, false, false)
SS_SAMPLE_DIRECTION(sunsky_sample_direction_rgb_ref, false, false, false)
SS_SAMPLE_DIRECTION(sunsky_sample_direction_spec_fast, true, true, false)
SS_SAMPLE_DIRECTION(sunsky_sample_direction_spec_ref, false, true, false)
// the unsorted LEAN RGB fast form, kept for A/B timing against the wave-sorted product kernel
SS_SAMPLE_DIRECTION(sunsky_sample_direction_rgb_lean_plain_fast, true, false, true)
// reference-precision twin of the unsorted LEAN form (the C ABI loads every kernel in both precisions)
SS_SAMPLE_DIRECTION(sunsky_sample_direction_rgb_lean_plain_ref, false, false, true)
// LEAN spectral: Mitsuba's 4 wavelengths per sample take the unrolled branchless body
#define SS_SAMPLE_DIRECTION_SPEC_LEAN(NAME, FAST)                                                              \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_SPEC_SAMPLE_ATTR void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, const float* ux, const float* uy, const float* px, const float* py, const float* pz,   \
        const float* lam, size_t lstride, int nlam, const uint8_t* active, size_t n, float* dx, float* dy,     \
        float* dz, float* pdf, float* dist, float* opx, float* opy, float* opz, float* weight, size_t wstride) { \
        if (nlam == 4)                                                                                         \
            sample_direction_spec4_body<FAST>(*Kp, ux, uy, lam, lstride, n, dx, dy, dz, pdf, weight, wstride);   \
        else                                                                                                   \
            sample_direction_body<FAST, true, true>(*Kp, ux, uy, px, py, pz, lam, lstride, nlam, active, n, dx,  \
                                                    dy, dz, pdf, dist, opx, opy, opz, weight, wstride);        \
    }
SS_SAMPLE_DIRECTION_SPEC_LEAN(sunsky_sample_direction_spec_lean_fast, true)
SS_SAMPLE_DIRECTION_SPEC_LEAN(sunsky_sample_direction_spec_lean_ref, false)
// LEAN spectral sample_direction at 4 wavelengths in wave-sorted windows of SS_SPEC_SORT_R x 64
// samples (the C ABI's call when nlam == 4): bitwise the unsorted LEAN kernel
// (test_spectral_sorted_kernel_bitwise_vs_unsorted)
#ifndef SS_SPEC_SORT_R
#define SS_SPEC_SORT_R 3
#endif
// 4 waves/SIMD (127 VGPRs, 2 spilled; 131 and 3 waves without): interleaved A/B against the
// unsorted LEAN kernel 0.963 (3 waves: 1.027; R = 2: 0.999, at 4 waves 0.994), profiles/r03_v13_ab_spec_sorted.log
#ifndef SS_SPEC_SORTED_ATTR
#define SS_SPEC_SORTED_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#endif
#define SS_SAMPLE_DIRECTION_SPEC4_SORTED(NAME, FAST, R)                                                       \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_SPEC_SORTED_ATTR void NAME(                           \
        const SunskyKArgs* __restrict__ Kp, const float* ux, const float* uy, const float* px, const float* py, const float* pz,   \
        const float* lam, size_t lstride, int nlam, const uint8_t* active, size_t n, float* dx, float* dy,     \
        float* dz, float* pdf, float* dist, float* opx, float* opy, float* opz, float* weight, size_t wstride) { \
        sample_direction_spec4_sorted_body<FAST, R>(*Kp, ux, uy, lam, lstride, n, dx, dy, dz, pdf, weight, wstride); \
    }
SS_SAMPLE_DIRECTION_SPEC4_SORTED(sunsky_sample_direction_spec_lean4_sorted_fast, true, SS_SPEC_SORT_R)
SS_SAMPLE_DIRECTION_SPEC4_SORTED(sunsky_sample_direction_spec_lean4_sorted_ref, false, SS_SPEC_SORT_R)
// Mitsuba's unmasked spectral DirectionSample call (it.p in, ds.dist / ds.p out), 4 wavelengths
#define SS_SAMPLE_DIRECTION_SPEC4_POS_SORTED(NAME, FAST, R)                                                   \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_SPEC_SORTED_ATTR void NAME(                           \
        const SunskyKArgs* __restrict__ Kp, const float* ux, const float* uy, const float* px, const float* py, const float* pz,   \
        const float* lam, size_t lstride, int nlam, const uint8_t* active, size_t n, float* dx, float* dy,     \
        float* dz, float* pdf, float* dist, float* opx, float* opy, float* opz, float* weight, size_t wstride) { \
        sample_direction_spec4_sorted_body<FAST, R, true>(*Kp, ux, uy, lam, lstride, n, dx, dy, dz, pdf, weight, \
                                                          wstride, px, py, pz, dist, opx, opy, opz);          \
    }
SS_SAMPLE_DIRECTION_SPEC4_POS_SORTED(sunsky_sample_direction_spec_pos_sorted_fast, true, SS_SPEC_SORT_R)
SS_SAMPLE_DIRECTION_SPEC4_POS_SORTED(sunsky_sample_direction_spec_pos_sorted_ref, false, SS_SPEC_SORT_R)
// the previous LEAN spectral form (wavelength loop, lambda not prefetched), for A/B timing
SS_SAMPLE_DIRECTION(sunsky_sample_direction_spec_lean_loop_fast, true, true, true)

#define SS_SAMPLE_DIRECTION_SORTED(NAME, FAST, R, MODE)                                                           \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_RGB_SORTED_ATTR void NAME(                            \
        const SunskyKArgs* __restrict__ Kp, const float* ux, const float* uy, const float* px, const float* py, const float* pz,   \
        const float* lam, size_t lstride, int nlam, const uint8_t* active, size_t n, float* dx, float* dy,     \
        float* dz, float* pdf, float* dist, float* opx, float* opy, float* opz, float* weight, size_t wstride) { \
        sample_direction_sorted_body<FAST, R, MODE>(*Kp, ux, uy, px, py, pz, active, n, dx, dy, dz, pdf, dist, \
                                                    opx, opy, opz, weight, wstride);                           \
    }
// LEAN RGB sample_direction (the C ABI's common call): wave-sorted windows of 4 x 64
// samples.  R = 4 measured fastest (kbench sweep, profiles/r02_v11_ws_sweep.log): R = 2 / 3
// sort less of the divergence away, R = 5 / 6 are held to 3 waves/SIMD by their LDS.  Both
// precisions reproduce the general kernel's bits (test_sample_direction_lean_kernel_bitwise,
// test_wave_sorted_rgb_kernels_bitwise_vs_unsorted) since the file contracts within
// expressions only (the pragma at the top).
SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_lean_fast, true, SS_SORT_R, kSortLean)
SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_lean_ref, false, SS_SORT_R, kSortLean)
// The general call (it.p, ds.dist, ds.p, mask) in the same windows: bitwise the unsorted kernel
// (test_wave_sorted_rgb_kernels_bitwise_vs_unsorted) but slower: 2 % in round 2 (125 VGPRs and 28
// SGPR spills, profiles/r02_v13_ab_sample_full.log), 14 % against the round-3 unsorted general kernel,
// 10 % with the mask and it.p prefetched (114 VGPRs, 42 SGPR spills;
// profiles/r03_v23_ab_sample_full.log), so the C ABI keeps the unsorted general kernel and takes this one
// only with SUNSKY_AMD_SORTED_GENERAL_SAMPLING=1 (test_wave_sorted_rgb_kernels_bitwise_vs_unsorted).
SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_full_sorted_fast, true, 4, kSortFull)
SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_full_sorted_ref, false, 4, kSortFull)
// Mitsuba's DirectionSample call (it.p in, ds.dist / ds.p out, no mask: path.cpp:216 ->
// scene.cpp:295-348) in the LEAN windows, the next window's it.p prefetched with its u.
SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_pos_sorted_fast, true, SS_SORT_R, kSortPos)
SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_pos_sorted_ref, false, SS_SORT_R, kSortPos)


// The FAST 4-direction kernel at 8 waves/SIMD: left alone the compiler holds 96 SGPRs (7 waves);
// amdgpu_waves_per_eu(8) fits it in 78 without spills, 0.9 % faster at 64M and 2.3 % at 16M
// (interleaved A/B, profiles/r06_v17_ab_pdf_direction_8waves.log).  The reference form would
// spill 14 SGPRs there and keeps the default.
#define SS_PDF_W8 __attribute__((amdgpu_waves_per_eu(8)))
#define SS_PDF_DIRECTION(NAME, VEC, FAST, ATTR)                                                               \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) ATTR void NAME(                                          \
        const SunskyKArgs* __restrict__ Kp, const float* dx, const float* dy, const float* dz, const uint8_t* active, size_t n,     \
        float* pdf) {                                                                                          \
        pdf_direction_body<VEC, FAST>(*Kp, dx, dy, dz, active, n, pdf);                                          \
    }
SS_PDF_DIRECTION(sunsky_pdf_direction_v4_fast, 4, true, SS_PDF_W8)
SS_PDF_DIRECTION(sunsky_pdf_direction_v1_fast, 1, true, )
SS_PDF_DIRECTION(sunsky_pdf_direction_v4_ref, 4, false, )
SS_PDF_DIRECTION(sunsky_pdf_direction_v1_ref, 1, false, )

// TESTING ONLY (sunsky_emitter_sun_segments): the segment add_sun_terms picks for a disc
// direction with this cos theta, i.e. the index every eval / sampling kernel of the
// precision uses (sunsky.cpp:579-584).
template <bool FAST>
__device__ __forceinline__ void debug_sun_segments_body(const SunskyKArgs& K, const float* __restrict__ z, size_t n,
                                                        int* __restrict__ pos) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float3_ n_ = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
        DirTerms t = dir_terms<FAST>(K, n_, true);
        t.cos_theta = z[i];
        t.hit_sun = true;
        add_sun_terms<FAST>(K, t);
        pos[i] = t.sun_pos;
    }
}
#define SS_DEBUG_SUN_SEGMENTS(NAME, FAST)                                                                     \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(const SunskyKArgs* __restrict__ Kp, const float* z,  \
                                                                size_t n, int* pos) {                         \
        debug_sun_segments_body<FAST>(*Kp, z, n, pos);                                                         \
    }
SS_DEBUG_SUN_SEGMENTS(sunsky_debug_sun_segments_fast, true)
SS_DEBUG_SUN_SEGMENTS(sunsky_debug_sun_segments_ref, false)

#define SS_SAMPLE_WAVELENGTHS(NAME, FAST, SPEC)                                                               \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, const float* wx, const float* wy, const float* wz, const float* sample,                 \
        const uint8_t* active, size_t n, float* lam, size_t lstride, float* weight, size_t wstride) {          \
        sample_wavelengths_body<FAST, SPEC>(*Kp, wx, wy, wz, sample, active, n, lam, lstride, weight, wstride);  \
    }
SS_SAMPLE_WAVELENGTHS(sunsky_sample_wavelengths_rgb_fast, true, false)
SS_SAMPLE_WAVELENGTHS(sunsky_sample_wavelengths_rgb_ref, false, false)
SS_SAMPLE_WAVELENGTHS(sunsky_sample_wavelengths_spec_fast, true, true)
SS_SAMPLE_WAVELENGTHS(sunsky_sample_wavelengths_spec_ref, false, true)

#define SS_SAMPLE_RAY(NAME, FAST, SPEC)                                                                       \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        const SunskyKArgs* __restrict__ Kp, const float* wls, const float* s2x, const float* s2y, const float* s3x,                 \
        const float* s3y, const uint8_t* active, size_t n, float* ox, float* oy, float* oz, float* dx,         \
        float* dy, float* dz, float* lam, size_t lstride, float* weight, size_t wstride) {                     \
        sample_ray_body<FAST, SPEC>(*Kp, wls, s2x, s2y, s3x, s3y, active, n, ox, oy, oz, dx, dy, dz, lam,        \
                                    lstride, weight, wstride);                                                 \
    }
#ifndef SS_RAY_SORT_R
#define SS_RAY_SORT_R 4
#endif
// 4 waves/SIMD (125 VGPRs; 131 and 3 waves without): interleaved A/B against the unsorted
// kernel 0.922 (3 waves 0.976; R = 3: 0.946, at 4 waves 0.955), profiles/r03_v18_ab_sample_ray_sorted.log
#ifndef SS_RAY_SORTED_ATTR
#define SS_RAY_SORTED_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#endif
#define SS_SAMPLE_RAY_RGB_SORTED(NAME, FAST, R)                                                               \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_RAY_SORTED_ATTR void NAME(                           \
        const SunskyKArgs* __restrict__ Kp, const float* wls, const float* s2x, const float* s2y, const float* s3x,                 \
        const float* s3y, const uint8_t* active, size_t n, float* ox, float* oy, float* oz, float* dx,         \
        float* dy, float* dz, float* lam, size_t lstride, float* weight, size_t wstride) {                     \
        sample_ray_rgb_sorted_body<FAST, R>(*Kp, s2x, s2y, s3x, s3y, n, ox, oy, oz, dx, dy, dz, lam, lstride,   \
                                            weight, wstride);                                                  \
    }
// RGB sample_ray without a mask (the C ABI's call then): wave-sorted windows, bitwise the
// unsorted kernel (test_sample_ray_sorted_bitwise_vs_unsorted)
SS_SAMPLE_RAY_RGB_SORTED(sunsky_sample_ray_rgb_sorted_fast, true, SS_RAY_SORT_R)
SS_SAMPLE_RAY_RGB_SORTED(sunsky_sample_ray_rgb_sorted_ref, false, SS_RAY_SORT_R)
SS_SAMPLE_RAY(sunsky_sample_ray_rgb_fast, true, false)
SS_SAMPLE_RAY(sunsky_sample_ray_rgb_ref, false, false)
SS_SAMPLE_RAY(sunsky_sample_ray_spec_fast, true, true)
SS_SAMPLE_RAY(sunsky_sample_ray_spec_ref, false, true)

#ifndef SS_DIFFUSE_SPEC_ATTR   // probe builds: occupancy of the FAST spectral diffuse caller
#define SS_DIFFUSE_SPEC_ATTR
#endif
#define SS_DIRECT_DIFFUSE(NAME, FAST, SPEC, ATTR)                                                             \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) ATTR void NAME(                                         \
        const SunskyKArgs* __restrict__ Kp, const float* nx, const float* ny, const float* nz, const float* rho, const float* lam, \
        size_t lstride, int nlam, uint32_t seed, uint32_t spp, const uint8_t* vis, size_t vstride, size_t n,     \
        float* out, size_t ostride) {                                                                          \
        direct_diffuse_body<FAST, SPEC>(*Kp, nx, ny, nz, rho, lam, lstride, nlam, seed, spp, vis, vstride, n, out, \
                                        ostride);                                                              \
    }
SS_DIRECT_DIFFUSE(sunsky_direct_diffuse_rgb_fast, true, false, )
SS_DIRECT_DIFFUSE(sunsky_direct_diffuse_rgb_ref, false, false, )
SS_DIRECT_DIFFUSE(sunsky_direct_diffuse_spec_fast, true, true, SS_DIFFUSE_SPEC_ATTR)
SS_DIRECT_DIFFUSE(sunsky_direct_diffuse_spec_ref, false, true, )

#define SS_DIRECT_CONDUCTOR(NAME, FAST, SPEC, ATTR)                                                           \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) ATTR void NAME(                                          \
        const SunskyKArgs* __restrict__ Kp, ConductorArgs C, const float* nx, const float* ny, const float* nz,  \
        const float* vx, const float* vy, const float* vz, const float* lam, size_t lstride, int nlam, uint32_t seed, \
        uint32_t spp, const uint8_t* vis, size_t vstride, size_t n, float* out, size_t ostride) {              \
        direct_conductor_body<FAST, SPEC>(*Kp, C, nx, ny, nz, vx, vy, vz, lam, lstride, nlam, seed, spp, vis,    \
                                          vstride, n, out, ostride);                                           \
    }
// FAST at 4 waves/SIMD (128 VGPRs, 10 spilled): interleaved A/B 5.7 % faster than the
// compiler's 149 VGPRs at 3 waves (profiles/r03_v12_ab_conductor.log)
SS_DIRECT_CONDUCTOR(sunsky_direct_conductor_rgb_fast, true, false, SS_CONDUCTOR_ATTR)
SS_DIRECT_CONDUCTOR(sunsky_direct_conductor_rgb_ref, false, false, )
SS_DIRECT_CONDUCTOR(sunsky_direct_conductor_spec_fast, true, true, SS_CONDUCTOR_ATTR)
SS_DIRECT_CONDUCTOR(sunsky_direct_conductor_spec_ref, false, true, )

#define SS_DIRECT_CONDUCTOR_RAYS(NAME, FAST)                                                                  \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                              \
        const SunskyKArgs* __restrict__ Kp, ConductorArgs C, const float* nx, const float* ny, const float* nz,  \
        const float* vx, const float* vy, const float* vz, uint32_t seed, uint32_t spp, size_t n, float* ex,     \
        float* ey, float* ez, float* bx, float* by, float* bz, size_t rstride, float* bw, int nw) {            \
        direct_conductor_rays_body<FAST>(*Kp, C, nx, ny, nz, vx, vy, vz, seed, spp, n, ex, ey, ez, bx, by, bz,   \
                                         rstride, bw, nw);                                                     \
    }
SS_DIRECT_CONDUCTOR_RAYS(sunsky_direct_conductor_rays_fast, true)
SS_DIRECT_CONDUCTOR_RAYS(sunsky_direct_conductor_rays_ref, false)

#define SS_DIRECT_DIFFUSE_RAYS(NAME, FAST)                                                                    \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                              \
        const SunskyKArgs* __restrict__ Kp, const float* nx, const float* ny, const float* nz, uint32_t seed,   \
        uint32_t spp, size_t n, float* ex, float* ey, float* ez, float* bx, float* by, float* bz, size_t rstride) { \
        direct_diffuse_rays_body<FAST>(*Kp, nx, ny, nz, seed, spp, n, ex, ey, ez, bx, by, bz, rstride);         \
    }
SS_DIRECT_DIFFUSE_RAYS(sunsky_direct_diffuse_rays_fast, true)
SS_DIRECT_DIFFUSE_RAYS(sunsky_direct_diffuse_rays_ref, false)

extern "C" __global__ __launch_bounds__(SS_BLOCK) void sunsky_eval_jvp_rgb(
    const SunskyKArgs* __restrict__ Kp, const float* jvp, const float* wx, const float* wy, const float* wz, const uint8_t* active,
    size_t n, float* out, float* dout, size_t ostride, float sign) {
    eval_jvp_rgb_body(*Kp, jvp, wx, wy, wz, active, n, out, dout, ostride, sign);
}
extern "C" __global__ __launch_bounds__(SS_BLOCK) void sunsky_eval_jvp_spec(
    const SunskyKArgs* __restrict__ Kp, const float* jvp, const float* wx, const float* wy, const float* wz, const float* lam,
    size_t lstride, int nlam, const uint8_t* active, size_t n, float* out, float* dout, size_t ostride, float sign) {
    eval_jvp_spec_body(*Kp, jvp, wx, wy, wz, lam, lstride, nlam, active, n, out, dout, ostride, sign);
}

extern "C" __global__ __launch_bounds__(SS_BLOCK) void sunsky_eval_vjp_rgb(
    const SunskyKArgs* __restrict__ Kp, const float* vjp, const float* wx, const float* wy, const float* wz, const uint8_t* active,
    size_t n, const float* dout, size_t ostride, float sign, float* partials) {
    eval_vjp_rgb_body(*Kp, vjp, wx, wy, wz, active, n, dout, ostride, sign, partials);
}
#ifndef SS_VJP_SPEC_ATTR
#define SS_VJP_SPEC_ATTR
#endif
extern "C" __global__ __launch_bounds__(SS_BLOCK) SS_VJP_SPEC_ATTR void sunsky_eval_vjp_spec(
    const SunskyKArgs* __restrict__ Kp, const float* vjp, const float* wx, const float* wy, const float* wz, const float* lam,
    size_t lstride, int nlam, const uint8_t* active, size_t n, const float* dout, size_t ostride, float sign,
    float* partials) {
    eval_vjp_spec_body(*Kp, vjp, wx, wy, wz, lam, lstride, nlam, active, n, dout, ostride, sign, partials);
}
// grad[p] += sum over blocks (in block order) of partials[block][p]; one wave.
// grad[p] += sum over blocks of partials[b][p], one 256-thread workgroup: thread (s, p)
// sums blocks s, s + 16, s + 32, ... in order, then thread p adds the 16 segment sums
// in order.  A fixed summation order (deterministic), 16 independent load streams per
// gradient instead of one serial chain over all blocks.
extern "C" __global__ __launch_bounds__(256) void sunsky_grad_reduce(const float* partials, unsigned nblocks,
                                                                      float* grad) {
    constexpr int kSeg = 256 / kGradCount;
    __shared__ float seg[kSeg][kGradCount];
    const int p = threadIdx.x % kGradCount, sgi = threadIdx.x / kGradCount;
    float acc = 0.f;
    // 16 loads in flight per thread, then the adds in block order (the summation order of
    // the one-load-per-step loop, which waited out a load latency per block: 26 us per call)
    constexpr unsigned kU = 16;
    unsigned b = sgi;
    for (; b + (kU - 1) * kSeg < nblocks; b += kU * kSeg) {
        float v[kU];
#pragma unroll
        for (unsigned u = 0; u < kU; ++u) v[u] = partials[(size_t)(b + u * kSeg) * kGradCount + p];
#pragma unroll
        for (unsigned u = 0; u < kU; ++u) acc += v[u];
    }
    for (; b < nblocks; b += kSeg) acc += partials[(size_t)b * kGradCount + p];
    seg[sgi][p] = acc;
    __syncthreads();
    if (threadIdx.x < kGradCount) {
        float t = 0.f;
        for (int k = 0; k < kSeg; ++k) t += seg[k][threadIdx.x];
        grad[threadIdx.x] += t;
    }
}

#define SS_BAKE(NAME_RGB, NAME_SPEC, FAST)                                                                    \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME_RGB(const SunskyKArgs* __restrict__ Kp, LatLong G, float* out,      \
                                                                    size_t ostride) {                          \
        bake_rgb_body<FAST>(*Kp, G, out, ostride);                                                               \
    }                                                                                                          \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME_SPEC(const SunskyKArgs* __restrict__ Kp, LatLong G, LambdaSet L,    \
                                                                     float* out, size_t ostride) {             \
        bake_spec_body<FAST>(*Kp, G, L, out, ostride);                                                           \
    }
SS_BAKE(sunsky_bake_latlong_rgb_fast, sunsky_bake_latlong_spec_fast, true)
SS_BAKE(sunsky_bake_latlong_rgb_ref, sunsky_bake_latlong_spec_ref, false)

// ======================================================================
// Device staging of parameters_changed (sunsky.cpp:242-285): the radiance tables
// (compute_radiance_params, sunsky.h:158-231; compute_sun_params, :404-419) and the
// JIT sampling weight / wavelength distribution (estimate_sky_sun_ratio,
// sunsky.cpp:772-886) written straight into the emitter's device state, on the
// caller's stream.  The host writes the rest of the state (geometry, TGMM) with an
// async copy just before; launches that follow on the stream see the new state.
// ======================================================================
struct StageArgs {                 // mirrors the host-side struct (sunsky_capi.cpp)
    SunskyKArgs* state;            // the emitter's device state (sky[], fsky[] written)
    float* sun_table;              // its turbidity-lerped sun table (written)
    const float* sky_params_ds;    // (10 T, 2 albedo, 6 ctrl, nch, 9)
    const float* sky_rad_ds;       // (10, 2, 6, nch)
    const float* sun_rad_ds;       // (10, sun_block)
    RadianceStage rs;
    float albedo[kNbWavelengths];
    int nch, variant, sun_block;
    float sky_scale;
};

// One workgroup: every sky coefficient / radiance entry, every sun-table entry, then
// one thread per channel folds it (sunsky_staging.h: the host model's arithmetic).
extern "C" __global__ __launch_bounds__(256) void sunsky_stage_radiance(StageArgs A) {
    __shared__ float p[kNbWavelengths * kNbSkyParams];
    __shared__ float r[kNbWavelengths];
    const int t = threadIdx.x;
    const int np = A.nch * kNbSkyParams;
    for (int e = t; e < np; e += blockDim.x)
        p[e] = radiance_param(A.sky_params_ds, np, e, A.rs, A.albedo[e / kNbSkyParams]);
    for (int e = t; e < A.nch; e += blockDim.x) r[e] = radiance_param(A.sky_rad_ds, A.nch, e, A.rs, A.albedo[e]);
    for (int i = t; i < A.sun_block; i += blockDim.x) A.sun_table[i] = sun_param(A.sun_rad_ds, A.sun_block, i, A.rs);
    __syncthreads();
    if (t < A.nch) {
        SkyChannel ch;
        FastChannel f;
        fold_channel(&p[t * kNbSkyParams], r[t], A.variant, A.sky_scale, &ch, &f);
        A.state->sky[t] = ch;
        A.state->fsky[t] = f;
    }
}

constexpr int kQuadBlock = 256;    // one quadrature row per workgroup, one point per thread

// Tangent tables of eval_jvp / eval_vjp (sunsky_staging.h TangentArgs): one float per
// thread, fp64 Bezier derivatives of the device-resident datasets, the same code as the
// host model's eval_tangent.
extern "C" __global__ __launch_bounds__(256) void sunsky_stage_tangent(TangentArgs A) {
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < A.total; idx += gridDim.x * blockDim.x)
        A.out[idx] = tangent_buffer_value(A, idx);
}

struct QuadArgs {                  // mirrors the host-side struct (sunsky_capi.cpp)
    SunskyKArgs* state;
    const float* qx;               // 200 Gauss-Legendre nodes / weights (fp32)
    const float* qw;
    float* rows;                   // [2][nq][nch] row sums (sky, sun)
    int nq, nch;
    float cie_y[kNbWavelengths];
    float sky_scale, sun_scale;
    int* status;                   // set to 1 by a rejected staging (negative wavelength-distribution entry)
};

// Workgroup j = quadrature row j, thread i = point (i, j): its direction terms once,
// every channel's sky and sun terms, then a fixed-shape tree reduction over the row's
// points in LDS (deterministic: the same order on every run).
extern "C" __global__ __launch_bounds__(kQuadBlock) void sunsky_stage_quad_points(QuadArgs A) {
    __shared__ float red[2 * kNbWavelengths][kQuadBlock];
    const int j = blockIdx.x, i = threadIdx.x;
    const SunskyKArgs& K = *A.state;
    float as[kNbWavelengths], au[kNbWavelengths];
#pragma unroll
    for (int c = 0; c < kNbWavelengths; ++c) as[c] = au[c] = 0.f;
    if (i < A.nq) {
        const QuadDir d = quad_dir(K, A.qx, A.qw, i, j);
        const float wj = A.qw[j];
#pragma unroll
        for (int c = 0; c < kNbWavelengths; ++c)
            if (c < A.nch) quad_channel(K, K.sun_table, K.sun_ld, d, wj, c, &as[c], &au[c]);
    }
#pragma unroll
    for (int c = 0; c < kNbWavelengths; ++c) {
        red[c][i] = as[c];
        red[kNbWavelengths + c][i] = au[c];
    }
    __syncthreads();
    for (int h = kQuadBlock / 2; h > 0; h >>= 1) {
        if (i < h)
#pragma unroll
            for (int c = 0; c < 2 * kNbWavelengths; ++c) red[c][i] += red[c][i + h];
        __syncthreads();
    }
    if (i < A.nch) {
        A.rows[(size_t)j * A.nch + i] = red[i][0];
        A.rows[(size_t)(A.nq + j) * A.nch + i] = red[kNbWavelengths + i][0];
    }
}

// One workgroup: the row sums to LDS, thread c adds channel c's rows in row order, then
// one thread derives the sampling weight and the wavelength distribution (quad_finish).
extern "C" __global__ __launch_bounds__(256) void sunsky_stage_quad_finish(QuadArgs A) {
    __shared__ float rows[2 * 200 * kNbWavelengths];
    __shared__ float sky[kNbWavelengths], sun[kNbWavelengths];
    const int total = 2 * A.nq * A.nch;
    for (int i = threadIdx.x; i < total; i += blockDim.x) rows[i] = A.rows[i];
    __syncthreads();
    const int c = threadIdx.x;
    if (c < A.nch) {
        float s = 0.f, u = 0.f;
        for (int j = 0; j < A.nq; ++j) {
            s += rows[j * A.nch + c];
            u += rows[(A.nq + j) * A.nch + c];
        }
        sky[c] = s;
        sun[c] = u;
    }
    __syncthreads();
    if (c == 0) {
        const bool ok = quad_finish(A.state, sky, sun, A.cie_y, A.sky_scale, A.sun_scale);
        if (!ok) *A.status = 1;   // sticky until the host reads it back (sync_host)
    }
}
