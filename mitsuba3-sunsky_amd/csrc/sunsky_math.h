// sunsky_math.h -- the emitter's per-direction math, usable from the HIP
// kernels (device) and from the host staging (estimate_sky_sun_ratio's
// quadrature runs these same functions on the CPU).  Every function names the
// reference code it implements.  Third-party arithmetic the reference takes
// from Dr.Jit 1.0.4 (unit_angle, sphdir, lerp, erfinv) is written from the
// published algorithms.
#pragma once
#include <math.h>

#include "sunsky_types.h"

namespace sunsky {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kTwoPi = 6.28318530717958647692f;
constexpr float kHalfPi = 1.57079632679489661923f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kInvTwoPi = 0.15915494309189533577f;
constexpr float kSqrtTwo = 1.41421356237309504880f;
constexpr float kInvSqrtTwo = 0.70710678118654752440f;
constexpr float kEpsilon = 5.9604644775390625e-08f;        // dr::Epsilon<float> = 2^-24
constexpr float kOneMinusEpsilon = 0.99999994039535522461f;  // dr::OneMinusEpsilon<float>

struct float3_ { float x, y, z; };

SS_HD inline float3_ mk3(float x, float y, float z) { float3_ r = {x, y, z}; return r; }

// dr::lerp(a, b, t) = fmadd(b, t, fnmadd(a, t, a))
SS_HD inline float lerpf_(float a, float b, float t) { return fmaf(b, t, fmaf(-a, t, a)); }
SS_HD inline float safe_sqrtf_(float x) { return sqrtf(x > 0.f ? x : 0.f); }
SS_HD inline float mulsignf_(float a, float b) { return signbit(b) ? -a : a; }
SS_HD inline float mulsign_negf_(float a, float b) { return signbit(b) ? a : -a; }
SS_HD inline float dot3(float3_ a, float3_ b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
SS_HD inline float powif_(float x, int k) { float r = 1.f; for (int i = 0; i < k; ++i) r *= x; return r; }

// Transform::operator*(Vector) / transform_affine on vectors, transform.h:149-158
SS_HD inline float3_ xform_vec(const float* m, float3_ v) {
    return mk3(fmaf(m[2], v.z, fmaf(m[1], v.y, m[0] * v.x)),
               fmaf(m[5], v.z, fmaf(m[4], v.y, m[3] * v.x)),
               fmaf(m[8], v.z, fmaf(m[7], v.y, m[6] * v.x)));
}

// Dr.Jit unit_angle(a, b) (sunsky.cpp:311): 2 asin(|b -/+ a| / 2), robust near 0 and pi
SS_HD inline float unit_angle(float3_ a, float3_ b) {
    float d = dot3(a, b);
    float3_ v = mk3(b.x - mulsignf_(a.x, d), b.y - mulsignf_(a.y, d), b.z - mulsignf_(a.z, d));
    float temp = 2.f * asinf(0.5f * sqrtf(dot3(v, v)));
    return d >= 0.f ? temp : kPi - temp;
}

// Dr.Jit unit_angle_z(v) (sunsky.h:87)
SS_HD inline float unit_angle_z(float3_ v) {
    float dz = v.z - mulsignf_(1.f, v.z);
    float temp = 2.f * asinf(0.5f * sqrtf(fmaf(v.x, v.x, fmaf(v.y, v.y, dz * dz))));
    return v.z >= 0.f ? temp : kPi - temp;
}

// Dr.Jit sphdir(theta, phi) (sunsky.cpp:688)
SS_HD inline float3_ sphdir(float theta, float phi) {
    float st = sinf(theta), ct = cosf(theta), sp = sinf(phi), cp = cosf(phi);
    return mk3(cp * st, sp * st, ct);
}

// coordinate_system, include/mitsuba/core/vector.h:116-137
SS_HD inline void coordinate_system(float3_ n, float3_* s, float3_* t) {
    float sign = copysignf(1.f, n.z);
    float a = -1.f / (sign + n.z);
    float b = n.x * n.y * a;
    *s = mk3(mulsignf_(n.x * n.x * a, n.z) + 1.f, mulsignf_(b, n.z), mulsign_negf_(n.x, n.z));
    *t = mk3(b, fmaf(n.y, n.y * a, sign), -n.y);
}

// Frame::to_world, frame.h:36-38
SS_HD inline float3_ frame_to_world(float3_ s, float3_ t, float3_ n, float3_ v) {
    return mk3(fmaf(n.x, v.z, fmaf(t.x, v.y, s.x * v.x)),
               fmaf(n.y, v.z, fmaf(t.y, v.y, s.y * v.x)),
               fmaf(n.z, v.z, fmaf(t.z, v.y, s.z * v.x)));
}

// render_sky, sunsky.cpp:538-555 (one channel, reference operation order)
SS_HD inline float render_sky(const SkyChannel& k, float cos_theta, float gamma) {
    float cg = cosf(gamma), cg2 = cg * cg;
    float c1 = 1.f + k.A * expf(k.B / (cos_theta + 0.01f));
    float chi = (1.f + cg2) / powf(1.f + k.I * k.I - 2.f * k.I * cg, 1.5f);
    float c2 = k.C + k.D * expf(k.E * gamma) + k.F * cg2 + k.G * chi + k.H * safe_sqrtf_(cos_theta);
    return c1 * c2 * k.rad;
}

// compute_cos_psi, sunsky.h:385-392
SS_HD inline float cos_psi(float gamma, float inv_sin2_half_ap) {
    float sg = sinf(gamma);
    return safe_sqrtf_(1.f - inv_sin2_half_ap * sg * sg);
}

// Segment search of render_sun, sunsky.cpp:579-587
SS_HD inline int sun_segment(float cos_theta, float* x) {
    float elevation = kHalfPi - acosf(cos_theta);
    float seg = cbrtf(2.f * elevation * kInvPi) * (float)kNbSunSegments;
    int pos = seg > 0.f ? (int)floorf(seg) : 0;
    pos = pos < kNbSunSegments - 1 ? pos : kNbSunSegments - 1;
    float frac = (float)pos / (float)kNbSunSegments;
    *x = elevation - kHalfPi * (frac * frac * frac);
    return pos;
}

// render_sun, RGB branch (limb darkening baked in), sunsky.cpp:597-611
SS_HD inline float render_sun_rgb(const float* table, int pos, int c, float x, float cpsi) {
    const float* s = table + pos * (3 * kNbSunCtrlPts * kNbSunLdParams) + c * (kNbSunCtrlPts * kNbSunLdParams);
    float res = 0.f;
    for (int k = 0; k < kNbSunCtrlPts; ++k)
        for (int j = 0; j < kNbSunLdParams; ++j)
            res += powif_(x, k) * powif_(cpsi, j) * s[k * kNbSunLdParams + j];
    return res;
}

// render_sun, spectral branch, sunsky.cpp:590-596
SS_HD inline float render_sun_spec(const float* table, int pos, int c, float x) {
    const float* s = table + pos * (kNbWavelengths * kNbSunCtrlPts) + c * kNbSunCtrlPts;
    float res = 0.f;
SS_NO_UNROLL
    for (int k = 0; k < kNbSunCtrlPts; ++k) res += powif_(x, k) * s[k];
    return res;
}

// compute_sun_ld, sunsky.cpp:631-650 (hi channel 11 at lambda = 720 nm carries weight 0)
SS_HD inline float sun_limb_darkening(const float* ld, int lo, int hi, float f, float cpsi) {
    float res = 0.f;
SS_NO_UNROLL
    for (int j = 0; j < kNbSunLdParams; ++j) {
        float a = ld[lo * kNbSunLdParams + j];
        float coef = a;
        if (f != 0.f) coef = lerpf_(a, hi < kNbWavelengths ? ld[hi * kNbSunLdParams + j] : 0.f, f);
        res += powif_(cpsi, j) * coef;
    }
    return res;
}

// sample_tea_32 (include/mitsuba/core/random.h:77-90), 4 rounds
SS_HD inline void sample_tea_32(uint32_t* v0, uint32_t* v1) {
    uint32_t a = *v0, b = *v1, sum = 0;
    for (int i = 0; i < 4; ++i) {
        sum += 0x9e3779b9u;
        a += ((b << 4) + 0xa341316cu) ^ (b + sum) ^ ((b >> 5) + 0xc8013ea4u);
        b += ((a << 4) + 0xad90777du) ^ (a + sum) ^ ((a >> 5) + 0x7e95761eu);
    }
    *v0 = a;
    *v1 = b;
}

// PCG32 (M. O'Neill's pcg32_srandom_r / pcg32_random_r: XSH-RR output of a 64-bit
// LCG), the generator of Dr.Jit's PCG32 used by the independent sampler
// (src/samplers/independent.cpp:88-97).  Dr.Jit is not vendored:
// this is the published algorithm, seeded as PCG32Sampler::seed does
// (src/render/sampler.cpp:125-144): (v0, v1) = sample_tea_32(seed, lane index),
// rng.seed(initstate = v0, initseq = v1).
struct Pcg32 {
    uint64_t state, inc;
    SS_HD void seed(uint64_t initstate, uint64_t initseq) {
        state = 0;
        inc = (initseq << 1) | 1u;
        next_uint32();
        state += initstate;
        next_uint32();
    }
    SS_HD uint32_t next_uint32() {
        const uint64_t old = state;
        state = old * 0x5851f42d4c957f2dull + inc;
        const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
        const uint32_t rot = (uint32_t)(old >> 59);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    // next_float32: the 23 high bits as the mantissa of [1, 2), minus 1
    SS_HD float next_float() {
        const uint32_t bits = (next_uint32() >> 9) | 0x3f800000u;
        float f;
        __builtin_memcpy(&f, &bits, sizeof f);
        return f - 1.f;
    }
};

// warp::square_to_uniform_disk_concentric, warp.h:54-90
SS_HD inline void disk_concentric(float sx, float sy, float* ox, float* oy) {
    float x = fmaf(2.f, sx, -1.f), y = fmaf(2.f, sy, -1.f);
    bool is_zero = (x == 0.f) && (y == 0.f);
    bool q13 = fabsf(x) < fabsf(y);
    float r = q13 ? y : x, rp = q13 ? x : y;
    float phi = 0.25f * kPi * rp / r;
    if (q13) phi = 0.5f * kPi - phi;
    if (is_zero) phi = 0.f;
    *ox = r * cosf(phi);
    *oy = r * sinf(phi);
}

// warp::square_to_uniform_cone (approach 2), warp.h:533-551
SS_HD inline float3_ uniform_cone(float sx, float sy, float cos_cutoff) {
    float omc = 1.f - cos_cutoff, px, py;
    disk_concentric(sx, sy, &px, &py);
    float pn = fmaf(px, px, py * py);
    float z = cos_cutoff + omc * (1.f - pn);
    float sc = safe_sqrtf_(omc * (2.f - omc * pn));
    return mk3(px * sc, py * sc, z);
}

// gaussian_cdf, sunsky.h:113-115
SS_HD inline float gaussian_cdf(float mu, float sigma, float x) {
    return 0.5f * (1.f + erff(kInvSqrtTwo * (x - mu) / sigma));
}

// erfinv: M. Giles, "Approximating the erfinv function", GPU Computing Gems
// Jade (2011), single-precision coefficients (the algorithm Dr.Jit uses).
SS_HD inline float erfinvf_(float x) {
    float w = -logf(fmaf(x, -x, 1.f)), p;
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
        w = sqrtf(w) - 3.f;
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

}  // namespace sunsky
