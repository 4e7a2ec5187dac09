// sunsky_kernels.hip -- CDNA4 (gfx950) kernels of the sun/sky emitter.
//
// Compiled to a standalone code object (hipcc --genco --offload-arch=gfx950)
// and loaded by the C-ABI layer with hipModuleLoad / hipModuleGetFunction.
//
// Design (DESIGN.md "Kernels"):
//  * one direction per lane, VEC = 4 consecutive directions per lane so every
//    global access is a 16-byte-per-lane dwordx4 (1 KiB per wave instruction);
//  * SoA fp32 rays in HBM (x[], y[], z[] planes), SoA outputs (one plane per
//    channel / wavelength);
//  * every per-emitter constant arrives in the by-value SunskyKArgs kernarg
//    block -> s_load -> SGPRs; tables that lanes index with DIFFERENT
//    indices (TGMM components, per-ray spectral channels) are staged in LDS;
//  * the sun disc (~1e-5 of random directions) runs behind an exec-masked
//    branch that waves skip when no lane hits it; its 13 KB table is read
//    from L2.
//  * FAST = 1 folds the transcendental constants on the host (exp -> exp2
//    with log2(e)-prescaled coefficients, pow(x,1.5) -> x * rsqrt(x) chains,
//    cos(unit_angle) -> 1 - 2 h^2 identity); FAST = 0 follows the reference
//    operation order with full-precision libm calls.  Both are parity-tested.
#include <hip/hip_runtime.h>

#include "sunsky_math.h"
#include "sunsky_types.h"

using namespace sunsky;

#define SS_BLOCK 256
constexpr float kLog2e = 1.44269504088896340736f;

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

struct DirTerms {
    float cos_theta, gamma, cg, cg2;
    float r;        // 1 / (cos_theta + 0.01)
    float sq;       // safe_sqrt(cos_theta)
    bool active, hit_sun;
};

// Shared per-direction terms of eval(), sunsky.cpp:309-314.
template <bool FAST>
__device__ __forceinline__ DirTerms dir_terms(const SunskyKArgs& K, float3_ wo, bool mask) {
    DirTerms t;
    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    t.cos_theta = wo.z;
    float d = dot3(sn, wo);
    // unit_angle(n, wo): 2 asin(|wo -/+ n| / 2)
    float3_ v = mk3(wo.x - mulsignf_(sn.x, d), wo.y - mulsignf_(sn.y, d), wo.z - mulsignf_(sn.z, d));
    float h = 0.5f * sqrtf(dot3(v, v));
    float temp = 2.f * asinf(h);
    t.gamma = d >= 0.f ? temp : kPi - temp;
    if (FAST) {
        // cos(2 asin h) = 1 - 2 h^2 ; cos(pi - 2 asin h) = -(1 - 2 h^2)
        float c = fmaf(-2.f * h, h, 1.f);
        t.cg = d >= 0.f ? c : -c;
        t.r = fast_rcp(t.cos_theta + 0.01f);
    } else {
        t.cg = cosf(t.gamma);
        t.r = 1.f / (t.cos_theta + 0.01f);
    }
    t.cg2 = t.cg * t.cg;
    t.sq = safe_sqrtf_(t.cos_theta);
    t.active = mask && (t.cos_theta >= 0.f);
    t.hit_sun = t.active && (d >= K.cos_cutoff);
    return t;
}

// render_sky for one channel, sunsky.cpp:538-555
template <bool FAST>
__device__ __forceinline__ float sky_channel(const SkyChannel& k, const DirTerms& t) {
    if (FAST) {
        float c1 = fmaf(k.A, fast_exp2(k.Bl2 * t.r), 1.f);
        float b = fmaf(k.Q, t.cg, k.P);                 // 1 + I^2 - 2 I cos g
        float rs = fast_rsq(b);
        float chi = (1.f + t.cg2) * (rs * rs * rs);      // / b^1.5
        float c2 = fmaf(k.D, fast_exp2(k.El2 * t.gamma), k.C);
        c2 = fmaf(k.F, t.cg2, c2);
        c2 = fmaf(k.G, chi, c2);
        c2 = fmaf(k.H, t.sq, c2);
        return c1 * c2 * k.rad;
    } else {
        float c1 = 1.f + k.A * expf(k.B * t.r);
        float chi = (1.f + t.cg2) / powf(1.f + k.I * k.I - 2.f * k.I * t.cg, 1.5f);
        float c2 = k.C + k.D * expf(k.E * t.gamma) + k.F * t.cg2 + k.G * chi + k.H * t.sq;
        return c1 * c2 * k.rad;
    }
}

__device__ __forceinline__ float3_ to_local(const SunskyKArgs& K, float3_ v) {
    return K.identity_xform ? v : xform_vec(K.to_local, v);
}
__device__ __forceinline__ float3_ to_world(const SunskyKArgs& K, float3_ v) {
    return K.identity_xform ? v : xform_vec(K.to_world, v);
}

// Full RGB eval for one local direction (sunsky.cpp:317-323): out[3]
template <bool FAST>
__device__ __forceinline__ void eval_rgb_local(const SunskyKArgs& K, float3_ wo, bool mask, float out[3]) {
    DirTerms t = dir_terms<FAST>(K, wo, mask);
    const float cie = (float)kCieYNormalization;
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c] = K.sky_scale * sky_channel<FAST>(K.sky[c], t);
    if (t.hit_sun) {
        float xs;
        int pos = sun_segment(t.cos_theta, &xs);
        float cpsi = cos_psi(t.gamma, K.inv_sin2_half_ap);
        const float conv = (float)kSpecToRgbSunConv;
#pragma unroll
        for (int c = 0; c < 3; ++c)
            out[c] += K.sun_scale * render_sun_rgb(K.sun_table, pos, c, xs, cpsi) * K.area_ratio * conv;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c] = t.active ? out[c] * cie : 0.f;
}

// Spectral eval of one wavelength for one direction (sunsky.cpp:325-348) with the
// channel table in LDS (lanes index different channels).
template <bool FAST>
__device__ __forceinline__ float eval_spec_one(const SunskyKArgs& K, const SkyChannel* sky, const DirTerms& t,
                                               float lambda) {
    float nw = (lambda - kWavelength0) / kWavelengthStep;
    bool valid = (0.f <= nw) && (nw <= (float)(kNbWavelengths - 1));
    if (!(t.active && valid)) return 0.f;
    int lo = (int)floorf(nw), hi = lo + 1;
    float f = nw - (float)lo;
    float a = sky_channel<FAST>(sky[lo], t);
    float res = a;
    if (f != 0.f) res = lerpf_(a, hi < kNbWavelengths ? sky_channel<FAST>(sky[hi], t) : 0.f, f);
    res = K.sky_scale * res;
    if (t.hit_sun) {
        float xs;
        int pos = sun_segment(t.cos_theta, &xs);
        float sa = render_sun_spec(K.sun_table, pos, lo, xs);
        float sun = sa;
        if (f != 0.f) sun = lerpf_(sa, hi < kNbWavelengths ? render_sun_spec(K.sun_table, pos, hi, xs) : 0.f, f);
        float cpsi = cos_psi(t.gamma, K.inv_sin2_half_ap);
        float ld = sun_limb_darkening(K.sun_ld, lo, hi, f, cpsi);
        res += K.sun_scale * sun * ld * K.area_ratio;
    }
    return res;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, size_t i, float v[VEC]) {
    if constexpr (VEC == 4) {
        f32x4 q = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + i));
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
        v[0] = __builtin_nontemporal_load(p + i);
    }
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* p, size_t i, const float v[VEC]) {
    if constexpr (VEC == 4) {
        f32x4 q = {v[0], v[1], v[2], v[3]};
        __builtin_nontemporal_store(q, reinterpret_cast<f32x4*>(p + i));
    } else {
        __builtin_nontemporal_store(v[0], p + i);
    }
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
    } else {
        v[0] = m[i] != 0;
    }
}

// ======================================================================
// eval(): RGB.  out plane c at out + c * ostride.  sign = -1 for eval(si)
// (local_wo = M^-1 (-si.wi)), +1 for eval_direction (wi = -ds.d).
// ======================================================================
template <int VEC, bool FAST>
__device__ __forceinline__ void eval_rgb_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                              const float* __restrict__ wy, const float* __restrict__ wz,
                                              const uint8_t* __restrict__ active, size_t n,
                                              float* __restrict__ out, size_t ostride, float sign) {
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC], r[VEC], g[VEC], b[VEC];
        bool m[VEC];
        load_vec<VEC>(wx, i, x);
        load_vec<VEC>(wy, i, y);
        load_vec<VEC>(wz, i, z);
        load_mask<VEC>(active, i, m);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            float o[3];
            eval_rgb_local<FAST>(K, to_local(K, mk3(sign * x[j], sign * y[j], sign * z[j])), m[j], o);
            r[j] = o[0]; g[j] = o[1]; b[j] = o[2];
        }
        store_vec<VEC>(out, i, r);
        store_vec<VEC>(out + ostride, i, g);
        store_vec<VEC>(out + 2 * ostride, i, b);
    }
}

// ======================================================================
// eval(): spectral, one wavelength set broadcast to every direction (the
// test02/03 eval_full_spec layout and the C3 bench workload).  Wavelength k
// maps to channels (lo[k], hi[k], f[k]) computed on the host: wave-uniform,
// so the channel constants come from SGPRs.  out plane k at out + k*ostride.
// ======================================================================
struct LambdaSet {
    int m;
    int lo[kMaxBroadcastLambda];
    float f[kMaxBroadcastLambda];   // < 0: invalid wavelength (output 0)
};

template <int VEC, bool FAST>
__device__ __forceinline__ void eval_spec_bcast_body(const SunskyKArgs& K, const LambdaSet& L,
                                                     const float* __restrict__ wx, const float* __restrict__ wy,
                                                     const float* __restrict__ wz, const uint8_t* __restrict__ active,
                                                     size_t n, float* __restrict__ out, size_t ostride, float sign) {
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
        load_vec<VEC>(wx, i, x);
        load_vec<VEC>(wy, i, y);
        load_vec<VEC>(wz, i, z);
        load_mask<VEC>(active, i, m);
        DirTerms t[VEC];
        bool any_sun = false;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            t[j] = dir_terms<FAST>(K, to_local(K, mk3(sign * x[j], sign * y[j], sign * z[j])), m[j]);
            any_sun |= t[j].hit_sun;
        }
        for (int k = 0; k < L.m; ++k) {
            const int lo = L.lo[k];
            const float f = L.f[k];
            float o[VEC];
            if (f < 0.f) {
#pragma unroll
                for (int j = 0; j < VEC; ++j) o[j] = 0.f;
            } else {
                const SkyChannel& cl = K.sky[lo];
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    float a = sky_channel<FAST>(cl, t[j]);
                    o[j] = a;
                }
                if (f != 0.f) {
                    const int hi = lo + 1;
                    if (hi < kNbWavelengths) {
                        const SkyChannel& ch = K.sky[hi];
#pragma unroll
                        for (int j = 0; j < VEC; ++j) o[j] = lerpf_(o[j], sky_channel<FAST>(ch, t[j]), f);
                    } else {
#pragma unroll
                        for (int j = 0; j < VEC; ++j) o[j] = lerpf_(o[j], 0.f, f);
                    }
                }
#pragma unroll
                for (int j = 0; j < VEC; ++j) o[j] = K.sky_scale * o[j];
                if (any_sun) {
#pragma unroll
                    for (int j = 0; j < VEC; ++j) {
                        if (t[j].hit_sun) {
                            const int hi = lo + 1;
                            float xs;
                            int pos = sun_segment(t[j].cos_theta, &xs);
                            float sa = render_sun_spec(K.sun_table, pos, lo, xs), sun = sa;
                            if (f != 0.f)
                                sun = lerpf_(sa, hi < kNbWavelengths ? render_sun_spec(K.sun_table, pos, hi, xs) : 0.f, f);
                            float cpsi = cos_psi(t[j].gamma, K.inv_sin2_half_ap);
                            float ld = sun_limb_darkening(K.sun_ld, lo, hi, f, cpsi);
                            o[j] += K.sun_scale * sun * ld * K.area_ratio;
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < VEC; ++j) o[j] = t[j].active ? o[j] : 0.f;
            }
            store_vec<VEC>(out + (size_t)k * ostride, i, o);
        }
    }
}

// ======================================================================
// eval(): spectral with per-ray wavelengths (Mitsuba Spectrum<Float, k>):
// lambda plane k at lam + k*lstride, out plane k at out + k*ostride.
// ======================================================================
__device__ __forceinline__ void stage_sky_lds(const SunskyKArgs& K, SkyChannel* sky) {
    const int nwords = (int)(kNbWavelengths * sizeof(SkyChannel) / 4);
    const float* src = reinterpret_cast<const float*>(K.sky);
    float* dst = reinterpret_cast<float*>(sky);
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) dst[w] = src[w];
    __syncthreads();
}

template <bool FAST>
__device__ __forceinline__ void eval_spec_rays_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                                    const float* __restrict__ wy, const float* __restrict__ wz,
                                                    const float* __restrict__ lam, size_t lstride, int nlam,
                                                    const uint8_t* __restrict__ active, size_t n,
                                                    float* __restrict__ out, size_t ostride, float sign) {
    __shared__ SkyChannel sky[kNbWavelengths];
    stage_sky_lds(K, sky);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool m = active ? active[i] != 0 : true;
        DirTerms t = dir_terms<FAST>(K, to_local(K, mk3(sign * wx[i], sign * wy[i], sign * wz[i])), m);
        for (int k = 0; k < nlam; ++k) out[(size_t)k * ostride + i] = eval_spec_one<FAST>(K, sky, t, lam[(size_t)k * lstride + i]);
    }
}

// ======================================================================
// Sampling: TGMM sky + uniform-cone sun (sunsky.cpp:399-451, 661-763)
// ======================================================================
struct SamplerLds {
    Gaussian gauss[kNbMixture];
    SkyChannel sky[kNbWavelengths];
};

__device__ __forceinline__ void stage_sampler_lds(const SunskyKArgs& K, SamplerLds* s) {
    const int ng = (int)(sizeof(K.gauss) / 4), ns = (int)(sizeof(K.sky) / 4);
    const float* gsrc = reinterpret_cast<const float*>(K.gauss);
    const float* ssrc = reinterpret_cast<const float*>(K.sky);
    float* gdst = reinterpret_cast<float*>(s->gauss);
    float* sdst = reinterpret_cast<float*>(s->sky);
    for (int w = threadIdx.x; w < ng; w += blockDim.x) gdst[w] = gsrc[w];
    for (int w = threadIdx.x; w < ns; w += blockDim.x) sdst[w] = ssrc[w];
    __syncthreads();
}

// DiscreteDistribution::sample_reuse (distr_1d.h:173-183): JIT predicate
// ((cdf < s) || cdf == 0) && cdf != sum over [0, n-1] (:116-136) -- a prefix
// count against the SGPR-resident CDF; scalar variants search [first, last].
__device__ __forceinline__ int discrete_sample_reuse(const SunskyKArgs& K, float value, float* reused) {
    const float s = value * K.gauss_sum;
    int idx;
    if (K.semantics == kJit) {
        idx = 0;
        bool run = true;
#pragma unroll
        for (int i = 0; i < kNbMixture - 1; ++i) {
            const float c = K.gauss_cdf[i];
            run = run && ((c < s) || c == 0.f) && (c != K.gauss_sum);
            idx += run ? 1 : 0;
        }
    } else {
        idx = K.gauss_first;
#pragma unroll
        for (int i = 0; i < kNbMixture; ++i)
            if (i >= K.gauss_first && i < K.gauss_last && K.gauss_cdf[i] < s) idx = i + 1;
    }
    // pmf / cdf gathers by a per-lane index: select chain over the SGPR table
    float pmf = 0.f, cdf_prev = 0.f;
#pragma unroll
    for (int i = 0; i < kNbMixture; ++i) {
        pmf = (idx == i) ? K.gauss_pmf[i] : pmf;
        cdf_prev = (idx == i + 1) ? K.gauss_cdf[i] : cdf_prev;
    }
    *reused = (value - cdf_prev * K.gauss_norm) / (pmf * K.gauss_norm);
    return idx;
}

// sample_sky, sunsky.cpp:661-689
__device__ __forceinline__ float3_ sample_sky(const SunskyKArgs& K, const Gaussian* G, float ux, float uy) {
    float temp;
    int idx = discrete_sample_reuse(K, ux, &temp);
    const Gaussian& g = G[idx];
    float sx = lerpf_(g.cdf_a_phi, g.cdf_b_phi, temp);
    float sy = lerpf_(g.cdf_a_theta, g.cdf_b_theta, uy);
    sx = fminf(fmaxf(sx, kEpsilon), kOneMinusEpsilon);
    sy = fminf(fmaxf(sy, kEpsilon), kOneMinusEpsilon);
    float phi = kSqrtTwo * erfinvf_(2.f * sx - 1.f) * g.sigma_phi + g.mu_phi;
    float theta = kSqrtTwo * erfinvf_(2.f * sy - 1.f) * g.sigma_theta + g.mu_theta;
    phi += K.sun_phi - 0.5f * kPi;
    theta = fminf(theta, 0.5f * kPi - kEpsilon);
    return sphdir(theta, phi);
}

// sample_sun, sunsky.cpp:697-701
__device__ __forceinline__ float3_ sample_sun(const SunskyKArgs& K, float ux, float uy) {
    return frame_to_world(mk3(K.sun_s[0], K.sun_s[1], K.sun_s[2]), mk3(K.sun_t[0], K.sun_t[1], K.sun_t[2]),
                          mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]), uniform_cone(ux, uy, K.cos_cutoff));
}

// tgmm_pdf, sunsky.cpp:732-763, with the truncation volume hoisted to the host.
template <bool FAST>
__device__ __forceinline__ float tgmm_pdf(const SunskyKArgs& K, float phi, float theta, bool active) {
    phi -= K.sun_phi - 0.5f * kPi;
    phi = phi < 0.f ? phi + kTwoPi : phi;
    phi = phi > kTwoPi ? phi - kTwoPi : phi;
    active = active && (theta >= 0.f) && (theta <= 0.5f * kPi);
    float pdf = 0.f;
#pragma unroll
    for (int i = 0; i < kNbMixture; ++i) {
        const Gaussian& g = K.gauss[i];
        float sx = (phi - g.mu_phi) * g.inv_sigma_phi, sy = (theta - g.mu_theta) * g.inv_sigma_theta;
        float q = fmaf(sy, sy, sx * sx);
        float e = FAST ? fast_exp2((-0.5f * kLog2e) * q) : expf(-0.5f * q);
        pdf = fmaf(g.coef, kInvTwoPi * e, pdf);
    }
    return active ? pdf : 0.f;
}

// compute_pdfs, sunsky.cpp:711-723
template <bool FAST>
__device__ __forceinline__ void compute_pdfs(const SunskyKArgs& K, float3_ d, bool check_sun, bool active,
                                             float* sky_pdf, float* sun_pdf) {
    float sin_theta = safe_sqrtf_(fmaf(d.x, d.x, d.y * d.y));
    active = active && (d.z >= 0.f) && (sin_theta != 0.f);
    sin_theta = fmaxf(sin_theta, kEpsilon);
    float phi = atan2f(d.y, d.x), theta = unit_angle_z(d);
    *sky_pdf = tgmm_pdf<FAST>(K, phi, theta, active) / sin_theta;
    float cosg = dot3(mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]), d);
    *sun_pdf = (!check_sun || cosg >= K.cos_cutoff) ? K.sun_pdf : 0.f;
}

// sample_direction, sunsky.cpp:399-441.  nw = 3 (RGB) or the number of
// per-ray wavelengths (spectral).
template <bool FAST>
__device__ __forceinline__ void sample_direction_body(
    const SunskyKArgs& K, const float* __restrict__ ux, const float* __restrict__ uy,
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ pz,
    const float* __restrict__ lam, size_t lstride, int nlam, const uint8_t* __restrict__ active, size_t n,
    float* __restrict__ dx, float* __restrict__ dy, float* __restrict__ dz, float* __restrict__ pdf,
    float* __restrict__ dist, float* __restrict__ opx, float* __restrict__ opy, float* __restrict__ opz,
    float* __restrict__ weight, size_t wstride) {
    __shared__ SamplerLds S;
    stage_sampler_lds(K, &S);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool act = active ? active[i] != 0 : true;
        const float sx = ux[i], sy = uy[i];
        const bool pick_sky = sx < K.w_sky;
        float3_ sd;
        if (pick_sky) sd = sample_sky(K, S.gauss, sx / K.w_sky, sy);
        else sd = sample_sun(K, (sx - K.w_sky) / (1.f - K.w_sky), sy);
        act = act && (sd.z >= 0.f);
        float3_ itp = mk3(px ? px[i] : 0.f, py ? py[i] : 0.f, pz ? pz[i] : 0.f);
        float3_ rel = mk3(itp.x - K.bs_center[0], itp.y - K.bs_center[1], itp.z - K.bs_center[2]);
        float radius = fmaxf(K.bs_radius, sqrtf(dot3(rel, rel)));
        float dd = 2.f * radius;
        float3_ d = to_world(K, sd);
        float skyp, sunp;
        compute_pdfs<FAST>(K, sd, pick_sky, act, &skyp, &sunp);
        float pd = lerpf_(sunp, skyp, K.w_sky);
        dx[i] = d.x; dy[i] = d.y; dz[i] = d.z;
        pdf[i] = pd;
        if (dist) dist[i] = dd;
        if (opx) { opx[i] = fmaf(d.x, dd, itp.x); opy[i] = fmaf(d.y, dd, itp.y); opz[i] = fmaf(d.z, dd, itp.z); }
        // weight = eval(si{wi = -d}) / pdf, zeroed when not finite
        float3_ wo = to_local(K, d);
        if (K.variant == kRGB) {
            float e[3];
            eval_rgb_local<FAST>(K, wo, act, e);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float w = e[c] / pd;
                weight[(size_t)c * wstride + i] = isfinite(w) ? w : 0.f;
            }
        } else {
            DirTerms t = dir_terms<FAST>(K, wo, act);
            for (int k = 0; k < nlam; ++k) {
                float e = t.active ? eval_spec_one<FAST>(K, S.sky, t, lam[(size_t)k * lstride + i]) : 0.f;
                float w = e / pd;
                weight[(size_t)k * wstride + i] = isfinite(w) ? w : 0.f;
            }
        }
    }
}

// pdf_direction, sunsky.cpp:443-451
template <bool FAST>
__device__ __forceinline__ void pdf_direction_body(const SunskyKArgs& K, const float* __restrict__ dx,
                                                   const float* __restrict__ dy, const float* __restrict__ dz,
                                                   const uint8_t* __restrict__ active, size_t n,
                                                   float* __restrict__ pdf) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool act = active ? active[i] != 0 : true;
        float3_ l = to_local(K, mk3(dx[i], dy[i], dz[i]));
        float skyp, sunp;
        compute_pdfs<FAST>(K, l, true, true, &skyp, &sunp);
        float pd = lerpf_(sunp, skyp, K.w_sky);
        __builtin_nontemporal_store(act ? pd : 0.f, pdf + i);
    }
}

// ContinuousDistribution::sample_pdf (distr_1d.h:468-499) over [360, 720]
__device__ __forceinline__ float spectral_sample_pdf(const SunskyKArgs& K, float sample, float* pdf_out) {
    sample *= K.spec_integral;
    const int nint = K.spec_size - 1;
    int idx = 0;
    if (K.semantics == kJit) {
        bool run = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < nint - 1) {
                const float c = K.spec_cdf[i];
                run = run && ((c < sample) || c == 0.f) && (c != K.spec_integral);
                idx += run ? 1 : 0;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i < nint - 1 && K.spec_cdf[i] < sample) idx = i + 1;
    }
    float y0 = 0.f, y1 = 0.f, c0 = 0.f;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        y0 = idx == i ? K.spec_pdf[i] : y0;
        y1 = idx == i ? K.spec_pdf[i + 1] : y1;
        c0 = idx == i + 1 ? K.spec_cdf[i] : c0;
    }
    sample = (sample - c0) * K.spec_inv_interval;
    float t_linear = (y0 - safe_sqrtf_(fmaf(y0, y0, 2.f * sample * (y1 - y0)))) * (1.f / (y0 - y1));
    float t_const = sample * (1.f / y0);
    float t = (y0 == y1) ? t_const : t_linear;
    *pdf_out = fmaf(t, y1 - y0, y0) * K.spec_norm;
    return fmaf((float)idx + t, K.spec_interval, 360.f);
}

// sample_wavelengths, sunsky.cpp:463-480 (spectral: 4 shifted samples, Spectrum<Float, 4>)
template <bool FAST>
__device__ __forceinline__ void sample_wavelengths_one(const SunskyKArgs& K, const SkyChannel* sky, const DirTerms& t,
                                                       float sample, float lam[4], float w[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float s = sample + (float)k / 4.f;   // math::sample_shifted, math.h:408-431
        s = s > 1.f ? s - 1.f : s;
        float lpdf;
        lam[k] = spectral_sample_pdf(K, s, &lpdf);
        w[k] = eval_spec_one<FAST>(K, sky, t, lam[k]) / lpdf;
    }
}

template <bool FAST>
__device__ __forceinline__ void sample_wavelengths_body(const SunskyKArgs& K, const float* __restrict__ wx,
                                                        const float* __restrict__ wy, const float* __restrict__ wz,
                                                        const float* __restrict__ sample, const uint8_t* __restrict__ active,
                                                        size_t n, float* __restrict__ lam_out, size_t lstride,
                                                        float* __restrict__ weight, size_t wstride) {
    __shared__ SkyChannel sky[kNbWavelengths];
    stage_sky_lds(K, sky);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool act = active ? active[i] != 0 : true;
        float3_ wo = to_local(K, mk3(-wx[i], -wy[i], -wz[i]));
        if (K.variant == kRGB) {
            float e[3];
            eval_rgb_local<FAST>(K, wo, act, e);
            for (int c = 0; c < 3; ++c) weight[(size_t)c * wstride + i] = e[c];
            for (int k = 0; k < 4; ++k) lam_out[(size_t)k * lstride + i] = 0.f;
        } else {
            DirTerms t = dir_terms<FAST>(K, wo, act);
            float lam[4], w[4];
            sample_wavelengths_one<FAST>(K, sky, t, sample[i], lam, w);
            for (int k = 0; k < 4; ++k) {
                lam_out[(size_t)k * lstride + i] = lam[k];
                weight[(size_t)k * wstride + i] = w[k];
            }
        }
    }
}

// sample_ray, sunsky.cpp:354-397
template <bool FAST>
__device__ __forceinline__ void sample_ray_body(const SunskyKArgs& K, const float* __restrict__ wls,
                                                const float* __restrict__ s2x, const float* __restrict__ s2y,
                                                const float* __restrict__ s3x, const float* __restrict__ s3y,
                                                const uint8_t* __restrict__ active, size_t n,
                                                float* __restrict__ ox, float* __restrict__ oy, float* __restrict__ oz,
                                                float* __restrict__ dxo, float* __restrict__ dyo, float* __restrict__ dzo,
                                                float* __restrict__ lam_out, size_t lstride,
                                                float* __restrict__ weight, size_t wstride) {
    __shared__ SamplerLds S;
    stage_sampler_lds(K, &S);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool act = active ? active[i] != 0 : true;
        float offx, offy;
        disk_concentric(s2x[i], s2y[i], &offx, &offy);
        const float sx = s3x[i], sy = s3y[i];
        const bool pick_sky = sx < K.w_sky;
        float3_ d;
        if (pick_sky) d = sample_sky(K, S.gauss, sx / K.w_sky, sy);
        else d = sample_sun(K, (sx - K.w_sky) / (1.f - K.w_sky), sy);
        float3_ dw = to_world(K, mk3(-d.x, -d.y, -d.z));
        act = act && (d.z >= 0.f);
        float skyp, sunp;
        compute_pdfs<FAST>(K, d, pick_sky, act, &skyp, &sunp);
        float pd = lerpf_(sunp, skyp, K.w_sky);
        pd *= kInvPi * (1.f / (K.bs_radius * K.bs_radius));
        act = act && pd > 0.f;
        float3_ wo = to_local(K, mk3(-dw.x, -dw.y, -dw.z));
        float w[4];
        int nw;
        if (K.variant == kRGB) {
            eval_rgb_local<FAST>(K, wo, act, w);
            nw = 3;
            for (int k = 0; k < 4; ++k) lam_out[(size_t)k * lstride + i] = 0.f;
        } else {
            DirTerms t = dir_terms<FAST>(K, wo, act);
            float lam[4];
            sample_wavelengths_one<FAST>(K, S.sky, t, wls[i], lam, w);
            for (int k = 0; k < 4; ++k) lam_out[(size_t)k * lstride + i] = lam[k];
            nw = 4;
        }
        float3_ fs, ft;
        coordinate_system(dw, &fs, &ft);
        float3_ po = frame_to_world(fs, ft, dw, mk3(offx, offy, 0.f));
        ox[i] = K.bs_center[0] + (po.x - dw.x) * K.bs_radius;
        oy[i] = K.bs_center[1] + (po.y - dw.y) * K.bs_radius;
        oz[i] = K.bs_center[2] + (po.z - dw.z) * K.bs_radius;
        dxo[i] = dw.x; dyo[i] = dw.y; dzo[i] = dw.z;
        for (int k = 0; k < nw; ++k) {
            float v = w[k] / pd;
            weight[(size_t)k * wstride + i] = isfinite(v) ? v : 0.f;
        }
    }
}

// ======================================================================
// extern "C" entry points (hipModuleGetFunction names)
// ======================================================================
#define SS_EVAL_RGB(NAME, VEC, FAST)                                                                          \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, const float* wx, const float* wy, const float* wz, const uint8_t* active, size_t n,     \
        float* out, size_t ostride, float sign) {                                                              \
        eval_rgb_body<VEC, FAST>(K, wx, wy, wz, active, n, out, ostride, sign);                                \
    }
SS_EVAL_RGB(sunsky_eval_rgb_v4_fast, 4, true)
SS_EVAL_RGB(sunsky_eval_rgb_v1_fast, 1, true)
SS_EVAL_RGB(sunsky_eval_rgb_v4_ref, 4, false)
SS_EVAL_RGB(sunsky_eval_rgb_v1_ref, 1, false)

#define SS_EVAL_SPEC_BCAST(NAME, VEC, FAST)                                                                   \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, LambdaSet L, const float* wx, const float* wy, const float* wz, const uint8_t* active,  \
        size_t n, float* out, size_t ostride, float sign) {                                                    \
        eval_spec_bcast_body<VEC, FAST>(K, L, wx, wy, wz, active, n, out, ostride, sign);                      \
    }
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v4_fast, 4, true)
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v1_fast, 1, true)
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v4_ref, 4, false)
SS_EVAL_SPEC_BCAST(sunsky_eval_spec_bcast_v1_ref, 1, false)

#define SS_EVAL_SPEC_RAYS(NAME, FAST)                                                                         \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, const float* wx, const float* wy, const float* wz, const float* lam, size_t lstride,    \
        int nlam, const uint8_t* active, size_t n, float* out, size_t ostride, float sign) {                   \
        eval_spec_rays_body<FAST>(K, wx, wy, wz, lam, lstride, nlam, active, n, out, ostride, sign);           \
    }
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_fast, true)
SS_EVAL_SPEC_RAYS(sunsky_eval_spec_rays_ref, false)

#define SS_SAMPLE_DIRECTION(NAME, FAST)                                                                       \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, const float* ux, const float* uy, const float* px, const float* py, const float* pz,   \
        const float* lam, size_t lstride, int nlam, const uint8_t* active, size_t n, float* dx, float* dy,     \
        float* dz, float* pdf, float* dist, float* opx, float* opy, float* opz, float* weight, size_t wstride) { \
        sample_direction_body<FAST>(K, ux, uy, px, py, pz, lam, lstride, nlam, active, n, dx, dy, dz, pdf,     \
                                    dist, opx, opy, opz, weight, wstride);                                     \
    }
SS_SAMPLE_DIRECTION(sunsky_sample_direction_fast, true)
SS_SAMPLE_DIRECTION(sunsky_sample_direction_ref, false)

#define SS_PDF_DIRECTION(NAME, FAST)                                                                          \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, const float* dx, const float* dy, const float* dz, const uint8_t* active, size_t n,     \
        float* pdf) {                                                                                          \
        pdf_direction_body<FAST>(K, dx, dy, dz, active, n, pdf);                                               \
    }
SS_PDF_DIRECTION(sunsky_pdf_direction_fast, true)
SS_PDF_DIRECTION(sunsky_pdf_direction_ref, false)

#define SS_SAMPLE_WAVELENGTHS(NAME, FAST)                                                                     \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, const float* wx, const float* wy, const float* wz, const float* sample,                 \
        const uint8_t* active, size_t n, float* lam, size_t lstride, float* weight, size_t wstride) {          \
        sample_wavelengths_body<FAST>(K, wx, wy, wz, sample, active, n, lam, lstride, weight, wstride);        \
    }
SS_SAMPLE_WAVELENGTHS(sunsky_sample_wavelengths_fast, true)
SS_SAMPLE_WAVELENGTHS(sunsky_sample_wavelengths_ref, false)

#define SS_SAMPLE_RAY(NAME, FAST)                                                                             \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                               \
        SunskyKArgs K, const float* wls, const float* s2x, const float* s2y, const float* s3x,                 \
        const float* s3y, const uint8_t* active, size_t n, float* ox, float* oy, float* oz, float* dx,         \
        float* dy, float* dz, float* lam, size_t lstride, float* weight, size_t wstride) {                     \
        sample_ray_body<FAST>(K, wls, s2x, s2y, s3x, s3y, active, n, ox, oy, oz, dx, dy, dz, lam, lstride,     \
                              weight, wstride);                                                                \
    }
SS_SAMPLE_RAY(sunsky_sample_ray_fast, true)
SS_SAMPLE_RAY(sunsky_sample_ray_ref, false)
