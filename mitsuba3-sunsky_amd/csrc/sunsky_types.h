// sunsky_types.h -- data layout shared by the host staging (C++) and the HIP
// kernels.  Everything a kernel reads besides its ray batch travels in ONE
// by-value kernel argument (SunskyKArgs) that the hardware places in the
// kernarg segment: wave-uniform, fetched with s_load into SGPRs, snapshotted
// per launch (so parameters_changed() can never race an in-flight launch).
// Only the two sun tables (<=13 KB, read by the ~1e-5 of lanes that hit the
// sun disc) live in device memory.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SS_HD __host__ __device__
#define SS_NO_UNROLL _Pragma("unroll 1")
#else
#define SS_HD
#define SS_NO_UNROLL
#endif

namespace sunsky {

// Model constants, include/mitsuba/render/sunsky/sunsky.h:19-62
constexpr int kNbWavelengths = 11;    // NB_WAVELENGTHS
constexpr int kNbTurbidity = 10;      // NB_TURBIDITY
constexpr int kNbAlbedo = 2;          // NB_ALBEDO
constexpr int kNbSkyCtrlPts = 6;      // NB_SKY_CTRL_PTS
constexpr int kNbSkyParams = 9;       // NB_SKY_PARAMS
constexpr int kNbSunCtrlPts = 4;      // NB_SUN_CTRL_PTS
constexpr int kNbSunSegments = 45;    // NB_SUN_SEGMENTS
constexpr int kNbSunLdParams = 6;     // NB_SUN_LD_PARAMS
constexpr int kNbEtas = 30;           // NB_ETAS
constexpr int kNbGaussian = 5;        // NB_GAUSSIAN
constexpr int kNbGaussianParams = 5;  // NB_GAUSSIAN_PARAMS
constexpr int kNbMixture = 4 * kNbGaussian;  // 4 corner mixtures (sunsky.h:462-474)
constexpr float kWavelength0 = 320.f, kWavelengthStep = 40.f;  // sunsky.h:27-32
constexpr double kSunHalfApertureDeg = 0.5358 / 2.0;           // SUN_HALF_APERTURE, sunsky.h:54
constexpr double kSpecToRgbSunConv = 467.069280386;            // SPEC_TO_RGB_SUN_CONV, sunsky.h:62
constexpr double kCieYNormalization = 1.0 / 106.7502593994140625;  // MI_CIE_Y_NORMALIZATION
constexpr int kSunRgbTableSize = kNbSunSegments * 3 * kNbSunCtrlPts * kNbSunLdParams;    // 3240
constexpr int kSunSpecTableSize = kNbSunSegments * kNbWavelengths * kNbSunCtrlPts;       // 1980
constexpr int kMaxLambdaPerRay = 16;   // Mitsuba uses 4 (Spectrum<Float, 4>)
constexpr int kMaxBroadcastLambda = 32;
constexpr int kGaussGuideSize = 256;   // CDF-inversion guide buckets (power of two)
constexpr int kSunRowsStaged = 8;      // RGB sun-table segments staged for the disc (sampling kernels)

enum Variant : int { kRGB = 0, kSpectral = 1 };
enum Semantics : int { kJit = 0, kScalar = 1 };

// One sky channel (render_sky, sunsky.cpp:538-555) with the per-channel
// constants of the formula folded on the host:
//   c1  = 1 + A exp(B / (cos_theta + 0.01))
//   chi = (1 + cos^2 g) / (1 + I^2 - 2 I cos g)^1.5
//   c2  = C + D exp(E g) + F cos^2 g + G chi + H sqrt(cos_theta)
//   L   = c1 c2 rad
struct SkyChannel {
    float A, B, C, D, E, F, G, H, I;
    float P;     // 1 + I*I   (host fp32, same rounding as the per-lane reference op)
    float rad;   // sky radiance of the channel
    float Bl2;   // B * log2(e)   -- exp(B r) = exp2(Bl2 r)
    float El2;   // E * log2(e)   -- exp(E g) = exp2(El2 g)
    float Q;     // -2 I          -- 1 + I^2 - 2 I cos g = fma(Q, cos g, P)
    float pad[2];
};

// The same channel with the output scale folded in for the FAST kernels:
// Rs = rad * sky_scale (* MI_CIE_Y_NORMALIZATION for RGB) multiplies C..H, so
// L = (1 + A exp2(Bl2 r)) (Cs + Ds exp2(El2 g) + Fs cos^2 g + Gs chi + Hs sqrt(cos_theta)).
// 48 bytes, 16-byte aligned: a per-lane channel gather from LDS is three
// ds_read_b128 (full LDS read rate) instead of five ds_read2_b32 (half rate).
struct alignas(16) FastChannel {
    float A, Bl2, El2, P, Q;
    float Cs, Ds, Fs, Gs, Hs;
    float pad[2];
};
static_assert(sizeof(FastChannel) == 48, "FastChannel LDS stride");

// One truncated Gaussian of the TGMM (sunsky.cpp:661-689, :732-763) with
// its per-gaussian truncation constants hoisted out of the per-lane loop.
struct alignas(16) Gaussian {
    float mu_phi, mu_theta, sigma_phi, sigma_theta;
    float weight;                          // mixture weight x corner lerp factor
    float inv_sigma_phi, inv_sigma_theta;
    float coef;                            // weight / volume, volume = (cdf_b-cdf_a).x (cdf_b-cdf_a).y sigma.x sigma.y
    float cdf_a_phi, cdf_b_phi, cdf_a_theta, cdf_b_theta;  // gaussian_cdf at a=(0,0), b=(2pi, pi/2)
};

struct SunskyKArgs {
    // -------- geometry
    float to_world[9];       // 3x3 linear part of to_world (row-major)
    float to_local[9];       // its inverse (transform_affine on vectors, transform.h:149-158)
    float sun_n[3], sun_s[3], sun_t[3];   // local sun frame (Frame3f(local_sun_dir))
    float sun_phi, sun_theta;             // m_sun_angles (from_spherical)
    float cos_cutoff;        // cos(sun_half_aperture)
    float half_aperture;     // m_sun_half_aperture
    float inv_sin2_half_ap;  // 1 / sin^2(half_aperture)  (compute_cos_psi, sunsky.h:385-392)
    // FAST cos psi: 1 / sin^2 of the half aperture in fp64 (0.5 x the fp32 aperture in
    // degrees, converted in fp64), as an unevaluated float pair hi + lo
    float cpsi_inv_hi, cpsi_inv_lo;
    float area_ratio;        // get_area_ratio(half_aperture)
    float sky_scale, sun_scale;
    float sun_pdf;           // InvTwoPi / (1 - cos_cutoff) (warp.h:568-577)
    float w_sky;             // m_sky_sampling_w
    float bs_center[3], bs_radius;        // bounding sphere (set_scene)
    int   variant, semantics, nch;
    int   identity_xform;      // to_world linear part == I: skip the 3x3 products
    // -------- radiance
    SkyChannel sky[kNbWavelengths];
    FastChannel fsky[kNbWavelengths];
    float sun_mul;           // sun_scale * area_ratio (* SPEC_TO_RGB_SUN_CONV * CIE_Y_NORMALIZATION for RGB)
    const float* sun_table;  // device: 45x3x4x6 (RGB) or 45x11x4 (spectral), turbidity-lerped
    const float* sun_ld;     // device: 11x6 limb darkening (spectral only)
    int   sun_row_lo;        // first elevation segment a direction inside the sun disc can reach
    int   sun_row_hi;        // last one (both with a margin far above fp32 rounding)
    // render_sun's segment decision (sunsky.cpp:579-584, pos = floor(cbrt(2 elevation / pi) 45)
    // with elevation = pi/2 - acos(cos theta), all fp32) as cos theta thresholds: sun_seg_z[j]
    // is the smallest fp32 cos theta whose decision is >= j (the decision is monotone in
    // cos theta; checked for every fp32 in [0, 1] by tests/test_capi_cpu.py).  A disc
    // direction's segment is sun_row_lo + #{sun_row_lo < j <= sun_row_hi : cos theta >=
    // sun_seg_z[j]}: the reference's index bit for bit, without acos / cbrt.  [0] = 0.
    float sun_seg_z[kNbSunSegments];
    // -------- sky sampling (TGMM + DiscreteDistribution)
    Gaussian gauss[kNbMixture];
    float gauss_cdf[kNbMixture];   // unnormalised inclusive prefix sum
    float gauss_pmf[kNbMixture];
    float gauss_sum, gauss_norm;
    int   gauss_first, gauss_last; // scalar-variant search bounds (distr_1d.h:233-265)
    // Guide table of the CDF inversion: for value in [b/256, (b+1)/256) the sampled
    // index lies in [gauss_guide[b], gauss_guide[b] + gauss_guide_span] (the search
    // predicate is monotone in value), so a lane tests at most gauss_guide_span
    // entries instead of all 20.  Same predicate, same result.
    int   gauss_guide_span;
    uint8_t gauss_guide[kGaussGuideSize];
    // tgmm_pdf terms with a non-zero coefficient, in mixture order: a gaussian whose
    // corner weight is 0 (integer turbidity / table-node elevation) adds exactly +0
    int   tgmm_count;
    uint8_t tgmm_idx[kNbMixture];
    // The sky pdf at a SUN pick (the FAST sampling kernels).  A sun pick's pdf is
    // (1 - w) sun_pdf + w sky_pdf(d) (sunsky.cpp:711-723 with check_sun = false), d inside the
    // disc, and sky_pdf = tgmm_pdf / sin(theta) is smooth over the 0.27-degree disc.  The host
    // fits it with a quadratic in the disc coordinates (a, b) of the sun frame
    // (square_to_uniform_cone's x, y; sun_sky_fit[6]: c0 + a (c1 + c3 a + c4 b) + b (c2 + c5 b)),
    // bounds the fit's deviation over the disc (sun_sky_fit_dev, with the smallest value
    // sun_sky_fit_fmin), and the staging turns it on only where w dev stays below
    // kSunSkyFitTol of the smallest total pdf (decide_sun_sky_fit, once w_sky is known).
    float sun_sky_fit[6];
    float sun_sky_fit_dev, sun_sky_fit_fmin;
    int   sun_sky_fit_ok;          // host: the disc lies away from the zenith, the horizon and the phi wrap
    int   sun_sky_fit_on;          // staging: sun_sky_fit_ok and the bound holds for this w_sky
    // -------- wavelength sampling (ContinuousDistribution over [360, 720])
    int   spec_size;               // 10 (JIT) / 2 (scalar) / 0 (RGB)
    float spec_pdf[10], spec_cdf[9];
    float spec_integral, spec_norm, spec_interval, spec_inv_interval;
};

static_assert(sizeof(SunskyKArgs) < 3584, "kernarg segment budget");

}  // namespace sunsky
