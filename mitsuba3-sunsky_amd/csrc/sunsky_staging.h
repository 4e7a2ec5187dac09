// sunsky_staging.h -- the per-entry arithmetic of the emitter's parameter staging,
// shared by the host model (sunsky_model.cpp: host-only emitters, the CPU tests)
// and the device staging kernels (sunsky_kernels.hip: parameters_changed of a GPU
// emitter, stream-ordered).  One definition, one operation order, contraction off:
// the polynomial staging (compute_radiance_params, compute_sun_params, the channel
// folding) is bitwise the same on both sides.  The host computes the few libm
// scalars (x = cbrt(2 eta / pi), floor(T)) once and hands them to the device.
#pragma once
#include "sunsky_math.h"

#if defined(__clang__)
#define SS_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define SS_NO_CONTRACT
#endif

namespace sunsky {

// Scalars of compute_radiance_params / compute_sun_params (sunsky.h:158-231, 404-419)
// for one (turbidity, eta): computed on the host, shared by every table entry.
struct RadianceStage {
    float x;        // cbrt(2 eta / pi)
    float t_rem;    // turbidity - floor(turbidity)
    int t_low, t_high;
    int in_range;   // 0 <= eta <= pi/2, else every sky coefficient is 0 (sunsky.h:230)
};

// bezier_interpolate + compute_radiance_params for entry e of a (nch x npar) result,
// sunsky.h:158-231.  ds: (10 T, 2 albedo, 6 ctrl, result_size) fp32.
SS_HD inline float radiance_param(const float* ds, int result_size, int e, const RadianceStage& s,
                                  float albedo) {
    SS_NO_CONTRACT
    const float coefs[kNbSkyCtrlPts] = {1, 5, 10, 10, 5, 1};
    const int a_block = kNbSkyCtrlPts * result_size, t_block = kNbAlbedo * a_block;
    float bez[2][2];
    for (int ti = 0; ti < 2; ++ti) {
        const int t = ti ? s.t_high : s.t_low;
        for (int a = 0; a < 2; ++a) {
            float res = 0.f;
            if (t >= 0 && t < kNbTurbidity)   // gather mask "t < NB_TURBIDITY"
                for (int k = 0; k < kNbSkyCtrlPts; ++k) {
                    const float data = ds[(size_t)t * t_block + a * a_block + k * result_size + e];
                    float term = coefs[k] * powif_(s.x, k);
                    term = term * powif_(1.f - s.x, kNbSkyCtrlPts - 1 - k);
                    term = term * data;
                    res = res + term;
                }
            bez[ti][a] = res;
        }
    }
    const float ra_low = lerpf_(bez[0][0], bez[1][0], s.t_rem);
    const float ra_high = lerpf_(bez[0][1], bez[1][1], s.t_rem);
    const float v = lerpf_(ra_low, ra_high, albedo);
    return s.in_range ? v : 0.f;
}

// compute_sun_params entry i (lerp over turbidity of the sun table), sunsky.h:404-419
SS_HD inline float sun_param(const float* ds, int block, int i, const RadianceStage& s) {
    const float lo = (s.t_low >= 0 && s.t_low < kNbTurbidity) ? ds[(size_t)s.t_low * block + i] : 0.f;
    const float hi = (s.t_high >= 0 && s.t_high < kNbTurbidity) ? ds[(size_t)s.t_high * block + i] : 0.f;
    return lerpf_(lo, hi, s.t_rem);
}

// ---------------------------------------------------------------- AD staging
// Tangent of the staging for one differentiable parameter (traverse(), sunsky.cpp:220-240)
// at the current (turbidity, eta, albedo): what Dr.Jit's forward mode propagates through
// compute_radiance_params / compute_sun_params (sunsky.h:158-231, 404-419) before eval.
// The host fills the few scalars (x = cbrt(2 eta / pi) and dx = dx/deta x deta, t_rem,
// the albedo tangent); every table entry is then radiance_param_tangent / sun_param_tangent,
// run by the host model (eval_tangent) and by the device kernel sunsky_stage_tangent in
// fp64 with integer powers by repeated products: the same bits on both sides.
struct TangentStage {
    double x, dx;                 // Bezier abscissa and its tangent
    double t_rem, dT;             // turbidity lerp factor (d t_rem / dT = 1, floor(T) constant)
    int t_low, t_high, in_range, nch;
    double albedo[kNbWavelengths], dalbedo[kNbWavelengths];
    float dsun_local[3];          // tangent of the local sun direction (sun_direction)
    double deta, dx_per_eta;      // the sun elevation's tangent; dx = dx_per_eta * deta
};

SS_HD inline double powid_(double x, int k) {
    double r = 1.0;
    for (int i = 0; i < k; ++i) r *= x;
    return r;
}

// d compute_radiance_params entry e of a (nch x npar) result (sunsky.h:158-231): the
// quintic Bezier and its derivative, the turbidity lerp, the albedo lerp.
SS_HD inline double radiance_param_tangent(const float* ds, int npar, int e, const TangentStage& s) {
    SS_NO_CONTRACT
    const double coefs[kNbSkyCtrlPts] = {1, 5, 10, 10, 5, 1};
    const int result_size = s.nch * npar, a_block = kNbSkyCtrlPts * result_size, t_block = kNbAlbedo * a_block;
    if (!s.in_range) return 0.0;
    double bez[2][2], dbez[2][2];
    for (int ti = 0; ti < 2; ++ti) {
        const int t = ti ? s.t_high : s.t_low;
        for (int a = 0; a < 2; ++a) {
            double v = 0.0, dv = 0.0;
            if (t >= 0 && t < kNbTurbidity)
                for (int k = 0; k < kNbSkyCtrlPts; ++k) {
                    const double data = ds[(size_t)t * t_block + a * a_block + k * result_size + e];
                    const int m = kNbSkyCtrlPts - 1 - k;
                    v += coefs[k] * powid_(s.x, k) * powid_(1.0 - s.x, m) * data;
                    double db = 0.0;
                    if (k > 0) db += k * powid_(s.x, k - 1) * powid_(1.0 - s.x, m);
                    if (m > 0) db -= m * powid_(s.x, k) * powid_(1.0 - s.x, m - 1);
                    dv += coefs[k] * db * data;
                }
            bez[ti][a] = v;
            dbez[ti][a] = dv * s.dx;
        }
    }
    const double ra_low = bez[0][0] + s.t_rem * (bez[1][0] - bez[0][0]);
    const double ra_high = bez[0][1] + s.t_rem * (bez[1][1] - bez[0][1]);
    const double dra_low = dbez[0][0] + s.t_rem * (dbez[1][0] - dbez[0][0]) + (bez[1][0] - bez[0][0]) * s.dT;
    const double dra_high = dbez[0][1] + s.t_rem * (dbez[1][1] - dbez[0][1]) + (bez[1][1] - bez[0][1]) * s.dT;
    const int c = e / npar;
    return dra_low + s.albedo[c] * (dra_high - dra_low) + (ra_high - ra_low) * s.dalbedo[c];
}

// d compute_sun_params entry i (sunsky.h:404-419): the turbidity lerp's slope times dT
SS_HD inline float sun_param_tangent(const float* ds, int block, int i, const TangentStage& s) {
    SS_NO_CONTRACT
    if (s.dT == 0.0) return 0.f;
    const double lo = (s.t_low >= 0 && s.t_low < kNbTurbidity) ? ds[(size_t)s.t_low * block + i] : 0.0;
    const double hi = (s.t_high >= 0 && s.t_high < kNbTurbidity) ? ds[(size_t)s.t_high * block + i] : 0.0;
    return (float)((hi - lo) * s.dT);
}

// Layouts of the tangent tables the AD kernels read (sunsky_kernels.hip): per basis a
// block of kTanBlock floats, d{A..I, rad} of channel c at c * 10 (+ q) -- the VJP reads
// blocks 0-2 only (turbidity, albedo, the unit-elevation tangent its sun axes share);
// blocks 3-4 stay reserved and zero -- the local sun direction's tangent at kTanSunLocal
// (JVP) or kVjpSunLocal + 3 k (VJP, sun axis k); the sun table's at kJvpSunOffset (JVP) /
// kVjpSunOffset (VJP, turbidity basis).
constexpr int kTanBlock = kNbWavelengths * 10;   // 110
constexpr int kTanSunLocal = kTanBlock;          // JVP: 110..112
constexpr int kJvpSunOffset = 128;
constexpr int kVjpBases = 5;                     // turbidity, albedo (diagonal), sun x / y / z
constexpr int kVjpSunLocal = kVjpBases * kTanBlock;   // 550..558
// VJP: d eta of the 3 sun axes (559..561).  The sky tables of a sun axis are d eta times
// those of a unit elevation tangent, which the VJP stages as its basis 2 (eval_vjp_*_body)
constexpr int kVjpSunEta = kVjpSunLocal + 9;
constexpr int kVjpSunOffset = 576;
static_assert(kVjpSunEta + 3 <= kVjpSunOffset, "VJP buffer layout");

// Sky-channel entry j = c x 10 + q (< nch x 10) of one basis' tangent block: d{A..I}
// (q < 9) from the sky parameter dataset, d rad (q = 9) from the sky radiance dataset.
SS_HD inline float tangent_value(const float* sky_params_ds, const float* sky_rad_ds, const TangentStage& s, int j) {
    const int c = j / 10, q = j % 10;
    return (float)(q < kNbSkyParams ? radiance_param_tangent(sky_params_ds, kNbSkyParams, c * kNbSkyParams + q, s)
                                    : radiance_param_tangent(sky_rad_ds, 1, c, s));
}

// Arguments of the device tangent staging (sunsky_stage_tangent): `nbasis` tangents, the
// sky blocks of the first `nsky` of them at out + b x kTanBlock (the VJP's sun axes
// share basis 2's unit-elevation block, so it stages 3 of its 5), the local sun tangents
// of bases [sun_local_first, nbasis) at out + sun_local_off (3 each), basis 0's sun-table
// tangent at out + sun_off; every other float of [0, total) is written 0.
struct TangentArgs {
    const float* sky_params_ds;
    const float* sky_rad_ds;
    const float* sun_rad_ds;
    float* out;
    int nbasis, nsky, sun_local_off, sun_local_first, sun_off, sun_block, total;
    TangentStage st[kVjpBases];
    int eta_off;   // > 0: d eta of bases [sun_local_first, nbasis) at out + eta_off (VJP)
};

// Float idx of the tangent buffer described by A (the device kernel's per-thread work).
SS_HD inline float tangent_buffer_value(const TangentArgs& A, int idx) {
    if (idx < A.nsky * kTanBlock) {
        const int b = idx / kTanBlock, j = idx % kTanBlock;
        return j < A.st[b].nch * 10 ? tangent_value(A.sky_params_ds, A.sky_rad_ds, A.st[b], j) : 0.f;
    }
    const int nloc = 3 * (A.nbasis - A.sun_local_first);
    if (A.eta_off > 0 && idx >= A.eta_off && idx < A.eta_off + nloc / 3)
        return (float)A.st[A.sun_local_first + (idx - A.eta_off)].deta;
    if (idx >= A.sun_local_off && idx < A.sun_local_off + nloc) {
        const int k = (idx - A.sun_local_off) / 3, r = (idx - A.sun_local_off) % 3;
        return A.st[A.sun_local_first + k].dsun_local[r];
    }
    if (idx >= A.sun_off && idx < A.sun_off + A.sun_block)
        return sun_param_tangent(A.sun_rad_ds, A.sun_block, idx - A.sun_off, A.st[0]);
    return 0.f;
}

// One staged sky channel from its 9 coefficients and radiance: the reference-order
// record (render_sky) and the FAST record with the output scale folded in
// (sky_scale, x MI_CIE_Y_NORMALIZATION for RGB; sunsky.cpp:303-352).
SS_HD inline void fold_channel(const float* p, float rad, int variant, float sky_scale, SkyChannel* ch,
                               FastChannel* f) {
    SS_NO_CONTRACT
    ch->A = p[0]; ch->B = p[1]; ch->C = p[2]; ch->D = p[3]; ch->E = p[4];
    ch->F = p[5]; ch->G = p[6]; ch->H = p[7]; ch->I = p[8];
    ch->P = 1.f + ch->I * ch->I;
    ch->rad = rad;
    ch->Bl2 = (float)((double)ch->B * 1.4426950408889634074);
    ch->El2 = (float)((double)ch->E * 1.4426950408889634074);
    ch->Q = -2.f * ch->I;
    ch->pad[0] = ch->pad[1] = 0.f;
    const float Rs = variant == kRGB ? ch->rad * sky_scale * (float)kCieYNormalization : ch->rad * sky_scale;
    f->A = ch->A; f->Bl2 = ch->Bl2; f->El2 = ch->El2; f->P = ch->P; f->Q = ch->Q;
    f->Cs = ch->C * Rs; f->Ds = ch->D * Rs; f->Fs = ch->F * Rs; f->Gs = ch->G * Rs; f->Hs = ch->H * Rs;
    f->pad[0] = f->pad[1] = 0.f;
}

// estimate_sky_sun_ratio (sunsky.cpp:772-886): quadrature point (i, j) of the
// 200 x 200 Gauss-Legendre grid, sky over the hemisphere and sun over its cone.  The
// direction terms are shared by every channel; row j's per-channel sums over i, in
// i order, are the unit the host and the device reduce identically.
struct QuadDir {
    float cos_theta, gamma, wij;   // sky point
    int sun_ok, pos;               // sun point above the horizon; its elevation segment
    float xs, cpsi;
};

SS_HD inline QuadDir quad_dir(const SunskyKArgs& K, const float* x, const float* w, int i, int j) {
    SS_NO_CONTRACT
    QuadDir d;
    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    d.cos_theta = 0.5f * (x[j] + 1.f);
    const float sin_theta = safe_sqrtf_(1.f - d.cos_theta * d.cos_theta);
    const float cc = K.cos_cutoff;
    const float cos_gamma = 0.5f * ((1.f - cc) * x[j] + (1.f + cc));
    const float sin_gamma = safe_sqrtf_(1.f - cos_gamma * cos_gamma);
    const float phi = kPi * (x[i] + 1.f);
    const float sp = sinf(phi), cp = cosf(phi);
    d.gamma = unit_angle(sn, mk3(sin_theta * cp, sin_theta * sp, d.cos_theta));
    d.wij = w[i];
    const float3_ sw = mk3(sin_gamma * cp, sin_gamma * sp, cos_gamma);
    const float g2 = unit_angle_z(sw);
    const float3_ wl = frame_to_world(mk3(K.sun_s[0], K.sun_s[1], K.sun_s[2]), mk3(K.sun_t[0], K.sun_t[1], K.sun_t[2]),
                                      sn, sw);
    d.sun_ok = wl.z >= 0.f;
    d.pos = 0;
    d.xs = d.cpsi = 0.f;
    if (d.sun_ok) {
        // render_sun's segment (sunsky.cpp:579-587) from the staged cos theta thresholds, as
        // every eval / sampling / AD kernel takes it (SunskyKArgs::sun_seg_z), not from this
        // build's acosf / cbrtf: host and device staging and the kernels agree at segment starts
        int pos = 0;
        for (int s = 1; s < kNbSunSegments; ++s) pos += wl.z >= K.sun_seg_z[s] ? 1 : 0;
        const float frac = (float)pos / (float)kNbSunSegments;
        d.pos = pos;
        d.xs = (kHalfPi - acosf(wl.z)) - kHalfPi * (frac * frac * frac);
        d.cpsi = cos_psi(g2, K.inv_sin2_half_ap);
    }
    return d;
}

// channel c's sky and sun terms at a quadrature point (w_j: the row's weight)
SS_HD inline void quad_channel(const SunskyKArgs& K, const float* sun_table, const float* sun_ld, const QuadDir& d,
                               float w_j, int c, float* sky_v, float* sun_v) {
    SS_NO_CONTRACT
    *sky_v = render_sky(K.sky[c], d.cos_theta, d.gamma) * d.wij * w_j;
    *sun_v = 0.f;
    if (!d.sun_ok) return;
    if (K.variant == kSpectral) {
        const float v = render_sun_spec(sun_table, d.pos, c, d.xs) * d.wij * w_j;
        *sun_v = v * sun_limb_darkening(sun_ld, c, c, 0.f, d.cpsi);
    } else {
        *sun_v = render_sun_rgb(sun_table, d.pos, c, d.xs, d.cpsi) * d.wij * w_j;
    }
}

// Relative bound on a sun pick's total pdf from the quadratic sky-pdf fit (SunskyKArgs::
// sun_sky_fit): 1e-7, a hundredth of the 1e-5 parity bar.
constexpr float kSunSkyFitTol = 1e-7f;

// Turn the fit on when w dev <= tol ((1 - w) sun_pdf + w fmin) for the staged w_sky: the
// error of the sky term, relative to the smallest pdf a sun pick can have.
SS_HD inline void decide_sun_sky_fit(SunskyKArgs* k) {
    SS_NO_CONTRACT
    const float w = k->w_sky;
    k->sun_sky_fit_on = (k->sun_sky_fit_ok &&
                         w * k->sun_sky_fit_dev <= kSunSkyFitTol * ((1.f - w) * k->sun_pdf + w * k->sun_sky_fit_fmin))
                            ? 1 : 0;
}

// The end of estimate_sky_sun_ratio: the per-channel sums of the quadrature rows (added
// in row order by the caller), luminance, the sky sampling weight and (spectral) the
// wavelength distribution (ContinuousDistribution over [360, 720] of avg_spec[1..10],
// JIT compute_cdf, distr_1d.h:513-538).  Returns false when the distribution has a
// negative entry (the reference throws).
SS_HD inline bool quad_finish(SunskyKArgs* k, const float* sky_sum, const float* sun_sum, const float* cie_y,
                              float sky_scale, float sun_scale) {
    SS_NO_CONTRACT
    const int nch = k->nch;
    const bool spec = k->variant == kSpectral;
    float sky[kNbWavelengths] = {0}, sun[kNbWavelengths] = {0};
    for (int c = 0; c < nch; ++c) { sky[c] = sky_sum[c]; sun[c] = sun_sum[c]; }
    const float J_sky = 0.5f * kPi, J_sun = 0.5f * kPi * (1.f - k->cos_cutoff);
    for (int c = 0; c < nch; ++c) { sky[c] *= J_sky; sun[c] *= J_sun; }
    float sky_lum = sky_scale, sun_lum = sun_scale;
    if (!spec) {
        sky_lum *= sky[0] * 0.212671f + sky[1] * 0.715160f + sky[2] * 0.072169f;
        sun_lum *= (sun[0] * 0.212671f + sun[1] * 0.715160f + sun[2] * 0.072169f) * k->area_ratio *
                   (float)kSpecToRgbSunConv;
    } else {
        float ls = 0.f, lu = 0.f;
        for (int c = 0; c < kNbWavelengths; ++c) { ls += cie_y[c] * sky[c]; lu += cie_y[c] * sun[c]; }
        sky_lum *= ls / (float)kNbWavelengths;
        sun_lum *= lu / (float)kNbWavelengths * k->area_ratio;
    }
    float res = sky_lum / (sky_lum + sun_lum);
    if (res != res) res = 0.f;
    k->w_sky = res;
    decide_sun_sky_fit(k);
    if (!spec) {
        k->spec_size = 0;
        return true;
    }
    const int size = kNbWavelengths - 1;
    bool all_zero = true, ok = true;
    for (int i = 0; i < size; ++i) {
        k->spec_pdf[i] = sun[i + 1] + sky[i + 1];
        all_zero &= k->spec_pdf[i] == 0.f;
    }
    if (all_zero)
        for (int i = 0; i < size; ++i) k->spec_pdf[i] += 1.f;
    for (int i = 0; i < size; ++i) ok &= !(k->spec_pdf[i] < 0.f);
    k->spec_size = size;
    float interval = (720.f - 360.f) / (float)(size - 1), prefix = 0.f, pre[kNbWavelengths];
    for (int i = 0; i < size; ++i) { prefix += k->spec_pdf[i]; pre[i] = prefix; }
    for (int i = 1; i < size; ++i)
        k->spec_cdf[i - 1] = interval * (pre[i] - 0.5f * k->spec_pdf[0] - 0.5f * k->spec_pdf[i]);
    k->spec_interval = interval;
    k->spec_integral = k->spec_cdf[size - 2];
    k->spec_norm = 1.f / k->spec_integral;
    k->spec_inv_interval = 1.f / interval;
    return ok;
}

}  // namespace sunsky
