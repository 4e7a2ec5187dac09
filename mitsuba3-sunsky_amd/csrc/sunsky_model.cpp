// sunsky_model.cpp -- host staging of the sun/sky emitter (see sunsky_model.h).
// All staging arithmetic is fp32 like the reference's float variants, where
// the tables are read as fp64 and cast to fp32 (sunsky.cpp:182-199).
#include "sunsky_model.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

#include "sunsky_math.h"
#include "sunsky_staging.h"

namespace sunsky {

namespace {

std::string fmt(const char* f, double v) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), f, v);
    return buf;
}

bool is_dir(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::vector<float> to_f32(const Table& t) {
    std::vector<float> r(t.size());
    for (size_t i = 0; i < t.size(); ++i) r[i] = (float)t.data[i];
    return r;
}

// bezier_interpolate + compute_radiance_params, sunsky.h:158-231 (per-entry
// arithmetic shared with the device staging kernel: sunsky_staging.h)
void compute_radiance_params(const std::vector<float>& ds, int nch, int npar, const std::vector<float>& albedo,
                             const RadianceStage& rs, std::vector<float>* out) {
    const int result_size = nch * npar;
    out->assign(result_size, 0.f);
    for (int e = 0; e < result_size; ++e) (*out)[e] = radiance_param(ds.data(), result_size, e, rs, albedo[e / npar]);
}

// Forward-mode derivative of compute_radiance_params (sunsky.h:158-231) along
// (dT, dalbedo[c], deta), in fp64: d/dx of the quintic Bezier, dx/deta of
// x = cbrt(2 eta / pi), and the derivatives of the turbidity / albedo lerps
// (floor(T) is piecewise constant, so d t_rem / dT = 1).
// compute_sun_params, sunsky.h:404-419
void compute_sun_params(const std::vector<float>& ds, int block, const RadianceStage& rs, std::vector<float>* out) {
    out->assign(block, 0.f);
    for (int i = 0; i < block; ++i) (*out)[i] = sun_param(ds.data(), block, i, rs);
}

float clipf_(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

void invert3(const double* m, double* inv) {
    double det = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
                 m[2] * (m[3] * m[7] - m[4] * m[6]);
    if (det == 0.0) throw std::invalid_argument("to_world transform is singular");
    inv[0] = (m[4] * m[8] - m[5] * m[7]) / det; inv[1] = (m[2] * m[7] - m[1] * m[8]) / det;
    inv[2] = (m[1] * m[5] - m[2] * m[4]) / det; inv[3] = (m[5] * m[6] - m[3] * m[8]) / det;
    inv[4] = (m[0] * m[8] - m[2] * m[6]) / det; inv[5] = (m[2] * m[3] - m[0] * m[5]) / det;
    inv[6] = (m[3] * m[7] - m[4] * m[6]) / det; inv[7] = (m[1] * m[6] - m[0] * m[7]) / det;
    inv[8] = (m[0] * m[4] - m[1] * m[3]) / det;
}

}  // namespace

// ------------------------------------------------------------ free helpers
void compute_sun_coordinates(const DateTime& t, const Location& l, float out[3]) {
    float dec_hours = t.hour - l.timezone + (t.minute + t.second / 60.f) / 60.f;
    int li_aux_1 = (t.month - 14) / 12;
    int li_aux_2 = (1461 * (t.year + 4800 + li_aux_1)) / 4 + (367 * (t.month - 2 - 12 * li_aux_1)) / 12 -
                   (3 * ((t.year + 4900 + li_aux_1) / 100)) / 4 + t.day - 32075;
    float d_julian_date = (float)li_aux_2 - 0.5f + dec_hours / 24.f;
    float elapsed = d_julian_date - 2451545.f;

    float omega = 2.1429f - 0.0010394594f * elapsed;
    float mean_longitude = 4.8950630f + 0.017202791698f * elapsed;
    float anomaly = 6.2400600f + 0.0172019699f * elapsed;
    float ecl_long = mean_longitude + 0.03341607f * sinf(anomaly) + 0.00034894f * sinf(2 * anomaly) -
                     0.0001134f - 0.0000203f * sinf(omega);
    float ecl_obl = 0.4090928f - 6.2140e-9f * elapsed + 0.0000396f * cosf(omega);

    float sin_ecl = sinf(ecl_long);
    float dy = cosf(ecl_obl) * sin_ecl, dx = cosf(ecl_long);
    float ra = atan2f(dy, dx);
    ra += ra < 0.f ? kTwoPi : 0.f;
    float decl = asinf(sinf(ecl_obl) * sin_ecl);

    float gmst = 6.6974243242f + 0.0657098283f * elapsed + dec_hours;
    const float deg2rad = (float)(3.14159265358979323846 / 180.0);
    float lmst = (gmst * 15 + l.longitude) * deg2rad;
    float lat = l.latitude * deg2rad;
    float cos_lat = cosf(lat), sin_lat = sinf(lat);
    float ha = lmst - ra, cos_ha = cosf(ha);
    float elevation = acosf(cos_lat * cos_ha * cosf(decl) + sinf(decl) * sin_lat);
    dy = -sinf(ha);
    dx = tanf(decl) * cos_lat - sin_lat * cos_ha;
    float azimuth = atan2f(dy, dx);
    azimuth += azimuth < 0.f ? kTwoPi : 0.f;
    elevation += (float)(6371.01 / 149597890.0) * sinf(elevation);   // parallax
    float3_ d = sphdir(elevation, azimuth - kPi);
    out[0] = d.x; out[1] = d.y; out[2] = d.z;
}

void gauss_legendre(int n, std::vector<double>* nodes, std::vector<double>* weights) {
    auto legendre_pd = [](int l, double x, double* lv, double* dv) {   // math.h:93-120
        double l_cur = 0, d_cur = 0;
        if (l > 1) {
            double l_p = 1, l_pred = x, d_p = 0, d_pred = 1, k0 = 3, k1 = 2, k2 = 1;
            for (int ki = 2; ki <= l; ++ki) {
                l_cur = (k0 * x * l_pred - k2 * l_p) / k1;
                d_cur = d_p + k0 * l_pred;
                l_p = l_pred; l_pred = l_cur; d_p = d_pred; d_pred = d_cur;
                k2 = k1; k0 += 2; k1 += 1;
            }
        } else if (l == 0) { l_cur = 1; d_cur = 0; } else { l_cur = x; d_cur = 1; }
        *lv = l_cur; *dv = d_cur;
    };
    nodes->assign(n, 0.0);
    weights->assign(n, 0.0);
    if (n < 1) throw std::invalid_argument("gauss_legendre(): n must be >= 1");
    n--;
    if (n == 0) { (*nodes)[0] = 0; (*weights)[0] = 2; return; }
    if (n == 1) { (*nodes)[0] = -std::sqrt(1.0 / 3.0); (*nodes)[1] = -(*nodes)[0]; (*weights)[0] = (*weights)[1] = 1; }
    int m = (n + 1) / 2;
    for (int i = 0; i < m; ++i) {
        double x = -std::cos((double)(2 * i + 1) / (double)(2 * n + 2) * 3.14159265358979323846);
        for (int it = 0;; ++it) {
            if (it >= 20) throw std::runtime_error("gauss_legendre: did not converge");
            double lv, dv;
            legendre_pd(n + 1, x, &lv, &dv);
            double step = lv / dv;
            x -= step;
            if (std::fabs(step) <= 4 * std::fabs(x) * 1.1102230246251565e-16) break;
        }
        double lv, dv;
        legendre_pd(n + 1, x, &lv, &dv);
        (*weights)[i] = (*weights)[n - i] = 2 / ((1 - x * x) * (dv * dv));
        (*nodes)[i] = x;
        (*nodes)[n - i] = -x;
    }
    if ((n % 2) == 0) {
        double lv, dv;
        legendre_pd(n + 1, 0.0, &lv, &dv);
        (*weights)[n / 2] = 2.0 / (dv * dv);
        (*nodes)[n / 2] = 0;
    }
}

// ------------------------------------------------------------ SunskyModel
SunskyModel::SunskyModel(const Properties& props, int variant, int semantics, const std::string& datasets,
                         bool radiance_on_host)
    : variant_(variant), semantics_(semantics) {
    if (variant != kRGB && variant != kSpectral)
        throw std::invalid_argument("Unsupported spectrum type, can only render in Spectral or RGB modes!");
    if (semantics != kJit && semantics != kScalar) throw std::invalid_argument("unknown variant semantics");
    nch_ = variant == kSpectral ? kNbWavelengths : 3;
    std::memset(&k_, 0, sizeof(k_));

    // ---------------- init_from_props, sunsky.cpp:889-948
    sun_scale_ = (float)props.get_float("sun_scale", 1.0);
    if (sun_scale_ < 0.f) throw std::invalid_argument(fmt("Invalid sun scale: %f, must be positive!", sun_scale_));
    sky_scale_ = (float)props.get_float("sky_scale", 1.0);
    if (sky_scale_ < 0.f) throw std::invalid_argument(fmt("Invalid sky scale: %f, must be positive!", sky_scale_));
    float turb = (float)props.get_float("turbidity", 3.0);
    if (turb < 1.f || 10.f < turb) throw std::invalid_argument(fmt("Turbidity value %f is out of range [1, 10]", turb));
    turbidity_ = turb;
    const float deg2rad = (float)(3.14159265358979323846 / 180.0);
    sun_aperture_deg_ = (float)props.get_float("sun_aperture", 0.5358);
    sun_half_aperture_ = (0.5f * sun_aperture_deg_) * deg2rad;
    if (sun_half_aperture_ <= 0.f || 0.5f * kPi <= sun_half_aperture_)
        throw std::invalid_argument(fmt("Invalid sun aperture angle: %f, must be in ]0, 90[ degrees!",
                                        2.0 * sun_half_aperture_ / deg2rad));
    extract_albedo(props);

    // Endpoint base: to_world (default identity)
    static const float ident[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const Properties::Value* tw = props.get_typed("to_world", Properties::Type::Transform);
    std::memcpy(to_world_, tw ? tw->m : ident, sizeof(to_world_));
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) to_world_d_[r * 3 + c] = to_world_[r * 4 + c];
    invert3(to_world_d_, to_local_d_);
    for (int i = 0; i < 9; ++i) { k_.to_world[i] = (float)to_world_d_[i]; k_.to_local[i] = (float)to_local_d_[i]; }
    k_.identity_xform = 1;
    for (int i = 0; i < 9; ++i)
        if (k_.to_world[i] != ((i % 4) == 0 ? 1.f : 0.f) || k_.to_local[i] != ((i % 4) == 0 ? 1.f : 0.f)) k_.identity_xform = 0;

    const char* tl_keys[] = {"latitude", "longitude", "timezone", "year", "month", "day", "hour", "minute", "second"};
    if (props.has("sun_direction")) {
        for (const char* key : tl_keys)
            if (props.has(key))
                throw std::invalid_argument(
                    "Both the 'sun_direction' and parameters for time/location were provided, both "
                    "information cannot be given at the same time!");
        active_record_ = false;
        const Properties::Value* v = props.get_typed("sun_direction", Properties::Type::Vector3);
        float3_ d = mk3(v->m[0], v->m[1], v->m[2]);
        float inv = 1.f / sqrtf(dot3(d, d));
        sun_dir_[0] = d.x * inv; sun_dir_[1] = d.y * inv; sun_dir_[2] = d.z * inv;
    } else {
        location_.latitude = (float)props.get_float("latitude", 35.6894);
        location_.longitude = (float)props.get_float("longitude", 139.6917);
        location_.timezone = (float)props.get_float("timezone", 9.0);
        time_.year = (int)props.get_int("year", 2010);
        time_.month = (int)props.get_int("month", 7);
        time_.day = (int)props.get_int("day", 10);
        time_.hour = (float)props.get_float("hour", 15.0);
        time_.minute = (float)props.get_float("minute", 0.0);
        time_.second = (float)props.get_float("second", 0.0);
        active_record_ = true;
        float s[3];
        compute_sun_coordinates(time_, location_, s);
        if (s[2] < 0.f) warnings.push_back("The sun is below the horizon at the specified time and location!");
        float3_ w = xform_vec(k_.to_world, mk3(s[0], s[1], s[2]));
        sun_dir_[0] = w.x; sun_dir_[1] = w.y; sun_dir_[2] = w.z;
    }
    (void)props.find("dataset_path");  // consumed by the C-ABI layer

    // ---------------- ctor body, sunsky.cpp:174-217
    float3_ local = xform_vec(k_.to_local, mk3(sun_dir_[0], sun_dir_[1], sun_dir_[2]));
    float lv[3] = {local.x, local.y, local.z};
    update_angles(lv);
    load_datasets(datasets);
    sky_params_.assign((size_t)nch_ * kNbSkyParams, 0.f);
    sky_rad_.assign(nch_, 0.f);
    stage(radiance_on_host);
    k_.bs_center[0] = k_.bs_center[1] = k_.bs_center[2] = 0.f;   // unit bounding sphere until set_scene
    k_.bs_radius = 1.f;
    commit();

    std::vector<std::string> unq = props.unqueried();
    if (!unq.empty()) {
        std::string s = "Unreferenced property \"" + unq[0] + "\" in sunsky plugin";
        throw std::invalid_argument(s);
    }
}

void SunskyModel::extract_albedo(const Properties& props) {
    albedo_.assign(nch_, 0.f);
    const Properties::Value* v = props.find("albedo");
    if (!v) {
        std::fill(albedo_.begin(), albedo_.end(), 0.3f);
    } else if (v->type == Properties::Type::Float || v->type == Properties::Type::Int) {
        float a = v->type == Properties::Type::Float ? (float)v->f : (float)v->i;
        std::fill(albedo_.begin(), albedo_.end(), a);
    } else if (v->type == Properties::Type::Spectrum) {
        if ((int)v->a.size() == 1) std::fill(albedo_.begin(), albedo_.end(), v->a[0]);
        else if ((int)v->a.size() == nch_) albedo_ = v->a;
        else throw std::invalid_argument("albedo: expected 1 or " + std::to_string(nch_) + " values");
    } else if (v->type == Properties::Type::Irregular) {
        if (variant_ != kSpectral)
            throw std::invalid_argument("irregular albedo spectra are only supported in spectral variants");
        // IrregularSpectrum::eval at the model wavelengths (linear, 0 outside its range)
        const std::vector<float>& wl = v->a;
        const std::vector<float>& val = v->b;
        if (wl.size() < 2 || wl.size() != val.size())
            throw std::invalid_argument("irregular albedo spectrum needs >= 2 (wavelength, value) pairs");
        for (int c = 0; c < nch_; ++c) {
            float lam = kWavelength0 + kWavelengthStep * c, r = 0.f;
            if (lam >= wl.front() && lam <= wl.back()) {
                size_t i = 0;
                while (i + 2 < wl.size() && wl[i + 1] < lam) ++i;
                float w1 = (lam - wl[i]) / (wl[i + 1] - wl[i]), w0 = 1.f - w1;
                r = fmaf(w0, val[i], w1 * val[i + 1]);
            }
            albedo_[c] = r;
        }
    } else {
        throw std::invalid_argument("Expected a non-spatially varying radiance spectra!");
    }
    for (float a : albedo_)
        if (a < 0.f || a > 1.f) throw std::invalid_argument(fmt("Albedo values must be in [0, 1], got: %f", a));
}

void SunskyModel::load_datasets(const std::string& where) {
    const bool spec = variant_ == kSpectral;
    auto check = [](const Table& t, size_t n, const char* name) {
        if (t.size() != n) throw std::runtime_error(std::string("dataset '") + name + "' has an unexpected size");
    };
    Table sp, sr, sun, ld, tg;
    std::string err;
    if (is_dir(where)) {
        // Reference layout: <dir>/{sky,sun}_{rgb,spec}_*.bin (path_to_dataset, sunsky.h:124-141)
        std::string d = where + "/", ty = spec ? "_spec_" : "_rgb_";
        if (!read_array_file(d + "sky" + ty + "params.bin", 2, &sp, &err) ||
            !read_array_file(d + "sky" + ty + "rad.bin", 2, &sr, &err) ||
            !read_array_file(d + "sun" + ty + "rad.bin", 2, &sun, &err) ||
            !read_array_file(d + "sun_spec_ld.bin", 2, &ld, &err) ||
            !read_array_file(d + "tgmm_tables.bin", 1, &tg, &err))
            throw std::runtime_error(err);
        // CIE Y at the model wavelengths (spectrum.cpp:158 table, 5 nm grid)
        static const float cie_y_nodes[kNbWavelengths] = {0.f, 3.917e-06f, 0.000396f, 0.023f, 0.13902f,
                                                          0.71f, 0.995f, 0.631f, 0.175f, 0.017f, 0.001047f};
        std::memcpy(cie_y_, cie_y_nodes, sizeof(cie_y_));
    } else {
        DatasetPack pack;
        Table cie;
        if (!pack.open(where, &err) || !pack.get(spec ? "sky_spec_params" : "sky_rgb_params", &sp, &err) ||
            !pack.get(spec ? "sky_spec_rad" : "sky_rgb_rad", &sr, &err) ||
            !pack.get(spec ? "sun_spec_rad" : "sun_rgb_rad", &sun, &err) || !pack.get("sun_spec_ld", &ld, &err) ||
            !pack.get("tgmm_tables", &tg, &err) || !pack.get("cie_y_nodes", &cie, &err))
            throw std::runtime_error(err);
        check(cie, kNbWavelengths, "cie_y_nodes");
        for (int i = 0; i < kNbWavelengths; ++i) cie_y_[i] = (float)cie.data[i];
    }
    check(sp, (size_t)kNbTurbidity * kNbAlbedo * kNbSkyCtrlPts * nch_ * kNbSkyParams, "sky params");
    check(sr, (size_t)kNbTurbidity * kNbAlbedo * kNbSkyCtrlPts * nch_, "sky radiance");
    check(sun, (size_t)kNbTurbidity * (spec ? kSunSpecTableSize : kSunRgbTableSize), "sun radiance");
    check(ld, (size_t)kNbWavelengths * kNbSunLdParams, "sun limb darkening");
    check(tg, (size_t)(kNbTurbidity - 1) * kNbEtas * kNbGaussian * kNbGaussianParams, "tgmm tables");
    sky_params_ds_ = to_f32(sp);
    sky_rad_ds_ = to_f32(sr);
    sun_rad_ds_ = to_f32(sun);
    sun_ld_ = to_f32(ld);   // only read in spectral mode (sunsky.cpp:193-195)
    tgmm_tables_ = to_f32(tg);
}

void SunskyModel::update_angles(const float l[3]) {
    float3_ local = mk3(l[0], l[1], l[2]);
    k_.sun_phi = atan2f(local.y, local.x);            // from_spherical, sunsky.h:84-89
    k_.sun_theta = unit_angle_z(local);
    float3_ s, t;
    coordinate_system(local, &s, &t);                  // Frame3f(local_sun_dir)
    k_.sun_n[0] = local.x; k_.sun_n[1] = local.y; k_.sun_n[2] = local.z;
    k_.sun_s[0] = s.x; k_.sun_s[1] = s.y; k_.sun_s[2] = s.z;
    k_.sun_t[0] = t.x; k_.sun_t[1] = t.y; k_.sun_t[2] = t.z;
}

// Scalars of the radiance / sun-table staging for the current (turbidity, eta)
RadianceStage SunskyModel::radiance_stage() const {
    const float eta = 0.5f * kPi - k_.sun_theta;
    RadianceStage r;
    r.x = cbrtf(2.f * kInvPi * eta);
    r.t_high = (int)floorf(turbidity_);
    r.t_low = r.t_high - 1;
    r.t_rem = turbidity_ - (float)r.t_high;
    r.in_range = (0.f <= eta) && (eta <= 0.5f * kPi);
    return r;
}

// compute_radiance_params x2 + compute_sun_params + channel folding (sunsky.h:158-231,
// 404-419): the part of parameters_changed a GPU emitter runs on the device instead.
void SunskyModel::stage_radiance() {
    const bool spec = variant_ == kSpectral;
    const RadianceStage rs = radiance_stage();
    compute_radiance_params(sky_params_ds_, nch_, kNbSkyParams, albedo_, rs, &sky_params_);
    compute_radiance_params(sky_rad_ds_, nch_, 1, albedo_, rs, &sky_rad_);
    for (int c = 0; c < nch_; ++c)
        fold_channel(&sky_params_[c * kNbSkyParams], sky_rad_[c], variant_, sky_scale_, &k_.sky[c], &k_.fsky[c]);
    compute_sun_params(sun_rad_ds_, spec ? kSunSpecTableSize : kSunRgbTableSize, rs, &sun_table_);
}

// Host staging.  radiance_on_host = false (GPU emitters): the sky channels, the sun
// table and the JIT quadrature are left to the device staging kernels
// (sunsky_stage_*), which write them into the emitter's device state; the host copy
// of those fields is then stale until adopt_device_stage().
void SunskyModel::stage(bool radiance_on_host) {
    stage_geometry();
    if (radiance_on_host) {
        stage_radiance();
        estimate_sky_sun_ratio();
    } else if (semantics_ == kScalar) {
        estimate_sky_sun_ratio();   // constants only (sunsky.cpp:778-783)
    }
    radiance_stale_ = !radiance_on_host;
}

void SunskyModel::adopt_device_stage(const SunskyKArgs& dk, const float* sun_table) {
    for (int c = 0; c < nch_; ++c) {
        k_.sky[c] = dk.sky[c];
        k_.fsky[c] = dk.fsky[c];
        const SkyChannel& ch = dk.sky[c];
        const float p[kNbSkyParams] = {ch.A, ch.B, ch.C, ch.D, ch.E, ch.F, ch.G, ch.H, ch.I};
        for (int q = 0; q < kNbSkyParams; ++q) sky_params_[(size_t)c * kNbSkyParams + q] = p[q];
        sky_rad_[c] = ch.rad;
    }
    k_.w_sky = dk.w_sky;
    k_.sun_sky_fit_on = dk.sun_sky_fit_on;
    k_.spec_size = dk.spec_size;
    std::memcpy(k_.spec_pdf, dk.spec_pdf, sizeof(k_.spec_pdf));
    std::memcpy(k_.spec_cdf, dk.spec_cdf, sizeof(k_.spec_cdf));
    k_.spec_integral = dk.spec_integral;
    k_.spec_norm = dk.spec_norm;
    k_.spec_interval = dk.spec_interval;
    k_.spec_inv_interval = dk.spec_inv_interval;
    sun_table_.assign(sun_table, sun_table + (variant_ == kSpectral ? kSunSpecTableSize : kSunRgbTableSize));
    radiance_stale_ = false;
}

// Everything of the staging that does not depend on the radiance tables: scales,
// aperture, pdf constants, the sun-disc row bound and the TGMM / discrete distribution.
void SunskyModel::stage_geometry() {
    const float eta = 0.5f * kPi - k_.sun_theta;
    k_.variant = variant_;
    k_.semantics = semantics_;
    k_.nch = nch_;
    k_.sky_scale = sky_scale_;
    k_.sun_scale = sun_scale_;
    k_.half_aperture = sun_half_aperture_;
    k_.cos_cutoff = cosf(sun_half_aperture_);
    float sh = sinf(sun_half_aperture_);
    k_.inv_sin2_half_ap = 1.f / (sh * sh);
    {
        const double shd = std::sin(0.5 * (double)sun_aperture_deg_ * (3.14159265358979323846 / 180.0));
        const double inv = 1.0 / (shd * shd);
        k_.cpsi_inv_hi = (float)inv;
        k_.cpsi_inv_lo = (float)(inv - (double)k_.cpsi_inv_hi);
    }
    // get_area_ratio, sunsky.h:99-101
    k_.area_ratio = (1.f - cosf((float)(kSunHalfApertureDeg * (3.14159265358979323846 / 180.0)))) /
                    (1.f - cosf(sun_half_aperture_));
    k_.sun_pdf = kInvTwoPi / (1.f - k_.cos_cutoff);   // square_to_uniform_cone_pdf, warp.h:568-577

    k_.sun_mul = variant_ == kRGB
                     ? sun_scale_ * k_.area_ratio * (float)kSpecToRgbSunConv * (float)kCieYNormalization
                     : sun_scale_ * k_.area_ratio;
    {
        // Segments of render_sun's search (sunsky.cpp:579-587) over the elevations of the
        // directions inside the disc, [eta - aperture / 2, eta + aperture / 2], with a margin
        // far above fp32 rounding: the sampling kernels stage kSunRowsStaged segments from
        // sun_row_lo (a lane outside them reads the device table), and every kernel counts the
        // cos theta thresholds in (sun_row_lo, sun_row_hi] for a disc direction's segment.
        constexpr double kPiD = 3.14159265358979323846;
        auto seg_of = [](double elev) {
            const double seg = std::cbrt(2.0 * std::min(std::max(elev, 0.0), 0.5 * kPiD) / kPiD) * (double)kNbSunSegments;
            return std::min((int)std::floor(seg), kNbSunSegments - 1);
        };
        k_.sun_row_lo = seg_of((double)eta - (double)sun_half_aperture_ - 1e-3);
        k_.sun_row_hi = seg_of((double)eta + (double)sun_half_aperture_ + 1e-3);
        const std::array<float, kNbSunSegments>& z = sun_segment_thresholds();
        std::copy(z.begin(), z.end(), k_.sun_seg_z);
    }

    // ---------------- TGMM, sunsky.h:438-501
    {
        float eta_deg = eta * (float)(180.0 / 3.14159265358979323846);
        float eta_idx_f = clipf_((eta_deg - 2.f) / 3.f, 0.f, (float)(kNbEtas - 1));
        float t_idx_f = clipf_(turbidity_ - 2.f, 0.f, (float)(kNbTurbidity - 2));
        int eta_lo = (int)floorf(eta_idx_f), t_lo = (int)floorf(t_idx_f);
        int eta_hi = std::min(eta_lo + 1, kNbEtas - 1), t_hi = std::min(t_lo + 1, kNbTurbidity - 2);
        float eta_rem = eta_idx_f - (float)eta_lo, t_rem = t_idx_f - (float)t_lo;
        const int result_size = kNbGaussian * kNbGaussianParams, t_block = kNbEtas * result_size;
        const int idx[4] = {t_lo * t_block + eta_lo * result_size, t_lo * t_block + eta_hi * result_size,
                            t_hi * t_block + eta_lo * result_size, t_hi * t_block + eta_hi * result_size};
        const float lf[4] = {(1 - t_rem) * (1 - eta_rem), (1 - t_rem) * eta_rem, t_rem * (1 - eta_rem),
                             t_rem * eta_rem};
        for (int m = 0; m < 4; ++m)
            for (int i = 0; i < result_size; ++i) {
                float v = tgmm_tables_[idx[m] + i];
                if (i % kNbGaussianParams == kNbGaussianParams - 1) v = v * lf[m];
                gauss_raw_[m * result_size + i] = v;
            }
        for (int g = 0; g < kNbMixture; ++g) {
            const float* r = &gauss_raw_[g * kNbGaussianParams];
            Gaussian& G = k_.gauss[g];
            G.mu_phi = r[0]; G.mu_theta = r[1]; G.sigma_phi = r[2]; G.sigma_theta = r[3]; G.weight = r[4];
            G.inv_sigma_phi = 1.f / r[2];
            G.inv_sigma_theta = 1.f / r[3];
            G.cdf_a_phi = gaussian_cdf(r[0], r[2], 0.f);
            G.cdf_b_phi = gaussian_cdf(r[0], r[2], kTwoPi);
            G.cdf_a_theta = gaussian_cdf(r[1], r[3], 0.f);
            G.cdf_b_theta = gaussian_cdf(r[1], r[3], 0.5f * kPi);
            float volume = (G.cdf_b_phi - G.cdf_a_phi) * (G.cdf_b_theta - G.cdf_a_theta) * (r[2] * r[3]);
            G.coef = r[4] / volume;
            k_.gauss_pmf[g] = r[4];
        }
        k_.tgmm_count = 0;
        for (int g = 0; g < kNbMixture; ++g)
            if (k_.gauss[g].coef != 0.f) k_.tgmm_idx[k_.tgmm_count++] = (uint8_t)g;
        // DiscreteDistribution(mis_weights): JIT prefix_sum in fp32 (distr_1d.h:218-231),
        // scalar accumulation in fp64 + first/last nonzero bounds (:233-265)
        bool any_pos = false;
        for (int g = 0; g < kNbMixture; ++g) {
            if (k_.gauss_pmf[g] < 0.f) throw std::runtime_error("DiscreteDistribution: entries must be non-negative!");
            any_pos |= k_.gauss_pmf[g] > 0.f;
        }
        if (!any_pos) throw std::runtime_error("DiscreteDistribution: no probability mass found!");
        k_.gauss_first = -1;
        k_.gauss_last = -1;
        if (semantics_ == kJit) {
            float acc = 0.f;
            for (int g = 0; g < kNbMixture; ++g) { acc += k_.gauss_pmf[g]; k_.gauss_cdf[g] = acc; }
            k_.gauss_first = 0;
            k_.gauss_last = kNbMixture - 1;
        } else {
            double acc = 0.0;
            for (int g = 0; g < kNbMixture; ++g) {
                acc += (double)k_.gauss_pmf[g];
                k_.gauss_cdf[g] = (float)acc;
                if (k_.gauss_pmf[g] > 0.f) {
                    if (k_.gauss_first < 0) k_.gauss_first = g;
                    k_.gauss_last = g;
                }
            }
        }
        k_.gauss_sum = k_.gauss_cdf[k_.gauss_last];
        k_.gauss_norm = 1.f / k_.gauss_sum;
        build_gauss_guide();
    }
    stage_sun_sky_fit();

    k_.sun_table = nullptr;   // device pointers are patched in by the C-ABI layer
    k_.sun_ld = nullptr;
}

const std::array<float, kNbSunSegments>& sun_segment_thresholds() {
    // Committed constants, not derived at run time from whatever libm loads the
    // library: [j] is the smallest fp32 cos theta in [0, 1] whose render_sun segment
    // (sunsky.cpp:579-584: min(floor(cbrt(2 (pi/2 - acosf z) / pi) 45), 44) in fp32, no
    // contraction) is >= j, found by bisection over the fp32 bit patterns of [0, 1] (the decision
    // is monotone there) with glibc 2.35's acosf / cbrtf.
    // tests/test_capi_cpu.py checks EVERY fp32 cos theta in [0, 1] against the oracle's fp32
    // decision on the libm the tests run on (a libm whose decision moves fails that test).
    static const std::array<float, kNbSunSegments> z = {{
    0x0.0p+0f, 0x1.204442p-16f, 0x1.210888p-13f, 0x1.e80444p-12f, 0x1.21310ep-10f,
    0x1.1a6c7cp-9f, 0x1.e8044p-9f, 0x1.837bbp-8f, 0x1.21322ep-7f, 0x1.9bc35cp-7f,
    0x1.1a68fep-6f, 0x1.77dfap-6f, 0x1.e7f51ap-6f, 0x1.362b4ep-5f, 0x1.83578cp-5f,
    0x1.dc527ap-5f, 0x1.20f644p-4f, 0x1.5a7926p-4f, 0x1.9b14ccp-4f, 0x1.e328dep-4f,
    0x1.1987b2p-3f, 0x1.458df6p-3f, 0x1.75ccb4p-3f, 0x1.aa63e2p-3f, 0x1.e36c74p-3f,
    0x1.107b84p-2f, 0x1.3184c4p-2f, 0x1.54cea4p-2f, 0x1.7a4e12p-2f, 0x1.a1eed8p-2f,
    0x1.cb9202p-2f, 0x1.f70bfap-2f, 0x1.12114ap-1f, 0x1.29457ap-1f, 0x1.40f3aap-1f,
    0x1.58e25cp-1f, 0x1.70cc56p-1f, 0x1.885fa2p-1f, 0x1.9f3c7cp-1f, 0x1.b4f4b8p-1f,
    0x1.c90b3p-1f, 0x1.daf3dap-1f, 0x1.ea1422p-1f, 0x1.f5c448p-1f, 0x1.fd5146p-1f,
    }};
    return z;
}

// Index returned by the kernels' discrete_sample_reuse for s = value * sum:
// JIT, the prefix count of ((cdf < s) || cdf == 0) && cdf != sum over [0, n-1)
// (distr_1d.h:116-136); scalar, first + #{i in [first, last) : cdf[i] < s}.
// Both are monotone in s (cdf is non-decreasing).
int SunskyModel::gauss_search(float s) const {
    if (semantics_ == kJit) {
        int idx = 0;
        for (int i = 0; i < kNbMixture - 1; ++i) {
            const float c = k_.gauss_cdf[i];
            if (!(((c < s) || c == 0.f) && (c != k_.gauss_sum))) break;
            ++idx;
        }
        return idx;
    }
    int idx = k_.gauss_first;
    for (int i = k_.gauss_first; i < k_.gauss_last; ++i)
        if (k_.gauss_cdf[i] < s) idx = i + 1;
    return idx;
}

// Guide table for the device search (SunskyKArgs::gauss_guide).  For value in
// [b/B, (b+1)/B) the fp32 product s = value * sum lies in [fl(b/B sum),
// fl((b+1)/B sum)] (rounding is monotone; b/B is exact), so the index lies in
// [search(s_lo), search(s_hi)].
void SunskyModel::build_gauss_guide() {
    int span = 0;
    for (int b = 0; b < kGaussGuideSize; ++b) {
        const float v0 = (float)b / (float)kGaussGuideSize, v1 = (float)(b + 1) / (float)kGaussGuideSize;
        const int lo = gauss_search(v0 * k_.gauss_sum), hi = gauss_search(v1 * k_.gauss_sum);
        k_.gauss_guide[b] = (uint8_t)lo;
        span = std::max(span, hi - lo);
    }
    k_.gauss_guide_span = span;
}

// The sky pdf over the sun disc, for the FAST samplers' sun picks (SunskyKArgs::sun_sky_fit).
// f(a, b) = tgmm_pdf(phi, theta) / sin(theta) (sunsky.cpp:711-763) of the local direction
// a s + b t + sqrt(1 - a^2 - b^2) n, (a, b) in the disc of radius rho = sin(half aperture),
// in fp64 from the staged fp32 gaussians.  Least-squares quadratic on 12 x 24 polar points,
// then the deviation and the smallest value over a 41 x 96 polar grid (rim included); the
// bound kept is twice the grid deviation plus 4e-7 of the largest value (the kernels
// evaluate the fp32 coefficients in fp32).  Not used (sun_sky_fit_ok = 0) when the disc
// comes within 16 rho of the zenith (1 / sin(theta) varies fast there), within 2 rho of the
// horizon (the pdf's mask), or near the wrap of phi.
void SunskyModel::stage_sun_sky_fit() {
    k_.sun_sky_fit_ok = 0;
    k_.sun_sky_fit_on = 0;
    for (float& c : k_.sun_sky_fit) c = 0.f;
    k_.sun_sky_fit_dev = k_.sun_sky_fit_fmin = 0.f;
    const double cc = (double)k_.cos_cutoff, rho = std::sqrt(std::max(0.0, 1.0 - cc * cc));
    const double n[3] = {k_.sun_n[0], k_.sun_n[1], k_.sun_n[2]}, s[3] = {k_.sun_s[0], k_.sun_s[1], k_.sun_s[2]},
                 t[3] = {k_.sun_t[0], k_.sun_t[1], k_.sun_t[2]};
    const double pi = 3.14159265358979323846, phi0 = (double)k_.sun_phi - 0.5 * (double)kPi;
    if (!(rho > 0.0) || !(n[2] > 2.0 * rho) || std::sqrt(n[0] * n[0] + n[1] * n[1]) < 16.0 * rho) return;
    bool ok = true;
    auto f = [&](double x, double y) {   // x, y: disc coordinates / rho
        const double a = x * rho, b = y * rho, z = std::sqrt(std::max(0.0, 1.0 - a * a - b * b));
        const double d[3] = {a * s[0] + b * t[0] + z * n[0], a * s[1] + b * t[1] + z * n[1],
                             a * s[2] + b * t[2] + z * n[2]};
        const double st = std::sqrt(d[0] * d[0] + d[1] * d[1]), th = std::atan2(st, d[2]);
        double ph = std::atan2(d[1], d[0]) - phi0;
        if (ph < 0.0) ph += 2.0 * pi;
        if (ph > 2.0 * pi) ph -= 2.0 * pi;
        if (!(d[2] > rho) || ph < 0.25 || ph > 2.0 * pi - 0.25 || th > 0.5 * pi) ok = false;
        double pdf = 0.0;
        for (int i = 0; i < k_.tgmm_count; ++i) {
            const Gaussian& g = k_.gauss[k_.tgmm_idx[i]];
            const double sx = (ph - g.mu_phi) / g.sigma_phi, sy = (th - g.mu_theta) / g.sigma_theta;
            pdf += (double)g.coef * std::exp(-0.5 * (sx * sx + sy * sy)) / (2.0 * pi);
        }
        return pdf / st;
    };
    auto basis = [](double x, double y, double* v) { v[0] = 1; v[1] = x; v[2] = y; v[3] = x * x; v[4] = x * y; v[5] = y * y; };
    double A[6][7] = {};
    for (int i = 0; i < 12; ++i)
        for (int j = 0; j < 24; ++j) {
            const double r = std::sqrt((i + 0.5) / 12.0), ang = 2.0 * pi * (j + 0.5 * (i & 1)) / 24.0;
            const double x = r * std::cos(ang), y = r * std::sin(ang), v0 = f(x, y);
            double v[6];
            basis(x, y, v);
            for (int p = 0; p < 6; ++p) {
                for (int q = 0; q < 6; ++q) A[p][q] += v[p] * v[q];
                A[p][6] += v[p] * v0;
            }
        }
    for (int c = 0; c < 6; ++c) {   // Gaussian elimination, partial pivoting
        int piv = c;
        for (int r = c + 1; r < 6; ++r)
            if (std::fabs(A[r][c]) > std::fabs(A[piv][c])) piv = r;
        for (int q = 0; q < 7; ++q) std::swap(A[c][q], A[piv][q]);
        for (int r = 0; r < 6; ++r) {
            if (r == c) continue;
            const double m = A[r][c] / A[c][c];
            for (int q = c; q < 7; ++q) A[r][q] -= m * A[c][q];
        }
    }
    double cn[6];
    for (int c = 0; c < 6; ++c) cn[c] = A[c][6] / A[c][c];
    double dev = 0.0, fmin = 1e300, fmax = 0.0;
    for (int i = 0; i <= 40; ++i)
        for (int j = 0; j < 96; ++j) {
            const double r = i / 40.0, ang = 2.0 * pi * j / 96.0, x = r * std::cos(ang), y = r * std::sin(ang);
            const double v0 = f(x, y);
            double v[6], p = 0.0;
            basis(x, y, v);
            for (int q = 0; q < 6; ++q) p += cn[q] * v[q];
            dev = std::max(dev, std::fabs(p - v0));
            fmin = std::min(fmin, v0);
            fmax = std::max(fmax, v0);
        }
    if (!ok || !(fmin > 0.0) || !std::isfinite(dev)) return;
    // unnormalised coefficients: x = a / rho, y = b / rho
    const double sc[6] = {1.0, 1.0 / rho, 1.0 / rho, 1.0 / (rho * rho), 1.0 / (rho * rho), 1.0 / (rho * rho)};
    for (int c = 0; c < 6; ++c) k_.sun_sky_fit[c] = (float)(cn[c] * sc[c]);
    k_.sun_sky_fit_dev = (float)(2.0 * dev + 4e-7 * fmax);
    k_.sun_sky_fit_fmin = (float)(0.99 * fmin);
    k_.sun_sky_fit_ok = 1;
}

// estimate_sky_sun_ratio, sunsky.cpp:772-886
void SunskyModel::estimate_sky_sun_ratio() {
    const bool spec = variant_ == kSpectral;
    if (semantics_ == kScalar) {
        // Mean ratio + uniform spectral sampling (:778-783)
        k_.w_sky = 0.5f;
        decide_sun_sky_fit(&k_);
        if (spec) {
            k_.spec_size = 2;
            k_.spec_pdf[0] = k_.spec_pdf[1] = 1.f;
            double interval = 720.0 - 360.0, integral = 0.5 * interval * 2.0;
            k_.spec_cdf[0] = (float)integral;
            k_.spec_interval = (float)interval;
            k_.spec_integral = k_.spec_cdf[0];
            k_.spec_norm = 1.f / k_.spec_integral;
            k_.spec_inv_interval = 1.f / k_.spec_interval;
        } else {
            k_.spec_size = 0;
        }
        return;
    }
    std::vector<float> x, w;
    quadrature_nodes(&x, &w);
    const int NQ = (int)x.size();
    // Row partial sums in parallel, rows added in a fixed order: deterministic for any
    // thread count, and the same reduction the device staging kernels run.
    std::vector<float> row_sky((size_t)NQ * nch_), row_sun((size_t)NQ * nch_);
#pragma omp parallel for schedule(static)
    for (int j = 0; j < NQ; ++j) {
        float as[kNbWavelengths] = {0}, au[kNbWavelengths] = {0};
        for (int i = 0; i < NQ; ++i) {
            const QuadDir d = quad_dir(k_, x.data(), w.data(), i, j);
            for (int c = 0; c < nch_; ++c) {
                float vs, vu;
                quad_channel(k_, sun_table_.data(), sun_ld_.data(), d, w[j], c, &vs, &vu);
                as[c] += vs;
                au[c] += vu;
            }
        }
        for (int c = 0; c < nch_; ++c) {
            row_sky[(size_t)j * nch_ + c] = as[c];
            row_sun[(size_t)j * nch_ + c] = au[c];
        }
    }
    float sky[kNbWavelengths] = {0}, sun[kNbWavelengths] = {0};
    for (int j = 0; j < NQ; ++j)
        for (int c = 0; c < nch_; ++c) { sky[c] += row_sky[(size_t)j * nch_ + c]; sun[c] += row_sun[(size_t)j * nch_ + c]; }
    if (!quad_finish(&k_, sky, sun, cie_y_, sky_scale_, sun_scale_))
        throw std::runtime_error("ContinuousDistribution: entries must be non-negative!");
}

// quad::gauss_legendre<Float>(200) nodes and weights, fp64 -> fp32 (sunsky.cpp:789-790)
void SunskyModel::quadrature_nodes(std::vector<float>* x, std::vector<float>* w) {
    constexpr int NQ = 200;
    std::vector<double> xd, wd;
    gauss_legendre(NQ, &xd, &wd);
    x->resize(NQ);
    w->resize(NQ);
    for (int i = 0; i < NQ; ++i) { (*x)[i] = (float)xd[i]; (*w)[i] = (float)wd[i]; }
}

void SunskyModel::validate() const {
    if (sun_scale_ < 0.f) throw std::invalid_argument(fmt("Invalid sun scale: %f, must be positive!", sun_scale_));
    if (sky_scale_ < 0.f) throw std::invalid_argument(fmt("Invalid sky scale: %f, must be positive!", sky_scale_));
    if (turbidity_ < 1.f || 10.f < turbidity_)
        throw std::invalid_argument(fmt("Turbidity value %f is out of range [1, 10]", turbidity_));
    for (float a : albedo_)
        if (a < 0.f || a > 1.f) throw std::invalid_argument(fmt("Albedo values must be in [0, 1], got: %f", a));
}

TangentStage SunskyModel::tangent_stage(int param, const float* tangent, int count) const {
    if (!tangent) throw std::invalid_argument("null tangent");
    TangentStage s;
    std::memset(&s, 0, sizeof(s));
    double deta = 0.0;
    switch (param) {
        case kJvpTurbidity:
            if (count != 1) throw std::invalid_argument("turbidity tangent has 1 value");
            s.dT = tangent[0];
            break;
        case kJvpAlbedo:
            if (count != 1 && count != nch_)
                throw std::invalid_argument("albedo tangent has 1 or " + std::to_string(nch_) + " values");
            for (int c = 0; c < nch_; ++c) s.dalbedo[c] = tangent[count == 1 ? 0 : c];
            break;
        case kJvpSunDirection: {
            if (active_record_) throw std::invalid_argument("sun_direction is not differentiable in time/location mode");
            if (count != 3) throw std::invalid_argument("sun_direction tangent has 3 values");
            // local = M^-1 m_sun_dir (parameters_changed, sunsky.cpp:258-263)
            double dl[3];
            for (int r = 0; r < 3; ++r)
                dl[r] = to_local_d_[r * 3] * tangent[0] + to_local_d_[r * 3 + 1] * tangent[1] +
                        to_local_d_[r * 3 + 2] * tangent[2];
            for (int r = 0; r < 3; ++r) s.dsun_local[r] = (float)dl[r];
            // theta = unit_angle_z(local) (from_spherical, sunsky.h:84-89); eta = pi/2 - theta
            const double lz = k_.sun_n[2];
            const double w[3] = {k_.sun_n[0], k_.sun_n[1], lz - (std::signbit(lz) ? -1.0 : 1.0)};
            const double h = 0.5 * std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            if (h > 0.0) {
                const double dtemp = (w[0] * dl[0] + w[1] * dl[1] + w[2] * dl[2]) / (2.0 * h * std::sqrt(1.0 - h * h));
                const double dtheta = lz >= 0.0 ? dtemp : -dtemp;
                deta = -dtheta;
            }
            break;
        }
        default: throw std::invalid_argument("unknown differentiable parameter");
    }
    // the staging scalars of compute_radiance_params (sunsky.h:158-231) and their tangents:
    // x = cbrt(2 eta / pi), dx = 2 / (3 pi x^2) deta; t_rem = T - floor(T), d t_rem / dT = 1
    const float eta = 0.5f * kPi - k_.sun_theta;
    s.x = std::cbrt(2.0 * eta / 3.14159265358979323846);
    s.deta = deta;
    s.dx_per_eta = s.x > 0.0 ? (2.0 / (3.0 * 3.14159265358979323846)) / (s.x * s.x) : 0.0;
    s.dx = s.x > 0.0 ? s.dx_per_eta * deta : 0.0;
    s.t_high = (int)std::floor(turbidity_);
    s.t_low = s.t_high - 1;
    s.t_rem = (double)turbidity_ - s.t_high;
    s.in_range = (0.f <= eta) && (eta <= 0.5f * kPi);
    s.nch = nch_;
    for (int c = 0; c < nch_; ++c) s.albedo[c] = albedo_[c];
    return s;
}

EvalTangent SunskyModel::eval_tangent(int param, const float* tangent, int count) const {
    const TangentStage s = tangent_stage(param, tangent, count);
    EvalTangent out;
    out.dsky.assign((size_t)nch_ * 10, 0.f);
    for (int j = 0; j < nch_ * 10; ++j) out.dsky[j] = tangent_value(sky_params_ds_.data(), sky_rad_ds_.data(), s, j);
    std::memcpy(out.dsun_local, s.dsun_local, sizeof(out.dsun_local));
    // sun table: lerp over turbidity (compute_sun_params, sunsky.h:404-419)
    const int block = variant_ == kSpectral ? kSunSpecTableSize : kSunRgbTableSize;
    out.dsun.assign(block, 0.f);
    for (int i = 0; i < block; ++i) out.dsun[i] = sun_param_tangent(sun_rad_ds_.data(), block, i, s);
    return out;
}

void SunskyModel::set_param(const std::string& name, const float* v, int count) {
    auto need = [&](int n) {
        if (count != n) throw std::invalid_argument("parameter '" + name + "' expects " + std::to_string(n) + " value(s)");
    };
    auto need_record = [&]() {
        if (!active_record_) throw std::invalid_argument("parameter '" + name + "' is not exposed (sun_direction mode)");
    };
    if (name == "turbidity") { need(1); turbidity_ = v[0]; }
    else if (name == "sky_scale") { need(1); sky_scale_ = v[0]; }
    else if (name == "sun_scale") { need(1); sun_scale_ = v[0]; }
    else if (name == "albedo") {
        if (count == 1) std::fill(albedo_.begin(), albedo_.end(), v[0]);
        else { need(nch_); albedo_.assign(v, v + nch_); }
    }
    else if (name == "latitude") { need_record(); need(1); location_.latitude = v[0]; }
    else if (name == "longitude") { need_record(); need(1); location_.longitude = v[0]; }
    else if (name == "timezone") { need_record(); need(1); location_.timezone = v[0]; }
    else if (name == "year") { need_record(); need(1); time_.year = (int)v[0]; }
    else if (name == "month") { need_record(); need(1); time_.month = (int)v[0]; }
    else if (name == "day") { need_record(); need(1); time_.day = (int)v[0]; }
    else if (name == "hour") { need_record(); need(1); time_.hour = v[0]; }
    else if (name == "minute") { need_record(); need(1); time_.minute = v[0]; }
    else if (name == "second") { need_record(); need(1); time_.second = v[0]; }
    else if (name == "sun_direction") {
        if (active_record_) throw std::invalid_argument("parameter 'sun_direction' is not exposed (time/location mode)");
        need(3);
        std::memcpy(sun_dir_, v, 3 * sizeof(float));
    }
    else if (name == "to_world") {
        need(16);
        std::memcpy(to_world_, v, sizeof(to_world_));
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) to_world_d_[r * 3 + c] = to_world_[r * 4 + c];
        invert3(to_world_d_, to_local_d_);
        for (int i = 0; i < 9; ++i) { k_.to_world[i] = (float)to_world_d_[i]; k_.to_local[i] = (float)to_local_d_[i]; }
        k_.identity_xform = 1;
        for (int i = 0; i < 9; ++i)
            if (k_.to_world[i] != ((i % 4) == 0 ? 1.f : 0.f) || k_.to_local[i] != ((i % 4) == 0 ? 1.f : 0.f))
                k_.identity_xform = 0;
    }
    else throw std::invalid_argument("unknown parameter '" + name + "'");
}

void SunskyModel::parameters_changed(bool radiance_on_host) {
    try {
        validate();
        float local[3];
        if (active_record_) {
            compute_sun_coordinates(time_, location_, local);
            float3_ w = xform_vec(k_.to_world, mk3(local[0], local[1], local[2]));
            sun_dir_[0] = w.x; sun_dir_[1] = w.y; sun_dir_[2] = w.z;
        } else {
            float3_ l = xform_vec(k_.to_local, mk3(sun_dir_[0], sun_dir_[1], sun_dir_[2]));
            local[0] = l.x; local[1] = l.y; local[2] = l.z;
        }
        update_angles(local);
        stage(radiance_on_host);
    } catch (...) {
        rollback();
        throw;
    }
    commit();
}

void SunskyModel::commit() {
    Snapshot& c = committed_;
    c.turbidity = turbidity_; c.sky_scale = sky_scale_; c.sun_scale = sun_scale_;
    c.albedo = albedo_; c.time = time_; c.location = location_;
    std::memcpy(c.sun_dir, sun_dir_, sizeof(sun_dir_));
    std::memcpy(c.to_world, to_world_, sizeof(to_world_));
    std::memcpy(c.to_world_d, to_world_d_, sizeof(to_world_d_));
    std::memcpy(c.to_local_d, to_local_d_, sizeof(to_local_d_));
    c.sky_params = sky_params_; c.sky_rad = sky_rad_; c.sun_table = sun_table_;
    std::memcpy(c.gauss_raw, gauss_raw_, sizeof(gauss_raw_));
    c.k = k_;
    c.radiance_stale = radiance_stale_;
}

void SunskyModel::rollback() {
    const Snapshot& c = committed_;
    turbidity_ = c.turbidity; sky_scale_ = c.sky_scale; sun_scale_ = c.sun_scale;
    albedo_ = c.albedo; time_ = c.time; location_ = c.location;
    std::memcpy(sun_dir_, c.sun_dir, sizeof(sun_dir_));
    std::memcpy(to_world_, c.to_world, sizeof(to_world_));
    std::memcpy(to_world_d_, c.to_world_d, sizeof(to_world_d_));
    std::memcpy(to_local_d_, c.to_local_d, sizeof(to_local_d_));
    sky_params_ = c.sky_params; sky_rad_ = c.sky_rad; sun_table_ = c.sun_table;
    std::memcpy(gauss_raw_, c.gauss_raw, sizeof(gauss_raw_));
    const float bs[4] = {k_.bs_center[0], k_.bs_center[1], k_.bs_center[2], k_.bs_radius};
    k_ = c.k;
    k_.bs_center[0] = bs[0]; k_.bs_center[1] = bs[1]; k_.bs_center[2] = bs[2]; k_.bs_radius = bs[3];
    radiance_stale_ = c.radiance_stale;
}

void SunskyModel::revert_to_accepted() {
    committed_ = accepted_;
    rollback();
}

int SunskyModel::get_param(const std::string& name, float* out, int cap) const {
    std::vector<float> v;
    if (name == "turbidity") v = {turbidity_};
    else if (name == "sky_scale") v = {sky_scale_};
    else if (name == "sun_scale") v = {sun_scale_};
    else if (name == "albedo") v = albedo_;
    else if (name == "latitude") v = {location_.latitude};
    else if (name == "longitude") v = {location_.longitude};
    else if (name == "timezone") v = {location_.timezone};
    else if (name == "year") v = {(float)time_.year};
    else if (name == "month") v = {(float)time_.month};
    else if (name == "day") v = {(float)time_.day};
    else if (name == "hour") v = {time_.hour};
    else if (name == "minute") v = {time_.minute};
    else if (name == "second") v = {time_.second};
    else if (name == "sun_direction") v.assign(sun_dir_, sun_dir_ + 3);
    else if (name == "to_world") v.assign(to_world_, to_world_ + 16);
    else throw std::invalid_argument("unknown parameter '" + name + "'");
    for (int i = 0; i < (int)v.size() && i < cap; ++i) out[i] = v[i];
    return (int)v.size();
}

void SunskyModel::set_scene(bool bbox_valid, const float center[3], float radius) {
    const float ray_eps = 5.9604644775390625e-08f * 1500.f;   // math::RayEpsilon<float>
    if (bbox_valid) {
        k_.bs_center[0] = center[0]; k_.bs_center[1] = center[1]; k_.bs_center[2] = center[2];
        k_.bs_radius = std::max(ray_eps, radius * (1.f + ray_eps));
    } else {
        k_.bs_center[0] = k_.bs_center[1] = k_.bs_center[2] = 0.f;
        k_.bs_radius = ray_eps;
    }
}

std::string SunskyModel::to_string() const {
    std::ostringstream oss;
    oss << "SunskyEmitter[\n  bsphere = BoundingSphere3f[center = [" << k_.bs_center[0] << ", " << k_.bs_center[1]
        << ", " << k_.bs_center[2] << "], radius = " << k_.bs_radius << "]\n  turbidity = " << turbidity_
        << "\n  sky_scale = " << sky_scale_ << "\n  sun_scale = " << sun_scale_ << "\n  albedo = [";
    for (size_t i = 0; i < albedo_.size(); ++i) oss << (i ? ", " : "") << albedo_[i];
    oss << "]\n  sun aperture (\xc2\xb0) = " << 2.0 * sun_half_aperture_ * 180.0 / 3.14159265358979323846 << "\n";
    if (active_record_)
        oss << "  location = LocationRecord[latitude = " << location_.latitude << ", longitude = " << location_.longitude
            << ", timezone = " << location_.timezone << "]\n  date_time = DateTimeRecord[year = " << time_.year
            << ", month= " << time_.month << ", day = " << time_.day << ", hour = " << time_.hour
            << ", minute = " << time_.minute << ", second = " << time_.second << "]\n";
    else
        oss << "  sun_dir = [" << sun_dir_[0] << ", " << sun_dir_[1] << ", " << sun_dir_[2] << "]\n";
    oss << "]";
    return oss.str();
}

}  // namespace sunsky
