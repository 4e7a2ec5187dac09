// sunsky_amd.hpp -- header-only C++17 facade over the C ABI (sunsky_amd.h).
//
// The host-side mirror of the reference plugin's interface for the renderer
// that links this library instead of src/emitters/sunsky.cpp: the same
// methods as mitsuba::Emitter / Endpoint (include/mitsuba/render/endpoint.h:99-313,
// emitter.h:53-95; overrides in sunsky.cpp:220-500) with the same argument
// meaning, batched: every Dr.Jit array becomes a structure-of-arrays batch of
// device pointers and a count.  Errors come back as sunsky_amd::Error carrying
// the reference's message (the reference throws via Log(Error, ...),
// logger.cpp:55-60); sample_position raises NotImplementedError like
// sunsky.cpp:483-495.  No HIP types appear here: streams are `void*`
// (a hipStream_t), so callers need only this header and libsunsky_amd.so.
#pragma once

#include <cmath>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "sunsky_amd.h"

namespace sunsky_amd {

struct Error : std::runtime_error {
    int status;
    Error(int s, const std::string& what) : std::runtime_error(what), status(s) {}
};
struct NotImplementedError : Error {
    explicit NotImplementedError(const std::string& what) : Error(SUNSKY_ERROR_NOT_IMPLEMENTED, what) {}
};

inline void check(int status) {
    if (status == SUNSKY_OK) return;
    std::string msg = sunsky_last_error();
    if (status == SUNSKY_ERROR_NOT_IMPLEMENTED) throw NotImplementedError(msg);
    throw Error(status, msg);
}

enum class Variant { RGB = SUNSKY_VARIANT_RGB, Spectral = SUNSKY_VARIANT_SPECTRAL };
enum class Semantics { JIT = SUNSKY_SEMANTICS_JIT, Scalar = SUNSKY_SEMANTICS_SCALAR };
enum class Precision { Fast = SUNSKY_PRECISION_FAST, Reference = SUNSKY_PRECISION_REFERENCE };
// Differentiable traverse() parameters (sunsky.cpp:220-240)
enum class Param {
    Turbidity = SUNSKY_PARAM_TURBIDITY,
    Albedo = SUNSKY_PARAM_ALBEDO,
    SunDirection = SUNSKY_PARAM_SUN_DIRECTION
};

// mitsuba::Properties subset consumed by SunskyEmitter::init_from_props (sunsky.cpp:889-948).
class Properties {
public:
    Properties() { check(sunsky_props_create(&p_)); }
    ~Properties() { sunsky_props_destroy(p_); }
    Properties(const Properties&) = delete;
    Properties& operator=(const Properties&) = delete;

    Properties& set_float(const char* name, double v) { check(sunsky_props_set_float(p_, name, v)); return *this; }
    Properties& set_int(const char* name, int64_t v) { check(sunsky_props_set_int(p_, name, v)); return *this; }
    Properties& set_vector3(const char* name, float x, float y, float z) {
        check(sunsky_props_set_vector3(p_, name, x, y, z));
        return *this;
    }
    Properties& set_transform(const char* name, const float m[16]) {
        check(sunsky_props_set_transform(p_, name, m));
        return *this;
    }
    Properties& set_spectrum(const char* name, const std::vector<float>& v) {
        check(sunsky_props_set_spectrum(p_, name, v.data(), (int)v.size()));
        return *this;
    }
    Properties& set_irregular_spectrum(const char* name, const std::vector<float>& wl, const std::vector<float>& v) {
        if (wl.size() != v.size()) throw Error(SUNSKY_ERROR_INVALID_VALUE, "wavelength / value size mismatch");
        check(sunsky_props_set_irregular_spectrum(p_, name, wl.data(), v.data(), (int)v.size()));
        return *this;
    }
    const sunsky_props* get() const { return p_; }

private:
    sunsky_props* p_ = nullptr;
};

// ---------------------------------------------------------------- batches
// Vector3f / Point3f batch: three fp32 device planes.
struct Vector3 { const float *x = nullptr, *y = nullptr, *z = nullptr; };
struct Vector3Out { float *x = nullptr, *y = nullptr, *z = nullptr; };
struct Point2 { const float *x = nullptr, *y = nullptr; };

// Spectrum batch: `channels` planes at data + c * stride (3 RGB, 4 in Mitsuba's spectral variants).
struct SpectrumOut { float* data = nullptr; size_t stride = 0; };
struct Wavelengths { const float* data = nullptr; int count = 0; size_t stride = 0; };

// SurfaceInteraction3f fields eval() reads (sunsky.cpp:303-352): wi and wavelengths.
struct SurfaceInteraction { Vector3 wi; Wavelengths wavelengths; size_t n = 0; };
// Interaction3f fields sample/pdf_direction read: p and wavelengths.
struct Interaction { Vector3 p; Wavelengths wavelengths; size_t n = 0; };
// DirectionSample3f: d and pdf always; dist / p optional (nullptr = not produced).
struct DirectionSample { Vector3Out d; float* pdf = nullptr; float* dist = nullptr; Vector3Out p; };
struct DirectionSampleIn { Vector3 d; };
struct Ray { Vector3Out o, d; float* wavelengths = nullptr; size_t wl_stride = 0; };

struct BoundingBox3f {
    float min[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                    std::numeric_limits<float>::infinity()};
    float max[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                    -std::numeric_limits<float>::infinity()};
    bool valid() const { return min[0] <= max[0] && min[1] <= max[1] && min[2] <= max[2]; }
};

// ---------------------------------------------------------------- emitter
class SunskyEmitter {
public:
    // SunskyEmitter(const Properties&), sunsky.cpp:162-218; tables staged on the
    // host and uploaded to the current HIP device.
    SunskyEmitter(const Properties& props, Variant variant, Semantics semantics = Semantics::JIT,
                  const char* dataset_path = nullptr) {
        check(sunsky_emitter_create(props.get(), (int)variant, (int)semantics, dataset_path, &e_));
    }
    // Host-only staging (no device): tables, info and to_string, no batch calls.
    static SunskyEmitter host_only(const Properties& props, Variant variant, Semantics semantics = Semantics::JIT,
                                   const char* dataset_path = nullptr) {
        sunsky_emitter* e = nullptr;
        check(sunsky_emitter_create_host(props.get(), (int)variant, (int)semantics, dataset_path, &e));
        return SunskyEmitter(e);
    }
    ~SunskyEmitter() { if (e_) sunsky_emitter_destroy(e_); }
    SunskyEmitter(SunskyEmitter&& o) noexcept : e_(std::exchange(o.e_, nullptr)) {}
    SunskyEmitter& operator=(SunskyEmitter&& o) noexcept {
        if (this != &o) {
            if (e_) sunsky_emitter_destroy(e_);
            e_ = std::exchange(o.e_, nullptr);
        }
        return *this;
    }
    SunskyEmitter(const SunskyEmitter&) = delete;
    SunskyEmitter& operator=(const SunskyEmitter&) = delete;

    // ------------------------------------------------ Emitter interface
    // eval(si, active), sunsky.cpp:303-352
    void eval(const SurfaceInteraction& si, SpectrumOut out, const uint8_t* active = nullptr,
              void* stream = nullptr) const {
        check(sunsky_eval(e_, vin(si.wi), si.wavelengths.data, si.wavelengths.count, si.wavelengths.stride, active,
                          si.n, out.data, out.stride ? out.stride : si.n, stream));
    }
    // eval_direction(it, ds, active), sunsky.cpp:453-461
    void eval_direction(const Interaction& it, const DirectionSampleIn& ds, SpectrumOut out,
                        const uint8_t* active = nullptr, void* stream = nullptr) const {
        check(sunsky_eval_direction(e_, vin(ds.d), it.wavelengths.data, it.wavelengths.count, it.wavelengths.stride,
                                    active, it.n, out.data, out.stride ? out.stride : it.n, stream));
    }
    // sample_direction(it, sample, active) -> (ds, weight), sunsky.cpp:399-441
    void sample_direction(const Interaction& it, Point2 sample, DirectionSample ds, SpectrumOut weight,
                          const uint8_t* active = nullptr, void* stream = nullptr) const {
        check(sunsky_sample_direction(e_, sample.x, sample.y, vin(it.p), it.wavelengths.data, it.wavelengths.count,
                                      it.wavelengths.stride, active, it.n, vout(ds.d), ds.pdf, ds.dist, vout(ds.p),
                                      weight.data, weight.stride ? weight.stride : it.n, stream));
    }
    // pdf_direction(it, ds, active), sunsky.cpp:443-451
    void pdf_direction(size_t n, const DirectionSampleIn& ds, float* pdf, const uint8_t* active = nullptr,
                       void* stream = nullptr) const {
        check(sunsky_pdf_direction(e_, vin(ds.d), active, n, pdf, stream));
    }
    // sample_ray(time, wavelength_sample, sample2, sample3, active), sunsky.cpp:354-397
    void sample_ray(size_t n, const float* wavelength_sample, Point2 sample2, Point2 sample3, Ray ray,
                    SpectrumOut weight, const uint8_t* active = nullptr, void* stream = nullptr) const {
        check(sunsky_sample_ray(e_, wavelength_sample, sample2.x, sample2.y, sample3.x, sample3.y, active, n,
                                vout(ray.o), vout(ray.d), ray.wavelengths, ray.wl_stride ? ray.wl_stride : n,
                                weight.data, weight.stride ? weight.stride : n, stream));
    }
    // sample_wavelengths(si, sample, active), sunsky.cpp:463-480
    void sample_wavelengths(const SurfaceInteraction& si, const float* sample, float* wavelengths, size_t wl_stride,
                            SpectrumOut weight, const uint8_t* active = nullptr, void* stream = nullptr) const {
        check(sunsky_sample_wavelengths(e_, vin(si.wi), sample, active, si.n, wavelengths,
                                        wl_stride ? wl_stride : si.n, weight.data,
                                        weight.stride ? weight.stride : si.n, stream));
    }
    // sample_position, sunsky.cpp:483-495: not implemented in the reference either
    [[noreturn]] void sample_position() const {
        check(sunsky_sample_position(e_));
        throw NotImplementedError("sample_position");
    }
    // eval(si) and its forward-mode derivative along `tangent` of `param` (the
    // reference's dr::forward_from(param) + dr::grad(eval(si))); d_out mirrors out.
    void eval_jvp(const SurfaceInteraction& si, Param param, const std::vector<float>& tangent, SpectrumOut out,
                  SpectrumOut d_out, const uint8_t* active = nullptr, void* stream = nullptr) const {
        const size_t stride = out.stride ? out.stride : si.n;
        if ((d_out.stride ? d_out.stride : si.n) != stride)
            throw Error(SUNSKY_ERROR_INVALID_VALUE, "out and d_out must share one plane stride");
        check(sunsky_eval_jvp(e_, (int)param, tangent.data(), (int)tangent.size(), vin(si.wi), si.wavelengths.data,
                              si.wavelengths.count, si.wavelengths.stride, active, si.n, out.data, d_out.data, stride,
                              stream));
    }
    // Reverse mode: grad (device, SUNSKY_GRAD_COUNT floats) += sum(d_out * d eval(si) / d param);
    // layout SUNSKY_GRAD_TURBIDITY / _ALBEDO + c / _SUN_DIRECTION + k.
    void eval_vjp(const SurfaceInteraction& si, const float* d_out, size_t d_out_stride, float* grad,
                  const uint8_t* active = nullptr, void* stream = nullptr) const {
        check(sunsky_eval_vjp(e_, vin(si.wi), si.wavelengths.data, si.wavelengths.count, si.wavelengths.stride,
                              active, si.n, d_out, d_out_stride ? d_out_stride : si.n, grad, stream));
    }
    // Lat-long environment map of the sky (sunsky_bake_latlong): planes [c][height * width]
    void bake_latlong(int width, int height, float theta0, float theta1, float phi0, float phi1, SpectrumOut out,
                      const std::vector<float>& wavelengths = {}, void* stream = nullptr) const {
        const size_t n = (size_t)width * (size_t)height;
        check(sunsky_bake_latlong(e_, width, height, theta0, theta1, phi0, phi1,
                                  wavelengths.empty() ? nullptr : wavelengths.data(), (int)wavelengths.size(),
                                  out.data, out.stride ? out.stride : n, stream));
    }
    // Direct sun + sky light at diffuse points (sunsky_direct_diffuse): one vertex of
    // PathIntegrator::sample (path.cpp:176-250) with diffuse.cpp's BSDF, spp samples per point.
    // Spectral: wavelengths = the points' si.wavelengths (<= 4 planes).  visibility: NULL
    // (unoccluded) or the tracer's verdicts [spp][vis_stride] on direct_diffuse_rays' rays.
    void direct_diffuse(Vector3 normal, size_t n, uint32_t seed, uint32_t spp, SpectrumOut out,
                        const float* reflectance = nullptr, Wavelengths wavelengths = {},
                        void* stream = nullptr, const uint8_t* visibility = nullptr,
                        size_t vis_stride = 0) const {
        check(sunsky_direct_diffuse(e_, vin(normal), reflectance, wavelengths.data, wavelengths.count,
                                    wavelengths.stride ? wavelengths.stride : n, seed, spp, visibility,
                                    vis_stride ? vis_stride : n, n, out.data, out.stride ? out.stride : n,
                                    stream));
    }
    // The shadow and BSDF rays of direct_diffuse's samples (sunsky_direct_diffuse_rays):
    // planes [spp][ray_stride] per component, (0,0,0) where no ray is needed.
    void direct_diffuse_rays(Vector3 normal, size_t n, uint32_t seed, uint32_t spp, Vector3Out emitter_dir,
                             Vector3Out bsdf_dir, size_t ray_stride = 0, void* stream = nullptr) const {
        check(sunsky_direct_diffuse_rays(e_, vin(normal), seed, spp, n, vout(emitter_dir), vout(bsdf_dir),
                                         ray_stride ? ray_stride : n, stream));
    }
    // The same vertex at rough-conductor points (sunsky_direct_conductor): roughconductor.cpp with
    // a Beckmann / GGX distribution and visible-normal sampling (isotropic alpha, or alpha_u /
    // alpha_v through the _aniso forms).  wi: the points'
    // si.wi in world space; eta / k: complex IOR per RGB channel (spectral: the first).
    enum class Microfacet { Beckmann = SUNSKY_MICROFACET_BECKMANN, GGX = SUNSKY_MICROFACET_GGX };
    void direct_conductor(Vector3 normal, Vector3 wi, size_t n, Microfacet distribution, float alpha,
                          const float eta[3], const float k[3], uint32_t seed, uint32_t spp, SpectrumOut out,
                          Wavelengths wavelengths = {}, void* stream = nullptr, const uint8_t* visibility = nullptr,
                          size_t vis_stride = 0) const {
        check(sunsky_direct_conductor(e_, vin(normal), vin(wi), (int)distribution, alpha, eta, k, wavelengths.data,
                                      wavelengths.count, wavelengths.stride ? wavelengths.stride : n, seed, spp,
                                      visibility, vis_stride ? vis_stride : n, n, out.data,
                                      out.stride ? out.stride : n, stream));
    }
    void direct_conductor_aniso(Vector3 normal, Vector3 wi, size_t n, Microfacet distribution, float alpha_u,
                                float alpha_v, const float eta[3], const float k[3], uint32_t seed, uint32_t spp,
                                SpectrumOut out, Wavelengths wavelengths = {}, void* stream = nullptr,
                                const uint8_t* visibility = nullptr, size_t vis_stride = 0) const {
        check(sunsky_direct_conductor_aniso(e_, vin(normal), vin(wi), (int)distribution, alpha_u, alpha_v, eta, k,
                                            wavelengths.data, wavelengths.count,
                                            wavelengths.stride ? wavelengths.stride : n, seed, spp, visibility,
                                            vis_stride ? vis_stride : n, n, out.data, out.stride ? out.stride : n,
                                            stream));
    }
    // Its shadow and BSDF rays, and (bsdf_weight not null) the BSDF samples' weights F G1 per
    // channel at bsdf_weight[(c * spp + s) * ray_stride + i] (c < 3 RGB, c < 1 spectral).
    void direct_conductor_rays(Vector3 normal, Vector3 wi, size_t n, Microfacet distribution, float alpha,
                               uint32_t seed, uint32_t spp, Vector3Out emitter_dir, Vector3Out bsdf_dir,
                               float* bsdf_weight = nullptr, const float eta[3] = nullptr,
                               const float k[3] = nullptr, size_t ray_stride = 0, void* stream = nullptr) const {
        check(sunsky_direct_conductor_rays(e_, vin(normal), vin(wi), (int)distribution, alpha, eta, k, seed, spp, n,
                                           vout(emitter_dir), vout(bsdf_dir), bsdf_weight,
                                           ray_stride ? ray_stride : n, stream));
    }
    void direct_conductor_rays_aniso(Vector3 normal, Vector3 wi, size_t n, Microfacet distribution, float alpha_u,
                                     float alpha_v, uint32_t seed, uint32_t spp, Vector3Out emitter_dir,
                                     Vector3Out bsdf_dir, float* bsdf_weight = nullptr, const float eta[3] = nullptr,
                                     const float k[3] = nullptr, size_t ray_stride = 0,
                                     void* stream = nullptr) const {
        check(sunsky_direct_conductor_rays_aniso(e_, vin(normal), vin(wi), (int)distribution, alpha_u, alpha_v, eta, k,
                                                 seed, spp, n, vout(emitter_dir), vout(bsdf_dir), bsdf_weight,
                                                 ray_stride ? ray_stride : n, stream));
    }
    // Spectral eval of one wavelength list broadcast to every ray (test_sunsky.py:42-59 layout)
    void eval_spectral_broadcast(Vector3 wi, size_t n, const std::vector<float>& wavelengths, SpectrumOut out,
                                 const uint8_t* active = nullptr, void* stream = nullptr) const {
        check(sunsky_eval_spectral_broadcast(e_, vin(wi), wavelengths.data(), (int)wavelengths.size(), active, n,
                                             out.data, out.stride ? out.stride : n, stream));
    }

    // ------------------------------------------------ scene / parameters
    // bbox(), sunsky.cpp:498-500: an invalid box
    BoundingBox3f bbox() const {
        BoundingBox3f b;
        check(sunsky_emitter_bbox(e_, b.min, b.max));
        return b;
    }
    // set_scene(scene), sunsky.cpp:287-301: bounding sphere of the scene's bbox
    void set_scene(const BoundingBox3f& scene_bbox) {
        if (scene_bbox.valid()) {
            // ScalarBoundingBox3f::bounding_sphere in fp32 (bbox.h:343-346)
            float c[3], r2 = 0.f;
            for (int i = 0; i < 3; ++i) {
                c[i] = (scene_bbox.max[i] + scene_bbox.min[i]) * 0.5f;
                float h = c[i] - scene_bbox.max[i];
                r2 += h * h;
            }
            check(sunsky_emitter_set_scene(e_, 1, c, std::sqrt(r2)));
        } else {
            check(sunsky_emitter_set_scene(e_, 0, nullptr, 0.f));
        }
    }
    // traverse() + Parameters.update(): set one differentiable / updatable
    // parameter (sunsky.cpp:220-240), then restage (parameters_changed, :242-285).
    void set_parameter(const char* name, const std::vector<float>& values) {
        check(sunsky_emitter_set_param(e_, name, values.data(), (int)values.size()));
    }
    // Blocking restage on the default stream (state read back to the host).
    void parameters_changed() { check(sunsky_emitter_parameters_changed(e_)); }
    // Stream-ordered restage: the staging kernels run on `stream`; launches queued on it
    // afterwards see the new state (sunsky_emitter_parameters_changed_async).
    void parameters_changed(void* stream) { check(sunsky_emitter_parameters_changed_async(e_, stream)); }
    // Current value of a traverse() parameter (sunsky_emitter_get_param).
    std::vector<float> parameter(const char* name) const {
        float buf[16];
        int n = 0;
        check(sunsky_emitter_get_param(e_, name, buf, 16, &n));
        return std::vector<float>(buf, buf + n);
    }
    void set_precision(Precision p) { check(sunsky_emitter_set_precision(e_, (int)p)); }

    sunsky_info info() const {
        sunsky_info i;
        check(sunsky_emitter_get_info(e_, &i));
        return i;
    }
    uint32_t flags() const { return info().flags; }
    bool is_environment() const { return (flags() & SUNSKY_FLAG_INFINITE) != 0; }
    std::vector<float> table(sunsky_table_id id) const {
        size_t count = 0;
        check(sunsky_emitter_get_table(e_, (int)id, nullptr, 0, &count));
        std::vector<float> v(count);
        check(sunsky_emitter_get_table(e_, (int)id, v.data(), v.size(), &count));
        return v;
    }
    std::string to_string() const {
        std::vector<char> buf(8192);
        check(sunsky_emitter_to_string(e_, buf.data(), buf.size()));
        return std::string(buf.data());
    }
    const sunsky_emitter* handle() const { return e_; }

private:
    explicit SunskyEmitter(sunsky_emitter* e) : e_(e) {}
    static sunsky_vec3_in vin(const Vector3& v) { return sunsky_vec3_in{v.x, v.y, v.z}; }
    static sunsky_vec3_out vout(const Vector3Out& v) { return sunsky_vec3_out{v.x, v.y, v.z}; }
    sunsky_emitter* e_ = nullptr;
};

// mi.hosek_sun_rad (sunsky_v.cpp:19): Hosek-Wilkie solar radiance, fp64; dataset nullptr = bundled pack
inline double hosek_sun_rad(double turbidity, double wavelength, double elevation, double gamma,
                            const char* dataset = nullptr) {
    double out = 0.0;
    check(sunsky_hosek_sun_rad(dataset, turbidity, wavelength, elevation, gamma, &out));
    return out;
}

}  // namespace sunsky_amd
