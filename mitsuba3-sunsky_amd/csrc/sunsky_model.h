// sunsky_model.h -- host-side state and table staging of the sun/sky
// emitter: the constructor / parameters_changed() work of the reference
// (sunsky.cpp:162-301, 772-978; sunsky.h:158-501).  Produces a SunskyKArgs
// block plus the two small device tables; owns no device memory itself.
#pragma once
#include <array>
#include <string>
#include <vector>

#include "sunsky_dataset.h"
#include "sunsky_props.h"
#include "sunsky_staging.h"
#include "sunsky_types.h"

namespace sunsky {

struct DateTime { int year = 2010, month = 7, day = 10; float hour = 15.f, minute = 0.f, second = 0.f; };
struct Location { float latitude = 35.6894f, longitude = 139.6917f, timezone = 9.f; };

// compute_sun_coordinates, sunsky.h:284-374 (fp32, Int32 Julian-day arithmetic)
void compute_sun_coordinates(const DateTime& t, const Location& l, float out[3]);
// quad::gauss_legendre, quad.h:27-86 (fp64 nodes/weights)
void gauss_legendre(int n, std::vector<double>* nodes, std::vector<double>* weights);

// Forward-mode tangent of the staged eval tables with respect to one
// differentiable parameter of traverse() (sunsky.cpp:220-240): what Dr.Jit's
// dr::forward_from(param) propagates into the staging before eval runs.
enum JvpParam { kJvpTurbidity = 0, kJvpAlbedo = 1, kJvpSunDirection = 2 };
struct EvalTangent {
    std::vector<float> dsky;   // nch x 10: d{A, B, C, D, E, F, G, H, I, rad} per channel
    std::vector<float> dsun;   // d sun radiance table (turbidity), else all zero
    float dsun_local[3] = {0, 0, 0};   // d local sun direction (sun_direction)
};

// SunskyKArgs::sun_seg_z: [j] = the smallest fp32 cos theta in [0, 1] whose render_sun
// elevation segment (sunsky.cpp:579-584, fp32: min(floor(cbrt(2 (pi/2 - acos z) / pi) 45), 44))
// is >= j ([0] = 0); committed constants (sunsky_model.cpp).
const std::array<float, kNbSunSegments>& sun_segment_thresholds();

class SunskyModel {
public:
    // SunskyEmitter(const Properties&), sunsky.cpp:162-218.  Throws std::invalid_argument /
    // std::runtime_error with the reference's messages.  radiance_on_host = false leaves the
    // radiance tables and the JIT quadrature to the device staging kernels (GPU emitters).
    SunskyModel(const Properties& props, int variant, int semantics, const std::string& dataset_dir_or_pack,
                bool radiance_on_host = true);

    // traverse() parameters (sunsky.cpp:220-240): turbidity, sky_scale, sun_scale,
    // albedo (1 or nch values), latitude, longitude, timezone, year, day, month,
    // hour, minute, second, sun_direction (3), to_world (16, row-major).
    void set_param(const std::string& name, const float* v, int count);
    // parameters_changed, sunsky.cpp:242-285.  A rejected update (validation or staging
    // error) restores the last committed state before rethrowing.
    void parameters_changed(bool radiance_on_host = true);
    // Current value of a traverse() parameter (set_param's names) -> count values.
    int get_param(const std::string& name, float* out, int cap) const;
    // set_scene, sunsky.cpp:287-301
    void set_scene(bool bbox_valid, const float center[3], float radius);

    const SunskyKArgs& kargs() const { return k_; }
    const std::vector<float>& sun_table() const { return sun_table_; }
    const std::vector<float>& sun_ld() const { return sun_ld_; }
    int variant() const { return variant_; }
    int nch() const { return nch_; }
    bool active_record() const { return active_record_; }
    const float* sun_dir_world() const { return sun_dir_; }
    float turbidity() const { return turbidity_; }
    const std::vector<float>& albedo() const { return albedo_; }
    const std::vector<float>& sky_params() const { return sky_params_; }
    const std::vector<float>& sky_radiance() const { return sky_rad_; }
    const float* gaussians_raw() const { return gauss_raw_; }
    std::string to_string() const;
    // device staging: the libm scalars of compute_radiance_params for the current state,
    // the raw datasets the staging kernels read, the quadrature nodes, and the adoption of
    // the device-staged fields (sky channels, sun table, w_sky, wavelength distribution)
    RadianceStage radiance_stage() const;
    const std::vector<float>& sky_params_ds() const { return sky_params_ds_; }
    const std::vector<float>& sky_rad_ds() const { return sky_rad_ds_; }
    const std::vector<float>& sun_rad_ds() const { return sun_rad_ds_; }
    const float* cie_y() const { return cie_y_; }
    float sky_scale() const { return sky_scale_; }
    float sun_scale() const { return sun_scale_; }
    int semantics() const { return semantics_; }
    bool radiance_stale() const { return radiance_stale_; }
    void adopt_device_stage(const SunskyKArgs& device_kargs, const float* sun_table);
    // The device staging rejected the last committed update: make the commit before it the
    // committed state again and restore it (the caller restages the device).
    // The device staging's verdict, known only at a read-back: mark_accepted records the
    // committed state as accepted; revert_to_accepted restores the last such state.
    void mark_accepted() { accepted_ = committed_; has_accepted_ = true; }
    bool has_accepted() const { return has_accepted_; }
    void revert_to_accepted();
    // Drop parameter values set since the last commit (an update refused before staging).
    void discard_pending() { rollback(); }
    static void quadrature_nodes(std::vector<float>* x, std::vector<float>* w);
    // Tangent of the eval tables for param (JvpParam) along `tangent`
    // (turbidity: 1 value; albedo: 1 or nch; sun_direction: 3, world space).
    EvalTangent eval_tangent(int param, const float* tangent, int count) const;
    // The scalars of that tangent (validates param / count), for the device tangent staging
    TangentStage tangent_stage(int param, const float* tangent, int count) const;
    std::vector<std::string> warnings;

private:
    void load_datasets(const std::string& where);
    void extract_albedo(const Properties& props);
    void update_angles(const float local_sun[3]);
    void stage(bool radiance_on_host);   // geometry (+ radiance + sampling weight)
    void stage_geometry();               // scales, aperture, TGMM, discrete distribution
    void stage_radiance();               // sky channels + sun table (host-only emitters)
    int gauss_search(float s) const;
    void build_gauss_guide();
    void stage_sun_sky_fit();            // SunskyKArgs::sun_sky_fit (the FAST samplers' sun-pick sky pdf)
    void estimate_sky_sun_ratio();
    void validate() const;

    int variant_, semantics_, nch_;
    // datasets (fp64 on disk -> fp32, array_from_file<Float64, Float>)
    std::vector<float> sky_params_ds_, sky_rad_ds_, sun_rad_ds_, sun_ld_, tgmm_tables_;
    float cie_y_[kNbWavelengths] = {0};
    // parameters
    float turbidity_ = 3.f, sky_scale_ = 1.f, sun_scale_ = 1.f, sun_half_aperture_ = 0.f, sun_aperture_deg_ = 0.5358f;
    std::vector<float> albedo_;
    bool active_record_ = true;
    DateTime time_;
    Location location_;
    float sun_dir_[3] = {0, 0, 1};   // world space (m_sun_dir)
    float to_world_[16];
    double to_world_d_[9], to_local_d_[9];
    // staged
    std::vector<float> sky_params_, sky_rad_, sun_table_;
    float gauss_raw_[kNbMixture * kNbGaussianParams];
    SunskyKArgs k_;
    bool radiance_stale_ = false;   // sky channels / sun table / w_sky live on the device only
    // last committed state (rollback of a rejected parameters_changed)
    struct Snapshot {
        float turbidity, sky_scale, sun_scale;
        std::vector<float> albedo;
        DateTime time;
        Location location;
        float sun_dir[3], to_world[16];
        double to_world_d[9], to_local_d[9];
        std::vector<float> sky_params, sky_rad, sun_table;
        float gauss_raw[kNbMixture * kNbGaussianParams];
        SunskyKArgs k;
        bool radiance_stale;
    };
    Snapshot committed_, accepted_;
    bool has_accepted_ = false;
    void commit();
    void rollback();
};

}  // namespace sunsky
