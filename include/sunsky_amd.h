/*
 * sunsky_amd.h -- C ABI of the MI355X-native sun/sky emitter.
 *
 * Drop-in replacement for the `sunsky` emitter plugin of
 * matttsss/mitsuba3-sunsky (src/emitters/sunsky.cpp).  Each entry point names
 * the reference interface it replaces (file:line under the reference tree).
 * Conventions:
 *   - every function returns an int status (SUNSKY_OK = 0); on failure the
 *     thread-local message from sunsky_last_error() carries the reference's
 *     error text (the reference throws through Log(Error, ...), logger.cpp:55-60);
 *     nothing throws across this boundary;
 *   - batch inputs/outputs are DEVICE pointers (HBM), structure-of-arrays,
 *     one fp32 plane per component -- the layout Dr.Jit gives the JIT variants;
 *     multi-channel outputs are planes at `out + c * out_stride`;
 *   - `active` is an optional per-ray uint8 mask (NULL = all active), the
 *     `Mask active` argument of the reference methods;
 *   - `stream` is a hipStream_t (NULL = default stream); every batch call is
 *     asynchronous and stream-ordered.  The hot-path calls (eval,
 *     eval_direction, eval_spectral_broadcast, sample_direction, pdf_direction,
 *     sample_ray, sample_wavelengths, direct_diffuse, direct_diffuse_rays)
 *     allocate nothing, make no host-synchronous call and may be captured into
 *     a hipGraph (tests/test_graph_capture.py).  Kernels read the emitter state
 *     from device memory, which parameters_changed_async rewrites in place on
 *     the caller's stream, so a captured graph replays with the state current at
 *     replay.  eval_jvp and eval_vjp restage their tangent tables (host fp64
 *     derivative of the staging, stream-ordered copy from pinned memory) when
 *     the emitter state (or, for eval_jvp, the tangent) changed since the
 *     previous call; they and bake_latlong order successive calls on the same
 *     emitter through events and are not capturable;
 *   - every batch entry point opens a roctx range "<ProfilerPhase>:<entry>"
 *     (the reference's MI_MASKED_FUNCTION scopes; SUNSKY_AMD_ROCTX=0 disables);
 *   - create/update/destroy are host-synchronous and must not race batch calls
 *     on the same emitter (the reference's parameters_changed() contract).
 */
#ifndef SUNSKY_AMD_H
#define SUNSKY_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SUNSKY_AMD_ABI_VERSION 7   /* 3: direct_diffuse visibility, direct_diffuse_rays; 4: direct_conductor(_rays),
                                     emitter_tangent_tables, direct_diffuse draws sample_1 (path.cpp:233);
                                     5: direct_conductor(_rays)_aniso (alpha_u, alpha_v);
                                     6: SUNSKY_TABLE_SUN_SKY_FIT, emitter_inject_staging_fault (testing),
                                        a rejected update reverts to the last accepted one;
                                     7: SUNSKY_TABLE_SUN_SEGMENTS, emitter_sun_segments (testing) */

typedef enum sunsky_status {
    SUNSKY_OK = 0,
    SUNSKY_ERROR_INVALID_VALUE = 1,   /* bad parameter (reference: Log(Error, ...))      */
    SUNSKY_ERROR_FILE = 2,            /* dataset missing / unreadable (sunsky.h:519-520) */
    SUNSKY_ERROR_FORMAT = 3,          /* dataset header / size mismatch (sunsky.h:531)   */
    SUNSKY_ERROR_HIP = 4,             /* HIP runtime / code object failure               */
    SUNSKY_ERROR_NOT_IMPLEMENTED = 5, /* sample_position (sunsky.cpp:483-495)            */
    SUNSKY_ERROR_INTERNAL = 6,
    SUNSKY_ERROR_COMM = 7             /* RCCL unavailable / communicator failure         */
} sunsky_status;

typedef enum sunsky_variant {     /* mitsuba.conf variants: *_rgb / *_spectral */
    SUNSKY_VARIANT_RGB = 0,
    SUNSKY_VARIANT_SPECTRAL = 1
} sunsky_variant;

typedef enum sunsky_semantics {
    SUNSKY_SEMANTICS_JIT = 0,     /* llvm_* / cuda_*: quadrature sky/sun ratio (sunsky.cpp:784-885) */
    SUNSKY_SEMANTICS_SCALAR = 1   /* scalar_*: ratio 0.5, uniform wavelength pdf (:778-783)         */
} sunsky_semantics;

typedef enum sunsky_precision {
    SUNSKY_PRECISION_FAST = 0,      /* host-folded transcendental constants (default) */
    SUNSKY_PRECISION_REFERENCE = 1  /* reference operation order, full-precision libm */
} sunsky_precision;

typedef enum sunsky_table_id {      /* staged tables, for inspection / parity tests */
    SUNSKY_TABLE_SKY_PARAMS = 0,    /* nch x 9  (m_sky_params)            */
    SUNSKY_TABLE_SKY_RADIANCE = 1,  /* nch      (m_sky_radiance)          */
    SUNSKY_TABLE_SUN_RADIANCE = 2,  /* 45x3x4x6 or 45x11x4 (m_sun_radiance) */
    SUNSKY_TABLE_SUN_LD = 3,        /* 11 x 6   (m_sun_ld)                 */
    SUNSKY_TABLE_GAUSSIANS = 4,     /* 20 x 5   (m_gaussians)              */
    SUNSKY_TABLE_GAUSSIAN_CDF = 5,  /* 20       (DiscreteDistribution cdf) */
    SUNSKY_TABLE_SPECTRAL_PDF = 6,  /* m_spectral_distr pdf                */
    SUNSKY_TABLE_SPECTRAL_CDF = 7,  /* m_spectral_distr cdf                */
    SUNSKY_TABLE_ALBEDO = 8,        /* extract_albedo() result             */
    SUNSKY_TABLE_SUN_SKY_FIT = 9,   /* 10: the FAST samplers' sun-pick sky pdf fit: c0..c5, bound,
                                       smallest value, usable (0/1), in use for this w_sky (0/1) */
    SUNSKY_TABLE_SUN_SEGMENTS = 10  /* 47: render_sun's segment decision (sunsky.cpp:579-584) as cos theta
                                       thresholds z[0..44] (z[j] = smallest fp32 cos theta whose segment
                                       is >= j), then the disc's first and last segment */
} sunsky_table_id;

#define SUNSKY_FLAG_INFINITE 0x04u          /* EmitterFlags::Infinite (emitter.h:29-30) */
#define SUNSKY_FLAG_SPATIALLY_VARYING 0x10u /* EmitterFlags::SpatiallyVarying (emitter.h:39-40) */

typedef struct sunsky_props sunsky_props;
typedef struct sunsky_emitter sunsky_emitter;

typedef struct sunsky_vec3_in { const float *x, *y, *z; } sunsky_vec3_in;
typedef struct sunsky_vec3_out { float *x, *y, *z; } sunsky_vec3_out;

typedef struct sunsky_info {
    int variant, semantics, nb_channels, active_record;
    float turbidity, sky_scale, sun_scale;
    float sun_half_aperture, cos_cutoff, area_ratio;
    float sun_dir_world[3];       /* m_sun_dir                 */
    float sun_dir_local[3];       /* m_local_sun_frame.n       */
    float sun_angles[2];          /* m_sun_angles (phi, theta) */
    float sky_sampling_w;         /* m_sky_sampling_w          */
    float bsphere_center[3], bsphere_radius;
    unsigned flags;               /* SUNSKY_FLAG_*             */
    int device;                   /* HIP device owning the tables */
    int precision;                /* sunsky_precision          */
} sunsky_info;

/* ------------------------------------------------------------ library */
int sunsky_abi_version(void);
const char *sunsky_last_error(void);

/* --------------------------------------------------- property bag
 * mitsuba::Properties as consumed by init_from_props (sunsky.cpp:889-948):
 * "turbidity", "sky_scale", "sun_scale", "sun_aperture" (deg), "albedo"
 * (float / per-channel spectrum / irregular spectrum), "sun_direction" (vector)
 * XOR {"latitude","longitude","timezone","year","month","day","hour",
 * "minute","second"}, "to_world" (4x4 row-major).  Unqueried names are an
 * error at create time, like the XML/dict loader (src/core/xml.cpp:1085-1102). */
int sunsky_props_create(sunsky_props **out);
void sunsky_props_destroy(sunsky_props *p);
int sunsky_props_set_float(sunsky_props *p, const char *name, double value);
int sunsky_props_set_int(sunsky_props *p, const char *name, int64_t value);
int sunsky_props_set_vector3(sunsky_props *p, const char *name, float x, float y, float z);
int sunsky_props_set_transform(sunsky_props *p, const char *name, const float matrix_row_major[16]);
int sunsky_props_set_spectrum(sunsky_props *p, const char *name, const float *values, int count);
int sunsky_props_set_irregular_spectrum(sunsky_props *p, const char *name, const float *wavelengths,
                                        const float *values, int count);

/* ------------------------------------------------------------ emitter
 * SunskyEmitter(const Properties&) -- sunsky.cpp:162-218.  The emitter lives on the
 * CURRENT HIP device: its state (one SunskyKArgs block + tables) is allocated there,
 * the radiance tables and the JIT sampling quadrature are staged there by kernels,
 * and every later call on the emitter runs on that device whatever device is current.  dataset_path: NULL for the
 * bundled pack, a .pack file, or a directory holding the reference's
 * resources/sunsky/datasets/<table>.bin files (path_to_dataset, sunsky.h:124-141). */
int sunsky_emitter_create(const sunsky_props *props, int variant, int semantics,
                          const char *dataset_path, sunsky_emitter **out);
/* Same staging without a device: batch calls on it fail; for inspecting the
 * staged tables (get_info / get_table / to_string) on machines without a GPU. */
int sunsky_emitter_create_host(const sunsky_props *props, int variant, int semantics,
                               const char *dataset_path, sunsky_emitter **out);
void sunsky_emitter_destroy(sunsky_emitter *e);
/* traverse() parameters, sunsky.cpp:220-240 (name, 1/3/11/16 floats).  Values take
 * effect at the next parameters_changed; a rejected update (e.g. turbidity 12) restores
 * the last committed values. */
int sunsky_emitter_set_param(sunsky_emitter *e, const char *name, const float *values, int count);
/* Current value of a traverse() parameter: *count values written to out (<= capacity). */
int sunsky_emitter_get_param(const sunsky_emitter *e, const char *name, float *out, int capacity,
                             int *count);
/* parameters_changed(), sunsky.cpp:242-285, stream-ordered: validation and the cheap
 * geometry / TGMM staging run on the host; the radiance tables (sunsky.h:158-231,
 * 404-419) and the JIT quadrature (estimate_sky_sun_ratio, sunsky.cpp:772-886) run as
 * kernels on `stream`, writing the emitter's device state in place.  Batch calls on
 * `stream` after this one see the new state; the call does not wait for the device.
 * Work on other streams must be ordered by the caller (the reference's contract:
 * parameters_changed is not concurrent with rendering).  Not capturable: called on a
 * stream that is capturing a hipGraph it returns SUNSKY_ERROR_INVALID_VALUE and changes
 * nothing (update outside the capture; captured batch calls read the current state).
 * An update the device staging rejects (a negative wavelength-distribution node, as
 * ContinuousDistribution's constructor checks) is reported by the next call that reads
 * the state back (get_info / get_table / the blocking form), which restores and restages
 * the parameters of the last staging known to be accepted (every update queued since that
 * read-back is rolled back: the rejection status is sticky across stagings, so one
 * rejected update among several queued ones is never lost). */
int sunsky_emitter_parameters_changed_async(sunsky_emitter *e, void *stream);
/* TESTING ONLY (tests/test_graph_capture.py): the next `count` device stagings of `e`
 * report a rejected wavelength distribution, so the rollback path above can be exercised
 * without a parameter set that produces one.  0 turns it off. */
int sunsky_emitter_inject_staging_fault(sunsky_emitter *e, int count);
/* TESTING ONLY (tests/test_gpu_parity.py): pos[i] = the elevation segment render_sun
 * (sunsky.cpp:579-584) takes for a direction inside the sun disc whose cos theta is
 * cos_theta[i], decided by the code the emitter's eval and sampling kernels run (its
 * precision).  Device int32 output; defined for the cos theta of disc directions. */
int sunsky_emitter_sun_segments(const sunsky_emitter *e, const float *cos_theta, size_t n, int *pos, void *stream);
/* Blocking form: _async on the default (null) stream, then waits for the staging. */
int sunsky_emitter_parameters_changed(sunsky_emitter *e);
/* set_scene(), sunsky.cpp:287-301: bounding sphere of the scene bbox */
int sunsky_emitter_set_scene(sunsky_emitter *e, int bbox_valid, const float center[3], float radius);
int sunsky_emitter_set_precision(sunsky_emitter *e, int precision);
int sunsky_emitter_get_info(const sunsky_emitter *e, sunsky_info *out);
int sunsky_emitter_get_table(const sunsky_emitter *e, int table_id, float *out, size_t capacity,
                             size_t *count);
/* to_string(), sunsky.cpp:502-519 */
int sunsky_emitter_to_string(const sunsky_emitter *e, char *buf, size_t capacity);
/* bbox(), sunsky.cpp:498-500: always an invalid box (min=+inf, max=-inf) */
int sunsky_emitter_bbox(const sunsky_emitter *e, float out_min[3], float out_max[3]);

/* ------------------------------------------------------ batched hot path */
/* eval(si, active), sunsky.cpp:303-352.  wi = si.wi.
 * RGB: out = 3 planes.  Spectral: wavelengths = n_wavelengths planes (per-ray
 * si.wavelengths, Mitsuba uses 4) at `wavelengths + k * wl_stride`; out likewise. */
int sunsky_eval(const sunsky_emitter *e, sunsky_vec3_in wi, const float *wavelengths,
                int n_wavelengths, size_t wl_stride, const uint8_t *active, size_t n,
                float *out, size_t out_stride, void *stream);
/* eval_direction(it, ds, active), sunsky.cpp:453-461: eval with wi = -ds.d */
int sunsky_eval_direction(const sunsky_emitter *e, sunsky_vec3_in d, const float *wavelengths,
                          int n_wavelengths, size_t wl_stride, const uint8_t *active, size_t n,
                          float *out, size_t out_stride, void *stream);
/* Spectral eval of ONE host-side wavelength list broadcast to every ray (the
 * eval_full_spec layout of test_sunsky.py:42-59): out plane k = lambda[k]. */
int sunsky_eval_spectral_broadcast(const sunsky_emitter *e, sunsky_vec3_in wi,
                                   const float *wavelengths_host, int n_wavelengths,
                                   const uint8_t *active, size_t n, float *out,
                                   size_t out_stride, void *stream);
/* sample_direction(it, sample, active), sunsky.cpp:399-441.
 * it_p: interaction positions (x == NULL -> origin).  Outputs ds.d (required),
 * ds.pdf (required), ds.dist / ds.p (optional, NULL to skip); weight planes:
 * 3 (RGB) or n_wavelengths (spectral, wavelengths = it.wavelengths). */
int sunsky_sample_direction(const sunsky_emitter *e, const float *sample_x, const float *sample_y,
                            sunsky_vec3_in it_p, const float *wavelengths, int n_wavelengths,
                            size_t wl_stride, const uint8_t *active, size_t n, sunsky_vec3_out ds_d,
                            float *ds_pdf, float *ds_dist, sunsky_vec3_out ds_p, float *weight,
                            size_t weight_stride, void *stream);
/* pdf_direction(it, ds, active), sunsky.cpp:443-451 */
int sunsky_pdf_direction(const sunsky_emitter *e, sunsky_vec3_in ds_d, const uint8_t *active,
                         size_t n, float *pdf, void *stream);
/* sample_ray(time, wavelength_sample, sample2, sample3, active), sunsky.cpp:354-397.
 * Outputs ray.o, ray.d, ray.wavelengths (4 planes; zeros in RGB) and weight
 * (3 planes RGB / 4 spectral). */
int sunsky_sample_ray(const sunsky_emitter *e, const float *wavelength_sample, const float *sample2_x,
                      const float *sample2_y, const float *sample3_x, const float *sample3_y,
                      const uint8_t *active, size_t n, sunsky_vec3_out ray_o, sunsky_vec3_out ray_d,
                      float *ray_wavelengths, size_t wl_stride, float *weight, size_t weight_stride,
                      void *stream);
/* sample_wavelengths(si, sample, active), sunsky.cpp:463-480 (wi = si.wi).
 * Outputs 4 wavelength planes and 4 (spectral) / 3 (RGB) weight planes. */
int sunsky_sample_wavelengths(const sunsky_emitter *e, sunsky_vec3_in wi, const float *sample,
                              const uint8_t *active, size_t n, float *wavelengths, size_t wl_stride,
                              float *weight, size_t weight_stride, void *stream);
/* sample_position(), sunsky.cpp:483-495: NotImplementedError in the reference */
int sunsky_sample_position(const sunsky_emitter *e);

/* Lat-long bake of the sky (a caller of eval, as sunsky-testing/sky_data_test.py:58-79
 * builds an environment map from eval over helpers.py get_spherical_rays): pixel (x, y)
 * of a width x height image holds eval(si.wi = -sphdir(theta_y, phi_x)) with
 * theta_y = linspace(theta0, theta1, height)[y], phi_x = linspace(phi0, phi1, width)[x]
 * (z-up, local frame of to_world applied).  Planes [c][height * width], row-major:
 * 3 RGB planes, or one per host wavelength (spectral).  Directions are generated on the
 * device: the bake only writes HBM. */
int sunsky_bake_latlong(const sunsky_emitter *e, int width, int height, float theta0, float theta1,
                        float phi0, float phi1, const float *wavelengths_host, int n_wavelengths,
                        float *out, size_t out_stride, void *stream);

/* A caller of sample_direction / pdf_direction / eval: the sun-and-sky light a
 * smooth-diffuse point receives, gathered as the path integrator does at one vertex
 * (src/integrators/path.cpp:176-250; src/bsdfs/diffuse.cpp:100-180): emitter
 * sampling + cosine-hemisphere BSDF sampling combined with the power heuristic, spp
 * samples per point from PCG32Sampler-seeded streams (src/render/sampler.cpp:125-144:
 * sample_tea_32(seed, point index)), each sample drawing next_2d (emitter), next_1d
 * (sample_1, unused by this BSDF) and next_2d (BSDF) as path.cpp:216-234 does.
 * normal: unit world-space normals; reflectance: gray per point (NULL = 1).
 * out planes: 3 (RGB) or n_wavelengths <= 4 (spectral, per-point wavelengths).
 * visibility: NULL for unoccluded points, else one byte per (sample s, point i) at
 * visibility[s * vis_stride + i] with the caller's tracer verdicts on the rays
 * sunsky_direct_diffuse_rays wrote for the same (seed, spp, normal): bit 0 = the
 * shadow ray along the emitter sample is unoccluded (path.cpp:216-219 ray_test),
 * bit 1 = the BSDF ray escapes to the environment (path.cpp:176-196).
 * n < 2^32. */
int sunsky_direct_diffuse(const sunsky_emitter *e, sunsky_vec3_in normal, const float *reflectance,
                          const float *wavelengths, int n_wavelengths, size_t wl_stride, uint32_t seed,
                          uint32_t spp, const uint8_t *visibility, size_t vis_stride, size_t n, float *out,
                          size_t out_stride, void *stream);
/* The rays a wavefront caller traces between the two halves of sunsky_direct_diffuse
 * (the shadow ray of the emitter sample, path.cpp:216-219, and the BSDF ray,
 * path.cpp:176-196), from the same streams and arithmetic as that call: for sample s
 * of point i, emitter_dir[s * ray_stride + i] is the world direction of the emitter
 * sample ((0,0,0) when the sample contributes nothing: pdf 0 or below the point's
 * horizon) and bsdf_dir[s * ray_stride + i] the cosine-sampled world direction
 * ((0,0,0) when its pdf is 0).  ray_stride >= n; n < 2^32. */
int sunsky_direct_diffuse_rays(const sunsky_emitter *e, sunsky_vec3_in normal, uint32_t seed, uint32_t spp,
                               size_t n, sunsky_vec3_out emitter_dir, sunsky_vec3_out bsdf_dir,
                               size_t ray_stride, void *stream);

/* A caller with a glossy vertex: the light a rough conductor (src/bsdfs/roughconductor.cpp,
 * Beckmann or GGX, visible-normal sampling, include/mitsuba/render/microfacet.h)
 * reflects towards wi, gathered as path.cpp:176-250 does at one vertex: per sample the
 * emitter sample (next_2d) weighted by f cos / pdf and the power heuristic, sample_1
 * (next_1d, unused by this BSDF), then the BSDF sample (next_2d): reflected direction,
 * weight F G1(wo), its escaped ray through eval() and pdf_direction().
 * normal, wi: unit world vectors (wi towards the viewer, si.wi in world space).
 * eta, k: complex IOR per RGB channel (3 values); spectral emitters use eta[0], k[0]
 * for every wavelength.  alpha: roughness (clamped to 1e-4 as the reference).
 * visibility: as sunsky_direct_diffuse, for the rays of sunsky_direct_conductor_rays. */
#define SUNSKY_MICROFACET_BECKMANN 0
#define SUNSKY_MICROFACET_GGX 1
int sunsky_direct_conductor(const sunsky_emitter *e, sunsky_vec3_in normal, sunsky_vec3_in wi, int distribution,
                            float alpha, const float *eta, const float *k, const float *wavelengths,
                            int n_wavelengths, size_t wl_stride, uint32_t seed, uint32_t spp,
                            const uint8_t *visibility, size_t vis_stride, size_t n, float *out,
                            size_t out_stride, void *stream);
/* The shadow rays and BSDF rays of sunsky_direct_conductor's samples (same streams and
 * arithmetic): (0,0,0) where the emitter sample contributes nothing (pdf 0 or f cos = 0)
 * or the BSDF sample is invalid.  bsdf_weight (NULL to skip; then eta / k may be NULL):
 * the BSDF sample's weight F(wi.m) G1(wo, m) (roughconductor.cpp sample(), the path
 * throughput factor of a multi-bounce caller) at bsdf_weight[(c * spp + s) * ray_stride + i]
 * for c < 3 (RGB) or c < 1 (spectral: eta[0], k[0]), 0 where the sample is invalid.
 * ray_stride >= n; n < 2^32. */
int sunsky_direct_conductor_rays(const sunsky_emitter *e, sunsky_vec3_in normal, sunsky_vec3_in wi,
                                 int distribution, float alpha, const float *eta, const float *k, uint32_t seed,
                                 uint32_t spp, size_t n, sunsky_vec3_out emitter_dir, sunsky_vec3_out bsdf_dir,
                                 float *bsdf_weight, size_t ray_stride, void *stream);
/* The same two calls with an anisotropic distribution: roughconductor's alpha_u / alpha_v
 * (microfacet.h:92-95, eval :186-207, smith_g1 :330-354, the visible-normal stretch
 * :301-316), alpha_u along the shading frame's first tangent (coordinate_system(normal),
 * include/mitsuba/core/vector.h:116-137) and alpha_v along the second; each clamped to
 * 1e-4.  alpha_u == alpha_v gives the isotropic calls' results bit for bit. */
int sunsky_direct_conductor_aniso(const sunsky_emitter *e, sunsky_vec3_in normal, sunsky_vec3_in wi,
                                  int distribution, float alpha_u, float alpha_v, const float *eta, const float *k,
                                  const float *wavelengths, int n_wavelengths, size_t wl_stride, uint32_t seed,
                                  uint32_t spp, const uint8_t *visibility, size_t vis_stride, size_t n, float *out,
                                  size_t out_stride, void *stream);
int sunsky_direct_conductor_rays_aniso(const sunsky_emitter *e, sunsky_vec3_in normal, sunsky_vec3_in wi,
                                       int distribution, float alpha_u, float alpha_v, const float *eta,
                                       const float *k, uint32_t seed, uint32_t spp, size_t n,
                                       sunsky_vec3_out emitter_dir, sunsky_vec3_out bsdf_dir, float *bsdf_weight,
                                       size_t ray_stride, void *stream);

/* ------------------------------------------------ forward-mode derivatives */
typedef enum sunsky_param {         /* Differentiable traverse() parameters, sunsky.cpp:220-240 */
    SUNSKY_PARAM_TURBIDITY = 0,     /* tangent: 1 value                               */
    SUNSKY_PARAM_ALBEDO = 1,        /* tangent: 1 value or one per channel (3 / 11)   */
    SUNSKY_PARAM_SUN_DIRECTION = 2  /* tangent: 3 values, world space (m_sun_dir)     */
} sunsky_param;
/* eval(si) and its forward-mode derivative along `tangent` of `param`: what
 * dr::enable_grad(param); dr::set_grad(param, tangent); dr::forward_from(param);
 * dr::grad(eval(si)) computes in the reference's AD variants (exercised by
 * sunsky-testing/traversal_test.py:94-145).  Layout as sunsky_eval; d_out has the
 * planes of out.  The tangent of the staged tables is staged by a device kernel
 * (fp64, stream-ordered on `stream`) when the emitter or the tangent changed, then the
 * rays are processed on `stream`. */
int sunsky_eval_jvp(const sunsky_emitter *e, int param, const float *tangent, int tangent_count,
                    sunsky_vec3_in wi, const float *wavelengths, int n_wavelengths, size_t wl_stride,
                    const uint8_t *active, size_t n, float *out, float *d_out, size_t out_stride,
                    void *stream);
/* Reverse mode: grad[p] += sum over rays and output planes of d_out * d eval / d p,
 * i.e. the parameter gradients dr.backward(dr.sum(d_out * eval(si))) accumulates in the
 * reference.  `grad` is a DEVICE array of SUNSKY_GRAD_COUNT floats:
 *   [SUNSKY_GRAD_TURBIDITY]          turbidity
 *   [SUNSKY_GRAD_ALBEDO + c]         albedo of channel c (c < 3 RGB, < 11 spectral;
 *                                    a uniform albedo's gradient is their sum)
 *   [SUNSKY_GRAD_SUN_DIRECTION + k]  sun_direction, world axis k (0 in time/location mode)
 * Accumulation is deterministic (fixed-order workgroup and block reductions). */
#define SUNSKY_GRAD_COUNT 16
#define SUNSKY_GRAD_TURBIDITY 0
#define SUNSKY_GRAD_ALBEDO 1
#define SUNSKY_GRAD_SUN_DIRECTION 12
int sunsky_eval_vjp(const sunsky_emitter *e, sunsky_vec3_in wi, const float *wavelengths, int n_wavelengths,
                    size_t wl_stride, const uint8_t *active, size_t n, const float *d_out, size_t out_stride,
                    float *grad, void *stream);
/* The tangent of the staged tables along `tangent` of `param` -- what dr::forward_from(param)
 * propagates into compute_radiance_params / compute_sun_params (sunsky.h:158-231, 404-419)
 * before eval: SUNSKY_TANGENT_FLOATS floats, d{A..I, rad} of channel c at c * 10 (+ q), the
 * local sun direction's tangent at 110..112, the sun table's at 128.  on_device = 1 stages
 * them with the kernel eval_jvp uses (blocking, on the null stream), 0 on the host (also
 * for host-only emitters); both compute the same fp64 arithmetic. */
#define SUNSKY_TANGENT_FLOATS (128 + 3240)
int sunsky_emitter_tangent_tables(const sunsky_emitter *e, int param, const float *tangent, int tangent_count,
                                  int on_device, float *out, size_t capacity, size_t *count);

/* --------------------------------------------- dataset I/O (sunsky_v.cpp:16-18) */
/* array_from_file_d / _f (sunsky.h:516-561): file_dtype 0 = infer, 1 = fp32, 2 = fp64.
 * Writes min(count, capacity) fp64 values; shape gets up to 16 dims. */
int sunsky_array_from_file(const char *path, int file_dtype, double *out, size_t capacity,
                           size_t *count, uint64_t *shape, int *ndims);
/* array_to_file (sunsky.h:573-597) */
int sunsky_array_to_file(const char *path, const float *data, size_t count, const uint64_t *shape,
                         int ndims);
/* mi.hosek_sun_rad (sunsky_v.cpp:19): arhosekskymodel_solar_radiance_internal2
 * (ArHosekSkyModel.c:686-784), the Hosek-Wilkie solar radiance in fp64 for a
 * turbidity, a wavelength (nm), the sun elevation and the angle gamma from the sun
 * centre (radians).  dataset_path: NULL for the bundled pack. */
int sunsky_hosek_sun_rad(const char *dataset_path, double turbidity, double wavelength, double elevation,
                         double gamma, double *out);

/* Plugin identification of MI_EXPORT_PLUGIN (class.h:220-225; sunsky.cpp:1037):
 * plugin_name() = "sunsky". */
const char *plugin_name(void);
const char *plugin_descr(void);

/* Path of the bundled dataset pack the library resolves by default. */
int sunsky_default_dataset_path(char *buf, size_t capacity);

/* ------------------------------------------------------------ multi-GPU gather
 * configs[4]: one process per GPU, each evaluating its contiguous
 * slice of the ray batch; the only exchange is the gather of the radiance planes to
 * one rank (the reference's ncclGather, rccl.h:745-746).  RCCL is loaded on first use
 * (dlopen librccl.so.1); without it these calls return SUNSKY_ERROR_COMM. */
#define SUNSKY_COMM_ID_BYTES 128
typedef struct sunsky_comm sunsky_comm;
/* ncclGetUniqueId: rank 0 makes the id, the caller hands it to every rank (any channel). */
int sunsky_comm_get_unique_id(unsigned char id[SUNSKY_COMM_ID_BYTES]);
/* ncclCommInitRank on the CURRENT HIP device (collective over the nranks processes). */
int sunsky_comm_create(const unsigned char id[SUNSKY_COMM_ID_BYTES], int nranks, int rank, sunsky_comm **out);
void sunsky_comm_destroy(sunsky_comm *comm);
int sunsky_comm_info(const sunsky_comm *comm, int *rank, int *nranks, int *device);
/* Gather every rank's shard into root's final planes, stream-ordered: rank r sends nplanes
 * planes of counts[r] floats (plane p at send + p * send_stride); on root they land at
 * recv + p * recv_stride + sum(counts[0..r)).  counts[] (nranks entries) is the same on
 * every rank; recv is only read on root.  Grouped ncclSend / ncclRecv: no padding and no
 * re-layout copy; root's own shard is a device copy (none when already in place). */
int sunsky_gather_radiance(sunsky_comm *comm, int root, const float *send, size_t send_stride, int nplanes,
                           const size_t *counts, float *recv, size_t recv_stride, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SUNSKY_AMD_H */
