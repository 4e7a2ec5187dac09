/*
 * sunsky_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference sun/sky emitter (matttsss/mitsuba3-sunsky,
 * src/emitters/sunsky.cpp + include/mitsuba/render/sunsky/sunsky.h) used as
 * the parity checker for the HIP product path.  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load it; the product
 * (mitsuba3-sunsky_amd/) never links or calls it.
 *
 * Two instantiations of the same code:
 *   *_f32  follows the reference's fp32 variants op for op (tables cast fp64 ->
 *          fp32 as array_from_file<Float64, Float>, sunsky.h:558-560),
 *   *_f64  the same algorithm in fp64 (tables kept fp64) = the "ideal" answer
 *          for conditioning-aware parity checks.
 *
 * Pinning (see DESIGN.md "Oracle"): checked against every fixture the
 * reference's own tests hold for this path -- the 80 sun spectra
 * (resources/sunsky/test_data/spectrum/sun_spectrum_*.spd files, test_sunsky.py:154-196) and the
 * 7 EXR sky renders (test_sunsky.py:115-145) -- through tests/golden/.
 * The reference plugin itself cannot be built here (Dr.Jit submodule absent)
 * and ArHosekSkyModel.c needs Dr.Jit symbols (c:758-763), so no oracle/_ref.
 */
#ifndef SUNSKY_ORACLE_H
#define SUNSKY_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_params {
    int   spectral;        /* 0 = *_rgb variants, 1 = *_spectral variants           */
    int   jit_semantics;   /* 1 = llvm_/cuda_ variants (quadrature w_sky, sunsky.cpp:784-885),
                              0 = scalar_ variants (w_sky = 0.5, uniform lambda pdf, :778-783) */
    float turbidity;       /* [1, 10]                                              */
    float sky_scale, sun_scale;
    float sun_aperture_deg;/* full aperture in degrees (default 0.5358, :904)        */
    int   albedo_n;        /* 1 (uniform) or NB_CHANNELS (3 / 11) per-channel values */
    float albedo[11];
    int   use_sun_direction;
    float sun_direction[3];/* world space, normalised inside (:923)                  */
    float latitude, longitude, timezone;
    int   year, month, day;
    float hour, minute, second;
    float to_world[16];    /* row-major 4x4                                          */
    float bsphere_center[3];
    float bsphere_radius;  /* after set_scene (sunsky.cpp:287-301); default 1        */
} oracle_params;

typedef struct oracle_f32 oracle_f32;
typedef struct oracle_f64 oracle_f64;

/* Staged state exported for staging-parity tests (Appendix B of SURVEY.md). */
typedef struct oracle_info {
    double sun_dir_world[3], sun_dir_local[3], sun_angles[2];
    double frame_s[3], frame_t[3];
    double sun_eta, w_sky, area_ratio, cos_cutoff;
    int    nb_channels;
    double sky_params[11 * 9], sky_radiance[11];
    double gaussians[20 * 5], gauss_cdf[20];
    double gauss_sum;
    double spec_pdf[10], spec_cdf[9], spec_integral;
    int    spec_size; /* 10 (jit) or 2 (scalar) */
} oracle_info;

const char *oracle_last_error(void);
void oracle_set_threads(int n);
/* estimate_sky_sun_ratio's sums: 0 (default) the fp32 terms added exactly, 1 sequentially in R */
void oracle_set_quadrature_sum(int sequential);
int oracle_get_quadrature_sum(void);
int  oracle_get_threads(void);

/* Restated helper exposed for tests: Gauss-Legendre nodes (quad.h:27-86). */
void oracle_gauss_legendre(int n, double *nodes, double *weights);
/* Restated compute_sun_coordinates (sunsky.h:284-374), fp32 like the reference. */
void oracle_sun_coordinates(int year, int month, int day, float hour, float minute,
                            float second, float latitude, float longitude, float timezone,
                            float out[3]);

#define ORACLE_DECL(SFX, R)                                                                     \
    int  oracle_create_##SFX(const oracle_params *p, const char *pack_path, oracle_##SFX **out); \
    void oracle_destroy_##SFX(oracle_##SFX *o);                                                  \
    void oracle_info_##SFX(const oracle_##SFX *o, oracle_info *info);                            \
    /* sun table after turbidity lerp; returns element count */                                 \
    size_t oracle_sun_table_##SFX(const oracle_##SFX *o, R *out, size_t cap);                    \
    /* eval(): wi SoA; spectral: lambda[k*n + i] for k < n_lambda, out[k*n + i] */              \
    void oracle_eval_##SFX(const oracle_##SFX *o, const float *wx, const float *wy,              \
                           const float *wz, const float *lambda, int n_lambda, size_t n,         \
                           R *out);                                                              \
    /* sample_direction(): it.p may be NULL (origin); lambda as in eval */                      \
    void oracle_sample_direction_##SFX(const oracle_##SFX *o, const float *ux, const float *uy, \
                           const float *px, const float *py, const float *pz,                    \
                           const float *lambda, int n_lambda, size_t n,                          \
                           R *dx, R *dy, R *dz, R *pdf, R *dist, R *weight);                     \
    void oracle_pdf_direction_##SFX(const oracle_##SFX *o, const float *dx, const float *dy,     \
                           const float *dz, size_t n, R *pdf);                                   \
    /* sample_ray(): spectral -> 4 wavelengths per ray (lambda_out[k*n+i]) */                   \
    void oracle_sample_ray_##SFX(const oracle_##SFX *o, const float *wavelength_sample,          \
                           const float *s2x, const float *s2y, const float *s3x,                 \
                           const float *s3y, size_t n, R *ox, R *oy, R *oz, R *dx, R *dy,        \
                           R *dz, R *lambda_out, R *weight);                                     \
    /* sample_wavelengths(si, sample): spectral -> 4 shifted samples per ray; RGB -> eval */  \
    void oracle_sample_wavelengths_##SFX(const oracle_##SFX *o, const float *wx, const float *wy,\
                           const float *wz, const float *sample, size_t n, R *lambda_out,        \
                           R *weight);                                                           \
    /* test hook: adopt another implementation's staged sky/sun sampling weight */             \
    void oracle_override_w_sky_##SFX(oracle_##SFX *o, double w_sky);                            \
    /* test hook: adopt another implementation's staged wavelength-distribution nodes (the    \
       pdf values of sunsky.cpp:870-885) and rebuild the CDF from them (distr_1d.h:513-585);  \
       returns 0, or 1 if size is not 2..10 or a value is negative / not finite */            \
    int oracle_override_spectral_distr_##SFX(oracle_##SFX *o, const double *pdf, int size);    \
    /* test hooks: evaluate with fp32 staged tables (the reference's staging precision,      \
       sunsky.cpp:182-195): round this oracle's own in place, or adopt another                 \
       implementation's with its fp32 local sun direction and disc cutoff (returns 1 on a size \
       mismatch); both take the fp32 segment decision */\
    void oracle_round_staged_tables_##SFX(oracle_##SFX *o);                                      \
    int oracle_adopt_tables_##SFX(oracle_##SFX *o, const float *sky_params, size_t n_sky,        \
                           const float *sky_rad, size_t n_rad, const float *sun_rad,             \
                           size_t n_sun, const float *sun_ld, size_t n_ld,                       \
                           const float *sun_local /* NULL: keep */, float cos_cutoff,           \
                           float area_ratio /* < 0: keep */);                                   \
    /* HW solar radiance (restates ArHosekSkyModel.c:686-784 on the packed tables) */          \
    R oracle_hw_sun_radiance_##SFX(const oracle_##SFX *o, R turbidity, R wavelength,            \
                           R elevation, R gamma);                                                \
    /* render_sun's elevation segment of a cos theta (sunsky.cpp:579-584) */                    \
    int oracle_sun_segment_##SFX(R cos_theta);

ORACLE_DECL(f32, float)
ORACLE_DECL(f64, double)

/* every fp32 cos theta in [0, 1] through the fp32 segment decision against a threshold
   table z[0..44]: the number of mismatches (first bad bit pattern in *first) */
long oracle_check_sun_segment_thresholds(const float *z, unsigned *first);

#ifdef __cplusplus
}
#endif
#endif
