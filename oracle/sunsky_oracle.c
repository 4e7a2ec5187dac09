/*
 * sunsky_oracle.c -- TEST INFRASTRUCTURE ONLY (see sunsky_oracle.h).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  FMA
 * contraction is disabled so that every fused multiply-add in this file is
 * one the reference (Dr.Jit fmadd/lerp) also fuses.
 */
#include "sunsky_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static __thread char g_err[512];

static void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const char *oracle_last_error(void) { return g_err; }

void oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int oracle_get_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------------------- pack file */
typedef struct {
    unsigned char *buf;
    size_t size;
    unsigned n;
} pack_file;

#define PACK_ENTRY_SIZE 96

static uint32_t crc32_calc(const unsigned char *p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return ~c;
}

static int pack_open(pack_file *pk, const char *path) {
    memset(pk, 0, sizeof(*pk));
    FILE *f = fopen(path, "rb");
    if (!f) { set_error("oracle: cannot open dataset pack '%s'", path); return 1; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    pk->buf = (unsigned char *)malloc((size_t)sz);
    if (fread(pk->buf, 1, (size_t)sz, f) != (size_t)sz) {
        fclose(f); free(pk->buf); set_error("oracle: short read on '%s'", path); return 1;
    }
    fclose(f);
    pk->size = (size_t)sz;
    if (pk->size < 16 || memcmp(pk->buf, "SSKYPAK1", 8) != 0) {
        free(pk->buf); set_error("oracle: '%s' is not a sunsky dataset pack", path); return 1;
    }
    uint32_t version, n;
    memcpy(&version, pk->buf + 8, 4);
    memcpy(&n, pk->buf + 12, 4);
    if (version != 1 || 16 + (size_t)n * PACK_ENTRY_SIZE > pk->size) {
        free(pk->buf); set_error("oracle: unsupported pack version %u", version); return 1;
    }
    pk->n = n;
    return 0;
}

static void pack_close(pack_file *pk) { free(pk->buf); pk->buf = NULL; }

static const unsigned char *pack_entry(const pack_file *pk, const char *name) {
    for (unsigned i = 0; i < pk->n; ++i) {
        const unsigned char *e = pk->buf + 16 + (size_t)i * PACK_ENTRY_SIZE;
        if (strncmp((const char *)e, name, 24) == 0) return e;
    }
    return NULL;
}

static int pack_dtype(const pack_file *pk, const char *name) {
    const unsigned char *e = pack_entry(pk, name);
    uint32_t dt = 0;
    if (e) memcpy(&dt, e + 24, 4);
    return (int)dt;
}

static const void *pack_find(const pack_file *pk, const char *name, size_t *count) {
    const unsigned char *e = pack_entry(pk, name);
    *count = 0;
    if (!e) return NULL;
    uint32_t dt, ndims, nbytes, crc;
    uint64_t shape[6], off;
    memcpy(&dt, e + 24, 4);
    memcpy(&ndims, e + 28, 4);
    memcpy(shape, e + 32, 48);
    memcpy(&off, e + 80, 8);
    memcpy(&nbytes, e + 88, 4);
    memcpy(&crc, e + 92, 4);
    size_t cnt = 1;
    for (uint32_t d = 0; d < ndims && d < 6; ++d) cnt *= (size_t)shape[d];
    size_t esz = dt == 2 ? 8 : 4;
    if (off + nbytes > pk->size || cnt * esz != nbytes) return NULL;
    if (crc32_calc(pk->buf + off, nbytes) != crc) {
        set_error("oracle: crc mismatch on pack entry '%s'", name);
        return NULL;
    }
    *count = cnt;
    return pk->buf + off;
}

/* ------------------------------------------- math::legendre_pd, math.h:93-120 */
static void legendre_pd(int l, double x, double *lv, double *dv) {
    double l_cur = 0, d_cur = 0;
    if (l > 1) {
        double l_p_pred = 1, l_pred = x, d_p_pred = 0, d_pred = 1;
        double k0 = 3, k1 = 2, k2 = 1;
        for (int ki = 2; ki <= l; ++ki) {
            l_cur = (k0 * x * l_pred - k2 * l_p_pred) / k1;
            d_cur = d_p_pred + k0 * l_pred;
            l_p_pred = l_pred; l_pred = l_cur;
            d_p_pred = d_pred; d_pred = d_cur;
            k2 = k1; k0 += 2; k1 += 1;
        }
    } else if (l == 0) {
        l_cur = 1; d_cur = 0;
    } else {
        l_cur = x; d_cur = 1;
    }
    *lv = l_cur;
    *dv = d_cur;
}

/* quad::gauss_legendre, quad.h:27-86 (double precision; caller rounds) */
void oracle_gauss_legendre(int n, double *nodes, double *weights) {
    if (n < 1) return;
    n--;
    if (n == 0) { nodes[0] = 0; weights[0] = 2; return; }
    if (n == 1) { nodes[0] = -sqrt(1.0 / 3.0); nodes[1] = -nodes[0]; weights[0] = weights[1] = 1; }
    int m = (n + 1) / 2;
    for (int i = 0; i < m; ++i) {
        double x = -cos((double)(2 * i + 1) / (double)(2 * n + 2) * 3.14159265358979323846);
        for (int it = 0; it < 20; ++it) {
            double lv, dv;
            legendre_pd(n + 1, x, &lv, &dv);
            double step = lv / dv;
            x -= step;
            if (fabs(step) <= 4 * fabs(x) * 1.1102230246251565e-16) break;
        }
        double lv, dv;
        legendre_pd(n + 1, x, &lv, &dv);
        weights[i] = weights[n - i] = 2 / ((1 - x * x) * (dv * dv));
        nodes[i] = x;
        nodes[n - i] = -x;
    }
    if ((n % 2) == 0) {
        double lv, dv;
        legendre_pd(n + 1, 0.0, &lv, &dv);
        weights[n / 2] = 2.0 / (dv * dv);
        nodes[n / 2] = 0;
    }
}

/* compute_sun_coordinates, sunsky.h:284-374, in fp32 like the float variants
   (Int32 Julian-day arithmetic with C truncating division). */
void oracle_sun_coordinates(int year, int month, int day, float hour, float minute,
                            float second, float latitude, float longitude, float timezone,
                            float out[3]) {
    const float pi = 3.14159265358979323846f, two_pi = 6.28318530717958647692f;
    float dec_hours = hour - timezone + (minute + second / 60.f) / 60.f;
    int li_aux_1 = (month - 14) / 12;
    int li_aux_2 = (1461 * (year + 4800 + li_aux_1)) / 4 + (367 * (month - 2 - 12 * li_aux_1)) / 12 -
                   (3 * ((year + 4900 + li_aux_1) / 100)) / 4 + day - 32075;
    float d_julian_date = (float)li_aux_2 - 0.5f + dec_hours / 24.f;
    float elapsed = d_julian_date - 2451545.f;

    float omega = 2.1429f - 0.0010394594f * elapsed;
    float mean_longitude = 4.8950630f + 0.017202791698f * elapsed;
    float anomaly = 6.2400600f + 0.0172019699f * elapsed;
    float ecl_long = mean_longitude + 0.03341607f * sinf(anomaly) + 0.00034894f * sinf(2 * anomaly) -
                     0.0001134f - 0.0000203f * sinf(omega);
    float ecl_obl = 0.4090928f - 6.2140e-9f * elapsed + 0.0000396f * cosf(omega);

    float sin_el = sinf(ecl_long);
    float dy = cosf(ecl_obl) * sin_el, dx = cosf(ecl_long);
    float ra = atan2f(dy, dx);
    ra += ra < 0.f ? two_pi : 0.f;
    float decl = asinf(sinf(ecl_obl) * sin_el);

    float gmst = 6.6974243242f + 0.0657098283f * elapsed + dec_hours;
    const float deg2rad = (float)(3.14159265358979323846 / 180.0);
    float lmst = (gmst * 15 + longitude) * deg2rad;
    float lat = latitude * deg2rad;
    float cos_lat = cosf(lat), sin_lat = sinf(lat);
    float hour_angle = lmst - ra;
    float cos_ha = cosf(hour_angle);
    float elevation = acosf(cos_lat * cos_ha * cosf(decl) + sinf(decl) * sin_lat);
    dy = -sinf(hour_angle);
    dx = tanf(decl) * cos_lat - sin_lat * cos_ha;
    float azimuth = atan2f(dy, dx);
    azimuth += azimuth < 0.f ? two_pi : 0.f;
    elevation += (float)(6371.01 / 149597890.0) * sinf(elevation);

    float theta = elevation, phi = azimuth - pi;
    out[0] = cosf(phi) * sinf(theta);
    out[1] = sinf(phi) * sinf(theta);
    out[2] = cosf(theta);
}

/* estimate_sky_sun_ratio's two 40,000-term sums (dr::sum_inner, sunsky.cpp:815, 849).
   Dr.Jit leaves the reduction order to its backend (LLVM: blocked SIMD partial sums,
   CUDA: a tree), so the oracle's default adds the fp32 terms exactly (an fp64
   accumulator, rounded once): the order-independent value every reasonable reduction
   approximates.  1 = the terms added one by one in R, the worst-case order (the
   round-1..3 restatement), kept for reporting. */
static int g_quad_sum_sequential = 0;
void oracle_set_quadrature_sum(int sequential) { g_quad_sum_sequential = sequential != 0; }
int oracle_get_quadrature_sum(void) { return g_quad_sum_sequential; }

/* -------------------------------------------------- precision instantiation */
#define R float
#define SFX f32
#define F(fn) fn##f
#include "oracle_impl.inc"
#undef R
#undef SFX
#undef F

#define R double
#define SFX f64
#define F(fn) fn
#include "oracle_impl.inc"
#undef R
#undef SFX
#undef F

/* Every fp32 cos theta in [0, 1] (bit patterns 0 .. 0x3f800000): does the fp32 segment
   decision (sun_segment_f32, sunsky.cpp:579-584) equal the count of thresholds z[1..44] it
   passes (the product's SunskyKArgs::sun_seg_z)?  Returns the number of mismatches; first
   mismatching bit pattern in *first (0xffffffff when none).  OpenMP over the range. */
long oracle_check_sun_segment_thresholds(const float *z, unsigned *first) {
    long bad = 0;
    unsigned first_bad = 0xffffffffu;
    const long n = 0x3f800001L;
#pragma omp parallel for reduction(+ : bad) schedule(static)
    for (long b = 0; b < n; ++b) {
        unsigned u = (unsigned)b;
        float f;
        memcpy(&f, &u, 4);
        int lo = 0, hi = 44;          /* largest j with f >= z[j] (z[0] = 0) */
        while (lo < hi) {
            int mid = (lo + hi + 1) / 2;
            if (f >= z[mid]) lo = mid; else hi = mid - 1;
        }
        if (lo != oracle_sun_segment_f32(f)) {
            ++bad;
#pragma omp critical
            if (u < first_bad) first_bad = u;
        }
    }
    if (first) *first = first_bad;
    return bad;
}
