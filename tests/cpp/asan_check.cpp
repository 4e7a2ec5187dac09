// asan_check.cpp -- AddressSanitizer + UBSan run of the host code (the
// reference's MI_SANITIZE_ADDRESS build option, CMakeLists.txt:34-36).  Built by
// tests/cpp/Makefile from the product's host sources (C ABI, staging, datasets, Hošek
// sun radiance, comm argument checks) and the oracle, all with -fsanitize=address,
// undefined; no device code and no HIP call is made (host-only emitters).  Run by
// tests/test_asan.py; prints "asan ok" and exits 0 when nothing was reported.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sunsky_amd.h"
#include "sunsky_oracle.h"

namespace {

int g_fail = 0;
#define EXPECT(cond)                                                              \
    do {                                                                          \
        if (!(cond)) {                                                            \
            std::fprintf(stderr, "FAILED %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, \
                         sunsky_last_error());                                    \
            ++g_fail;                                                             \
        }                                                                         \
    } while (0)

std::string g_pack;

sunsky_props* angles_props(double t, double elev_deg, int nalb, const float* alb) {
    sunsky_props* p = nullptr;
    EXPECT(sunsky_props_create(&p) == SUNSKY_OK);
    EXPECT(sunsky_props_set_float(p, "turbidity", t) == SUNSKY_OK);
    const double e = elev_deg * M_PI / 180.0;
    EXPECT(sunsky_props_set_vector3(p, "sun_direction", (float)(std::cos(e) * 0.6), (float)(std::cos(e) * 0.8),
                                    (float)std::sin(e)) == SUNSKY_OK);
    if (nalb == 1) EXPECT(sunsky_props_set_float(p, "albedo", alb[0]) == SUNSKY_OK);
    else EXPECT(sunsky_props_set_spectrum(p, "albedo", alb, nalb) == SUNSKY_OK);
    return p;
}

void exercise_emitter(sunsky_emitter* e, int variant) {
    sunsky_info info;
    EXPECT(sunsky_emitter_get_info(e, &info) == SUNSKY_OK);
    EXPECT(info.nb_channels == (variant ? 11 : 3));
    for (int id = SUNSKY_TABLE_SKY_PARAMS; id <= SUNSKY_TABLE_ALBEDO; ++id) {
        size_t count = 0;
        EXPECT(sunsky_emitter_get_table(e, id, nullptr, 0, &count) == SUNSKY_OK);
        std::vector<float> v(count + 1, -1.f);
        size_t c2 = 0;
        EXPECT(sunsky_emitter_get_table(e, id, v.data(), count, &c2) == SUNSKY_OK && c2 == count);
        EXPECT(v[count] == -1.f);   // wrote exactly `count` values
        if (count > 2) EXPECT(sunsky_emitter_get_table(e, id, v.data(), 2, &c2) == SUNSKY_OK);   // truncated copy
    }
    EXPECT(sunsky_emitter_get_table(e, 99, nullptr, 0, nullptr) != SUNSKY_OK);
    char buf[4096];
    EXPECT(sunsky_emitter_to_string(e, buf, sizeof(buf)) == SUNSKY_OK && std::strlen(buf) > 10);
    char small[8];
    EXPECT(sunsky_emitter_to_string(e, small, sizeof(small)) == SUNSKY_OK && std::strlen(small) == 7);
    float mn[3], mx[3];
    EXPECT(sunsky_emitter_bbox(e, mn, mx) == SUNSKY_OK && mn[0] > mx[0]);
    const float c[3] = {1.f, 2.f, 3.f};
    EXPECT(sunsky_emitter_set_scene(e, 1, c, 10.f) == SUNSKY_OK);
    // traverse()/update(): a valid update, then a rejected one that rolls back
    const float t = 5.5f;
    EXPECT(sunsky_emitter_set_param(e, "turbidity", &t, 1) == SUNSKY_OK);
    EXPECT(sunsky_emitter_parameters_changed(e) == SUNSKY_OK);
    const float bad = 12.f;
    EXPECT(sunsky_emitter_set_param(e, "turbidity", &bad, 1) == SUNSKY_OK);
    EXPECT(sunsky_emitter_parameters_changed(e) != SUNSKY_OK);
    float got[16];
    int n = 0;
    EXPECT(sunsky_emitter_get_param(e, "turbidity", got, 16, &n) == SUNSKY_OK && n == 1 && got[0] == t);
    EXPECT(sunsky_emitter_get_param(e, "albedo", got, 16, &n) == SUNSKY_OK && n >= 1);
    EXPECT(sunsky_emitter_get_param(e, "no_such_parameter", got, 16, &n) != SUNSKY_OK);
    std::vector<float> alb(variant ? 11 : 3, 0.4f);
    EXPECT(sunsky_emitter_set_param(e, "albedo", alb.data(), (int)alb.size()) == SUNSKY_OK);
    EXPECT(sunsky_emitter_parameters_changed(e) == SUNSKY_OK);
    const float dir[3] = {0.2f, -0.3f, 0.9f};
    if (!info.active_record) {   // sun_direction mode; time/location mode does not expose it
        EXPECT(sunsky_emitter_set_param(e, "sun_direction", dir, 3) == SUNSKY_OK);
        EXPECT(sunsky_emitter_parameters_changed(e) == SUNSKY_OK);
    } else {
        EXPECT(sunsky_emitter_set_param(e, "sun_direction", dir, 3) != SUNSKY_OK);
    }
    // batch calls on a host-only emitter fail cleanly
    float x = 0.f;
    sunsky_vec3_in w = {&x, &x, &x};
    float out[3];
    EXPECT(sunsky_eval(e, w, nullptr, 0, 1, nullptr, 1, out, 1, nullptr) != SUNSKY_OK);
    EXPECT(sunsky_sample_position(e) == SUNSKY_ERROR_NOT_IMPLEMENTED);
}

void product_host_paths() {
    const float a1 = 0.3f, a3[3] = {0.1f, 0.5f, 0.9f};
    std::vector<float> a11(11);
    for (int i = 0; i < 11; ++i) a11[i] = 0.05f + 0.08f * (float)i;
    struct Case { int variant, semantics; double t, elev; int nalb; const float* alb; };
    const Case cases[] = {{0, 0, 3.0, 45.0, 1, &a1}, {0, 1, 6.2, 12.0, 3, a3}, {1, 0, 2.5, 30.0, 11, a11.data()},
                          {1, 1, 9.9, 80.0, 1, &a1}, {0, 0, 1.0, 0.5, 1, &a1}};
    for (const Case& cs : cases) {
        sunsky_props* p = angles_props(cs.t, cs.elev, cs.nalb, cs.alb);
        sunsky_emitter* e = nullptr;
        EXPECT(sunsky_emitter_create_host(p, cs.variant, cs.semantics, g_pack.c_str(), &e) == SUNSKY_OK);
        if (e) exercise_emitter(e, cs.variant);
        sunsky_emitter_destroy(e);
        sunsky_props_destroy(p);
    }
    // time/location mode, irregular albedo spectrum, to_world
    {
        sunsky_props* p = nullptr;
        EXPECT(sunsky_props_create(&p) == SUNSKY_OK);
        EXPECT(sunsky_props_set_float(p, "latitude", 35.6894) == SUNSKY_OK);
        EXPECT(sunsky_props_set_float(p, "longitude", 139.6917) == SUNSKY_OK);
        EXPECT(sunsky_props_set_float(p, "timezone", 9) == SUNSKY_OK);
        EXPECT(sunsky_props_set_int(p, "year", 2010) == SUNSKY_OK);
        EXPECT(sunsky_props_set_int(p, "month", 7) == SUNSKY_OK);
        EXPECT(sunsky_props_set_int(p, "day", 10) == SUNSKY_OK);
        EXPECT(sunsky_props_set_float(p, "hour", 11.7753) == SUNSKY_OK);
        const float wl[5] = {300.f, 420.f, 555.f, 640.f, 800.f}, v[5] = {0.1f, 0.3f, 0.2f, 0.6f, 0.4f};
        EXPECT(sunsky_props_set_irregular_spectrum(p, "albedo", wl, v, 5) == SUNSKY_OK);
        const float m[16] = {1, 0, 0, 0, 0, 0, -1, 0, 0, 1, 0, 0, 0, 0, 0, 1};
        EXPECT(sunsky_props_set_transform(p, "to_world", m) == SUNSKY_OK);
        sunsky_emitter* e = nullptr;
        EXPECT(sunsky_emitter_create_host(p, 1, 0, g_pack.c_str(), &e) == SUNSKY_OK);
        if (e) exercise_emitter(e, 1);
        sunsky_emitter_destroy(e);
        sunsky_props_destroy(p);
    }
    // rejected constructions: unqueried property, out-of-range turbidity, both sun modes, bad pack
    {
        sunsky_props* p = angles_props(3.0, 40.0, 1, &a1);
        EXPECT(sunsky_props_set_float(p, "not_a_property", 1.0) == SUNSKY_OK);
        sunsky_emitter* e = nullptr;
        EXPECT(sunsky_emitter_create_host(p, 0, 0, g_pack.c_str(), &e) != SUNSKY_OK && e == nullptr);
        sunsky_props_destroy(p);
        p = angles_props(11.0, 40.0, 1, &a1);
        EXPECT(sunsky_emitter_create_host(p, 0, 0, g_pack.c_str(), &e) != SUNSKY_OK);
        EXPECT(sunsky_props_set_float(p, "hour", 10.0) == SUNSKY_OK);
        EXPECT(sunsky_emitter_create_host(p, 0, 0, g_pack.c_str(), &e) != SUNSKY_OK);
        sunsky_props_destroy(p);
        p = angles_props(3.0, 40.0, 1, &a1);
        EXPECT(sunsky_emitter_create_host(p, 0, 0, "/nonexistent/pack", &e) == SUNSKY_ERROR_FILE);
        sunsky_props_destroy(p);
    }
    // file formats (sunsky.h:516-597) and the Hošek sun radiance binding
    {
        const char* path = "build/asan_array.bin";
        std::vector<float> data(2 * 3 * 5);
        for (size_t i = 0; i < data.size(); ++i) data[i] = 0.25f * (float)i - 1.f;
        const uint64_t shape[3] = {2, 3, 5};
        EXPECT(sunsky_array_to_file(path, data.data(), data.size(), shape, 3) == SUNSKY_OK);
        size_t count = 0;
        uint64_t sh[16];
        int nd = 0;
        EXPECT(sunsky_array_from_file(path, 1, nullptr, 0, &count, sh, &nd) == SUNSKY_OK && count == data.size());
        std::vector<double> back(count);
        EXPECT(sunsky_array_from_file(path, 1, back.data(), back.size(), &count, sh, &nd) == SUNSKY_OK);
        EXPECT(nd == 3 && sh[2] == 5 && back[7] == (double)data[7]);
        EXPECT(sunsky_array_from_file("build/does_not_exist.bin", 1, nullptr, 0, &count, sh, &nd) ==
               SUNSKY_ERROR_FILE);
        double r = 0.0;
        EXPECT(sunsky_hosek_sun_rad(g_pack.c_str(), 3.0, 550.0, 0.5, 0.001, &r) == SUNSKY_OK && r > 0.0);
        EXPECT(sunsky_hosek_sun_rad(g_pack.c_str(), 3.0, 550.0, 0.5, 0.001, nullptr) != SUNSKY_OK);
    }
    // the multi-GPU entry points' argument checks (no communicator is created)
    EXPECT(sunsky_gather_radiance(nullptr, 0, nullptr, 0, 1, nullptr, nullptr, 0, nullptr) != SUNSKY_OK);
}

template <typename O, typename R>
void oracle_paths(int (*create)(const oracle_params*, const char*, O**), void (*destroy)(O*),
                  void (*info)(const O*, oracle_info*), size_t (*table)(const O*, R*, size_t),
                  void (*eval)(const O*, const float*, const float*, const float*, const float*, int, size_t, R*),
                  void (*sample)(const O*, const float*, const float*, const float*, const float*, const float*,
                                 const float*, int, size_t, R*, R*, R*, R*, R*, R*),
                  void (*pdf)(const O*, const float*, const float*, const float*, size_t, R*),
                  void (*sray)(const O*, const float*, const float*, const float*, const float*, const float*, size_t,
                               R*, R*, R*, R*, R*, R*, R*, R*),
                  void (*swl)(const O*, const float*, const float*, const float*, const float*, size_t, R*, R*)) {
    const size_t n = 37;   // ragged: not a multiple of any vector width
    std::vector<float> wx(n), wy(n), wz(n), ux(n), uy(n), lam(4 * n), s(n);
    unsigned state = 12345u;
    auto rnd = [&] { state = state * 1664525u + 1013904223u; return (float)((state >> 8) * (1.0 / 16777216.0)); };
    for (size_t i = 0; i < n; ++i) {
        const float ct = rnd(), ph = 6.2831853f * rnd(), st = std::sqrt(1.f - ct * ct);
        wx[i] = -st * std::cos(ph); wy[i] = -st * std::sin(ph); wz[i] = -ct;
        ux[i] = rnd(); uy[i] = rnd(); s[i] = rnd();
        for (int k = 0; k < 4; ++k) lam[k * n + i] = 360.f + 360.f * rnd();
    }
    for (int spectral = 0; spectral < 2; ++spectral)
        for (int jit = 0; jit < 2; ++jit) {
            oracle_params p;
            std::memset(&p, 0, sizeof(p));
            p.spectral = spectral; p.jit_semantics = jit; p.turbidity = 4.2f;
            p.sky_scale = 1.f; p.sun_scale = 1.f; p.sun_aperture_deg = 0.5358f;
            p.albedo_n = 1; p.albedo[0] = 0.3f; p.use_sun_direction = 1;
            p.sun_direction[0] = 0.3f; p.sun_direction[1] = 0.4f; p.sun_direction[2] = 0.6f;
            for (int i = 0; i < 4; ++i) p.to_world[i * 5] = 1.f;
            p.bsphere_radius = 1.f;
            O* o = nullptr;
            EXPECT(create(&p, g_pack.c_str(), &o) == 0 && o);
            if (!o) continue;
            oracle_info inf;
            info(o, &inf);
            std::vector<R> tab(table(o, nullptr, 0));
            EXPECT(table(o, tab.data(), tab.size()) == tab.size());
            const int nl = spectral ? 4 : 0;
            std::vector<R> out((spectral ? 4 : 3) * n), d(3 * n), pd(n), dist(n), w(4 * n), o3(3 * n), l4(4 * n);
            eval(o, wx.data(), wy.data(), wz.data(), spectral ? lam.data() : nullptr, nl, n, out.data());
            sample(o, ux.data(), uy.data(), nullptr, nullptr, nullptr, spectral ? lam.data() : nullptr, nl, n,
                   d.data(), d.data() + n, d.data() + 2 * n, pd.data(), dist.data(), w.data());
            std::vector<float> df(3 * n);
            for (size_t i = 0; i < 3 * n; ++i) df[i] = (float)d[i];
            pdf(o, df.data(), df.data() + n, df.data() + 2 * n, n, pd.data());
            sray(o, s.data(), ux.data(), uy.data(), uy.data(), ux.data(), n, o3.data(), o3.data() + n,
                 o3.data() + 2 * n, d.data(), d.data() + n, d.data() + 2 * n, l4.data(), w.data());
            swl(o, wx.data(), wy.data(), wz.data(), s.data(), n, l4.data(), w.data());
            for (size_t i = 0; i < n; ++i) EXPECT(std::isfinite((double)pd[i]));
            destroy(o);
        }
}

}  // namespace

int main(int argc, char** argv) {
    g_pack = argc > 1 ? argv[1] : "../../mitsuba3-sunsky_amd/data/sunsky_datasets.pack";
    product_host_paths();
    oracle_paths<oracle_f32, float>(oracle_create_f32, oracle_destroy_f32, oracle_info_f32, oracle_sun_table_f32,
                                    oracle_eval_f32, oracle_sample_direction_f32, oracle_pdf_direction_f32,
                                    oracle_sample_ray_f32, oracle_sample_wavelengths_f32);
    oracle_paths<oracle_f64, double>(oracle_create_f64, oracle_destroy_f64, oracle_info_f64, oracle_sun_table_f64,
                                     oracle_eval_f64, oracle_sample_direction_f64, oracle_pdf_direction_f64,
                                     oracle_sample_ray_f64, oracle_sample_wavelengths_f64);
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("asan ok\n");
    return 0;
}
