// facade_check.cpp -- drives the C++ facade (include/sunsky_amd.hpp) the way a
// C++ renderer would.  Test program for tests/test_cpp_facade.py:
//   facade_check host            host-only staging, errors, flags (no GPU)
//   facade_check gpu <out_dir>   eval / sample_direction / pdf_direction on the
//                                current HIP device; raw fp32 planes written to
//                                <out_dir> for the oracle comparison in pytest.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "sunsky_amd.hpp"

using namespace sunsky_amd;

#define HIPCK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 3;                                                                \
        }                                                                            \
    } while (0)

static void fill_props(Properties& p) {
    const double th = (90.0 - 45.0) * M_PI / 180.0;
    p.set_float("turbidity", 4.3).set_float("albedo", 0.2);
    p.set_vector3("sun_direction", (float)std::sin(th), 0.f, (float)std::cos(th));
}

static int host_mode() {
    Properties p;
    fill_props(p);
    SunskyEmitter em = SunskyEmitter::host_only(p, Variant::RGB);
    sunsky_info info = em.info();
    if (!em.is_environment() || info.nb_channels != 3) { std::puts("FAIL flags/channels"); return 1; }
    if (em.bbox().valid()) { std::puts("FAIL bbox should be invalid"); return 1; }
    if (em.table(SUNSKY_TABLE_SKY_PARAMS).size() != 27) { std::puts("FAIL sky params size"); return 1; }
    std::printf("to_string: %s\n", em.to_string().c_str());
    std::printf("w_sky=%.9g\n", info.sky_sampling_w);
    // reference error text: sunsky.cpp:889-948
    try {
        Properties bad;
        bad.set_float("turbidity", 12.0);
        SunskyEmitter::host_only(bad, Variant::RGB);
        std::puts("FAIL no error for turbidity 12");
        return 1;
    } catch (const Error& e) {
        std::printf("error: %s\n", e.what());
    }
    try {
        em.sample_position();
    } catch (const NotImplementedError& e) {
        std::printf("not implemented: %s\n", e.what());
    }
    std::printf("hosek_sun_rad=%.17g\n", hosek_sun_rad(3.5, 555.0, 0.7, 0.001));
    std::puts("host ok");
    return 0;
}

template <typename T>
static bool write_file(const std::string& path, const std::vector<T>& v) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fwrite(v.data(), sizeof(T), v.size(), f);
    std::fclose(f);
    return true;
}

static int gpu_mode(const std::string& dir) {
    const size_t n = 8192;
    std::vector<float> wi(3 * n), u(2 * n);
    std::mt19937 rng(11);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    for (size_t i = 0; i < n; ++i) {
        float ct = U(rng), ph = 2.f * (float)M_PI * U(rng), st = std::sqrt(std::max(0.f, 1.f - ct * ct));
        wi[i] = -st * std::cos(ph); wi[n + i] = -st * std::sin(ph); wi[2 * n + i] = -ct;
        u[i] = U(rng); u[n + i] = U(rng);
    }
    float *d_wi, *d_u, *d_rgb, *d_d, *d_pdf, *d_w, *d_pdf2, *d_jv, *d_djv;
    HIPCK(hipMalloc(&d_wi, 3 * n * 4)); HIPCK(hipMalloc(&d_u, 2 * n * 4)); HIPCK(hipMalloc(&d_rgb, 3 * n * 4));
    HIPCK(hipMalloc(&d_d, 3 * n * 4)); HIPCK(hipMalloc(&d_pdf, n * 4)); HIPCK(hipMalloc(&d_w, 3 * n * 4));
    HIPCK(hipMalloc(&d_pdf2, n * 4));
    HIPCK(hipMalloc(&d_jv, 3 * n * 4)); HIPCK(hipMalloc(&d_djv, 3 * n * 4));
    HIPCK(hipMemcpy(d_wi, wi.data(), 3 * n * 4, hipMemcpyHostToDevice));
    HIPCK(hipMemcpy(d_u, u.data(), 2 * n * 4, hipMemcpyHostToDevice));

    Properties p;
    fill_props(p);
    SunskyEmitter em(p, Variant::RGB);

    SurfaceInteraction si;
    si.wi = {d_wi, d_wi + n, d_wi + 2 * n};
    si.n = n;
    em.eval(si, {d_rgb, n});

    Interaction it;
    it.n = n;
    DirectionSample ds;
    ds.d = {d_d, d_d + n, d_d + 2 * n};
    ds.pdf = d_pdf;
    em.sample_direction(it, {d_u, d_u + n}, ds, {d_w, n});
    DirectionSampleIn dsi;
    dsi.d = {d_d, d_d + n, d_d + 2 * n};
    em.pdf_direction(n, dsi, d_pdf2);
    em.eval_jvp(si, Param::Turbidity, {1.f}, {d_jv, n}, {d_djv, n});   // d eval / d turbidity
    // direct light at upward diffuse points, 2 spp, seed 3
    float *d_nrm, *d_dd;
    HIPCK(hipMalloc(&d_nrm, 3 * n * 4)); HIPCK(hipMalloc(&d_dd, 3 * n * 4));
    {
        std::vector<float> nrm(3 * n, 0.f);
        std::fill(nrm.begin() + 2 * n, nrm.end(), 1.f);
        HIPCK(hipMemcpy(d_nrm, nrm.data(), 3 * n * 4, hipMemcpyHostToDevice));
    }
    em.direct_diffuse({d_nrm, d_nrm + n, d_nrm + 2 * n}, n, 3, 2, {d_dd, n});
    HIPCK(hipDeviceSynchronize());
    std::vector<float> direct(3 * n);
    HIPCK(hipMemcpy(direct.data(), d_dd, 3 * n * 4, hipMemcpyDeviceToHost));
    // the occluded form: the rays of the same samples, a tracer that blocks every shadow ray
    // below 30 deg elevation and lets every BSDF ray escape, then the shading call
    float *d_er, *d_br;
    uint8_t* d_vis;
    HIPCK(hipMalloc(&d_er, 3 * 2 * n * 4)); HIPCK(hipMalloc(&d_br, 3 * 2 * n * 4)); HIPCK(hipMalloc(&d_vis, 2 * n));
    em.direct_diffuse_rays({d_nrm, d_nrm + n, d_nrm + 2 * n}, n, 3, 2, {d_er, d_er + 2 * n, d_er + 4 * n},
                           {d_br, d_br + 2 * n, d_br + 4 * n});
    HIPCK(hipDeviceSynchronize());
    std::vector<float> er(3 * 2 * n);
    HIPCK(hipMemcpy(er.data(), d_er, er.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint8_t> vis(2 * n);
    for (size_t k = 0; k < 2 * n; ++k) vis[k] = (uint8_t)((er[4 * n + k] >= 0.5f ? 1 : 0) | 2);
    HIPCK(hipMemcpy(d_vis, vis.data(), vis.size(), hipMemcpyHostToDevice));
    em.direct_diffuse({d_nrm, d_nrm + n, d_nrm + 2 * n}, n, 3, 2, {d_dd, n}, nullptr, {}, nullptr, d_vis, n);
    HIPCK(hipDeviceSynchronize());
    std::vector<float> occluded(3 * n);
    HIPCK(hipMemcpy(occluded.data(), d_dd, 3 * n * 4, hipMemcpyDeviceToHost));
    // a rough-conductor vertex at the same points seen from one view direction: GGX, alpha 0.2,
    // gold-like eta / k, seed 5, 2 spp; then its rays' BSDF weights (F G1 per channel)
    float* d_wv;
    HIPCK(hipMalloc(&d_wv, 3 * n * 4));
    {
        std::vector<float> wv(3 * n);
        const float vx = 0.3f, vy = 0.1f, vz = 0.95f, l = std::sqrt(vx * vx + vy * vy + vz * vz);
        for (size_t i = 0; i < n; ++i) { wv[i] = vx / l; wv[n + i] = vy / l; wv[2 * n + i] = vz / l; }
        HIPCK(hipMemcpy(d_wv, wv.data(), 3 * n * 4, hipMemcpyHostToDevice));
    }
    const float eta[3] = {0.143f, 0.374f, 1.442f}, kk[3] = {3.983f, 2.385f, 1.603f};
    em.direct_conductor({d_nrm, d_nrm + n, d_nrm + 2 * n}, {d_wv, d_wv + n, d_wv + 2 * n}, n,
                        SunskyEmitter::Microfacet::GGX, 0.2f, eta, kk, 5, 2, {d_dd, n});
    HIPCK(hipDeviceSynchronize());
    std::vector<float> conductor(3 * n), cweights(3 * 2 * n);
    HIPCK(hipMemcpy(conductor.data(), d_dd, 3 * n * 4, hipMemcpyDeviceToHost));
    float* d_bw;
    HIPCK(hipMalloc(&d_bw, 3 * 2 * n * 4));
    em.direct_conductor_rays({d_nrm, d_nrm + n, d_nrm + 2 * n}, {d_wv, d_wv + n, d_wv + 2 * n}, n,
                             SunskyEmitter::Microfacet::GGX, 0.2f, 5, 2, {d_er, d_er + 2 * n, d_er + 4 * n},
                             {d_br, d_br + 2 * n, d_br + 4 * n}, d_bw, eta, kk);
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(cweights.data(), d_bw, cweights.size() * 4, hipMemcpyDeviceToHost));
    (void)hipFree(d_wv); (void)hipFree(d_bw);
    (void)hipFree(d_nrm); (void)hipFree(d_dd); (void)hipFree(d_er); (void)hipFree(d_br); (void)hipFree(d_vis);

    std::vector<float> rgb(3 * n), dd(3 * n), pdf(n), w(3 * n), pdf2(n), djv(3 * n);
    HIPCK(hipMemcpy(djv.data(), d_djv, 3 * n * 4, hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(rgb.data(), d_rgb, 3 * n * 4, hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(dd.data(), d_d, 3 * n * 4, hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(pdf.data(), d_pdf, n * 4, hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(w.data(), d_w, 3 * n * 4, hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(pdf2.data(), d_pdf2, n * 4, hipMemcpyDeviceToHost));
    bool ok = write_file(dir + "/wi.f32", wi) && write_file(dir + "/u.f32", u) && write_file(dir + "/rgb.f32", rgb) &&
              write_file(dir + "/d.f32", dd) && write_file(dir + "/pdf.f32", pdf) && write_file(dir + "/w.f32", w) &&
              write_file(dir + "/pdf2.f32", pdf2) && write_file(dir + "/drgb_dturbidity.f32", djv) &&
              write_file(dir + "/direct.f32", direct) && write_file(dir + "/occluded.f32", occluded) &&
              write_file(dir + "/emitter_rays.f32", er) && write_file(dir + "/vis.u8", vis) &&
              write_file(dir + "/conductor.f32", conductor) && write_file(dir + "/conductor_weights.f32", cweights);
    for (float* ptr : {d_wi, d_u, d_rgb, d_d, d_pdf, d_w, d_pdf2, d_jv, d_djv}) (void)hipFree(ptr);
    if (!ok) { std::puts("FAIL writing outputs"); return 1; }
    std::printf("gpu ok w_sky=%.9g\n", em.info().sky_sampling_w);
    return 0;
}

int main(int argc, char** argv) {
    try {
        if (argc >= 2 && std::strcmp(argv[1], "host") == 0) return host_mode();
        if (argc >= 3 && std::strcmp(argv[1], "gpu") == 0) return gpu_mode(argv[2]);
    } catch (const Error& e) {
        std::fprintf(stderr, "sunsky_amd::Error(%d): %s\n", e.status, e.what());
        return 2;
    }
    std::fprintf(stderr, "usage: facade_check host | gpu <out_dir>\n");
    return 2;
}
