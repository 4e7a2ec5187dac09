// kbench.cpp -- native kernel micro-benchmark for tuning (no Python, no torch).
//
// Stages a sunsky emitter with the product's host code (SunskyModel), uploads
// n uniform upper-hemisphere directions, and times kernels of the code object
// by name with hipEvents over back-to-back launches, for several grid sizes.
//
//   kbench <hsaco> <rgb|spec|sample|pdf> <n> <iters> <blocks_per_cu,...> <kernel> [kernel ...]
// rgb / spec: eval kernels on uniform upper-hemisphere directions (C2 / C3 emitters);
// sample / pdf: sample_direction (ds.dist, ds.p not requested) / pdf_direction (C4 emitter);
// sray / swl: sample_ray / sample_wavelengths (C4 emitter; KB_SAMPLE_SPEC=1 for spectral);
// conductor: direct_conductor (C4 emitter, GGX alpha 0.2 -- KB_BECKMANN=1 for Beckmann --,
// gold-like eta / k, 4 spp at random normals and views).
//
// Build: make -C tools kbench
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "sunsky_model.h"

using namespace sunsky;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

struct LambdaSet {
    int m;
    int lo[kMaxBroadcastLambda];
    float f[kMaxBroadcastLambda];
};

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: kbench <hsaco> <rgb|spec> <n> <iters> <bpcu,...> <kernel>...\n");
        return 2;
    }
    std::string hsaco = argv[1], mode = argv[2];
    size_t n = std::strtoull(argv[3], nullptr, 10);
    int iters = std::atoi(argv[4]);
    std::vector<int> bpcu;
    {
        std::stringstream ss(argv[5]);
        std::string tok;
        while (std::getline(ss, tok, ',')) bpcu.push_back(std::atoi(tok.c_str()));
    }
    const bool spec = mode == "spec";
    const bool rays = mode == "rays";   // per-ray spectral eval, 4 random wavelengths per ray (Spectrum<Float, 4>)
    const bool cond = mode == "conductor" || mode == "diffuse";   // the callers (diffuse: the normals only)
    const bool sray = mode == "sray", swl = mode == "swl";
    const bool sampling = mode == "sample" || mode == "pdf" || cond || sray || swl;
    const char* pack = std::getenv("SUNSKY_AMD_DATASET");
    std::string pack_path = pack ? pack : "mitsuba3-sunsky_amd/data/sunsky_datasets.pack";

    Properties props;
    props.set_float("turbidity", spec || sampling ? 3.0 : 2.0);
    props.set_float("albedo", spec || sampling ? 0.3 : 0.1);
    double th = (90.0 - (sampling ? 30.0 : 45.0)) * M_PI / 180.0;
    props.set_vector3("sun_direction", (float)std::sin(th), 0.f, (float)std::cos(th));
    // KB_SAMPLE_SPEC=1 (sample mode): the spectral emitter, 4 random wavelengths per sample
    const bool sspec = (mode == "sample" || sray || swl || cond) && std::getenv("KB_SAMPLE_SPEC") != nullptr;
    SunskyModel model(props, spec || sspec || rays ? kSpectral : kRGB, kJit, pack_path);

    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    float *d_sun, *d_ld;
    CK(hipMalloc(&d_sun, sizeof(float) * std::max(kSunRgbTableSize, kSunSpecTableSize)));
    CK(hipMalloc(&d_ld, sizeof(float) * 66));
    CK(hipMemcpy(d_sun, model.sun_table().data(), sizeof(float) * model.sun_table().size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ld, model.sun_ld().data(), sizeof(float) * 66, hipMemcpyHostToDevice));
    SunskyKArgs hk = model.kargs();
    hk.sun_table = d_sun;
    hk.sun_ld = d_ld;
    // kernels read the emitter state through a device pointer (sunsky_types.h)
    SunskyKArgs* K = nullptr;
    CK(hipMalloc(&K, sizeof(SunskyKArgs)));
    CK(hipMemcpy(K, &hk, sizeof(SunskyKArgs), hipMemcpyHostToDevice));

    // directions: cos theta = u1, phi = 2 pi u2; wi = -wo
    std::vector<float> hx(n), hy(n), hz(n);
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    for (size_t i = 0; i < n; ++i) {
        float ct = U(rng), ph = 2.f * (float)M_PI * U(rng), st = std::sqrt(std::max(0.f, 1 - ct * ct));
        hx[i] = -st * std::cos(ph); hy[i] = -st * std::sin(ph); hz[i] = -ct;
    }
    const int nout = spec ? 11 : (rays || sspec) ? 4 : (mode == "pdf" ? 1 : 3);
    // conductor mode: normals (mostly facing up) and views in their upper hemisphere
    struct ConductorArgs { int type; float alpha_u; float eta[4], k[4]; float alpha_v; };
    ConductorArgs cargs = {std::getenv("KB_BECKMANN") ? 0 : 1, 0.2f, {0.143f, 0.374f, 1.442f, 0.f}, {3.983f, 2.385f, 1.603f, 0.f},
                           0.2f};
    float *cnx = nullptr, *cny = nullptr, *cnz = nullptr, *cvx = nullptr, *cvy = nullptr, *cvz = nullptr;
    if (cond || swl) {
        std::normal_distribution<float> G(0.f, 1.f);
        std::vector<float> h(6 * n);
        for (size_t i = 0; i < n; ++i) {
            float a[3] = {G(rng), G(rng), std::fabs(G(rng)) + 0.2f}, b[3] = {G(rng), G(rng), G(rng)};
            float la = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
            float d = a[0] * b[0] + a[1] * b[1] + a[2] * b[2], sg = d < 0 ? -1.f : 1.f;
            float lb = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
            const float sn = swl ? -1.f : 1.f;   // swl: wi = -normal, so wo = -wi faces the sky
            for (int c = 0; c < 3; ++c) { h[c * n + i] = sn * a[c] / la; h[(3 + c) * n + i] = sg * b[c] / lb; }
        }
        float* buf = nullptr;
        CK(hipMalloc(&buf, 6 * n * 4));
        CK(hipMemcpy(buf, h.data(), 6 * n * 4, hipMemcpyHostToDevice));
        cnx = buf; cny = buf + n; cnz = buf + 2 * n; cvx = buf + 3 * n; cvy = buf + 4 * n; cvz = buf + 5 * n;
    }
    float *wx, *wy, *wz, *out;
    CK(hipMalloc(&wx, n * 4)); CK(hipMalloc(&wy, n * 4)); CK(hipMalloc(&wz, n * 4));
    // KB_OPAD=p: output planes at pitch n + p floats (eval modes; p a multiple of 4)
    const size_t opad = std::getenv("KB_OPAD") ? std::strtoull(std::getenv("KB_OPAD"), nullptr, 10) : 0;
    CK(hipMalloc(&out, (n + opad) * 4 * nout));
    CK(hipMemcpy(wx, hx.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wy, hy.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wz, hz.data(), n * 4, hipMemcpyHostToDevice));

    hipModule_t mod;
    CK(hipModuleLoad(&mod, hsaco.c_str()));
    LambdaSet L;
    std::memset(&L, 0, sizeof(L));
    L.m = 11;
    for (int k = 0; k < 11; ++k) { L.lo[k] = k; L.f[k] = 0.f; }
    const uint8_t* active = nullptr;
    size_t ostride = n + opad;
    float sign = -1.f;
    const double bytes = spec ? (12.0 + 44.0) * n : rays ? 44.0 * n : mode == "sample" ? 36.0 * n : mode == "pdf" ? 16.0 * n : 24.0 * n;
    // sampling inputs: u in [0,1)^2 (reuses wx / wy), outputs d (3 planes), pdf, RGB weight
    float *dd = nullptr, *pdf = nullptr, *wgt = nullptr;
    if (sampling) {
        std::vector<float> u(2 * n);
        for (auto& v : u) v = U(rng);
        // KB_SORT_U=1: u.x ascending, so every wave is all-sky or all-sun (the divergence-free
        // bound of sample_direction; outputs differ from the unsorted run by construction)
        // KB_SORT_U=2: only partitioned, sky picks (u.x < w_sky) first, each class in its
        // random order (the bound of removing the sky/sun divergence alone)
        // KB_UX_CLASS=sky / sun: every sample a sky (u.x in [0, w_sky)) or a sun pick (the
        // per-class cost of sample_direction)
        if (const char* uc = std::getenv("KB_UX_CLASS")) {
            const float ws = model.kargs().w_sky;
            const bool sky = std::string(uc) == "sky";
            for (size_t i = 0; i < n; ++i) u[i] = sky ? u[i] * ws * 0.999999f : ws + (1.f - ws) * u[i];
            for (size_t i = 0; i < n; ++i) u[i] = sky ? std::min(u[i], std::nextafter(ws, 0.f)) : std::max(u[i], ws);
        }
        if (const char* su = std::getenv("KB_SORT_U")) {
            if (std::atoi(su) == 2) {
                const float ws = model.kargs().w_sky;
                std::stable_partition(u.begin(), u.begin() + n, [ws](float x) { return x < ws; });
            } else {
                std::sort(u.begin(), u.begin() + n);
            }
        }
        CK(hipMemcpy(wx, u.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(wy, u.data() + n, n * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&dd, 3 * n * 4)); CK(hipMalloc(&pdf, n * 4)); CK(hipMalloc(&wgt, 4 * n * 4));
        if (mode == "pdf") {   // directions on the whole sphere
            for (size_t i = 0; i < n; ++i) {
                float ct = 2 * U(rng) - 1, ph = 2.f * (float)M_PI * U(rng), st = std::sqrt(std::max(0.f, 1 - ct * ct));
                hx[i] = st * std::cos(ph); hy[i] = st * std::sin(ph); hz[i] = ct;
            }
            CK(hipMemcpy(dd, hx.data(), n * 4, hipMemcpyHostToDevice));
            CK(hipMemcpy(dd + n, hy.data(), n * 4, hipMemcpyHostToDevice));
            CK(hipMemcpy(dd + 2 * n, hz.data(), n * 4, hipMemcpyHostToDevice));
        }
    }
    // KB_COLD=k: rotate over k distinct input batches so inputs cannot stay in the
    // 256 MiB Infinity Cache (rgb / spec modes).
    const int cold = std::getenv("KB_COLD") ? std::max(1, std::atoi(std::getenv("KB_COLD"))) : 1;
    std::vector<float*> cx(cold, wx), cy(cold, wy), cz(cold, wz);
    for (int c = 1; c < cold; ++c) {
        CK(hipMalloc(&cx[c], n * 4)); CK(hipMalloc(&cy[c], n * 4)); CK(hipMalloc(&cz[c], n * 4));
        CK(hipMemcpy(cx[c], wx, n * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(cy[c], wy, n * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(cz[c], wz, n * 4, hipMemcpyDeviceToDevice));
    }
    const float* nullf = nullptr;
    int nl4 = 4;
    float* lamp = nullptr;
    if (sspec || rays) {
        std::vector<float> l(4 * n);
        for (auto& v : l) v = 360.f + 360.f * U(rng);
        CK(hipMalloc(&lamp, 4 * n * 4));
        CK(hipMemcpy(lamp, l.data(), 4 * n * 4, hipMemcpyHostToDevice));
    }
    const bool full = std::getenv("KB_SAMPLE_FULL") != nullptr;
    const float *fpx = nullptr, *fpy = nullptr, *fpz = nullptr;
    float *fdist = nullptr, *fox = nullptr, *foy = nullptr, *foz = nullptr;
    if (full) {   // it.p: 3 distinct planes of random points (as bench.py's general call); outputs: 4 more planes
        std::vector<float> hp(3 * n);
        for (auto& v : hp) v = 20.f * U(rng) - 10.f;
        float* pin = nullptr;
        CK(hipMalloc(&pin, 3 * n * 4));
        CK(hipMemcpy(pin, hp.data(), 3 * n * 4, hipMemcpyHostToDevice));
        fpx = pin; fpy = pin + n; fpz = pin + 2 * n;
        float* buf = nullptr;
        CK(hipMalloc(&buf, 4 * n * 4));
        fdist = buf; fox = buf + n; foy = buf + 2 * n; foz = buf + 3 * n;
    }
    float* nullo = nullptr;
    size_t zero = 0;
    int nl0 = 0;
    float *ddy = dd ? dd + n : nullptr, *ddz = dd ? dd + 2 * n : nullptr;
    std::vector<float> ref;
    for (int a = 6; a < argc; ++a) {
        hipFunction_t f;
        CK(hipModuleGetFunction(&f, mod, argv[a]));
        std::string name = argv[a];
        int vec = name.find("_v4") != std::string::npos ? 4 : (name.find("_v2") != std::string::npos ? 2 : 1);
        if (name.find("_u2") != std::string::npos) vec = 8;
        if (name.find("_u4") != std::string::npos) vec = 16;
        for (int mult : bpcu) {
            size_t items = n / vec;
            unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>((items + 255) / 256, (size_t)cu * mult));
            void* args_rgb[] = {&K, &wx, &wy, &wz, &active, &n, &out, &ostride, &sign};
            void* args_spec[] = {&K, &L, &wx, &wy, &wz, &active, &n, &out, &ostride, &sign};
            void* args_sample[] = {&K, &wx, &wy, &nullf, &nullf, &nullf, sspec ? (void*)&lamp : (void*)&nullf,
                                   sspec ? (void*)&n : (void*)&zero, sspec ? (void*)&nl4 : (void*)&nl0, &active, &n,
                                   &dd, &ddy, &ddz, &pdf, &nullo, &nullo, &nullo, &nullo, &wgt, &n};
            // KB_SAMPLE_FULL=1: the general call, it.p in, ds.dist and ds.p out (Mitsuba's DirectionSample)
            void* args_sample_full[] = {&K, &wx, &wy, &fpx, &fpy, &fpz, sspec ? (void*)&lamp : (void*)&nullf,
                                        sspec ? (void*)&n : (void*)&zero, sspec ? (void*)&nl4 : (void*)&nl0, &active, &n,
                                        &dd, &ddy, &ddz, &pdf, &fdist, &fox, &foy, &foz, &wgt, &n};
            void* args_pdf[] = {&K, &dd, &ddy, &ddz, &active, &n, &pdf};
            void* args_rays[] = {&K, &wx, &wy, &wz, &lamp, &n, &nl4, &active, &n, &out, &ostride, &sign};
            uint32_t cseed = 7, cspp = 4;
            void* args_cond[] = {&K, &cargs, &cnx, &cny, &cnz, &cvx, &cvy, &cvz, sspec ? (void*)&lamp : (void*)&nullf,
                                 sspec ? (void*)&n : (void*)&zero, sspec ? (void*)&nl4 : (void*)&nl0, &cseed, &cspp,
                                 &active, &zero, &n, &out, &ostride};
            void* args_diff[] = {&K, &cnx, &cny, &cnz, &nullf, sspec ? (void*)&lamp : (void*)&nullf,
                                 sspec ? (void*)&n : (void*)&zero, sspec ? (void*)&nl4 : (void*)&nl0, &cseed, &cspp,
                                 &active, &zero, &n, &out, &ostride};
            // sample_ray: wavelength sample = u.x plane, sample2 = (u.x, u.y), sample3 = (u.y, u.x);
            // outputs o (3 planes of out), d (dd), lambda (lamo), weight (wgt)
            static float* lamo = nullptr;
            if ((sray || swl) && !lamo) CK(hipMalloc(&lamo, 4 * n * 4));
            static float* rayo = nullptr;
            if (sray && !rayo) CK(hipMalloc(&rayo, 3 * n * 4));
            float *ryx = rayo, *ryy = rayo ? rayo + n : nullptr, *ryz = rayo ? rayo + 2 * n : nullptr;
            void* args_sray[] = {&K, &wx, &wx, &wy, &wy, &wx, &active, &n, &ryx, &ryy, &ryz, &dd, &ddy, &ddz, &lamo, &n,
                                 &wgt, &n};
            void* args_swl[] = {&K, &cnx, &cny, &cnz, &wx, &active, &n, &lamo, &n, &wgt, &n};
            void** args = sray ? args_sray : swl ? args_swl : spec ? args_spec : rays ? args_rays
                                            : mode == "sample" ? (full ? args_sample_full : args_sample)
                                            : mode == "pdf" ? args_pdf : mode == "diffuse" ? args_diff
                                            : cond ? args_cond : args_rgb;
            // KB_LDS: dynamic LDS bytes per workgroup in the timed loop (an occupancy cap)
            const unsigned kb_lds = std::getenv("KB_LDS") ? std::atoi(std::getenv("KB_LDS")) : 0;
            for (int w = 0; w < 3; ++w) CK(hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, kb_lds, nullptr, args, nullptr));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0, nullptr));
            for (int it = 0; it < iters; ++it) {
                if (cold > 1) { wx = cx[it % cold]; wy = cy[it % cold]; wz = cz[it % cold]; }
                CK(hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, kb_lds, nullptr, args, nullptr));
            }
            wx = cx[0]; wy = cy[0]; wz = cz[0];
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            double us = 1e3 * ms / iters;
            // checksum against the first kernel
            // sample mode: d (3 planes), pdf and the weight (3 planes) all enter the check
            const bool samp7 = mode == "sample" || sray;
            std::vector<float> h((size_t)(samp7 ? 7 : nout) * n);
            if (samp7) {
                CK(hipMemcpy(h.data(), dd, 3 * n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h.data() + 3 * n, pdf, n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h.data() + 4 * n, wgt, 3 * n * 4, hipMemcpyDeviceToHost));
            } else {
                if (opad && !(sampling && !cond))
                    for (int c = 0; c < nout; ++c)
                        CK(hipMemcpy(h.data() + (size_t)c * n, out + (size_t)c * ostride, n * 4, hipMemcpyDeviceToHost));
                else
                    CK(hipMemcpy(h.data(), sampling && !cond ? (mode == "pdf" ? pdf : wgt) : out, h.size() * 4, hipMemcpyDeviceToHost));
            }
            double maxrel = 0;
            size_t ndiff = 0;
            if (ref.empty()) ref = h;
            else
                for (size_t i = 0; i < h.size(); ++i) {
                    if (std::memcmp(&h[i], &ref[i], 4) != 0) ++ndiff;
                    double d = std::fabs((double)h[i] - ref[i]) / std::max(1e-6, std::fabs((double)ref[i]));
                    if (d > maxrel) maxrel = d;
                }
            if (kb_lds) std::printf("[lds %u] ", kb_lds);
            std::printf("%-36s bpcu=%-4d grid=%-6u %9.2f us  %7.1f GB/s  %.3e evals/s  maxrel-vs-first=%.2e  "
                        "bitdiff=%zu\n",
                        argv[a], mult, grid, us, bytes / (us * 1e-6) / 1e9, (spec ? 11.0 : 1.0) * n / (us * 1e-6),
                        maxrel, ndiff);
            std::fflush(stdout);
            // KB_AB=<other.hsaco>: the same kernel from a second code object, timed in
            // alternating bursts (KB_AB_ROUNDS of them) so clock and thermal drift hit
            // both alike; prints medians and the median per-round ratio other/this.
            if (const char* ab = std::getenv("KB_AB")) {
                hipModule_t mod_b;
                CK(hipModuleLoad(&mod_b, ab));
                hipFunction_t fb;
                // KB_AB_NAME: a different kernel of the other code object (e.g. a variant)
                const char* bname = std::getenv("KB_AB_NAME") ? std::getenv("KB_AB_NAME") : argv[a];
                CK(hipModuleGetFunction(&fb, mod_b, bname));
                const int rounds = std::getenv("KB_AB_ROUNDS") ? std::atoi(std::getenv("KB_AB_ROUNDS")) : 20;
                std::vector<double> ta, tb, ratio;
                // KB_AB_LDS_A / KB_AB_LDS_B: dynamic LDS bytes per workgroup for this / the other
                // side (an occupancy cap without a code change)
                const unsigned lds_a = std::getenv("KB_AB_LDS_A") ? std::atoi(std::getenv("KB_AB_LDS_A")) : 0;
                const unsigned lds_b = std::getenv("KB_AB_LDS_B") ? std::atoi(std::getenv("KB_AB_LDS_B")) : 0;
                auto burst = [&](hipFunction_t fn) {
                    const unsigned lds = fn == f ? lds_a : lds_b;
                    CK(hipEventRecord(e0, nullptr));
                    for (int it = 0; it < iters; ++it)
                        CK(hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, lds, nullptr, args, nullptr));
                    CK(hipEventRecord(e1, nullptr));
                    CK(hipEventSynchronize(e1));
                    float t = 0;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    return 1e3 * t / iters;
                };
                for (int w = 0; w < 3; ++w) CK(hipModuleLaunchKernel(fb, grid, 1, 1, 256, 1, 1, 0, nullptr, args, nullptr));
                for (int r = 0; r < rounds; ++r) {
                    double x = burst(f), y = burst(fb);
                    ta.push_back(x); tb.push_back(y); ratio.push_back(y / x);
                }
                auto median = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
                std::printf("  A/B %-30s this %8.2f us  other(%s) %8.2f us  median(other/this) %.4f  (%d rounds x %d)\n",
                            argv[a], median(ta), bname, median(tb), median(ratio), rounds, iters);
                if (!sampling) {   // eval modes: the two code objects' outputs, bit for bit
                    std::vector<float> ha(h.size()), hb(h.size());
                    auto grab = [&](hipFunction_t fn, std::vector<float>& dst) {
                        CK(hipMemset(out, 0xFF, (n + opad) * 4 * nout));
                        CK(hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, nullptr, args, nullptr));
                        CK(hipDeviceSynchronize());
                        for (int c = 0; c < nout; ++c)
                            CK(hipMemcpy(dst.data() + (size_t)c * n, out + (size_t)c * ostride, n * 4, hipMemcpyDeviceToHost));
                    };
                    grab(f, ha);
                    grab(fb, hb);
                    size_t nd = 0;
                    for (size_t q = 0; q < ha.size(); ++q) nd += std::memcmp(&ha[q], &hb[q], 4) != 0;
                    std::printf("  A/B outputs: %zu of %zu floats differ\n", nd, ha.size());
                }
                std::fflush(stdout);
                CK(hipModuleUnload(mod_b));
            }
        }
    }
    return 0;
}
