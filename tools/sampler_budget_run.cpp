// sampler_budget_run.cpp -- runs the phase kernels of tools/sampler_budget.hip on the C4
// emitter (T = 3, albedo 0.3, sun at 30 deg) for 2^20 sky picks, so that rocprofv3 --pmc
// counts each phase's dynamic instructions (tools/sampler_budget.py --pmc reads them).
//   sampler_budget_run <sampler_budget.hsaco>
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "sunsky_model.h"

using namespace sunsky;

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: sampler_budget_run <sampler_budget.hsaco>\n");
        return 2;
    }
    const char* pack = std::getenv("SUNSKY_AMD_DATASET");
    Properties props;
    props.set_float("turbidity", 3.0);
    props.set_float("albedo", 0.3);
    const double th = (90.0 - 30.0) * M_PI / 180.0;
    props.set_vector3("sun_direction", (float)std::sin(th), 0.f, (float)std::cos(th));
    SunskyModel model(props, kRGB, kJit, pack ? pack : "mitsuba3-sunsky_amd/data/sunsky_datasets.pack");
    float *d_sun, *d_ld;
    CK(hipMalloc(&d_sun, sizeof(float) * kSunRgbTableSize));
    CK(hipMalloc(&d_ld, sizeof(float) * 66));
    CK(hipMemcpy(d_sun, model.sun_table().data(), sizeof(float) * model.sun_table().size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ld, model.sun_ld().data(), sizeof(float) * 66, hipMemcpyHostToDevice));
    SunskyKArgs hk = model.kargs();
    hk.sun_table = d_sun;
    hk.sun_ld = d_ld;
    SunskyKArgs* K = nullptr;
    CK(hipMalloc(&K, sizeof(SunskyKArgs)));
    CK(hipMemcpy(K, &hk, sizeof(SunskyKArgs), hipMemcpyHostToDevice));
    // the kernels index in[i], in[i + 65536], ... and out likewise: 65536 lanes per launch,
    // u.x a sky pick (u.x < w_sky), u.y uniform; 16 launches
    constexpr int n = 65536;
    std::mt19937 rng(3);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    std::vector<float> u(3 * n), d(3 * n);
    for (int i = 0; i < n; ++i) { u[i] = U(rng) * hk.w_sky * 0.999999f; u[n + i] = U(rng); u[2 * n + i] = 0.f; }
    float *din, *dout, *ddir;
    CK(hipMalloc(&din, 7 * n * 4));
    CK(hipMalloc(&dout, 7 * n * 4));
    CK(hipMalloc(&ddir, 3 * n * 4));
    CK(hipMemcpy(din, u.data(), 3 * n * 4, hipMemcpyHostToDevice));
    hipModule_t mod;
    CK(hipModuleLoad(&mod, argv[1]));
    auto run = [&](const char* name, float* in) {
        hipFunction_t f;
        CK(hipModuleGetFunction(&f, mod, name));
        void* args[] = {&K, &in, &dout};
        for (int r = 0; r < 16; ++r) CK(hipModuleLaunchKernel(f, n / 256, 1, 1, 256, 1, 1, 0, nullptr, args, nullptr));
        CK(hipDeviceSynchronize());
        std::printf("%s: 16 x %d lanes\n", name, n);
    };
    run("budget_baseline", din);
    run("budget_sky_direction", din);
    CK(hipMemcpy(ddir, dout, 3 * n * 4, hipMemcpyDeviceToDevice));   // the sampled directions feed pdf / eval
    run("budget_sky_pdf", ddir);
    run("budget_sky_eval", ddir);
    run("budget_sky_pick", din);
    // sun picks: u.x in [w_sky, 1)
    for (int i = 0; i < n; ++i) u[i] = hk.w_sky + (1.f - hk.w_sky) * U(rng);
    CK(hipMemcpy(din, u.data(), n * 4, hipMemcpyHostToDevice));
    run("budget_sun_pick", din);
    return 0;
}
