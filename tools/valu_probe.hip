// valu_probe.hip -- measures VALU issue rates on the device this runs on
// (fp32 FMA, packed FMA, v_exp_f32, v_rsq_f32), to ground the compute side
// of the emitter kernels' roofline (DESIGN.md "Roofline").
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float a, float b) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 0.001f + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_fmaf(x[j], a, b);
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pkfma(float* out, int iters, float a, float b) {
    f2 x[8];
    f2 va = {a, a}, vb = {b, b};
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (f2){threadIdx.x * 0.001f + j, j * 0.5f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_elementwise_fma(x[j], va, vb);
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
    if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_exp(float* out, int iters, float a, float b) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-6f + j * 1e-3f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_amdgcn_exp2f(x[j]) * a;
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_rsq(float* out, int iters, float a, float b) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = 1.f + threadIdx.x * 1e-6f + j * 1e-3f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_amdgcn_rsqf(x[j]);
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s;
}

template <typename K>
int run(const char* name, K kern, int blocks, int iters, double ops_per_iter_per_thread) {
    float* out;
    CK(hipMalloc(&out, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    kern<<<blocks, 256>>>(out, 10, 1.0000001f, 1e-7f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    kern<<<blocks, 256>>>(out, iters, 1.0000001f, 1e-7f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    double waves = blocks * 256.0 / 64.0;
    double winstr = waves * iters * ops_per_iter_per_thread;
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("%-8s blocks=%6d  %.3f ms  %.3e wave-instr/s  = %.2f SIMD-cycles/wave-instr @2.4GHz (%d CUs)\n", name, blocks,
           ms, winstr / (ms * 1e-3), (cu * 4 * 2.4e9) / (winstr / (ms * 1e-3)), cu);
    CK(hipFree(out));
    return 0;
}

int main() {
    for (int blocks : {2048, 8192}) {
        run("fma", k_fma, blocks, 20000, 8);
        run("pk_fma", k_pkfma, blocks, 20000, 8);
        run("exp2", k_exp, blocks, 5000, 16);   // exp + mul per element
        run("rsq", k_rsq, blocks, 5000, 8);
    }
    return 0;
}
