// valu_probe2.hip -- VALU issue cost per wave64 instruction on the device this runs on, with
// the instruction forced by inline asm (tools/valu_probe.hip let the compiler SLP-pack its
// "scalar" FMA chains into v_pk_fma_f32, so its scalar figure was a packed one).
// 8 independent chains per lane; every kernel launched with enough waves to fill all SIMDs
// (blocks x 4 waves, 1..8 waves per SIMD).  Prints SIMD-cycles per wave-instruction at the
// clock given by --clk (default 2.4 GHz) and the implied rate.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

#define BODY8(STMT) { STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7) }

__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 0.001f + j;
    for (int i = 0; i < iters; ++i) {
#define S(j) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(a), "v"(b));
        BODY8(S)
#undef S
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mul(float* out, int iters, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 0.001f + j;
    for (int i = 0; i < iters; ++i) {
#define S(j) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[j]) : "v"(a));
        BODY8(S)
#undef S
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s + b;
}

__global__ __launch_bounds__(256) void k_pkfma(float* out, int iters, float a, float b) {
    f2 x[8];
    f2 va = {a, a}, vb = {b, b};
    for (int j = 0; j < 8; ++j) x[j] = (f2){threadIdx.x * 0.001f + j, j * 0.5f};
    for (int i = 0; i < iters; ++i) {
#define S(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(va), "v"(vb));
        BODY8(S)
#undef S
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
    if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pkmul(float* out, int iters, float a, float b) {
    f2 x[8];
    f2 va = {a, a};
    for (int j = 0; j < 8; ++j) x[j] = (f2){threadIdx.x * 0.001f + j, j * 0.5f};
    for (int i = 0; i < iters; ++i) {
#define S(j) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x[j]) : "v"(va));
        BODY8(S)
#undef S
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
    if (s == 1.2345f) out[threadIdx.x] = s + b;
}

__global__ __launch_bounds__(256) void k_exp(float* out, int iters, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-6f + j * 1e-3f;
    for (int i = 0; i < iters; ++i) {
#define S(j) asm volatile("v_exp_f32 %0, %0" : "+v"(x[j]));
        BODY8(S)
#undef S
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s + a + b;
}

// 2 v_exp_f32 + 6 v_fma_f32 per iteration, independent: co-issue of the transcendental?
__global__ __launch_bounds__(256) void k_mix(float* out, int iters, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-6f + j * 1e-3f;
    for (int i = 0; i < iters; ++i) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[0]));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[1]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[2]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[3]) : "v"(a), "v"(b));
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[4]));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[5]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[7]) : "v"(a), "v"(b));
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_cndmask(float* out, int iters, float a, float b) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 0.001f + j;
    const bool c = threadIdx.x & 1;
    for (int i = 0; i < iters; ++i) {
#define S(j) x[j] = c ? x[j] + a : x[j]; asm volatile("" : "+v"(x[j]));
        BODY8(S)
#undef S
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    if (s == 1.2345f) out[threadIdx.x] = s + b;
}

template <typename K>
int run(const char* name, K kern, int blocks, int iters, double instr_per_iter, double clk) {
    float* out;
    CK(hipMalloc(&out, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    kern<<<blocks, 256>>>(out, 100, 1.0000001f, 1e-7f);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        kern<<<blocks, 256>>>(out, iters, 1.0000001f, 1e-7f);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    double waves = blocks * 256.0 / 64.0;
    double winstr = waves * iters * instr_per_iter;
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("%-8s blocks=%6d waves/SIMD=%5.1f  %8.3f ms  %.2f SIMD-cycles/wave-instr @%.2f GHz\n", name, blocks,
           waves / (cu * 4.0), best, (cu * 4 * clk) / (winstr / (best * 1e-3)), clk / 1e9);
    CK(hipFree(out));
    return 0;
}

int main(int argc, char** argv) {
    const double clk = argc > 1 ? atof(argv[1]) * 1e9 : 2.4e9;
    for (int blocks : {256, 1024, 2048}) {   // 1, 4, 8 waves per SIMD on 256 CUs
        run("fma", k_fma, blocks, 20000, 8, clk);
        run("mul", k_mul, blocks, 20000, 8, clk);
        run("pk_fma", k_pkfma, blocks, 20000, 8, clk);
        run("pk_mul", k_pkmul, blocks, 20000, 8, clk);
        run("exp", k_exp, blocks, 5000, 8, clk);
        run("mix2e6f", k_mix, blocks, 10000, 8, clk);
        run("cndmask", k_cndmask, blocks, 20000, 16, clk);   // v_add + v_cndmask per element
    }
    return 0;
}
