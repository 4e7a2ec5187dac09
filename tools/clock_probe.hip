// clock_probe.hip -- the shader clock of this GPU under a VALU-bound load, for reading the
// VALU-bound sampling lines of bench.py across boxes (their time scales with the clock the
// power manager grants).  Built as tools/build/clock_probe.hsaco; bench.py loads it with
// hipModuleLoad, launches 8 workgroups of 4 waves per CU (every SIMD busy with independent
// FMA chains for tens of ms) and divides each workgroup's shader-clock cycles (clock64,
// read at its start and end) by the launch's hipEvent time.  Reads the counter only;
// results leave through vector stores.  Not part of the product.
#include <hip/hip_runtime.h>

extern "C" __global__ __launch_bounds__(256) void sunsky_tools_clock_probe(unsigned long long* out, int iters,
                                                                             float a, float b) {
    __shared__ unsigned long long t0;
    if (threadIdx.x == 0) t0 = clock64();
    __syncthreads();
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3f + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_fmaf(x[j], a, b);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += x[j];
        out[2 * blockIdx.x] = clock64() - t0;
        out[2 * blockIdx.x + 1] = s == 1.2345f ? 1ull : 0ull;
    }
}

// The shader clock DURING another kernel's burst: one wave on a side stream counts shader-clock
// cycles (s_memtime) over `ticks` of the constant 100 MHz counter (s_memrealtime), sleeping
// between reads, then exits (a time-based exit every launch reaches).  Reads counters only;
// the result leaves through a vector store.  Not part of the product.
extern "C" __global__ __launch_bounds__(64) void sunsky_tools_clock_during(unsigned long long* out,
                                                                           unsigned long long ticks) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    unsigned long long r = r0;
    while (r - r0 < ticks) {
        __builtin_amdgcn_s_sleep(8);
        r = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r - r0;
    }
}
