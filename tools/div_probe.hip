// div_probe.hip -- checks div_by_rcp (csrc/sunsky_kernels.hip, Markstein) against the
// correctly rounded division on the device: every float a in [2^-100, 1) for a set
// of divisors b; prints the mismatch count and the first few mismatches.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float div_by_rcp(float a, float b, float rb) {
    if (fabsf(a) >= 0x1p-100f && fabsf(rb) <= 0x1p100f) {
        const float q = a * rb;
        return fmaf(fmaf(-q, b, a), rb, q);
    }
    return a / b;
}

__global__ void k(const float* bs, int nb, unsigned long long* bad, float* ex) {
    const unsigned lo = 0x0d800000u, hi = 0x3f800000u;   // [2^-100, 1)
    for (int j = 0; j < nb; ++j) {
        const float b = bs[j];
        const float rb = 1.f / b;
        for (unsigned u = lo + (blockIdx.x * blockDim.x + threadIdx.x); u < hi; u += gridDim.x * blockDim.x) {
            float a;
            __builtin_memcpy(&a, &u, 4);
            const float q1 = div_by_rcp(a, b, rb), q = a / b;
            if (q1 != q) {
                unsigned long long c = atomicAdd(bad, 1ull);
                if (c < 4) { ex[3 * c] = a; ex[3 * c + 1] = b; ex[3 * c + 2] = q1 - q; }
            }
        }
    }
}

int main() {
    const unsigned bbits[] = {0x3ead5aaa, 0x3dcb9ab4, 0x3eb5e8ec, 0x3d5dea29, 0x3e02c176, 0x3cf67a8b, 0x3cd9d85f,
                              0x3dae5a91, 0x3dc47d14, 0x3da2508b, 0x3d3e1979, 0x3e95d4d8};
    float bs[sizeof(bbits) / 4];
    std::memcpy(bs, bbits, sizeof(bbits));
    const int nb = sizeof(bs) / sizeof(bs[0]);
    float *dbs, *dex;
    unsigned long long* dbad;
    hipMalloc(&dbs, sizeof(bs));
    hipMalloc(&dex, 12 * 4);
    hipMalloc(&dbad, 8);
    hipMemcpy(dbs, bs, sizeof(bs), hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 8);
    k<<<4096, 256>>>(dbs, nb, dbad, dex);
    unsigned long long bad = 0;
    float ex[12];
    hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(ex, dex, 48, hipMemcpyDeviceToHost);
    printf("mismatches: %llu\n", bad);
    for (int i = 0; i < 4 && i < (int)bad; ++i) printf("a=%a b=%a diff=%a\n", ex[3 * i], ex[3 * i + 1], ex[3 * i + 2]);
    return 0;
}
