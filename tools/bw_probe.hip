// bw_probe.hip -- achievable HBM rate for the emitter kernels' access shapes:
// read 3 fp32 planes, write K fp32 planes (K = 3 RGB eval, 11 spectral broadcast),
// with trivial compute.  Calibrates the "achievable" ceiling of DESIGN.md §3.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int K, bool NT>
__global__ __launch_bounds__(256) void rw4(const float* x, const float* y, const float* z, float* out, size_t n) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f4 a = *(const f4*)(x + 4 * v), b = *(const f4*)(y + 4 * v), c = *(const f4*)(z + 4 * v);
        f4 s = a + b + c;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            f4 o = s * (float)(k + 1);
            if (NT) __builtin_nontemporal_store(o, (f4*)(out + (size_t)k * n + 4 * v));
            else *(f4*)(out + (size_t)k * n + 4 * v) = o;
        }
    }
}

template <int K, bool NT>
__global__ __launch_bounds__(256) void rw2(const float* x, const float* y, const float* z, float* out, size_t n) {
    size_t nv = n / 2, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f2 a = *(const f2*)(x + 2 * v), b = *(const f2*)(y + 2 * v), c = *(const f2*)(z + 2 * v);
        f2 s = a + b + c;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            f2 o = s * (float)(k + 1);
            if (NT) __builtin_nontemporal_store(o, (f2*)(out + (size_t)k * n + 2 * v));
            else *(f2*)(out + (size_t)k * n + 2 * v) = o;
        }
    }
}

// sample_direction's shape: read 2 planes (u), write 7 (d, pdf, RGB weight), VEC per lane
template <int VEC>
__global__ __launch_bounds__(256) void samp(const float* x, const float* y, const float* z, float* out, size_t n) {
    typedef float fv __attribute__((ext_vector_type(VEC)));
    size_t nv = n / VEC, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        fv a = *(const fv*)(x + VEC * v), b = *(const fv*)(y + VEC * v);
        fv s = a + b;
#pragma unroll
        for (int k = 0; k < 7; ++k) __builtin_nontemporal_store(s * (float)(k + 1), (fv*)(out + (size_t)k * n + VEC * v));
    }
}

// cold: rotate over 4 input batches (805 MB > the 256 MiB Infinity Cache)
static const float *g_cx[4], *g_cy[4], *g_cz[4];
static int g_cold = 1;

template <typename F>
int run(const char* name, F kern, int vec, int K, const float* x, const float* y, const float* z, float* out,
        size_t n, int cu, double bpe = 0) {
    for (int mult : {8, 16, 32, 64}) {
        unsigned grid = (unsigned)std::min<size_t>((n / vec + 255) / 256, (size_t)cu * mult);
        for (int w = 0; w < 3; ++w) kern<<<grid, 256>>>(x, y, z, out, n);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        const int it = 32;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; ++i) {
            if (g_cold > 1) { x = g_cx[i % g_cold]; y = g_cy[i % g_cold]; z = g_cz[i % g_cold]; }
            kern<<<grid, 256>>>(x, y, z, out, n);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        double us = 1e3 * ms / it, bytes = (bpe > 0 ? bpe : 12.0 + 4.0 * K) * n;
        printf("%-14s K=%2d vec=%d bpcu=%-3d %8.2f us  %7.1f GB/s\n", name, K, vec, mult, us, bytes / (us * 1e-6) / 1e9);
    }
    return 0;
}

int main() {
    const size_t n = 1 << 24;
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    float *x, *y, *z, *out;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&z, n * 4)); CK(hipMalloc(&out, n * 4 * 11));
    CK(hipMemset(x, 0, n * 4)); CK(hipMemset(y, 0, n * 4)); CK(hipMemset(z, 0, n * 4));
    run("rw4_nt", rw4<3, true>, 4, 3, x, y, z, out, n, cu);
    // the same with 4 rotating input batches (cold inputs)
    g_cold = 4;
    for (int c = 0; c < 4; ++c) {
        float *a, *b, *d;
        CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&d, n * 4));
        CK(hipMemset(a, 0, n * 4)); CK(hipMemset(b, 0, n * 4)); CK(hipMemset(d, 0, n * 4));
        g_cx[c] = a; g_cy[c] = b; g_cz[c] = d;
    }
    run("rw4_nt_cold", rw4<3, true>, 4, 3, x, y, z, out, n, cu);
    g_cold = 1;
    run("rw4_nt", rw4<11, true>, 4, 11, x, y, z, out, n, cu);
    run("rw4_plain", rw4<11, false>, 4, 11, x, y, z, out, n, cu);
    run("rw2_nt", rw2<11, true>, 2, 11, x, y, z, out, n, cu);
    run("rw2_plain", rw2<11, false>, 2, 11, x, y, z, out, n, cu);
    // sampling shape at C4's 64M samples: 8 B read + 28 B written per sample
    const size_t ns = (size_t)1 << 26;
    float *sx, *sy, *so;
    CK(hipMalloc(&sx, ns * 4)); CK(hipMalloc(&sy, ns * 4)); CK(hipMalloc(&so, ns * 4 * 7));
    CK(hipMemset(sx, 0, ns * 4)); CK(hipMemset(sy, 0, ns * 4));
    run("samp_r2w7", samp<1>, 1, 7, sx, sy, sy, so, ns, cu, 36.0);
    run("samp_r2w7", samp<2>, 2, 7, sx, sy, sy, so, ns, cu, 36.0);
    run("samp_r2w7", samp<4>, 4, 7, sx, sy, sy, so, ns, cu, 36.0);
    return 0;
}
