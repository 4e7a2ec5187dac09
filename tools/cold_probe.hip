// cold_probe.hip -- the headline's access shape (read 3 fp32 planes, write 3) with the
// inputs streamed from HBM (4 rotating 201 MB batches, more than the 256 MiB Infinity
// Cache), trivial compute, in several distributions of the work:
//   gs      grid-stride, one float4 per plane per lane (the eval kernel's shape)
//   gs_ntl  the same with non-temporal loads
//   blk     each workgroup sweeps a contiguous chunk of the planes (blocked)
//   gs2     grid-stride, two float4 per plane per lane, all loads issued first
//   xcd     grid-stride over chunks mapped so consecutive chunks stay on one XCD
// plus calibration shapes: copy (1 read, 1 write plane), read3 (3 planes read, one
// float per lane written), write3 (3 planes written from registers).
// Prints us per launch and GB/s of the algorithmic bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ldv(const float* p, bool nt) {
    return nt ? __builtin_nontemporal_load((const f4*)p) : *(const f4*)p;
}
__device__ __forceinline__ void stv(float* p, f4 v) { __builtin_nontemporal_store(v, (f4*)p); }

template <bool NTL>
__global__ __launch_bounds__(256) void gs(const float* x, const float* y, const float* z, float* out, size_t n) {
    const size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f4 a = ldv(x + 4 * v, NTL), b = ldv(y + 4 * v, NTL), c = ldv(z + 4 * v, NTL);
        stv(out + 4 * v, a + b);
        stv(out + n + 4 * v, b + c);
        stv(out + 2 * n + 4 * v, a + c);
    }
}

// blocked: workgroup g owns vec4 [g * chunk, (g + 1) * chunk)
__global__ __launch_bounds__(256) void blk(const float* x, const float* y, const float* z, float* out, size_t n) {
    const size_t nv = n / 4, chunk = (nv + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * chunk, hi = std::min(nv, lo + chunk);
    for (size_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
        f4 a = ldv(x + 4 * v, false), b = ldv(y + 4 * v, false), c = ldv(z + 4 * v, false);
        stv(out + 4 * v, a + b);
        stv(out + n + 4 * v, b + c);
        stv(out + 2 * n + 4 * v, a + c);
    }
}

// two float4 per plane per lane, 'half' vec4s apart so each instruction stays coalesced
__global__ __launch_bounds__(256) void gs2(const float* x, const float* y, const float* z, float* out, size_t n) {
    const size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x * 2 + threadIdx.x; v < nv; v += 2 * stride) {
        const size_t w = v + blockDim.x;
        const bool two = w < nv;
        f4 a = ldv(x + 4 * v, false), b = ldv(y + 4 * v, false), c = ldv(z + 4 * v, false);
        f4 a2 = two ? ldv(x + 4 * w, false) : a, b2 = two ? ldv(y + 4 * w, false) : b,
           c2 = two ? ldv(z + 4 * w, false) : c;
        stv(out + 4 * v, a + b);
        stv(out + n + 4 * v, b + c);
        stv(out + 2 * n + 4 * v, a + c);
        if (two) {
            stv(out + 4 * w, a2 + b2);
            stv(out + n + 4 * w, b2 + c2);
            stv(out + 2 * n + 4 * w, a2 + c2);
        }
    }
}

// XCD-aware: hardware dispatches workgroup b to XCD b % 8; remap so the workgroups on
// one XCD sweep one contiguous eighth of the planes (grid-stride inside it)
__global__ __launch_bounds__(256) void xcd(const float* x, const float* y, const float* z, float* out, size_t n) {
    const size_t nv = n / 4;
    const unsigned nx = 8, g = gridDim.x, per = g / nx;
    const unsigned xc = blockIdx.x % nx, local = blockIdx.x / nx;
    const size_t part = (nv + nx - 1) / nx, lo = (size_t)xc * part, hi = std::min(nv, lo + part);
    const size_t stride = (size_t)per * blockDim.x;
    for (size_t v = lo + (size_t)local * blockDim.x + threadIdx.x; v < hi; v += stride) {
        f4 a = ldv(x + 4 * v, false), b = ldv(y + 4 * v, false), c = ldv(z + 4 * v, false);
        stv(out + 4 * v, a + b);
        stv(out + n + 4 * v, b + c);
        stv(out + 2 * n + 4 * v, a + c);
    }
}

__global__ __launch_bounds__(256) void copy1(const float* x, const float*, const float*, float* out, size_t n) {
    const size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) stv(out + 4 * v, ldv(x + 4 * v, false));
}

__global__ __launch_bounds__(256) void read3(const float* x, const float* y, const float* z, float* out, size_t n) {
    const size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    f4 acc = {0, 0, 0, 0};
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride)
        acc += ldv(x + 4 * v, false) + ldv(y + 4 * v, false) + ldv(z + 4 * v, false);
    if (acc.x == 1234.5f) out[0] = acc.y;   // keeps the loads
}

__global__ __launch_bounds__(256) void write3(const float* x, const float*, const float*, float* out, size_t n) {
    const size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    const f4 s = {1.f, 2.f, 3.f, 4.f};
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        stv(out + 4 * v, s);
        stv(out + n + 4 * v, s);
        stv(out + 2 * n + 4 * v, s);
    }
}

static const float *g_x[4], *g_y[4], *g_z[4];

typedef void (*Kern)(const float*, const float*, const float*, float*, size_t);

int run(const char* name, Kern k, float* out, size_t n, int cu, int mult, double bytes_per_elem) {
    unsigned grid = (unsigned)std::min<size_t>((n / 4 + 255) / 256, (size_t)cu * mult);
    for (int w = 0; w < 4; ++w) k<<<grid, 256>>>(g_x[w], g_y[w], g_z[w], out, n);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int it = 40;
    CK(hipEventRecord(e0));
    for (int i = 0; i < it; ++i) k<<<grid, 256>>>(g_x[i % 4], g_y[i % 4], g_z[i % 4], out, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / it;
    printf("%-8s bpcu=%-3d %8.2f us  %7.1f GB/s\n", name, mult, us, bytes_per_elem * n / (us * 1e-6) / 1e9);
    return 0;
}

int main() {
    const size_t n = 1 << 24;
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    float* out;
    CK(hipMalloc(&out, n * 4 * 3));
    for (int c = 0; c < 4; ++c) {
        float *a, *b, *d;
        CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&d, n * 4));
        CK(hipMemset(a, 0, n * 4)); CK(hipMemset(b, 0, n * 4)); CK(hipMemset(d, 0, n * 4));
        g_x[c] = a; g_y[c] = b; g_z[c] = d;
    }
    struct { const char* name; Kern k; double bpe; } ks[] = {
        {"gs", gs<false>, 24}, {"gs_ntl", gs<true>, 24}, {"blk", blk, 24}, {"gs2", gs2, 24}, {"xcd", xcd, 24},
        {"copy", copy1, 8}, {"read3", read3, 12}, {"write3", write3, 12}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto& k : ks)
            for (int mult : {4, 8, 16, 32, 64})
                if (run(k.name, k.k, out, n, cu, mult, k.bpe)) return 1;
    return 0;
}
