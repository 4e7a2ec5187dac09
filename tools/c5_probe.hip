// c5_probe.hip -- access-shape ceiling of configs[4]'s per-rank leg (the C3 node kernel at
// 64M directions): read 3 fp32 planes, write 11, trivial compute.  At 64M the 805 MB of
// inputs and 2.95 GB of outputs exceed the 256 MiB Infinity Cache, so every launch is cold.
// Variants of the store shape: lanes x directions per lane, plain /
// non-temporal stores, grid-stride vs contiguous spans per workgroup, and LDS-staged writes
// that emit each plane in whole contiguous rows.  Also the reads-only and writes-only legs.
// usage: c5_probe [n_dirs]   (prints one line per variant and grid; best per variant last)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int K = 11;

template <int VEC> struct V;
template <> struct V<1> { typedef float t; };
template <> struct V<2> { typedef f2 t; };
template <> struct V<4> { typedef f4 t; };

// grid-stride, VEC directions per lane, one store per plane (the node kernel's shape at VEC 4)
template <int VEC, bool NT>
__global__ __launch_bounds__(256) void gs(const float* x, const float* y, const float* z, float* out, size_t n,
                                          size_t ostride) {
    typedef typename V<VEC>::t fv;
    size_t nv = n / VEC, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        fv a = *(const fv*)(x + VEC * v), b = *(const fv*)(y + VEC * v), c = *(const fv*)(z + VEC * v);
        fv s = a + b + c;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            fv o = s * (float)(k + 1);
            if (NT) __builtin_nontemporal_store(o, (fv*)(out + (size_t)k * ostride + VEC * v));
            else *(fv*)(out + (size_t)k * ostride + VEC * v) = o;
        }
    }
}

// contiguous span per workgroup: workgroup b owns directions [b * span, (b + 1) * span),
// walked in 1024-direction steps (VEC = 4)
__global__ __launch_bounds__(256) void span4(const float* x, const float* y, const float* z, float* out, size_t n,
                                             size_t ostride) {
    const size_t nv = n / 4, per = (nv + gridDim.x - 1) / gridDim.x;
    const size_t v0 = (size_t)blockIdx.x * per, v1 = v0 + per < nv ? v0 + per : nv;
    for (size_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
        f4 a = *(const f4*)(x + 4 * v), b = *(const f4*)(y + 4 * v), c = *(const f4*)(z + 4 * v);
        f4 s = a + b + c;
#pragma unroll
        for (int k = 0; k < K; ++k) __builtin_nontemporal_store(s * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * v));
    }
}

// loads of the next group issued before this group's stores (software pipelined, VEC 4)
__global__ __launch_bounds__(256) void gs4_pf(const float* x, const float* y, const float* z, float* out, size_t n,
                                              size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    f4 a = 0, b = 0, c = 0;
    if (v < nv) { a = *(const f4*)(x + 4 * v); b = *(const f4*)(y + 4 * v); c = *(const f4*)(z + 4 * v); }
    for (; v < nv; v += stride) {
        f4 s = a + b + c;
        size_t w = v + stride;
        if (w < nv) { a = *(const f4*)(x + 4 * w); b = *(const f4*)(y + 4 * w); c = *(const f4*)(z + 4 * w); }
#pragma unroll
        for (int k = 0; k < K; ++k) __builtin_nontemporal_store(s * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * v));
    }
}

// two groups of 4 directions per lane per iteration, 1024 directions apart: 22 stores in flight
__global__ __launch_bounds__(256) void gs4x2(const float* x, const float* y, const float* z, float* out, size_t n,
                                             size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x * 2;
    for (size_t v = (size_t)blockIdx.x * blockDim.x * 2 + threadIdx.x; v < nv; v += stride) {
        size_t w = v + blockDim.x;
        f4 s0 = *(const f4*)(x + 4 * v) + *(const f4*)(y + 4 * v) + *(const f4*)(z + 4 * v);
        f4 s1 = w < nv ? *(const f4*)(x + 4 * w) + *(const f4*)(y + 4 * w) + *(const f4*)(z + 4 * w) : f4{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) {
            __builtin_nontemporal_store(s0 * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * v));
            if (w < nv) __builtin_nontemporal_store(s1 * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * w));
        }
    }
}

// G groups of 4 directions per lane per iteration, 1024 directions apart (a workgroup covers
// 1024 G contiguous directions per iteration); SEQ: each group's 11 stores before the next
// group's loads (the node kernel computing one group at a time), else all loads first and the
// stores interleaved by plane
template <int G, bool SEQ>
__global__ __launch_bounds__(256) void gs4xg(const float* x, const float* y, const float* z, float* out, size_t n,
                                             size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x * G;
    for (size_t v = (size_t)blockIdx.x * blockDim.x * G + threadIdx.x; v < nv; v += stride) {
        if constexpr (SEQ) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const size_t w = v + (size_t)g * blockDim.x;
                if (w >= nv) break;
                f4 s0 = *(const f4*)(x + 4 * w) + *(const f4*)(y + 4 * w) + *(const f4*)(z + 4 * w);
#pragma unroll
                for (int k = 0; k < K; ++k) __builtin_nontemporal_store(s0 * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * w));
            }
        } else {
            f4 s[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const size_t w = v + (size_t)g * blockDim.x;
                s[g] = w < nv ? *(const f4*)(x + 4 * w) + *(const f4*)(y + 4 * w) + *(const f4*)(z + 4 * w) : f4{0, 0, 0, 0};
            }
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const size_t w = v + (size_t)g * blockDim.x;
                    if (w < nv) __builtin_nontemporal_store(s[g] * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * w));
                }
        }
    }
}

// 8 consecutive directions per lane (two 16-byte stores per plane, adjacent)
__global__ __launch_bounds__(256) void gs8(const float* x, const float* y, const float* z, float* out, size_t n,
                                           size_t ostride) {
    size_t nv = n / 8, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        const f4* X = (const f4*)(x + 8 * v); const f4* Y = (const f4*)(y + 8 * v); const f4* Z = (const f4*)(z + 8 * v);
        f4 s0 = X[0] + Y[0] + Z[0], s1 = X[1] + Y[1] + Z[1];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            f4* o = (f4*)(out + (size_t)k * ostride + 8 * v);
            __builtin_nontemporal_store(s0 * (float)(k + 1), o);
            __builtin_nontemporal_store(s1 * (float)(k + 1), o + 1);
        }
    }
}

// plane-outer: each lane writes plane k for its 4 directions, all lanes of the workgroup
// before the next plane (a __syncthreads between planes orders the workgroup's streams)
__global__ __launch_bounds__(256) void gs4_sync(const float* x, const float* y, const float* z, float* out, size_t n,
                                                size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v0 = (size_t)blockIdx.x * blockDim.x; v0 < nv; v0 += stride) {
        size_t v = v0 + threadIdx.x;
        f4 s = 0;
        if (v < nv) s = *(const f4*)(x + 4 * v) + *(const f4*)(y + 4 * v) + *(const f4*)(z + 4 * v);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (v < nv) __builtin_nontemporal_store(s * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * v));
            if (k == 5) __syncthreads();
        }
    }
}

// reads only (the 3 input planes; one conditional store that never fires keeps them live)
__global__ __launch_bounds__(256) void rd4(const float* x, const float* y, const float* z, float* out, size_t n,
                                           size_t) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    f4 acc = 0;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride)
        acc += *(const f4*)(x + 4 * v) + *(const f4*)(y + 4 * v) + *(const f4*)(z + 4 * v);
    if (acc.x == -1234.5f) out[0] = acc.y;
}

// writes only (the 11 output planes)
__global__ __launch_bounds__(256) void wr4(const float*, const float*, const float*, float* out, size_t n,
                                           size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f4 s = {(float)v, 1.f, 2.f, 3.f};
#pragma unroll
        for (int k = 0; k < K; ++k) __builtin_nontemporal_store(s * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * v));
    }
}

// writes only, KP planes of `n` floats each at plane pitch `ostride` (VERDICT r05 next 1:
// the same total bytes as 11 planes of the node kernel, split over 1 / 3 / 6 / 11 streams)
template <int KP>
__global__ __launch_bounds__(256) void wrk(const float*, const float*, const float*, float* out, size_t n,
                                           size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f4 s = {(float)v, 1.f, 2.f, 3.f};
#pragma unroll
        for (int k = 0; k < KP; ++k) __builtin_nontemporal_store(s * (float)(k + 1), (f4*)(out + (size_t)k * ostride + 4 * v));
    }
}

// full shape with the outputs interleaved [N][11]: lane's 4 directions x 11 values are 44
// consecutive floats; store j of the wave covers f4 index (64 * 11) * wave + 64 * j + lane,
// i.e. the wave writes 11 KB contiguously (the layout re-indexed so each store is coalesced;
// the element order inside a direction's record is a relabelling, not a transpose)
__global__ __launch_bounds__(256) void gs4_aos(const float* x, const float* y, const float* z, float* out, size_t n,
                                               size_t) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f4 s = *(const f4*)(x + 4 * v) + *(const f4*)(y + 4 * v) + *(const f4*)(z + 4 * v);
        const size_t wave = v / 64, lane = v % 64;
        f4* o = (f4*)out + wave * 64 * K + lane;
#pragma unroll
        for (int k = 0; k < K; ++k) __builtin_nontemporal_store(s * (float)(k + 1), o + 64 * k);
    }
}

// the node kernel's shape with NF dependent FMAs per output element (VALU work between
// the loads and each plane's store): does the time grow as max(memory, VALU) or as their sum?
template <int NF>
__global__ __launch_bounds__(256) void gs4_alu(const float* x, const float* y, const float* z, float* out, size_t n,
                                               size_t ostride) {
    size_t nv = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        f4 s = *(const f4*)(x + 4 * v) + *(const f4*)(y + 4 * v) + *(const f4*)(z + 4 * v);
#pragma unroll 1
        for (int k = 0; k < K; ++k) {
            f4 o = s;
#pragma unroll
            for (int i = 0; i < NF; ++i) o = o * 1.0001f + (float)k;
            __builtin_nontemporal_store(o, (f4*)(out + (size_t)k * ostride + 4 * v));
        }
    }
}

typedef void (*Kern)(const float*, const float*, const float*, float*, size_t, size_t);

double run(const char* name, Kern kern, int vec, const float* x, const float* y, const float* z, float* out, size_t n,
           int cu, double bytes_per_dir, std::vector<int> mults = {4, 8, 16, 32, 64}, size_t ostride = 0) {
    if (ostride == 0) ostride = n;
    double best = 1e30;
    int bm = 0;
    for (int mult : mults) {
        unsigned grid = (unsigned)std::min<size_t>((n / vec + 255) / 256, (size_t)cu * mult);
        for (int w = 0; w < 2; ++w) kern<<<grid, 256>>>(x, y, z, out, n, ostride);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int it = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; ++i) kern<<<grid, 256>>>(x, y, z, out, n, ostride);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        double us = 1e3 * ms / it;
        printf("%-10s vec=%d bpcu=%-3d %9.1f us  %7.1f GB/s\n", name, vec, mult, us, bytes_per_dir * n / (us * 1e-6) / 1e9);
        if (us < best) { best = us; bm = mult; }
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
    }
    printf("BEST %-10s %9.1f us at bpcu=%d  %7.1f GB/s\n", name, best, bm, bytes_per_dir * n / (best * 1e-6) / 1e9);
    fflush(stdout);
    return best;
}

int pitch_main(size_t n);

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "pitch") return pitch_main(argc > 2 ? std::strtoull(argv[2], nullptr, 0) : ((size_t)1 << 26));
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : ((size_t)1 << 26);
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    float *x, *y, *z, *out;
    CK(hipMalloc(&x, n * 4));
    CK(hipMalloc(&y, n * 4));
    CK(hipMalloc(&z, n * 4));
    CK(hipMalloc(&out, n * 4 * K));
    CK(hipMemset(x, 0, n * 4));
    CK(hipMemset(y, 0, n * 4));
    CK(hipMemset(z, 0, n * 4));
    printf("n = %zu directions, 3 read + %d write planes (%.1f MB in, %.1f MB out)\n", n, K, 12.0 * n / 1e6,
           4.0 * K * n / 1e6);
    const double b = 12.0 + 4.0 * K;
    double rd = run("reads", rd4, 4, x, y, z, out, n, cu, 12.0);
    double wr = run("writes", wr4, 4, x, y, z, out, n, cu, 4.0 * K);
    printf("SERIAL_SUM %9.1f us  %7.1f GB/s\n", rd + wr, b * n / ((rd + wr) * 1e-6) / 1e9);
    run("gs4_nt", gs<4, true>, 4, x, y, z, out, n, cu, b);
    run("gs2_nt", gs<2, true>, 2, x, y, z, out, n, cu, b);
    run("gs1_nt", gs<1, true>, 1, x, y, z, out, n, cu, b);
    run("gs4_plain", gs<4, false>, 4, x, y, z, out, n, cu, b);
    run("span4", span4, 4, x, y, z, out, n, cu, b, {1, 2, 4, 8});
    run("gs4_pf", gs4_pf, 4, x, y, z, out, n, cu, b);
    run("gs4x2", gs4x2, 8, x, y, z, out, n, cu, b);
    run("gs4x2_seq", gs4xg<2, true>, 8, x, y, z, out, n, cu, b);
    run("gs4x4", gs4xg<4, false>, 16, x, y, z, out, n, cu, b);
    run("gs4x4_seq", gs4xg<4, true>, 16, x, y, z, out, n, cu, b);
    run("gs8", gs8, 8, x, y, z, out, n, cu, b);
    run("gs4_sync", gs4_sync, 4, x, y, z, out, n, cu, b);
    return 0;
}

// is the 11-plane write ceiling (4.9 TB/s at 64M, pitch n = 2^28 B) a
// property of the power-of-two plane pitch or of the stream count?  Write-only legs at
// equal total bytes over K = 1, 3, 6, 11 planes and four pitches, then the full shapes
// (gs4_nt, gs4x4_seq) at the same pitches and the interleaved [N][11] layout.
int pitch_main(size_t n) {
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t pads[] = {0, 64, 1024 + 16, (2u << 20) / 4 + 4096 / 4};
    const size_t maxpad = (2u << 20) / 4 + 4096 / 4;
    float *x, *y, *z, *out;
    CK(hipMalloc(&x, n * 4));
    CK(hipMalloc(&y, n * 4));
    CK(hipMalloc(&z, n * 4));
    const size_t total = (size_t)K * n;   // floats written per launch
    CK(hipMalloc(&out, (total + (size_t)K * maxpad) * 4));
    CK(hipMemset(x, 0, n * 4));
    CK(hipMemset(y, 0, n * 4));
    CK(hipMemset(z, 0, n * 4));
    printf("pitch probe: n = %zu directions, %zu floats written per launch (%.1f MB)\n", n, total, 4.0 * total / 1e6);
    const std::vector<int> mults = {8, 16, 32, 64};
    char name[64];
    for (size_t pad : pads) {
        // write-only, KP planes of total / KP floats each (rounded down to a multiple of 4)
        const int kps[] = {1, 3, 6, 11};
        const Kern kk[] = {wrk<1>, wrk<3>, wrk<6>, wrk<11>};
        for (int i = 0; i < 4; ++i) {
            const size_t len = (total / kps[i]) & ~(size_t)3;
            snprintf(name, sizeof name, "wr_K%d_p+%zu", kps[i], pad);
            run(name, kk[i], 4, x, y, z, out, len, cu, 4.0 * kps[i], mults, len + pad);
        }
        snprintf(name, sizeof name, "gs4_nt_p+%zu", pad);
        run(name, gs<4, true>, 4, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults, n + pad);
        snprintf(name, sizeof name, "gs4x4seq_p+%zu", pad);
        run(name, gs4xg<4, true>, 16, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults, n + pad);
    }
    run("rd_only", rd4, 4, x, y, z, out, n, cu, 12.0, mults);
    run("gs4_alu0", gs4_alu<0>, 4, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults);
    run("gs4_alu8", gs4_alu<8>, 4, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults);
    run("gs4_alu16", gs4_alu<16>, 4, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults);
    run("gs4_alu32", gs4_alu<32>, 4, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults);
    run("gs4_alu64", gs4_alu<64>, 4, x, y, z, out, n, cu, 12.0 + 4.0 * K, mults);
    run("gs4_aos", gs4_aos, 4, x, y, z, out, n & ~(size_t)255, cu, 12.0 + 4.0 * K, mults);
    return 0;
}
