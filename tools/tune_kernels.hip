// tune_kernels.hip -- experimental variants of the product kernels for
// tools/kbench (never loaded by the product).  Includes the product source so
// every variant shares its device code.
#include "../mitsuba3-sunsky_amd/csrc/sunsky_kernels.hip"

#define TUNE_RGB(NAME, VEC, ATTR)                                                                          \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) ATTR void NAME(                                       \
        SunskyKArgs K, const float* wx, const float* wy, const float* wz, const uint8_t* active, size_t n,  \
        float* out, size_t ostride, float sign) {                                                           \
        (void)sign; eval_rgb_body<VEC, true, true>(K, wx, wy, wz, active, n, out, ostride);                             \
    }
#define NOATTR
TUNE_RGB(tune_rgb_v4_w8, 4, __attribute__((amdgpu_waves_per_eu(8, 8))))
TUNE_RGB(tune_rgb_v4_w4, 4, __attribute__((amdgpu_waves_per_eu(4, 4))))
TUNE_RGB(tune_rgb_v2, 2, NOATTR)
TUNE_RGB(tune_rgb_v2_w8, 2, __attribute__((amdgpu_waves_per_eu(8, 8))))

#define TUNE_SPEC(NAME, VEC, ATTR)                                                                         \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) ATTR void NAME(                                       \
        SunskyKArgs K, LambdaSet L, const float* wx, const float* wy, const float* wz, const uint8_t* active,\
        size_t n, float* out, size_t ostride, float sign) {                                                 \
        (void)L;                                                                                            \
        (void)sign; eval_spec_nodes_body<VEC, true, true>(K, wx, wy, wz, active, n, out, ostride);                      \
    }
TUNE_SPEC(tune_spec_nodes_v2_w8, 2, __attribute__((amdgpu_waves_per_eu(8, 8))))
TUNE_SPEC(tune_spec_nodes_v4, 4, NOATTR)
TUNE_SPEC(tune_spec_nodes_v1, 1, NOATTR)
TUNE_SPEC(tune_spec_nodes_v1_w8, 1, __attribute__((amdgpu_waves_per_eu(8, 8))))

// Grid-stride loop unrolled U times: each lane issues the loads of U vec4
// groups before computing any of them (more bytes in flight per wave).
template <int U, bool FAST>
__device__ __forceinline__ void eval_rgb_body_u(const SunskyKArgs& K, const float* __restrict__ wx,
                                                const float* __restrict__ wy, const float* __restrict__ wz,
                                                size_t n, float* __restrict__ out, size_t ostride, float sign) {
    const size_t nvec = n / 4;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v0 < nvec; v0 += U * stride) {
        float x[U][4], y[U][4], z[U][4];
        bool m[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = v0 + u * stride;
            if (v < nvec) load_dirs<4>(wx, wy, wz, nullptr, v * 4, x[u], y[u], z[u], m[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = v0 + u * stride;
            if (v >= nvec) break;
            float r[4], g[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float o[3];
                eval_rgb_local<FAST>(K, K.sun_table, to_local(K, mk3(sign * x[u][j], sign * y[u][j], sign * z[u][j])),
                                     m[u][j], o);
                r[j] = o[0]; g[j] = o[1]; b[j] = o[2];
            }
            store_vec<4>(out, v * 4, r);
            store_vec<4>(out + ostride, v * 4, g);
            store_vec<4>(out + 2 * ostride, v * 4, b);
        }
    }
}
#define TUNE_RGB_U(NAME, U)                                                                                 \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) void NAME(                                            \
        SunskyKArgs K, const float* wx, const float* wy, const float* wz, const uint8_t* active, size_t n,  \
        float* out, size_t ostride, float sign) {                                                           \
        (void)active;                                                                                       \
        eval_rgb_body_u<U, true>(K, wx, wy, wz, n, out, ostride, sign);                                     \
    }
TUNE_RGB_U(tune_rgb_u2, 2)
TUNE_RGB_U(tune_rgb_u4, 4)

// Software-pipelined grid-stride loop: the next group's loads are issued before
// the current group's compute.
template <bool FAST>
__device__ __forceinline__ void eval_rgb_body_pf(const SunskyKArgs& K, const float* __restrict__ wx,
                                                 const float* __restrict__ wy, const float* __restrict__ wz,
                                                 size_t n, float* __restrict__ out, size_t ostride, float sign) {
    const size_t nvec = n / 4;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    float nx[4], ny[4], nz[4];
    bool nm[4];
    if (v < nvec) load_dirs<4>(wx, wy, wz, nullptr, v * 4, nx, ny, nz, nm);
    for (; v < nvec; v += stride) {
        float x[4], y[4], z[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) { x[j] = nx[j]; y[j] = ny[j]; z[j] = nz[j]; }
        if (v + stride < nvec) load_dirs<4>(wx, wy, wz, nullptr, (v + stride) * 4, nx, ny, nz, nm);
        float r[4], g[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float o[3];
            eval_rgb_local<FAST>(K, K.sun_table, to_local(K, mk3(sign * x[j], sign * y[j], sign * z[j])), true, o);
            r[j] = o[0]; g[j] = o[1]; b[j] = o[2];
        }
        store_vec<4>(out, v * 4, r);
        store_vec<4>(out + ostride, v * 4, g);
        store_vec<4>(out + 2 * ostride, v * 4, b);
    }
}
extern "C" __global__ __launch_bounds__(SS_BLOCK) void tune_rgb_pf_v4(
    SunskyKArgs K, const float* wx, const float* wy, const float* wz, const uint8_t* active, size_t n,
    float* out, size_t ostride, float sign) {
    (void)active;
    eval_rgb_body_pf<true>(K, wx, wy, wz, n, out, ostride, sign);
}
