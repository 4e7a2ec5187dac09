// tune_kernels.hip -- experimental variants of the product kernels for
// tools/kbench (never loaded by the product).  Includes the product source so
// every variant shares its device code.
#include "../mitsuba3-sunsky_amd/csrc/sunsky_kernels.hip"

#define TUNE_RGB(NAME, VEC, ATTR)                                                                          \
    extern "C" __global__ __launch_bounds__(SS_BLOCK) ATTR void NAME(                                       \
        SunskyKArgs K, const float* wx, const float* wy, const float* wz, const uint8_t* active, size_t n,  \
        float* out, size_t ostride, float sign) {                                                           \
        eval_rgb_body<VEC, true>(K, wx, wy, wz, active, n, out, ostride, sign);                             \
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
        eval_spec_nodes_body<VEC, true>(K, wx, wy, wz, active, n, out, ostride, sign);                      \
    }
TUNE_SPEC(tune_spec_nodes_v2_w8, 2, __attribute__((amdgpu_waves_per_eu(8, 8))))
TUNE_SPEC(tune_spec_nodes_v4, 4, NOATTR)
TUNE_SPEC(tune_spec_nodes_v1, 1, NOATTR)
TUNE_SPEC(tune_spec_nodes_v1_w8, 1, __attribute__((amdgpu_waves_per_eu(8, 8))))
