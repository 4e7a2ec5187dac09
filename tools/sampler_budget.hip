// sampler_budget.hip -- instruction budget of the FAST RGB sample_direction per phase (VERDICT
// r05 next 5).  Each kernel runs ONE phase of sample_one_rgb (sunsky_kernels.hip) for one sample
// per lane, reading its inputs from and writing its outputs to global memory, so the listing of
// each holds that phase's code alone; tools/sampler_budget.py counts them (static instructions,
// rolled loops counted per trip) against a hand count of the minimum.  Probe only: compiled to
// an assembly listing, never run or shipped.
#include "sunsky_kernels.hip"

#define PHASE_KERNEL(NAME) extern "C" __global__ __launch_bounds__(256) void NAME( \
    const SunskyKArgs* __restrict__ Kp, const float* __restrict__ in, float* __restrict__ out)

// (1) the sky pick's direction: the reuse division, the guide-table search, 2 erfinv, 2 sincos
PHASE_KERNEL(budget_sky_direction) {
    const SunskyKArgs& K = *Kp;
    __shared__ SamplerLds<true, false> S;
    stage_sampler_lds<true, false>(K, &S);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float a, b;
    const float3_ d = sample_sky_or_sun<true>(K, S.tgmm, true, in[i], in[i + 65536], uniform_f(1.f / K.w_sky),
                                              uniform_f(1.f / (1.f - K.w_sky)), &a, &b);
    out[i] = d.x; out[i + 65536] = d.y; out[i + 131072] = d.z;
}

// (2) the sky pick's pdf: atan2 and the polar angle of d, the TGMM sum, the sun cone test
PHASE_KERNEL(budget_sky_pdf) {
    const SunskyKArgs& K = *Kp;
    __shared__ SamplerLds<true, false> S;
    stage_sampler_lds<true, false>(K, &S);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float skyp, sunp;
    sample_pdfs<true>(K, S.tgmm, mk3(in[i], in[i + 65536], in[i + 131072]), true, 0.f, 0.f, true, &skyp, &sunp);
    out[i] = lerpf_(sunp, skyp, K.w_sky);
}

// (3) the weight's eval() of a sky pick: dir terms, 3 sky channels (the disc branch present
// but not taken)
PHASE_KERNEL(budget_sky_eval) {
    const SunskyKArgs& K = *Kp;
    __shared__ SamplerLds<true, false> S;
    stage_sampler_lds<true, false>(K, &S);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float e[3];
    eval_rgb_local<true, true>(K, S.chans.c, K.sun_table, mk3(in[i], in[i + 65536], in[i + 131072]), true, e, S.rows);
    out[i] = e[0]; out[i + 65536] = e[1]; out[i + 131072] = e[2];
}

// (4) the whole sky pick (sample_one_rgb<FAST, sky-only>) and the whole sun pick
PHASE_KERNEL(budget_sky_pick) {
    const SunskyKArgs& K = *Kp;
    __shared__ SamplerLds<true, false> S;
    stage_sampler_lds<true, false>(K, &S);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float o[7];
    sample_one_rgb<true, 1, true>(K, S, in[i], in[i + 65536], true, uniform_f(1.f / K.w_sky),
                                  uniform_f(1.f / (1.f - K.w_sky)), o);
    for (int k = 0; k < 7; ++k) out[i + k * 65536] = o[k];
}

PHASE_KERNEL(budget_sun_pick) {
    const SunskyKArgs& K = *Kp;
    __shared__ SamplerLds<true, false> S;
    stage_sampler_lds<true, false>(K, &S);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float o[7];
    sample_one_rgb<true, 2, true>(K, S, in[i], in[i + 65536], true, uniform_f(1.f / K.w_sky),
                                  uniform_f(1.f / (1.f - K.w_sky)), o);
    for (int k = 0; k < 7; ++k) out[i + k * 65536] = o[k];
}

// the baseline every phase kernel carries: the sampler tables staged in LDS, the index, one
// load and one store
PHASE_KERNEL(budget_baseline) {
    const SunskyKArgs& K = *Kp;
    __shared__ SamplerLds<true, false> S;
    stage_sampler_lds<true, false>(K, &S);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] * S.chans.c[0].A;
}
