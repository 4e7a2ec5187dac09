#!/bin/bash
# Spectral LEAN sampling: bitwise test vs the general kernel, then an interleaved A/B of the
# 4-wavelength body against the previous loop form (same code object).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_entry_points.py -m gpu -q -x \
    -k "lean_kernel_bitwise or sample_direction_and_pdf or c4_sampling_at_30 or spectral_sampling_64M" --timeout 200 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 && \
KB_SAMPLE_SPEC=1 KB_AB=$H KB_AB_NAME=sunsky_sample_direction_spec_lean_loop_fast KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 \
    $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_spec_lean_fast > gpurun_out/ab.log 2>&1
