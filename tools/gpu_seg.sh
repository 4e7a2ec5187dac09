#!/bin/bash
# All GPU tests, then sample_direction (sorted LEAN) and direct_diffuse-free A/B: compare-based sun
# segment search (product) vs the cbrt search (tools/build/ab_base.hsaco built -DSS_PROBE_CBRT_SEGMENT).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=gpurun_out/seg.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=25 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=25 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_plain_fast >> $O 2>&1
