#!/bin/bash
# All GPU tests, then A/B against the HEAD build (KB_AB): the sorted LEAN sampling kernel, the
# headline and the C3 kernels; the sorted kernel vs the unsorted one; a grid sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=gpurun_out/ws5.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=30 timeout -k 10 200 $R/tools/build/kbench $H rgb 16777216 20 64 sunsky_eval_rgb_v4_fast >> $O 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H spec 16777216 20 64 sunsky_eval_spec_nodes_v4_fast >> $O 2>&1 || exit 1
KB_AB=$H KB_AB_NAME=sunsky_sample_direction_rgb_lean_plain_fast KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 20 16,32,64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1
