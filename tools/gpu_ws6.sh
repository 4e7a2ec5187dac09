#!/bin/bash
# Sorted LEAN sampling variants (hoisted channel constants, 4 waves/SIMD vs re-read per pass, 5 waves)
# against the HEAD build and the unsorted kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/ws6.log
timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast sunsky_sample_direction_rgb_lean_nh_fast >> $O 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
KB_AB=$H KB_AB_NAME=sunsky_sample_direction_rgb_lean_nh_fast KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
KB_AB=$H KB_AB_NAME=sunsky_sample_direction_rgb_lean_plain_fast KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1
