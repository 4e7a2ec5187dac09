#!/bin/bash
# General call without a mask (it.p in, ds.dist / ds.p out): sorted variants vs the unsorted kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/ws_pos.log
KB_SAMPLE_FULL=1 timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_fast sunsky_sample_direction_rgb_pos_sorted_fast sunsky_sample_direction_rgb_full_sorted_fast >> $O 2>&1 || exit 1
for B in sunsky_sample_direction_rgb_pos_sorted_fast sunsky_sample_direction_rgb_full_sorted_fast; do
KB_SAMPLE_FULL=1 KB_AB=$H KB_AB_NAME=$B KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_fast >> $O 2>&1 || exit 1
done
