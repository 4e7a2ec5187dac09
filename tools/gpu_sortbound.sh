#!/bin/bash
# Divergence-free bound of sample_direction: the LEAN kernel on u.x sorted (KB_SORT_U) vs unsorted.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/sortbound.log
for i in 1 2; do
timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 20 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
KB_SORT_U=1 timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 20 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
KB_SORT_U=2 timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 20 64 sunsky_sample_direction_rgb_lean_fast >> $O 2>&1 || exit 1
done
