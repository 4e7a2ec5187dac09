#!/bin/bash
# Grid sweep of the wave-sorted sample_direction kernels (plain kbench timings).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/ws_sweep.log
timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 20 ${BPCU:-4,8,16,32,64} sunsky_sample_direction_rgb_lean_fast ${VARIANTS:-sunsky_sample_direction_rgb_lean_plain_fast} >> $O 2>&1
