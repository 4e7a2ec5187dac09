#!/bin/bash
# sample_direction split: access shape alone (bw_probe samp_r2w7), compute alone
# (probe_nostore build), and the product kernel, 64M RGB samples.
set -o pipefail
R=$GRAFT_REPO_ROOT
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
O=$R/gpurun_out/split.log
mkdir -p $R/gpurun_out; : > $O
timeout -k 10 120 $R/tools/build/bw_probe >> $O 2>&1 || exit 1
K=sunsky_sample_direction_rgb_lean_fast
KB_AB=$R/tools/build/probe_nostore.hsaco KB_AB_ROUNDS=10 timeout -k 10 200 $R/tools/build/kbench \
    $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco sample 67108864 10 64 $K >> $O 2>&1 || exit 1
KB_AB=$R/tools/build/probe_nostore.hsaco KB_AB_ROUNDS=10 timeout -k 10 200 $R/tools/build/kbench \
    $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco pdf 67108864 10 64 sunsky_pdf_direction_v4_fast >> $O 2>&1 || exit 1
