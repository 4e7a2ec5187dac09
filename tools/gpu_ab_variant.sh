#!/bin/bash
# Interleaved A/B of two kernels of the SAME code object (kbench KB_AB + KB_AB_NAME),
# plus a plain kbench line for both (maxrel-vs-first = 0 means bitwise-equal outputs).
# usage: MODE=sample N=67108864 A=<kernel> B=<kernel> bash tools/gpu_ab_variant.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
timeout -k 10 200 $R/tools/build/kbench $H ${MODE:-sample} ${N:-67108864} 10 64 $A $B >> $R/gpurun_out/ab_variant.log 2>&1 && \
KB_AB=$H KB_AB_NAME=$B KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 300 \
    $R/tools/build/kbench $H ${MODE:-sample} ${N:-67108864} 10 64 $A >> $R/gpurun_out/ab_variant.log 2>&1
