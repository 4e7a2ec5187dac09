#!/bin/bash
# A/B timing of kernels: the product code object ("this") against
# tools/build/ab_base.hsaco ("other", a baseline build), interleaved burst by
# burst inside one kbench process (KB_AB).  median(other/this) > 1: product faster.
# usage: gpu_ab.sh <mode> <n> <kernel> [kernel...]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
O=$R/gpurun_out/ab.log
MODE=$1; N=$2; shift 2
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=${KB_AB_ROUNDS:-30} timeout -k 10 300 $R/tools/build/kbench \
    $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco $MODE $N 10 64 "$@" >> $O 2>&1
