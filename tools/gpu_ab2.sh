#!/bin/bash
# A/B timing of two code objects built from sources with the same SunskyKArgs layout:
# kernels of <this.hsaco> vs <other.hsaco>, interleaved burst by burst in one kbench
# process.  median(other/this) > 1: "this" faster.
# usage: gpu_ab2.sh <this.hsaco> <other.hsaco> <mode> <n> <kernel> [kernel...]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
O=$R/gpurun_out/ab.log
THIS=$1; OTHER=$2; MODE=$3; N=$4; shift 4
echo "== $THIS vs $OTHER ($MODE $N)" >> $O
KB_AB=$OTHER KB_AB_ROUNDS=${KB_AB_ROUNDS:-20} timeout -k 10 300 $R/tools/build/kbench $THIS $MODE $N 10 64 "$@" >> $O 2>&1
