#!/bin/bash
# A/B timing of one kernel: tools/build/ab_base.hsaco (baseline build) vs the product
# code object, interleaved in one process sequence on the same box.
# usage: gpu_ab.sh <mode> <n> <kernel> [kernel...]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/ab.log
: > $O
MODE=$1; N=$2; shift 2
for rep in 1 2 3; do
  echo "== base rep $rep" >> $O
  timeout -k 10 200 $KB $R/tools/build/ab_base.hsaco $MODE $N 10 64 "$@" >> $O 2>&1 || exit 1
  echo "== new rep $rep" >> $O
  timeout -k 10 200 $KB $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco $MODE $N 10 64 "$@" >> $O 2>&1 || exit 1
done
