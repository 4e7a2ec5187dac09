#!/bin/bash
# Interleaved A/B of product kernels against tools/build/ab_base.hsaco (tools/mk_ab_base.sh REV).
# KERNELS: "mode:kernel:n[:ENV=VAL]" entries.  Output gpurun_out/ab.log.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
: > $R/gpurun_out/ab.log
for e in $KERNELS; do
  IFS=: read -r m k n ev <<< "$e"
  env ${ev:-KB_X=0} KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 \
      $R/tools/build/kbench $H $m $n 10 64 $k >> $R/gpurun_out/ab.log 2>&1 || exit 1
done
