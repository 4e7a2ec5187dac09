#!/bin/bash
# A/B without the test suite: product kernels vs tools/build/ab_base.hsaco (KERNELS, as
# gpu_ab_sample.sh: "kernel" or "mode:kernel[:n]"), then same-object variants
# (VARIANTS: "mode:A:B" entries, gpu_ab_variant.sh).  Output: gpurun_out/ab.log, ab_variant.log.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
for mk in ${KERNELS:-}; do
  IFS=: read -r f1 f2 f3 <<< "$mk"
  if [ -z "$f2" ]; then m=sample; k=$f1; n=67108864; else m=$f1; k=$f2; n=${f3:-67108864}; fi
  KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 \
      $R/tools/build/kbench $H $m $n 10 64 $k >> $R/gpurun_out/ab.log 2>&1 || exit 1
done
for v in ${VARIANTS:-}; do
  IFS=: read -r m a b <<< "$v"
  MODE=$m A=$a B=$b bash $R/tools/gpu_ab_variant.sh || exit 1
done
