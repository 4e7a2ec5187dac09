#!/bin/bash
# Sampling parity tests, then A/B of sample_direction (product vs tools/build/ab_base.hsaco).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/t.log 2>&1 || exit 1
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
# KERNELS: "kernel" (kbench mode $MODE, default sample, 64M) or "mode:kernel[:n]"
for mk in ${KERNELS:-sunsky_sample_direction_rgb_lean_fast}; do
  IFS=: read -r f1 f2 f3 <<< "$mk"
  if [ -z "$f2" ]; then m=${MODE:-sample}; k=$f1; n=67108864; else m=$f1; k=$f2; n=${f3:-67108864}; fi
  KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 \
      $R/tools/build/kbench $H $m $n 10 64 $k >> gpurun_out/ab.log 2>&1 || exit 1
done
