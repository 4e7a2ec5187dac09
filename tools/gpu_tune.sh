#!/bin/bash
# Variant sweep (tools/tune_kernels.hip) against the product kernels, 16M directions,
# warm (one input batch) and cold (KB_COLD=4 rotating batches, 805 MB of inputs).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
T=$R/tools/build/tune_kernels.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/tune.log
: > $O
for cold in 1 4; do
  echo "== KB_COLD=$cold" >> $O
  KB_COLD=$cold timeout -k 10 200 $KB $T rgb 16777216 32 4,8,16,32,64 sunsky_eval_rgb_v4_fast tune_rgb_pf_v4 sunsky_eval_rgb_v4_fast >> $O 2>&1 || exit 1
done
