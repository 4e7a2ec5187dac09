#!/bin/bash
# Round-6 GPU batch D: cold (4 rotating batches) kbench timing of the headline kernel per build,
# alternating builds, two passes.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
mkdir -p gpurun_out/d
for pass in 1 2; do
  for h in mitsuba3-sunsky_amd/build/sunsky_kernels_ident tools/build/r05_kernels_ident tools/build/exp_v_ident tools/build/exp_nodisc_ident; do
    for cold in 4 1; do
      echo "== $h cold=$cold pass=$pass" >> gpurun_out/d/cold.log
      KB_COLD=$cold timeout -k 10 60 tools/build/kbench $R/$h.hsaco rgb 16777216 200 64 sunsky_eval_rgb_v4_fast >> gpurun_out/d/cold.log 2>&1 || exit 1
    done
  done
done
