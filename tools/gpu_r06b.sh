#!/bin/bash
# Round-6 GPU batch B: same-box A/B of this round's kernels against round 5's (built from
# git 8ed256b into tools/build/r05_kernels{,_ident}.hsaco; SunskyKArgs is unchanged), by
# running bench.py (no CPU baseline, no configs[4]) alternately with each code object pair.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/ab
for k in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu --no-c5 --steps 30 --warmup 5 > gpurun_out/ab/r06_$k.log 2>&1 || exit 1
  SUNSKY_AMD_CODE_OBJECT=$R/tools/build/r05_kernels.hsaco SUNSKY_AMD_CODE_OBJECT_IDENT=$R/tools/build/r05_kernels_ident.hsaco \
    timeout -k 10 240 python bench.py --no-cpu --no-c5 --steps 30 --warmup 5 > gpurun_out/ab/r05_$k.log 2>&1 || exit 1
done
