#!/bin/bash
# Wave-sorted sample_direction variants: plain timing + bitwise check against the LEAN
# kernel, the product LEAN kernel vs the HEAD build (KB_AB), and each variant vs LEAN
# interleaved in one process.  Output: gpurun_out/ws.log
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/ws.log
L=sunsky_sample_direction_rgb_lean_fast
timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 10 64 $L ${VARIANTS:-sunsky_sample_direction_rgb_lean_plain_fast} >> $O 2>&1 || exit 1
KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=${ROUNDS:-15} timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 $L >> $O 2>&1 || exit 1
for B in ${VARIANTS:-sunsky_sample_direction_rgb_lean_plain_fast}; do
  KB_AB=$H KB_AB_NAME=$B KB_AB_ROUNDS=${ROUNDS:-15} timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 $L >> $O 2>&1 || exit 1
done
