#!/bin/bash
# Round-6 GPU batch G: the C3/C5 node kernel at 64M with the product's occupancy cap (5 WG/CU via
# 32000 B of dynamic LDS) against the output plane pitch (KB_OPAD floats of padding per plane),
# three alternating passes; then the K = 11 write-only probe legs again for reproducibility.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
mkdir -p gpurun_out/g
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels_ident.hsaco
for pass in 1 2 3; do
  for pad in 0 525312 64 1049600; do
    echo "== pad=$pad pass=$pass" >> gpurun_out/g/nodes_pitch.log
    KB_LDS=32000 KB_OPAD=$pad timeout -k 10 60 tools/build/kbench $H spec 67108864 30 64 sunsky_eval_spec_nodes_v4_fast \
      >> gpurun_out/g/nodes_pitch.log 2>&1 || exit 1
    KB_LDS=32000 KB_OPAD=$pad timeout -k 10 60 tools/build/kbench $H spec 16777216 60 64 sunsky_eval_spec_nodes_v4_fast \
      >> gpurun_out/g/nodes_pitch.log 2>&1 || exit 1
  done
done
timeout -k 10 300 tools/build/c5_probe pitch > gpurun_out/g/c5_pitch_again.log 2>&1
