#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for B in sunsky_sample_direction_rgb_pf_fast sunsky_sample_direction_rgb_sorted_fast sunsky_sample_direction_rgb_sorted_v2_fast sunsky_sample_direction_rgb_sorted_v4_fast; do
  A=sunsky_sample_direction_rgb_lean_fast B=$B ROUNDS=15 bash $R/tools/gpu_ab_variant.sh || exit 1
done
