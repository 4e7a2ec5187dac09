#!/bin/bash
# Variant sweep (tools/tune_kernels.hip) against the product kernels, 16M directions.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
T=$R/tools/build/tune_kernels.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/tune.log
: > $O
timeout -k 10 200 $KB $T rgb 16777216 30 32,64 sunsky_eval_rgb_v4_fast tune_rgb_v4_w8 tune_rgb_v4_w4 tune_rgb_v2 tune_rgb_v2_w8 sunsky_eval_rgb_v4_fast >> $O 2>&1 && \
timeout -k 10 200 $KB $T spec 16777216 20 32,64 sunsky_eval_spec_nodes_v4_fast tune_spec_nodes_v2_w8 tune_spec_nodes_v4 tune_spec_nodes_v1 tune_spec_nodes_v1_w8 sunsky_eval_spec_nodes_v4_fast >> $O 2>&1
