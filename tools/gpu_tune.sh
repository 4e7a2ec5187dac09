#!/bin/bash
# Grid-size sweep of the streaming kernels (tools/kbench.cpp), 16M directions.
set -o pipefail
mkdir -p gpurun_out
H=mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
export SUNSKY_AMD_DATASET=mitsuba3-sunsky_amd/data/sunsky_datasets.pack
timeout -k 10 300 tools/build/kbench $H rgb 16777216 30 4,8,16,32,64,128 \
  sunsky_eval_rgb_v4_fast sunsky_eval_rgb_v4_ref > gpurun_out/tune_rgb.log 2>&1 && \
timeout -k 10 300 tools/build/kbench $H spec 16777216 20 4,8,16,32,64 \
  sunsky_eval_spec_nodes_v2_fast sunsky_eval_spec_bcast_v2_fast sunsky_eval_spec_nodes_v2_ref > gpurun_out/tune_spec.log 2>&1
