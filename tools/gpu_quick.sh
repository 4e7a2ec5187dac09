#!/bin/bash
# Quick kernel timing (kbench) of every hot kernel at its default grid, 16M / 64M items.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/quick.log
: > $O
timeout -k 10 120 $KB $H rgb 16777216 30 64 sunsky_eval_rgb_v4_fast >> $O 2>&1 && \
timeout -k 10 120 $KB $H spec 16777216 20 16,32,64 sunsky_eval_spec_nodes_v4_fast sunsky_eval_spec_bcast_v4_fast >> $O 2>&1 && \
timeout -k 10 200 $KB $H sample 67108864 10 16,32,64 sunsky_sample_direction_rgb_fast >> $O 2>&1 && \
timeout -k 10 200 $KB $H pdf 67108864 10 16,32,64 sunsky_pdf_direction_v4_fast >> $O 2>&1
