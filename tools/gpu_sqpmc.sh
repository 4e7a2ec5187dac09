#!/bin/bash
# SQ issue/stall counters for the sampling, pdf and eval kernels (one --pmc pass, kbench driver).
# Summaries -> gpurun_out/sqpmc/*.csv ; tools/sq_summary.py prints per-kernel ratios.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sqpmc
cd /tmp
export TMPDIR=/tmp
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
KB=$R/tools/build/kbench
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
timeout -k 10 300 rocprofv3 --pmc $C -d $R/gpurun_out/sqpmc/sample -o sample --output-format csv -- $KB $H sample 67108864 5 64 sunsky_sample_direction_rgb_fast > $R/gpurun_out/sqpmc/sample.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $C -d $R/gpurun_out/sqpmc/pdf -o pdf --output-format csv -- $KB $H pdf 67108864 5 64 sunsky_pdf_direction_v4_fast > $R/gpurun_out/sqpmc/pdf.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $C -d $R/gpurun_out/sqpmc/rgb -o rgb --output-format csv -- $KB $H rgb 16777216 5 64 sunsky_eval_rgb_v4_fast > $R/gpurun_out/sqpmc/rgb.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $C -d $R/gpurun_out/sqpmc/spec -o spec --output-format csv -- $KB $H spec 16777216 5 64 sunsky_eval_spec_nodes_v4_fast > $R/gpurun_out/sqpmc/spec.log 2>&1
