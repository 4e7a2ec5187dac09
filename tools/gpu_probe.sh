#!/bin/bash
# Calibration + counters for the non-headline kernels: HBM access-shape probe,
# grid sweeps of the sampling kernels, SQ counter passes (separate passes, no tracing domains).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/probe
mkdir -p $O
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
timeout -k 10 120 $R/tools/build/bw_probe > $O/bw_probe.log 2>&1 && \
timeout -k 10 200 $KB $H sample 67108864 10 8,16,32,64 sunsky_sample_direction_rgb_fast > $O/tune_sample.log 2>&1 && \
timeout -k 10 200 $KB $H pdf 67108864 10 8,16,32,64 sunsky_pdf_direction_v4_fast > $O/tune_pdf.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 && \
pmc() { local nm=$1 mode=$2 n=$3 k=$4 bp=$5; shift 5
  timeout -k 10 180 rocprofv3 --pmc "$@" -d $O/$nm -o $nm --output-format csv -- $KB $H $mode $n 3 $bp $k > $O/$nm.log 2>&1; } && \
pmc spec_sq1 spec 16777216 sunsky_eval_spec_nodes_v4_fast 32 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pmc spec_sq2 spec 16777216 sunsky_eval_spec_nodes_v4_fast 32 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
pmc sample_sq1 sample 67108864 sunsky_sample_direction_rgb_fast 16 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pmc sample_sq2 sample 67108864 sunsky_sample_direction_rgb_fast 16 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
pmc pdf_sq1 pdf 67108864 sunsky_pdf_direction_v4_fast 16 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pmc rgb_sq1 rgb 16777216 sunsky_eval_rgb_v4_fast 64 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
echo "probe rc=$?" >> $O/done.txt
