#!/bin/bash
# Spectral C3 kernel split: compute-only timing (stores suppressed) + SQ counter passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/specprobe
mkdir -p $O
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
P=$R/tools/build/probe_nostore.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
timeout -k 10 120 $KB $H spec 16777216 20 32,64 sunsky_eval_spec_nodes_v4_fast > $O/time.log 2>&1 && \
timeout -k 10 120 $KB $P spec 16777216 20 32,64 sunsky_eval_spec_nodes_v4_fast sunsky_eval_spec_bcast_v4_fast > $O/time_nostore.log 2>&1 && \
timeout -k 10 120 $KB $P sample 67108864 5 32 sunsky_sample_direction_rgb_fast >> $O/time_nostore.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
pmc() { local nm=$1; shift
  timeout -k 10 180 rocprofv3 --pmc "$@" -d $O/$nm -o $nm --output-format csv -- $KB $H spec 16777216 3 64 sunsky_eval_spec_nodes_v4_fast > $O/$nm.log 2>&1; } && \
pmc a SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_IFETCH && \
pmc b SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
echo "rc=$?" > $O/done.txt
