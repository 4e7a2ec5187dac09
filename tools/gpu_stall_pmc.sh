#!/bin/bash
# Stall / issue breakdown of one kbench kernel: rocprofv3 --list-avail (saved), then one --pmc
# pass of SQ issue/wait counters (<= 8 SQ counters, no tracing domains).
# usage: KERNEL=<name> MODE=<kbench mode> [N=..] [KB_SAMPLE_SPEC=1] bash tools/gpu_stall_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/stall
cd /tmp
export TMPDIR=/tmp
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
KB=$R/tools/build/kbench
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/stall/avail.txt 2>&1 || true
C1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $C1 -d $R/gpurun_out/stall/p1 -o p1 --output-format csv -- \
    $KB $H ${MODE:-sample} ${N:-67108864} 5 64 $KERNEL > $R/gpurun_out/stall/p1.log 2>&1
C2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $C2 -d $R/gpurun_out/stall/p2 -o p2 --output-format csv -- \
    $KB $H ${MODE:-sample} ${N:-67108864} 5 64 $KERNEL > $R/gpurun_out/stall/p2.log 2>&1
