#!/bin/bash
# PMC passes over the sampling kernels under kbench (64M samples; spectral: 4 lambda per
# sample): VALU / transcendental / SALU / LDS instruction counts, VALU-active and wave
# cycles, LDS bank conflicts and LDS waits.  One rocprofv3 --pmc pass per counter set.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/spmc
cd /tmp
export TMPDIR=/tmp
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=${HSACO:-$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco}
KB=$R/tools/build/kbench
C1="SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
run() {   # tag env counters kernel
  env $2 timeout -s KILL 90 rocprofv3 --pmc $3 -d $R/gpurun_out/spmc/$1 -o $1 --output-format csv -- $KB $H sample 67108864 3 64 $4 > $R/gpurun_out/spmc/$1.log 2>&1
}
run spec1 KB_SAMPLE_SPEC=1 "$C1" sunsky_sample_direction_spec_lean_fast && \
run spec2 KB_SAMPLE_SPEC=1 "$C2" sunsky_sample_direction_spec_lean_fast && \
run rgb1 KB_X=0 "$C1" sunsky_sample_direction_rgb_lean_fast && \
run rgb2 KB_X=0 "$C2" sunsky_sample_direction_rgb_lean_fast && \
python3 $R/tools/spmc_summary.py $R/gpurun_out/spmc > $R/gpurun_out/spmc/summary.json
