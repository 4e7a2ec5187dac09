#!/bin/bash
# VALU-roofline counters (one rocprofv3 --pmc pass per kernel; 8 SQ + 1 GRBM counters):
# VALU / transcendental wave-instructions, VALU-active and wave cycles, waves, GPU-active cycles.
# Summary: python tools/valu_summary.py gpurun_out/valu > profiles/rNN_vM_valu_roofline.json
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/valu
cd /tmp
export TMPDIR=/tmp
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels_ident.hsaco   # what the product launches for kbench's identity to_world
KB=$R/tools/build/kbench
C="SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
# second pass per kernel: where the wave cycles go (8 SQ counters)
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
run() {   # name mode n kernel   (KB_* environment passes through to kbench)
  timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/valu/$1 -o $1 --output-format csv -- $KB $H $2 $3 5 64 $4 > $R/gpurun_out/valu/$1.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc $C2 -d $R/gpurun_out/valu/$1_stall -o $1_stall --output-format csv -- $KB $H $2 $3 5 64 $4 > $R/gpurun_out/valu/$1_stall.log 2>&1
}
run sample sample 67108864 ${SAMPLE_KERNEL:-sunsky_sample_direction_rgb_lean_fast} && \
run sample_plain sample 67108864 sunsky_sample_direction_rgb_lean_plain_fast && \
run pdf pdf 67108864 sunsky_pdf_direction_v4_fast && \
run rgb rgb 16777216 sunsky_eval_rgb_v4_fast && \
run spec spec 16777216 sunsky_eval_spec_nodes_v4_fast && \
run rays rays 16777216 sunsky_eval_spec_rays4_v4_fast && \
KB_SAMPLE_SPEC=1 run sample_spec sample 67108864 sunsky_sample_direction_spec_lean4_sorted_fast && \
KB_SAMPLE_FULL=1 run sample_pos sample 67108864 sunsky_sample_direction_rgb_pos_sorted_fast && \
run spec64 spec 67108864 sunsky_eval_spec_nodes_v4_fast && \
KB_SAMPLE_SPEC=1 KB_SAMPLE_FULL=1 run sample_spec_pos sample 67108864 sunsky_sample_direction_spec_pos_sorted_fast
