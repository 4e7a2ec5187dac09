#!/bin/bash
# Session v14: parity tests, smoke, bench, rocprof stats, PMC traffic (tools/gpu_round.sh), VALU counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round.sh && \
bash tools/gpu_valu.sh && \
python3 tools/valu_summary.py gpurun_out/valu > gpurun_out/valu_roofline.json
