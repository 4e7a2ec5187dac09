#!/bin/bash
# Session v11: parity tests, smoke, bench, rocprof stats, PMC traffic (tools/gpu_round.sh), then the
# VALU counters (tools/gpu_valu.sh) and the wave-sorted vs plain sampling sweep / A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round.sh && \
bash tools/gpu_valu.sh && \
python3 tools/valu_summary.py gpurun_out/valu > gpurun_out/valu_roofline.json && \
VARIANTS=sunsky_sample_direction_rgb_lean_plain_fast BPCU=16,32,64 bash tools/gpu_ws_sweep.sh && \
VARIANTS=sunsky_sample_direction_rgb_lean_plain_fast ROUNDS=20 bash tools/gpu_ws.sh
