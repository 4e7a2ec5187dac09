#!/bin/bash
# Iteration loop on the GPU box: full GPU test suite, then kernel timings (gpu_quick.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
bash tools/gpu_quick.sh
