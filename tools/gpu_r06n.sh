#!/bin/bash
# Round-6 GPU batch N: every -m gpu test, smoke, then tools/gpu_prof.sh (bench, burst trace, PMC)
# on the final kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
bash tools/gpu_prof.sh
