#!/bin/bash
# Round-6 GPU batch E: every -m gpu test on the final kernels (one process, per-test timeout).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1
