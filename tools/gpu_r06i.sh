#!/bin/bash
# Round-6 GPU batch I: every -m gpu test and the bench after the pdf_direction occupancy change.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
