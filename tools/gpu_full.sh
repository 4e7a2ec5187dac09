#!/bin/bash
# Full GPU check: every -m gpu test (one process, per-test timeout), smoke, bench.
# Steps chained with &&; each under its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 30 --warmup 5} > gpurun_out/bench.log 2>&1
