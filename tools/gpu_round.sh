#!/bin/bash
# Combined GPU session: parity tests -> smoke -> [grid sweep] -> bench -> rocprof stats -> PMC traffic.
# Each GPU step has its own time limit; steps chained with && (stop at first failure).
# TUNE=1 adds the tools/gpu_tune.sh grid sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rs > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && \
{ [ "${TUNE:-0}" != 1 ] || bash tools/gpu_tune.sh; } && \
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 && \
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/gpurun_out/prof_bench.log 2>&1 ) && \
bash tools/gpu_pmc.sh
