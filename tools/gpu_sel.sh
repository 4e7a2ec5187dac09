#!/bin/bash
# GPU tests selected by a pytest -k expression (spaces allowed), then optionally a bench run.
# usage: bash tools/gpu_sel.sh "<files>" "<-k expression>" [bench args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $1 -k "$2" -m gpu -v -s --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_sel.log
[ $rc -le 1 ] && [ "${3:-}" != "" ] && timeout -k 10 600 python bench.py $3 > gpurun_out/bench.log 2>&1
exit $rc
