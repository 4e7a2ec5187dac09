#!/bin/bash
# GPU tests of a file/selection with printed parity figures, then a bench run.
# usage: bash tools/gpu_tests.sh "<pytest selection>" [bench args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${1:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -s --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_sel.log
[ $rc -le 1 ] && [ "${2:-}" != "" ] && timeout -k 10 600 python bench.py $2 > gpurun_out/bench.log 2>&1
exit $rc
