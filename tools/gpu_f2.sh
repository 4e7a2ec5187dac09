#!/bin/bash
# f2: AD tests (device tangent staging bitwise the host tangent, JVP vs finite differences, VJP
# vs JVP contractions), then the restage latency under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R && timeout -k 10 300 python -u -m pytest tests/test_eval_jvp.py tests/test_graph_capture.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_f2.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_f2 -o f2 --output-format csv -- python3 $R/tools/jvp_restage_bench.py $R/gpurun_out/jvp_restage.json > $R/gpurun_out/jvp_restage.log 2>&1
