#!/bin/bash
# Round-6 GPU batch K: the driver's exact N = 8 command at FULL size (64M directions per rank for
# configs[4]) on the one-GPU box, 8 rank processes, the C5 gather through the multi-process RCCL
# double: measures rank 0's post-teardown tail and the job's wall time instead of projecting them.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/k
t0=$(date +%s.%N)
SUNSKY_BENCH_RCCL_DOUBLE=$R/tests/cpp/build/libfake_rccl_ipc.so timeout -k 10 900 \
    python bench.py --gpus 8 > gpurun_out/k/rehearse8_full.log 2> gpurun_out/k/rehearse8_full.err
rc=$?
t1=$(date +%s.%N)
python3 -c "print('wall_s', $t1 - $t0, 'rc', $rc)" >> gpurun_out/k/rehearse8_full.log
exit $rc
