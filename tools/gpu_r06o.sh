#!/bin/bash
# Round-6 GPU batch O: the driver's N = 2 and N = 4 commands at full size on the one-GPU box
# (rank processes sharing the GPU, C5 gather through the multi-process RCCL double).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/o
for n in 2 4; do
  SUNSKY_BENCH_RCCL_DOUBLE=$R/tests/cpp/build/libfake_rccl_ipc.so timeout -k 10 600 \
      python bench.py --gpus $n > gpurun_out/o/rehearse${n}_full.log 2> gpurun_out/o/rehearse${n}_full.err || exit 1
done
