#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box (2 ranks share the GPU over gloo), then the
# C5 watchdog forced to fire (SUNSKY_BENCH_C5_TIMEOUT=1): the line must still print, exit 0.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --c5-dirs 4194304 > gpurun_out/rehearse2.log 2>&1 && \
SUNSKY_BENCH_C5_TIMEOUT=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-secondary > gpurun_out/rehearse2_watchdog.log 2>&1
echo "rc=$?" >> gpurun_out/rehearse2_watchdog.log
