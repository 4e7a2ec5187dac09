#!/bin/bash
# RCCL gather through the C ABI: GPU tests + a 2-rank bench rehearsal of configs[4].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gather.py -m gpu -v -s --timeout 300 --timeout-method thread -rs > gpurun_out/pytest_gather.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 10 --warmup 2 --no-secondary --no-cpu --c5 --c5-dirs 4194304 --gather > gpurun_out/bench_2rank.log 2>&1
