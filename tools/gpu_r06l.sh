#!/bin/bash
# Round-6 GPU batch L: the multi-process gather through the hipIpc double at growing shard sizes,
# with per-operation timings (SUNSKY_FAKE_RCCL_DEBUG), to find why the full-size 8-rank rehearsal
# timed out.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/l
for n in 16777216 67108864 134217728; do
  echo "== world 2, n=$n" >> gpurun_out/l/ipc_sizes.log
  pids=()
  for r in 0 1; do
    SUNSKY_AMD_RCCL=$R/tests/cpp/build/libfake_rccl_ipc.so SUNSKY_FAKE_RCCL_DEBUG=1 SUNSKY_FAKE_RCCL_TIMEOUT=60 \
    MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + n % 1000)) WORLD_SIZE=2 RANK=$r GATHER_N=$n \
      timeout -k 10 240 python tests/gpu_gather_worker.py > gpurun_out/l/w${r}_$n.log 2>&1 &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=1; done
  cat gpurun_out/l/w0_$n.log gpurun_out/l/w1_$n.log | grep -v "amdgpu.ids\|Gloo" >> gpurun_out/l/ipc_sizes.log
  [ $rc = 0 ] || exit 1
done
