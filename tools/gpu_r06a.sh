#!/bin/bash
# Round-6 GPU batch A: the multi-process RCCL-double gather tests, the sampler instruction
# budget (PMC), and the 8-rank rehearsal whose C5 gather takes the C-ABI branch through the
# double.  Steps chained with &&, each under its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/budget
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gather.py -v -s --timeout 200 --timeout-method thread -rs \
    > gpurun_out/pytest_gather.log 2>&1 && \
( cd /tmp && SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack timeout -s KILL 120 \
    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
    -d $R/gpurun_out/budget -o budget --output-format csv -- \
    $R/tools/build/sampler_budget_run $R/tools/build/sampler_budget.hsaco > $R/gpurun_out/budget/run.log 2>&1 ) && \
SUNSKY_BENCH_RCCL_DOUBLE=$R/tests/cpp/build/libfake_rccl_ipc.so timeout -k 10 700 \
    python bench.py --gpus 8 --c5-dirs 4194304 > gpurun_out/rehearse8_double.log 2>&1
