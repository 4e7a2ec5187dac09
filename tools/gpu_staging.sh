set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_device_staging.py -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 && \
timeout -k 10 120 python tools/staging_bench.py > gpurun_out/staging.json 2>&1 && \
( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stage -o run --output-format csv -- python3 $R/tools/staging_bench.py > $R/gpurun_out/prof_stage.log 2>&1 )
