#!/bin/bash
# Headline measurement: full bench, then a rocprofv3 kernel trace of the timed headline burst
# alone (bench.py --headline-only) with its per-launch statistics, then the PMC traffic of
# the same burst (separate FETCH_SIZE / WRITE_SIZE passes, no tracing domains with --pmc).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
export TMPDIR=/tmp
STEPS=${STEPS:-100}
cd $R && timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_burst -o burst --output-format csv -- \
    python3 $R/bench.py --headline-only --steps $STEPS --warmup 10 > $R/gpurun_out/prof_burst.log 2>&1 && \
python3 $R/tools/burst_stats.py $(find $R/gpurun_out/prof_burst -name '*kernel_trace.csv') sunsky_eval_rgb_v4_fast $STEPS \
    $R/gpurun_out/burst_stats.json > /dev/null && \
B="$R/bench.py --headline-only --steps 20 --warmup 2" && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc/fetch -o fetch --output-format csv -- python3 $B > $R/gpurun_out/pmc/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc/write -o write --output-format csv -- python3 $B > $R/gpurun_out/pmc/write.log 2>&1 && \
python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/pmc/fetch -name '*counter_collection.csv') \
    $(find $R/gpurun_out/pmc/write -name '*counter_collection.csv') $R/gpurun_out/pmc/pmc_traffic.json
