#!/bin/bash
# HBM traffic of the bench's kernels: two separate rocprofv3 --pmc passes over
# bench.py (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), no tracing
# domains combined with --pmc.  Summary -> gpurun_out/pmc/pmc_traffic.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp
export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 1 --no-cpu --no-pmc"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc/fetch -o fetch --output-format csv -- python3 $B > $R/gpurun_out/pmc/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc/write -o write --output-format csv -- python3 $B > $R/gpurun_out/pmc/write.log 2>&1 && \
python3 $R/tools/pmc_summary.py $(find $R/gpurun_out/pmc/fetch -name '*counter_collection.csv') \
    $(find $R/gpurun_out/pmc/write -name '*counter_collection.csv') $R/gpurun_out/pmc/pmc_traffic.json
