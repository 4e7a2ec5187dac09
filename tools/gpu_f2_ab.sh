#!/bin/bash
# JVP / VJP restage latency: this tree vs a previous build in tools/build/head_pkg (same box).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 200 python3 tools/jvp_restage_bench.py gpurun_out/jvp_restage_new.json > gpurun_out/jvp_restage_ab.log 2>&1 && \
timeout -k 10 200 python3 tools/jvp_restage_bench.py gpurun_out/jvp_restage_old.json $R/tools/build/head_pkg >> gpurun_out/jvp_restage_ab.log 2>&1
