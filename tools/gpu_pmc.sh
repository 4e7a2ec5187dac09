#!/bin/bash
# PMC counter passes (one counter group per pass; no tracing domains combined with --pmc).
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp
R=$GRAFT_REPO_ROOT
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1
K="sunsky_eval_rgb_v4_fast"
S="sunsky_eval_spec_nodes_v2_fast"
run() { # name, mode, kernel, counters...
  local nm=$1 mode=$2 k=$3; shift 3
  timeout -k 10 180 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc/$nm -o $nm --output-format csv -- $R/tools/build/kbench $H $mode 16777216 5 64 $k > $R/gpurun_out/pmc/$nm.log 2>&1
}
run rgb_fetch rgb $K FETCH_SIZE && \
run rgb_write rgb $K WRITE_SIZE && \
run rgb_sq rgb $K SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run spec_sq spec $S SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run spec_fetch spec $S FETCH_SIZE && \
run spec_write spec $S WRITE_SIZE
echo done
