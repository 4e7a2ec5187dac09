#!/bin/bash
# A/B of the LEAN sample_direction kernels against the general ones (same code
# object, interleaved bursts), after the sampling parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_direct_diffuse.py tests/test_graph_capture.py > gpurun_out/t.log 2>&1 || exit 1
for v in rgb; do   # kbench stages an RGB emitter
  KB_AB=$H KB_AB_NAME=sunsky_sample_direction_${v}_fast KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 \
      $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_${v}_lean_fast >> gpurun_out/ab.log 2>&1 || exit 1
done
