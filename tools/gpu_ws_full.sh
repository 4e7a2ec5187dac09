#!/bin/bash
# Sampling tests, then the general-call (it.p in, ds.dist / ds.p out) sorted vs unsorted A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sample or sorted or sun_disc or beyond" > gpurun_out/pytest_samp.log 2>&1 || exit 1
KB_SAMPLE_FULL=1 timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_full_sorted_fast sunsky_sample_direction_rgb_fast >> gpurun_out/ws_full.log 2>&1 || exit 1
KB_SAMPLE_FULL=1 KB_AB=$H KB_AB_NAME=sunsky_sample_direction_rgb_fast KB_AB_ROUNDS=20 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_full_sorted_fast >> gpurun_out/ws_full.log 2>&1
