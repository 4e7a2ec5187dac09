#!/bin/bash
# Spectral sampling iteration: the spectral sampling / lean-vs-general bitwise tests, then an
# interleaved A/B of the spectral LEAN kernel against tools/build/ab_base.hsaco.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_entry_points.py tests/test_graph_capture.py -m gpu -q -x \
    -k "lean or spectral or c4 or sample_ray or wavelengths or replay" --timeout 200 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 && \
KB_SAMPLE_SPEC=1 KB_AB=$R/tools/build/ab_base.hsaco KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 \
    $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_spec_lean_fast > gpurun_out/ab.log 2>&1
