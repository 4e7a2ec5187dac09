#!/bin/bash
# Interleaved A/B (kbench KB_AB) of the product kernels against tools/build/ab_base.hsaco
# for: RGB headline eval (16M), RGB LEAN sampling (64M), spectral LEAN sampling (64M x 4 lambda).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
B=$R/tools/build/ab_base.hsaco
L=$R/gpurun_out/ab.log
: > $L
KB_AB=$B KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 $R/tools/build/kbench $H rgb 16777216 20 64 sunsky_eval_rgb_v4_fast >> $L 2>&1 && \
KB_AB=$B KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $L 2>&1 && \
KB_SAMPLE_SPEC=1 KB_AB=$B KB_AB_ROUNDS=${ROUNDS:-20} timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_spec_lean_fast >> $L 2>&1
