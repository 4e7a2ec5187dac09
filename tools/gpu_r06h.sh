#!/bin/bash
# Round-6 GPU batch H: pdf_direction at 8 waves/SIMD (amdgpu_waves_per_eu(8): 78 SGPRs, no
# spills; the product build holds 96 SGPRs -> 7 waves) against the product build, interleaved
# A/B in kbench at 64M and 16M, twice.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
mkdir -p gpurun_out/h
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels_ident.hsaco
for pass in 1 2; do
  for n in 67108864 16777216; do
    echo "== n=$n pass=$pass" >> gpurun_out/h/pdf_w8.log
    KB_AB=$R/tools/build/exp_w8_ident.hsaco KB_AB_ROUNDS=30 timeout -k 10 120 \
      tools/build/kbench $H pdf $n 20 64 sunsky_pdf_direction_v4_fast >> gpurun_out/h/pdf_w8.log 2>&1 || exit 1
  done
done
