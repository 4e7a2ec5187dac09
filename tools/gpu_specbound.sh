#!/bin/bash
# Spectral LEAN sample_direction (4 random wavelengths per sample): random inputs vs inputs
# partitioned sky picks first (KB_SORT_U=2), the divergence bound a wave-sorted form could reach.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/specbound.log
for i in 1 2; do
KB_SAMPLE_SPEC=1 timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_spec_lean_fast >> $O 2>&1 || exit 1
KB_SAMPLE_SPEC=1 KB_SORT_U=2 timeout -k 10 120 $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_spec_lean_fast >> $O 2>&1 || exit 1
done
