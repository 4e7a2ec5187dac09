#!/bin/bash
# (the ws2/ws3/ws4 spectral variants were removed after this measurement: profiles/r02_v17_ab_spec_sorted_reverted.log)
# Spectral wave-sorted sample_direction variants (R = 2, 3, 4) vs the spectral LEAN kernel,
# 64M samples x 4 wavelengths (kbench KB_SAMPLE_SPEC): bitwise check + interleaved A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
O=$R/gpurun_out/specws.log
export KB_SAMPLE_SPEC=1
L=sunsky_sample_direction_spec_lean_fast
timeout -k 10 150 $R/tools/build/kbench $H sample 67108864 10 64 $L ${VARIANTS:-sunsky_sample_direction_spec_ws2_fast sunsky_sample_direction_spec_ws3_fast sunsky_sample_direction_spec_ws4_fast} >> $O 2>&1 || exit 1
for B in ${VARIANTS:-sunsky_sample_direction_spec_ws2_fast sunsky_sample_direction_spec_ws3_fast sunsky_sample_direction_spec_ws4_fast}; do
  KB_AB=$H KB_AB_NAME=$B KB_AB_ROUNDS=15 timeout -k 10 200 $R/tools/build/kbench $H sample 67108864 10 64 $L >> $O 2>&1 || exit 1
done
