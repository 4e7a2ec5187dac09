#!/bin/bash
# Cost ablations of the LEAN RGB sample_direction kernel as interleaved A/B ratios:
# product code object vs each probe build (tools/Makefile), 64M samples.
set -o pipefail
R=$GRAFT_REPO_ROOT
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
O=$R/gpurun_out/abl_ab.log
mkdir -p $R/gpurun_out; : > $O
K=${K:-sunsky_sample_direction_rgb_lean_fast}
for p in no_sky_sample no_pdf no_weight no_sun_disc nostore; do
  echo "== probe_$p" >> $O
  KB_AB=$R/tools/build/probe_$p.hsaco KB_AB_ROUNDS=15 timeout -k 10 150 $R/tools/build/kbench \
      $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco sample 67108864 10 64 $K >> $O 2>&1 || exit 1
done
