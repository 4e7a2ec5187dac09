#!/bin/bash
# Cost ablation of the RGB LEAN (wave-sorted) sampling kernel against probe builds.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
: > $R/gpurun_out/ab_rgb.log
for p in ${PROBES:-no_sky_sample no_pdf no_sun_disc no_weight}; do
  echo "probe $p" >> $R/gpurun_out/ab_rgb.log
  KB_AB=$R/tools/build/probe_$p.hsaco KB_AB_ROUNDS=${ROUNDS:-15} timeout -k 10 200 \
      $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast >> $R/gpurun_out/ab_rgb.log 2>&1 || exit 1
done
