#!/bin/bash
# Cost ablation of the spectral LEAN sampling kernel: interleaved A/B of the product kernel
# against probe builds that drop one part (tools/Makefile probe_%.hsaco).  Output gpurun_out/ab_spec.log.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
: > $R/gpurun_out/ab_spec.log
for p in ${PROBES:-spec_no_sky spec_no_sun no_sky_sample no_pdf}; do
  echo "probe $p" >> $R/gpurun_out/ab_spec.log
  KB_SAMPLE_SPEC=1 KB_AB=$R/tools/build/probe_$p.hsaco KB_AB_ROUNDS=${ROUNDS:-15} timeout -k 10 200 \
      $R/tools/build/kbench $H sample 67108864 10 64 sunsky_sample_direction_spec_lean_fast >> $R/gpurun_out/ab_spec.log 2>&1 || exit 1
done
