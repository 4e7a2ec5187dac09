#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/abl.log
: > $O
for h in $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco $R/tools/build/probe_no_sky_sample.hsaco $R/tools/build/probe_no_pdf.hsaco $R/tools/build/probe_no_weight.hsaco $R/tools/build/probe_no_sun_disc.hsaco; do
  echo "== $h" >> $O
  timeout -k 10 120 $KB $h sample 67108864 10 64 sunsky_sample_direction_rgb_fast >> $O 2>&1 || exit 1
done
