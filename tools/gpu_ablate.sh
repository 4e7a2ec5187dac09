#!/bin/bash
# Cost ablations of the LEAN RGB sample_direction kernel (probe builds, tools/Makefile)
# plus a workgroups-per-CU sweep of the product kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/abl.log
mkdir -p $R/gpurun_out; : > $O
K=sunsky_sample_direction_rgb_lean_fast
echo "== bpcu sweep" >> $O
timeout -k 10 120 $KB $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco sample 67108864 10 4,8,16,32,64 $K >> $O 2>&1 || exit 1
for h in $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco $R/tools/build/probe_no_sky_sample.hsaco $R/tools/build/probe_no_pdf.hsaco $R/tools/build/probe_no_weight.hsaco $R/tools/build/probe_no_sun_disc.hsaco; do
  echo "== $h" >> $O
  timeout -k 10 120 $KB $h sample 67108864 10 64 $K >> $O 2>&1 || exit 1
done
