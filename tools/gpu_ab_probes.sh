#!/bin/bash
# Interleaved A/B of one product kernel against probe code objects tools/build/probe_<P>.hsaco.
# usage: KERNEL=<name> MODE=<kbench mode> [ENVS="KB_SAMPLE_SPEC=1"] PROBES="w5 w6" bash tools/gpu_ab_probes.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
: > $R/gpurun_out/ab_probes.log
for p in $PROBES; do
  echo "probe $p" >> $R/gpurun_out/ab_probes.log
  env ${ENVS:-KB_X=0} KB_AB=$R/tools/build/probe_$p.hsaco KB_AB_ROUNDS=${ROUNDS:-15} timeout -k 10 200 \
      $R/tools/build/kbench $H ${MODE:-sample} ${N:-67108864} 10 64 $KERNEL >> $R/gpurun_out/ab_probes.log 2>&1 || exit 1
done
