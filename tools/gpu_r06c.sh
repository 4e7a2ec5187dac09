#!/bin/bash
# Round-6 GPU batch C: the headline RGB eval kernel, this round's build against round 5's and two
# probe builds (tools/build/exp_v_ident.hsaco: the disc branch's constants through a VGPR-laundered
# K; exp_nodisc_ident.hsaco: no disc term at all -- the bound on what the disc branch costs),
# interleaved A/B in kbench, warm and cold (4 rotating batches); then per-wave instruction counts.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
mkdir -p gpurun_out/c
A=$R/mitsuba3-sunsky_amd/build/sunsky_kernels_ident.hsaco
K=sunsky_eval_rgb_v4_fast
for b in r05_kernels_ident exp_v_ident exp_nodisc_ident; do
  for cold in 1 4; do
    echo "== B=$b cold=$cold" >> gpurun_out/c/ab.log
    KB_COLD=$cold KB_AB=$R/tools/build/$b.hsaco KB_AB_ROUNDS=30 timeout -k 10 120 \
      tools/build/kbench $A rgb 16777216 40 64 $K >> gpurun_out/c/ab.log 2>&1 || exit 1
  done
done
for h in $A $R/tools/build/r05_kernels_ident.hsaco; do
  ( cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_RD \
      -d $R/gpurun_out/c/pmc_$(basename $h .hsaco) -o p --output-format csv -- \
      $R/tools/build/kbench $h rgb 16777216 5 64 $K > $R/gpurun_out/c/pmc_$(basename $h .hsaco).log 2>&1 ) || exit 1
done
