#!/bin/bash
# Interleaved A/B timing of kernels in one kbench process (KB_AB): bursts alternate
# between THIS (default: the product code object) and OTHER (default:
# tools/build/ab_base.hsaco, built by tools/mk_ab_base.sh from a git revision or a
# probe build).  median(other/this) > 1: THIS is faster.  Output appended to
# gpurun_out/ab.log.
# usage: [THIS=a.hsaco] [OTHER=b.hsaco] gpu_ab.sh <mode> <n> <kernel> [kernel...]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
O=$R/gpurun_out/ab.log
THIS=${THIS:-$R/mitsuba3-sunsky_amd/build/sunsky_kernels_ident.hsaco}   # kbench emitters have an identity to_world
OTHER=${OTHER:-$R/tools/build/ab_base.hsaco}
MODE=$1; N=$2; shift 2
echo "== $THIS vs $OTHER ($MODE $N: $*)" >> $O
KB_AB=$OTHER KB_AB_ROUNDS=${KB_AB_ROUNDS:-20} timeout -k 10 300 $R/tools/build/kbench $THIS $MODE $N 10 64 "$@" >> $O 2>&1
