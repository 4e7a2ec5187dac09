#!/bin/bash
# eval_vjp A/B: the AD tests on the product code object, then tools/ad_ab.py interleaved over
# the code objects given (ROUNDS rounds, one process per code object per round).
# usage: gpu_ad_ab.sh <a.hsaco> <b.hsaco> ...   (the product's own code object: "default")
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
O=$R/gpurun_out/ad_ab.log
cd $R && timeout -k 10 300 python -u -m pytest tests/test_eval_jvp.py tests/test_device_staging.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ad.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-5}); do
  for co in "$@"; do
    if [ "$co" = default ]; then
      timeout -k 10 120 python tools/ad_ab.py "r$r default" >> $O 2>&1 || exit 1
    else
      SUNSKY_AMD_CODE_OBJECT=$R/$co timeout -k 10 120 python tools/ad_ab.py "r$r $co" >> $O 2>&1 || exit 1
    fi
  done
done
