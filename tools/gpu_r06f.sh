#!/bin/bash
# Round-6 GPU batch F: smoke, then tools/gpu_prof.sh (full bench, rocprofv3 trace of the timed
# headline burst, PMC traffic passes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
bash tools/gpu_prof.sh
