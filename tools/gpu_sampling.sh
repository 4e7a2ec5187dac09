#!/bin/bash
# Sampling-kernel timing (kbench, 64M samples) + the sampling / caller parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
H=$R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
KB=$R/tools/build/kbench
O=$R/gpurun_out/sampling.log
: > $O
timeout -k 10 200 $KB $H sample 67108864 10 32,64 sunsky_sample_direction_rgb_fast sunsky_sample_direction_spec_fast >> $O 2>&1 && \
timeout -k 10 200 $KB $H pdf 67108864 10 64 sunsky_pdf_direction_v4_fast >> $O 2>&1 && \
cd $R && timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_direct_diffuse.py tests/test_cpp_facade.py -m gpu -x -q -k "sampl or direct or facade" >> $O 2>&1
