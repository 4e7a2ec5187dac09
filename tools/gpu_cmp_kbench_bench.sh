set -o pipefail
R=$GRAFT_REPO_ROOT
export SUNSKY_AMD_DATASET=$R/mitsuba3-sunsky_amd/data/sunsky_datasets.pack
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/build/kbench $R/mitsuba3-sunsky_amd/build/sunsky_kernels.hsaco sample 67108864 10 64 sunsky_sample_direction_rgb_lean_fast > $R/gpurun_out/kb_sample.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_full -o full --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $R/gpurun_out/prof_full.log 2>&1
