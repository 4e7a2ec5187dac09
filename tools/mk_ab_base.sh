#!/bin/bash
# Build tools/build/ab_base.hsaco from the kernels of a git revision (default HEAD)
# for tools/gpu_ab.sh.
set -e
REV=${1:-HEAD}
cd "$(dirname "$0")/.."
git show $REV:mitsuba3-sunsky_amd/csrc/sunsky_kernels.hip > mitsuba3-sunsky_amd/csrc/_ab_base.hip
trap 'rm -f mitsuba3-sunsky_amd/csrc/_ab_base.hip' EXIT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --genco -DSS_XFORM_IDENTITY -Iinclude -Imitsuba3-sunsky_amd/csrc \
    -o tools/build/ab_base.hsaco mitsuba3-sunsky_amd/csrc/_ab_base.hip
