#!/bin/bash
# orbslam3lib_amd/variants/liborbgpu_old.so: orb_kernels.hip as of git revision REV (default HEAD)
# linked with the other objects of the current build, for A/B timing with tools/time_variants.sh.
cd "$(dirname "$0")/.."
set -e
REV=${1:-HEAD}
O=orbslam3lib_amd/variants
mkdir -p $O
git show $REV:orbslam3lib_amd/csrc/orb_kernels.hip > orbslam3lib_amd/csrc/zz_old_kernels.hip
trap 'rm -f orbslam3lib_amd/csrc/zz_old_kernels.hip' EXIT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form \
  -c -o $O/orb_kernels_old.o orbslam3lib_amd/csrc/zz_old_kernels.hip
objs=$(ls orbslam3lib_amd/csrc/build/*.o | grep -v orb_kernels.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $O/liborbgpu_old.so $O/orb_kernels_old.o $objs
echo built $O/liborbgpu_old.so from $REV
