#!/bin/bash
# Measurement variants of liborbgpu.so: orb_kernels.hip rebuilt with extra defines, linked with
# the other objects of the normal build.  Usage: tools/build_variants.sh NAME "-DFOO=1" [...]
cd "$(dirname "$0")/.."
set -e
make -s orbslam3lib_amd/liborbgpu.so
O=orbslam3lib_amd/variants
mkdir -p $O
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form \
    $defs -c -o $O/orb_kernels_$name.o orbslam3lib_amd/csrc/orb_kernels.hip
  objs=$(ls orbslam3lib_amd/csrc/build/*.o | grep -v orb_kernels.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $O/liborbgpu_$name.so $O/orb_kernels_$name.o $objs
  echo built $O/liborbgpu_$name.so
done
