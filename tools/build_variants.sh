#!/bin/bash
# Measurement variants of liborbgpu.so: one translation unit (SRC, default orb_kernels.hip)
# rebuilt with extra defines, linked with the other objects of the normal build.
# Usage: [SRC=orb_fast.hip] tools/build_variants.sh NAME "-DFOO=1" [...]
cd "$(dirname "$0")/.."
set -e
SRC=${SRC:-orb_kernels.hip}
make -s orbslam3lib_amd/liborbgpu.so
O=orbslam3lib_amd/variants
mkdir -p $O
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form \
    $defs -c -o $O/${SRC%.hip}_$name.o orbslam3lib_amd/csrc/$SRC
  objs=$(ls orbslam3lib_amd/csrc/build/*.o | grep -v "$SRC.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $O/liborbgpu_$name.so $O/${SRC%.hip}_$name.o $objs
  echo built $O/liborbgpu_$name.so
done
