#!/bin/bash
# A variant library whose orb_kernels.hip (and csrc headers) come from git revision REV, linked
# with the current build's other objects (the BatchArgs layout must match).  For A/B against
# the working tree: tools/build_rev_variant.sh REV NAME
cd "$(dirname "$0")/.."
set -e
REV=$1; NAME=$2
T=$(mktemp -d)
for f in $(git ls-tree --name-only $REV orbslam3lib_amd/csrc/); do git show $REV:$f > $T/$(basename $f); done
sed -i "s#\"../../include/orbgpu.h\"#\"$PWD/include/orbgpu.h\"#" $T/*.h $T/*.hip $T/*.cpp 2>/dev/null || true
mkdir -p orbslam3lib_amd/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form -c -o $T/k.o $T/orb_kernels.hip
objs=$(ls orbslam3lib_amd/csrc/build/*.o | grep -v "orb_kernels.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o orbslam3lib_amd/variants/liborbgpu_$NAME.so $T/k.o $objs
rm -rf $T
echo built orbslam3lib_amd/variants/liborbgpu_$NAME.so
