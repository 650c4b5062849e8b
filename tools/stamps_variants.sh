#!/bin/bash
# octree phase stamps (one pair) for the default library and every variant build
cd "$(dirname "$0")/.."
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  echo "== $(basename $lib .so)"
  ORBGPU_LIB=$PWD/$lib timeout -k 10 120 python3 tools/octree_stamps.py ${1:-1} 2>&1 | grep -E "L0|L7" || exit 1
done
