#!/bin/bash
# C4 step time (tools/c4_time.py) for the default build and every variant library
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for rep in 1 2; do
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  VENV=""; [ -f ${lib%.so}.env ] && VENV="ORBGPU_DIAGNOSTICS=1 $(cat ${lib%.so}.env)"  # per-variant knobs
  echo "== $(basename $lib .so)"; env $VENV ORBGPU_LIB=$PWD/$lib timeout -k 10 120 python tools/c4_time.py | tail -2
done
done
