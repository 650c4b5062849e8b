#!/bin/bash
# Compute PMC (tools/pmc.sh groups) for the default build and every variant, one kernel's lines.
# Usage: tools/pmc_variants_all.sh KERNEL_SUBSTRING
cd "$(dirname "$0")/.."
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  ORBGPU_LIB=$PWD/$lib bash tools/pmc.sh gpurun_out/pmc_$n > /dev/null
  echo "== $n"; python3 tools/pmc_summary.py gpurun_out/pmc_$n | grep -A19 "$1" | head -20
done
