#!/bin/bash
# tools/pmc_mem.sh for the default build and every variant under orbslam3lib_amd/variants, then
# the summary lines of one kernel.  Usage: tools/pmc_mem_variants.sh KERNEL_SUBSTRING
cd "$(dirname "$0")/.."
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  ORBGPU_LIB=$PWD/$lib bash tools/pmc_mem.sh gpurun_out/pmc_mem_$n > /dev/null
  echo "== $n"; python3 tools/pmc_summary.py gpurun_out/pmc_mem_$n | grep -A14 "$1" | head -15
done
