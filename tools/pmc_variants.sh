#!/bin/bash
# tools/pmc.sh for the default build and each library under orbslam3lib_amd/variants, then the
# per-kernel summary of KERNEL (default k_fast_cells<48>).
cd "$(dirname "$0")/.."
K=${1:-k_fast_cells<48>}
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  ORBGPU_LIB=$PWD/$lib bash tools/pmc.sh gpurun_out/pmcv/$n > gpurun_out/pmcv_$n.log 2>&1 || { tail gpurun_out/pmcv_$n.log; exit 1; }
  echo "== $n"; python3 tools/pmc_summary.py gpurun_out/pmcv/$n | grep -A20 "$K" | head -21
done
