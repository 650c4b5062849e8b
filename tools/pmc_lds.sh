#!/bin/bash
# LDS bank-conflict pass over tools/profile_batch.py for the default library and every
# measurement variant under orbslam3lib_amd/variants.  Usage: tools/pmc_lds.sh OUTDIR
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/pmc_lds}
mkdir -p $OUT
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  ORBGPU_LIB=$PWD/$lib timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/$n -o pmc -- python3 tools/profile_batch.py > $OUT/$n.log 2>&1 || { echo "$n failed"; continue; }
  echo "== $n"; python3 tools/pmc_summary.py $OUT/$n | grep -A5 "k_fast_cells<48>"
done
