#!/bin/bash
# PMC passes (VALU / LDS / waves / wait counters) over tools/profile_batch.py for k_fast_sb
# (ORBGPU_FAST_SB=1) and then the default per-cell k_fast_cells.  Usage: tools/pmc_fast.sh OUTDIR
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/pmc_fast}
mkdir -p $OUT
i=0
for env in "ORBGPU_FAST_SB=1" "X=1"; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
    env $env timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/profile_batch.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
    i=$((i+1))
  done
done
echo pmc-done
