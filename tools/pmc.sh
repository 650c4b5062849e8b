#!/bin/bash
# PMC passes over tools/profile_batch.py (one counter group per rocprofv3 run, kernel trace only).
# One stream so each dispatch is one kernel over the whole batch.  Usage: tools/pmc.sh OUTDIR
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE SQ_LEVEL_WAVES SQ_INST_CYCLES_VMEM" ; do
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/profile_batch.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo pmc-done
