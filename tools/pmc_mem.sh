#!/bin/bash
# Vector-memory pipeline counters (TA / TD / TCP busy and stalls) over tools/profile_batch.py,
# one pass per group, each pass failing alone.  Usage: tools/pmc_mem.sh OUTDIR
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/pmc_mem}
mkdir -p $OUT
i=0
for grp in "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  timeout -k 10 60 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/profile_batch.py > $OUT/p$i.log 2>&1 || echo "pass $i failed"
  i=$((i+1))
done
echo pmc-done
