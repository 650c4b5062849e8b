#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes only (separate rocprofv3 runs, kernel trace only) over
# tools/profile_batch.py with one stream: every stage one whole-batch launch per step, the shape
# of bench.py's serialized pass.  Usage: tools/pmc_traffic.sh OUTDIR (PAIRS / STEPS as profile_batch)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/pmct}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p0 -o pmc -- python3 tools/profile_batch.py > $OUT/p0.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p1 -o pmc -- python3 tools/profile_batch.py > $OUT/p1.log 2>&1
echo traffic-done
