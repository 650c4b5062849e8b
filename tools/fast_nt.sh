#!/bin/bash
cd "$(dirname "$0")/.."
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
PAIRS_LIST=1,128 timeout -k 10 200 python3 tools/stage_scaling.py 2>&1 | tail -2 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit 1
head -c 420 gpurun_out/b.json; echo
ORBGPU_DIAGNOSTICS=1 ORBGPU_ISOLATE=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_noiso.json 2> gpurun_out/b_noiso.err || exit 1
head -c 420 gpurun_out/b_noiso.json; echo
