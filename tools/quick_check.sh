#!/bin/bash
# GPU parity + per-stage scaling + bench line (no CPU baseline); each step under its own limit.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
PAIRS_LIST=${PAIRS_LIST:-1,128} timeout -k 10 200 python3 tools/stage_scaling.py > gpurun_out/ss.log 2>&1
rc=$?; tail -4 gpurun_out/ss.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err
rc=$?; cat gpurun_out/b.json | head -c 600; echo; exit $rc
