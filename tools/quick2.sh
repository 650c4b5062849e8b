#!/bin/bash
cd "$(dirname "$0")/.."
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1
rc=$?; tail -30 gpurun_out/pt.log | grep -v "^$" | tail -25; [ $rc -eq 0 ] || exit $rc
bash tools/trace_serial.sh gpurun_out/trace2 | tail -15 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit 1
head -c 300 gpurun_out/b.json; echo
