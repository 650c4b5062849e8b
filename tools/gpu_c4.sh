#!/bin/bash
# combined extraction + match submission: its GPU tests, the facade test, bench C4, C4 trace
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/c4m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "run_batch_match or facade or two_contexts or caller_stream" > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
echo pytest-ok
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sbp --no-wire --no-stereo --no-grid > $O/bench.json 2> $O/bench.err || { echo bench-failed; tail -20 $O/bench.err; exit 1; }
bash tools/c4_trace.sh $O/c4 > $O/c4.txt 2>&1
echo all-ok
