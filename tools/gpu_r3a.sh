#!/bin/bash
# round-3 check: GPU tests, 1-GPU bench, 2-rank rehearsal on one GPU (gloo)
cd "$(dirname "$0")/.."
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
echo pytest-ok
timeout -k 10 300 python bench.py --steps 10 > $O/bench.json 2> $O/bench.err || { echo bench-failed; tail -20 $O/bench.err; exit 1; }
echo bench-ok
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --no-cpu-baseline --no-sbp --no-wire --no-configs > $O/bench2.json 2> $O/bench2.err || { echo bench2-failed; tail -20 $O/bench2.err; exit 1; }
echo all-ok
