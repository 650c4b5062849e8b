#!/bin/bash
# octree iteration: octree GPU tests, stamps (1 and 64 pairs), headline bench, C4 trace
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/oct2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "octree or adversarial or bench_batch or edges or parity" > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
echo pytest-ok
timeout -k 10 120 python3 tools/octree_stamps.py 1 > $O/stamps1.txt 2>&1 && timeout -k 10 120 python3 tools/octree_stamps.py 64 > $O/stamps64.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sbp --no-wire --no-stereo --no-grid > $O/bench.json 2> $O/bench.err || { echo bench-failed; tail -20 $O/bench.err; exit 1; }
bash tools/c4_trace.sh $O/c4 > $O/c4.txt 2>&1
echo all-ok
