#!/bin/bash
# octree work: GPU tests, stamps (1 and 64 pairs), bench (headline + C4), C4 trace
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/oct
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
echo pytest-ok
timeout -k 10 120 python3 tools/octree_stamps.py 1 > $O/stamps1.txt 2>&1 && timeout -k 10 120 python3 tools/octree_stamps.py 64 > $O/stamps64.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sbp --no-wire > $O/bench.json 2> $O/bench.err || { echo bench-failed; tail -20 $O/bench.err; exit 1; }
ORBGPU_DIAGNOSTICS=1 ORBGPU_OCT_PYR=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-sbp --no-wire > $O/bench_nopyr.json 2> $O/bench_nopyr.err || exit 1
bash tools/c4_trace.sh $O/c4 > $O/c4.txt 2>&1
echo all-ok
