#!/bin/bash
# GPU suite on the current build, single-stream kernel stats of K for the build and every variant,
# then the headline A/B (tools/bench_ab.sh, REPS rounds).  Stops at the first failure.
cd "$(dirname "$0")/.."
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 bash tools/time_variants.sh "${K:-k_}" > $O/ktime.txt 2>&1 || { tail -20 $O/ktime.txt; exit 1; }
cat $O/ktime.txt
REPS=${REPS:-3} timeout -k 10 900 bash tools/bench_ab.sh
