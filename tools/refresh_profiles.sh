#!/bin/bash
# One-call refresh of the round's evidence (run on the GPU box from the repo root):
# GPU parity log, the bench line, the rocprofv3 kernel-trace summary of the same bench
# command, and the FETCH_SIZE/WRITE_SIZE traffic passes.  Stops at the first failing step.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/refresh
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo pytest-done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo bench-done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/prof.log 2>&1
echo prof-done
bash tools/pmc_traffic.sh $O/pmct
python3 tools/traffic.py $O/pmct $O/traffic.json > /dev/null
python3 tools/roofline_check.py $O/bench.json $O/prof/run_kernel_trace.csv > $O/roofline_check.json
echo all-done
