#!/bin/bash
# One-call refresh of the round's evidence (run on the GPU box from the repo root):
# GPU parity log, the FETCH_SIZE/WRITE_SIZE traffic passes (written to profiles/traffic_$ROUND.json
# on the box so the bench line that follows carries them), the bench line, the rocprofv3
# kernel-trace summary of the same bench command, the roofline cross-check and the PMC
# instruction counters (before the bench: its roofline_valu reads them).  Stops at the first failing step.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${ROUND:-r03}
O=gpurun_out/refresh
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo pytest-done
bash tools/pmc_traffic.sh $O/pmct
python3 tools/traffic.py $O/pmct $O/traffic.json --images $((2 * ${PAIRS:-256})) --steps ${STEPS:-3} > /dev/null
cp $O/traffic.json profiles/traffic_$R.json
echo traffic-done
bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt
mkdir -p profiles/$R && cp $O/pmc_summary.txt profiles/$R/pmc_summary.txt  # the bench line's roofline_valu reads it
echo pmc-done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo bench-done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/prof.log 2>&1
echo prof-done
grep '"metric"' $O/prof.log > $O/bench_profiled.json
python3 tools/roofline_check.py $O/bench_profiled.json $O/prof/run_kernel_trace.csv > $O/roofline_check.json
python3 tools/roofline_check.py $O/bench.json $O/prof/run_kernel_trace.csv > $O/roofline_check_unprofiled_run.json
echo all-done
