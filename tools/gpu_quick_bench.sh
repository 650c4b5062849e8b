#!/bin/bash
# GPU tests, then the headline bench; prints value and the serialized stage table.
cd "$(dirname "$0")/.."
O=gpurun_out/qb
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in ${RUNS:-1}; do
timeout -k 10 300 python bench.py --steps 20 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo bench-failed; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms/step", d["ms_per_step"], "C4", d.get("other_configs", {}).get("C4", {}).get("ms_per_step"))
for k, s in d["stages"].items():
    print("  %-18s %8.1f us/step  traffic/alg %s" % (k, s["us_per_step"], s.get("traffic_over_algorithmic")))
PY
done
