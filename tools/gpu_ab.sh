#!/bin/bash
# GPU tests, then headline-only benches A/B/A/B between two environments (ENV_A / ENV_B, e.g.
# ORBGPU_FAST_FUSED=0).  Usage: OUT=gpurun_out/x ENV_A="..." ENV_B="..." bash tools/gpu_ab.sh [notest]
cd "$(dirname "$0")/.."
O=${OUT:-gpurun_out/ab}
mkdir -p $O
if [ "$1" != "notest" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
  echo pytest-ok
fi
H="--steps 20 --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-configs"
for k in 1 2; do
  env $ENV_A timeout -k 10 200 python bench.py $H > $O/a$k.json 2> $O/a$k.err || { echo bench-a-failed; tail $O/a$k.err; exit 1; }
  env $ENV_B timeout -k 10 200 python bench.py $H > $O/b$k.json 2> $O/b$k.err || { echo bench-b-failed; tail $O/b$k.err; exit 1; }
done
python3 - <<'PY'
import json, os
O = os.environ.get("OUT", "gpurun_out/ab")
for f in sorted(os.listdir(O)):
    if f.endswith(".json"):
        d = json.loads(open(os.path.join(O, f)).read().strip().splitlines()[-1])
        st = {k: v["us_per_step"] for k, v in d["stages"].items()}
        print(f, d["value"], d["ms_per_step"], json.dumps(st))
PY
echo all-ok
