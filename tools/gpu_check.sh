#!/bin/bash
# GPU parity tests + a short bench (no CPU baseline) from the repo root; stops at the first failure.
cd "$(dirname "$0")/.."
O=gpurun_out/check
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['matches']['value']);[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()]"
python3 -c "import json;d=json.load(open('$O/bench.json'));print('stereo',d.get('stereo_matches'));print('grid',d.get('undistort_grid'));print('wire',d.get('wire'));print('sbp',d.get('search_by_projection'));print('configs',d.get('other_configs'));print('cpu',d.get('cpu_baseline'))"
