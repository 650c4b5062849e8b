#!/bin/bash
# GPU parity (TESTS=..., default all) + bench without the CPU leg + single-stream kernel trace.
cd "$(dirname "$0")/.."
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['matches']['value']);print('fp',d['roofline_fast_pyramid']);[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()]"
bash tools/trace_levels.sh $O/trace | tail -${TRACE_TAIL:-16}
