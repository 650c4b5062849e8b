#!/bin/bash
# GPU suite, C4 trace and the bench (no CPU leg).  Stops at the first failure.
cd "$(dirname "$0")/.."
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 bash tools/c4_trace.sh $O/c4 > $O/c4.txt 2>&1 || { tail $O/c4.txt; exit 1; }
tail -12 $O/c4.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['matches']['value']);[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()];print('C4',d['other_configs']['C4']['ms_per_step'],'C3',d['other_configs']['C3']['mfeatures_s'],'C5',d['other_configs']['C5']['mfeatures_s'])"
