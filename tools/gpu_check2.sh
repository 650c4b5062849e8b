#!/bin/bash
# GPU parity tests (optionally a subset: TESTS=...) + the full bench line (CPU baseline included).
cd "$(dirname "$0")/.."
O=gpurun_out/check2
mkdir -p $O
echo "nproc $(nproc) affinity $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $O/host.txt
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/host.txt
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['matches']['value']);print('h2d',d['h2d']);print('roof',d['roofline']);print('fp',d['roofline_fast_pyramid']);print('knn',d['roofline_knn2']);print('cpu',d['cpu_baseline']);[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()]"
