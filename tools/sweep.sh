#!/bin/bash
# Env sweep of the bench: each argument is one env assignment list ("A=1 B=2"); prints value + stages.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
i=0
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/sweep/b$i.json 2> gpurun_out/sweep/b$i.err || { echo "FAIL $cfg"; tail -5 gpurun_out/sweep/b$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/sweep/b$i.json'));print(sys.argv[1],'|',d['value'],d['ms_per_step'],'|',' '.join('%s=%.0f'%(k,v['avg_us']) for k,v in d['stages'].items()))" "$cfg"
  i=$((i+1))
done
