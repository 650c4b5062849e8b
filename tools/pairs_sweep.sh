#!/bin/bash
# Headline throughput against the batch size (pairs per step), every side leg off.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pairs
for p in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-configs --pairs $p > gpurun_out/pairs/$p.json 2> gpurun_out/pairs/$p.err || { tail gpurun_out/pairs/$p.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/pairs/$p.json'));print('pairs',$p,d['value'],d['ms_per_step'], round(d['ms_per_step']/$p*1e3,2),'us/pair')"
done
