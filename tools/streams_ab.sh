#!/bin/bash
# Headline step vs chunk-stream count (ORBGPU_STREAMS), bench without CPU baseline / profiling.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sab
for n in ${LIST:-3 2 4 3}; do
  ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile > gpurun_out/sab/b$n.json 2> gpurun_out/sab/b$n.err || { tail -5 gpurun_out/sab/b$n.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('streams',sys.argv[2],d['value'],d['ms_per_step'])" gpurun_out/sab/b$n.json $n
done
