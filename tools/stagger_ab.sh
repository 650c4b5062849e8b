#!/bin/bash
# Headline step vs chunk-stream count and stagger (re-staggered after the serialized profiling
# pass by default; ORBGPU_STAGGER=0: none).  Usage: CASES="name:ENV=.. ..." tools/stagger_ab.sh
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/stg
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/stg/$name.json 2> gpurun_out/stg/$name.err || { tail -5 gpurun_out/stg/$name.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'],d['matches']['value'])" gpurun_out/stg/$name.json $name
}
for c in ${CASES:-default:X=1 s1:ORBGPU_DIAGNOSTICS=1,ORBGPU_STREAMS=1 s2:ORBGPU_DIAGNOSTICS=1,ORBGPU_STREAMS=2 s2nostg:ORBGPU_DIAGNOSTICS=1,ORBGPU_STREAMS=2,ORBGPU_STAGGER=0 s3:ORBGPU_DIAGNOSTICS=1,ORBGPU_STREAMS=3 s2b:ORBGPU_DIAGNOSTICS=1,ORBGPU_STREAMS=2}; do
  run ${c%%:*} $(echo ${c#*:} | tr ',' ' ')
done
