#!/bin/bash
# Headline only (every side leg off) under each environment setting: value and ms_per_step.
cd "$(dirname "$0")/.."
# the library honours ORBGPU_* knobs only with the diagnostics gate on
export ORBGPU_DIAGNOSTICS=1
mkdir -p gpurun_out/benchenvf
i=0
for setting in "$@"; do
  env $setting timeout -k 10 300 python bench.py --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-configs > gpurun_out/benchenvf/$i.json 2> gpurun_out/benchenvf/$i.err || { tail gpurun_out/benchenvf/$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/benchenvf/$i.json'));print('%-50s %8.2f %7.4f'%(sys.argv[1],d['value'],d['ms_per_step']))" "$setting"
  i=$((i+1))
done
