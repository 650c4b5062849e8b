#!/bin/bash
# bench.py (no CPU leg) under each environment setting: value and ms_per_step per setting.
cd "$(dirname "$0")/.."
# the library honours ORBGPU_* knobs only with the diagnostics gate on
export ORBGPU_DIAGNOSTICS=1
mkdir -p gpurun_out/benchenv
i=0
for setting in "$@"; do
  env $setting timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/benchenv/$i.json 2> gpurun_out/benchenv/$i.err || { tail gpurun_out/benchenv/$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/benchenv/$i.json'));print('%-70s %8.2f %7.4f'%(sys.argv[1],d['value'],d['ms_per_step']))" "$setting"
  i=$((i+1))
done
