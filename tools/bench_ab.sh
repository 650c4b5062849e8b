#!/bin/bash
# Headline bench (no CPU leg, no side legs) alternating the default build and every variant
# under orbslam3lib_amd/variants, REPS rounds: value and ms_per_step per run.
cd "$(dirname "$0")/.."
O=gpurun_out/bench_ab; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-configs --no-profile > /dev/null 2>&1  # warm-up
for rep in $(seq ${REPS:-3}); do
  for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
    n=$(basename $lib .so)
    VENV=""; [ -f ${lib%.so}.env ] && VENV="ORBGPU_DIAGNOSTICS=1 $(cat ${lib%.so}.env)"  # per-variant knobs
    env $VENV ORBGPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-configs --no-profile > $O/$n.$rep.json 2> $O/$n.$rep.err || { tail -5 $O/$n.$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('%-22s %8.2f %7.4f'%(sys.argv[2],d['value'],d['ms_per_step']))" $O/$n.$rep.json $n
  done
done
