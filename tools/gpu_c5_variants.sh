#!/bin/bash
# C5 / C3 side lines of the bench (other_configs) for the default build and every variant library
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for rep in 1 2; do
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  ORBGPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-profile > gpurun_out/c5_$n.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));o=d['other_configs'];print('%-22s C5 %.1f C3 %.1f C4 %.3f head %.1f'%(sys.argv[2],o['C5']['mfeatures_s'],o['C3']['mfeatures_s'],o['C4']['ms_per_step'],d['value']))" gpurun_out/c5_$n.json $n
done
done
