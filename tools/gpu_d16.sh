#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/d16; mkdir -p $O
timeout -k 10 60 ./tools/d16_probe
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/liborbgpu_d16w.so; do
  echo "== $lib"
  ORBGPU_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_adversarial.py tests/test_fast_thresholds.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > $O/$(basename $lib).log 2>&1; tail -3 $O/$(basename $lib).log
done
