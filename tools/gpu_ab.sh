#!/bin/bash
# A/B of measurement variants: parity of each variant on the FAST-heavy test files, then the
# single-stream kernel times of the default build and every variant (twice, interleaved).
cd "$(dirname "$0")/.."
O=gpurun_out/ab; mkdir -p $O
for lib in orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  ORBGPU_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest ${AB_TESTS:-tests/test_adversarial.py tests/test_fast_thresholds.py} -m gpu -x -q --timeout 200 --timeout-method thread > $O/$n.log 2>&1 || { echo "$n FAILED"; tail -5 $O/$n.log; }
  echo "$n: $(tail -1 $O/$n.log)"
done
for rep in 1 2; do bash tools/time_variants.sh "${AB_KERNEL:-k_fast_cells<48>}"; done
