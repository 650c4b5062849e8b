#!/bin/bash
# Blur tile height A/B: needs orbslam3lib_amd/variants/liborbgpu_th48.so, i.e. every source of the
# library built with -DBLUR_TH=48 (the host tiling follows kBlurTH).  Parity with the default and
# the variant, single-stream timing of both, then smoke().
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
ORBGPU_LIB=$PWD/orbslam3lib_amd/variants/liborbgpu_th48.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_batch_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt48.log 2>&1; rc=$?; tail -1 gpurun_out/pt48.log; [ $rc -eq 0 ] || exit $rc
bash tools/time_variants.sh k_blur > gpurun_out/tv3.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
