#!/bin/bash
# Variant libraries (orbslam3lib_amd/variants: 16-lane k_orient_desc, 16-wave kNN2) vs the
# default: parity of each, then single-stream timing, then the chunk-stream A/B.  The variants are
# full-library builds with -DOD_LANES=16 (the runtime sizes the orientation grid from it) and
# tools/build_variants.sh knn16 "-DKNN_WAVES=16" (16-wave kNN2, since removed from the source).
cd "$(dirname "$0")/.."
for v in od16 knn16; do
  ORBGPU_LIB=$PWD/orbslam3lib_amd/variants/liborbgpu_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_batch_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/pt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/time_variants.sh "k_" > gpurun_out/tv4.log 2>&1 || exit 1
grep -E "==|orient|knn2_mfma" gpurun_out/tv4.log
bash tools/streams_ab.sh
