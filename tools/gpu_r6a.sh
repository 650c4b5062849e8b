#!/bin/bash
# Round 6, first call: product GPU suite, the 4-wave kNN2 variant on test_batch_edges, and the
# repeatability check (tools/determinism.py) with both libraries.  A parity failure (exit 1)
# continues; any other non-zero exit (fault, abort, time limit) ends the script.
cd "$(dirname "$0")/.."
O=gpurun_out/r6a
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step det_product 240 python -u tools/determinism.py 6
ORBGPU_LIB=orbslam3lib_amd/variants/liborbgpu_knn4.so step edges_knn4 240 python -u -m pytest tests/test_batch_edges.py -q --timeout 120 --timeout-method thread
ORBGPU_LIB=orbslam3lib_amd/variants/liborbgpu_knn4.so step det_knn4 240 python -u tools/determinism.py 6
