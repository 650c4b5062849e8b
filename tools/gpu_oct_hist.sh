#!/bin/bash
# octree A/B against a variant (V): GPU suite, one-pair phase stamps, C4 step time, octree alone, bench A/B
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/octh
mkdir -p $O
V=$PWD/orbslam3lib_amd/variants/liborbgpu_head.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python3 tools/octree_stamps.py 1 2>&1 | tail -8
ORBGPU_LIB=$V timeout -k 10 120 python3 tools/octree_stamps.py 1 2>&1 | tail -8
timeout -k 10 120 python tools/c4_time.py
ORBGPU_LIB=$V timeout -k 10 120 python tools/c4_time.py
bash tools/time_variants.sh k_octree
REPS=2 bash tools/bench_ab.sh
