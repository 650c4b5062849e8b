#!/bin/bash
# GPU suite, single-stream kernel stats of every kernel (tools/time_variants.sh over the default
# build and any variants), then the bench without the CPU leg.  Stops at the first failure.
cd "$(dirname "$0")/.."
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
if [ -n "$VTESTS" ]; then  # parity of each variant build on the named tests (a failure is reported, not fatal)
  for lib in orbslam3lib_amd/variants/*.so; do
    n=$(basename $lib .so)
    ORBGPU_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest $VTESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$n.log 2>&1
    rc=$?; echo "$n parity rc=$rc: $(tail -1 $O/pytest_$n.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
fi
timeout -k 10 400 bash tools/time_variants.sh "${K:-k_}" > $O/ktime.txt 2>&1 || { tail -20 $O/ktime.txt; exit 1; }
cat $O/ktime.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['matches']['value']);[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()];print('C4',d['other_configs']['C4']['ms_per_step'])"
