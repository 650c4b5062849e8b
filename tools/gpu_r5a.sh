#!/bin/bash
# Round 5, first GPU call: the GPU suite, the full bench (no CPU leg), the C4 kernel trace and a
# sweep of the k_pyr_tail image threshold (ORBGPU_TAIL_MIN) over the headline + side configs.
cd "$(dirname "$0")/.."
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
summ() {
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));oc=d.get('other_configs',{})
print('%-22s C2 %.1f (%.4f ms)' % (sys.argv[2], d['value'], d['ms_per_step']), ' '.join('%s %.1f/%.4fms' % (k, v['mfeatures_s'], v['ms_per_step']) for k, v in sorted(oc.items())))" "$@"
}
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
summ $O/bench.json default
python3 -c "import json;d=json.load(open('$O/bench.json'));[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()]"
export ORBGPU_DIAGNOSTICS=1
for tm in 0 64 256 100000; do
  ORBGPU_TAIL_MIN=$tm timeout -k 10 300 python bench.py --no-cpu-baseline --no-stereo --no-grid --no-wire --no-sbp --no-profile > $O/tail_$tm.json 2> $O/tail_$tm.err || { tail -20 $O/tail_$tm.err; exit 1; }
  summ $O/tail_$tm.json "TAIL_MIN=$tm"
done
unset ORBGPU_DIAGNOSTICS
bash tools/c4_trace.sh $O/c4 | tail -30
