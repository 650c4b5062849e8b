#!/bin/bash
# chunk streams and batch size around the headline, plus the 2-rank gloo rehearsal of the bench
cd "$(dirname "$0")/.."
O=gpurun_out/sweep3
mkdir -p $O
B="--no-cpu-baseline --no-sbp --no-wire --no-stereo --no-grid --no-configs"
for st in 3 4 2 3; do
  ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=$st timeout -k 10 200 python bench.py $B > $O/s$st.json 2>/dev/null || exit 1
  echo "streams $st $(python3 -c "import json;d=json.load(open('$O/s$st.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 200 python bench.py $B --pairs 384 > $O/p384.json 2>/dev/null || exit 1
echo "pairs 384 $(python3 -c "import json;d=json.load(open('$O/p384.json'));print(d['value'],d['ms_per_step'])")"
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --no-cpu-baseline --no-sbp --no-wire --no-configs > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail $O/bench_2rank.err; exit 1; }
echo 2rank-ok
