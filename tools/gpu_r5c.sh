#!/bin/bash
# Round 5: GPU suite, single-stream kernel times of the default build and the measurement
# variants, the headline bench, and the PMC passes of the default build.
cd "$(dirname "$0")/.."
O=gpurun_out/${OUT:-r5c}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/time_variants.sh "k_" 2>&1 | grep -v "k_pack\|k_sbs\|k_undist\|k_stereo\|k_sbp\|k_fish"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'));oc=d.get('other_configs',{})
print('C2 %.1f (%.4f ms)' % (d['value'], d['ms_per_step']), ' '.join('%s %.1f/%.4fms' % (k, v['mfeatures_s'], v['ms_per_step']) for k, v in sorted(oc.items())))
[print(k,v['avg_us'],v['launches']) for k,v in d['stages'].items()]"
if [ -z "$NOPMC" ]; then
bash tools/pmc.sh $O/pmc > /dev/null && python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt && grep -A16 "k_fast_cells<48>\|k_orient_desc\|k_knn2_mfma_pairs" $O/pmc_summary.txt | head -60
fi
