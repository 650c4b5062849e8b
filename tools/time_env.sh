#!/bin/bash
# Single-stream kernel stats of tools/profile_batch.py under each environment setting given,
# e.g. tools/time_env.sh k_octree "ORBGPU_OCT_SPLIT=8" "ORBGPU_OCT_SPLIT=3"
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
K=$1; shift
i=0
for setting in "$@"; do
  O=gpurun_out/timeenv/$i
  mkdir -p $O
  env $setting timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/profile_batch.py > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
  f=$(find $O -name "run_kernel_stats.csv" | head -1)
  echo "== $setting"; python3 -c "import csv,sys;[print('%s  calls %s  avg_us %.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r['Name']]" $f "$K"
  i=$((i+1))
done
