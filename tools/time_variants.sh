#!/bin/bash
# Single-stream kernel stats of tools/profile_batch.py for each library under orbslam3lib_amd/variants
# (plus the default build).  Usage: tools/time_variants.sh [KERNEL_SUBSTRING]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
K=${1:-k_fast_cells}
# the first process on a fresh box runs slow (clocks, code-object load): one untimed warm-up run
timeout -k 10 120 python3 tools/profile_batch.py > /dev/null 2>&1
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  O=gpurun_out/variants/$n
  mkdir -p $O
  VENV=""; [ -f ${lib%.so}.env ] && VENV=$(cat ${lib%.so}.env)  # per-variant knobs, e.g. ORBGPU_OD_ITERS=2
  env $VENV ORBGPU_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/profile_batch.py > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
  f=$(find $O -name "run_kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "import csv,sys;[print('%s  calls %s  avg_us %.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r['Name']]" $f "$K"
done
