#!/bin/bash
# Kernel time (single stream) and FETCH_SIZE / WRITE_SIZE of one stage for the default build and
# each library under orbslam3lib_amd/variants.  Usage: tools/variant_traffic.sh KERNEL_SUBSTRING
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
K=${1:-k_octree}
for lib in orbslam3lib_amd/liborbgpu.so orbslam3lib_amd/variants/*.so; do
  n=$(basename $lib .so)
  O=gpurun_out/vt/$n
  mkdir -p $O
  export ORBGPU_LIB=$PWD/$lib
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 tools/profile_batch.py > $O/t.log 2>&1 || { tail $O/t.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p0 -o pmc -- python3 tools/profile_batch.py > $O/p0.log 2>&1 || { tail $O/p0.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p1 -o pmc -- python3 tools/profile_batch.py > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
  echo "== $n"
  python3 - "$O" "$K" <<'PY'
import csv, glob, sys, collections
o, k = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(glob.glob(o + "/t/**/run_kernel_stats.csv", recursive=True)[0])):
    if k in r["Name"]:
        print("  %-60s calls %s avg_us %.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
acc = collections.defaultdict(float)
for f in glob.glob(o + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print("  FETCH_SIZE %.1f MB  WRITE_SIZE %.1f MB (all launches)" % (acc["FETCH_SIZE"] / 1024, acc["WRITE_SIZE"] / 1024))
PY
done
