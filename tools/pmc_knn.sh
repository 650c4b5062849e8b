#!/bin/bash
# MFMA-pipe counters for the kNN kernel (tools/profile_batch.py, one stream); one pass per group.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/pmck}
mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" ; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/profile_batch.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    if "knn" not in k and "octree" not in k and "orient" not in k:
        continue
    print(k)
    for name, v in sorted(c.items()):
        print("   %-28s %.4g" % (name, v))
PY
