#!/bin/bash
# Kernel trace of the C4 shape (one stereo pair per step, kNN2): per-kernel durations and the
# timeline of the last step.  Usage: tools/c4_trace.sh [OUTDIR]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-gpurun_out/c4}
mkdir -p $O
STEPS=30 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/c4_run.py > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# steps start at the first k_blur_resize after a k_knn2
starts = [i for i, r in enumerate(rows) if ("k_blur_resize" in r["Kernel_Name"] or "k_pyr_chain" in r["Kernel_Name"]) and (i == 0 or "knn2" in rows[i - 1]["Kernel_Name"])]
for s0, s1 in zip(starts[-4:-1], starts[-3:]):
    t0 = int(rows[s0]["Start_Timestamp"]); t1 = int(rows[s1]["Start_Timestamp"])
    print("step %.1f us" % ((t1 - t0) / 1e3))
s0, s1 = starts[-2], starts[-1]
t0 = int(rows[s0]["Start_Timestamp"])
prev_end = t0
for r in rows[s0:s1]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  %8.1f +%6.1f  dur %7.1f  %s" % ((st - t0) / 1e3, (st - prev_end) / 1e3, (en - st) / 1e3, r["Kernel_Name"].split("(")[0][:50]))
    prev_end = en
PY
