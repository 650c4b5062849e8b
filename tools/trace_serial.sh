#!/bin/bash
# Kernel trace of the bench batch on one stream (each launch alone): per-launch durations.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
OUT=${1:-gpurun_out/trace1}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o tr -- python3 tools/profile_batch.py > $OUT/log 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/tr_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = rows[-30:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3; d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("%-34s grid %9s %8.1f %7.1f" % (r["Kernel_Name"].split("(")[0][-34:], r["Grid_Size_X"] + "x" + r["Grid_Size_Y"] + "x" + r["Grid_Size_Z"], s, d))
PY
