#!/bin/bash
# Kernel trace of a few single-stream batch steps (each dispatch = one stage over the whole batch):
# per-dispatch durations in order, for per-level timing of the pyramid kernels.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp ORBGPU_DIAGNOSTICS=1 ORBGPU_STREAMS=1
O=${1:-gpurun_out/trace}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/profile_batch.py > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-40:]
for r in last:
    print("%-40s %8.1f us" % (r["Kernel_Name"][:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
