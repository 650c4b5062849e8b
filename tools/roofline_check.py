"""Cross-check of bench.py's roofline kernel time against the rocprofv3 kernel trace of the same
bench command (tools/refresh_profiles.sh): the mean duration of the dominant kernel's launches in
the timed region (the last steps x chunks launches) and over all launches.
Usage: python tools/roofline_check.py BENCH_JSON KERNEL_TRACE_CSV [steps] [chunks]"""
import csv
import json
import sys

bench = json.load(open(sys.argv[1]))
steps = int(sys.argv[3]) if len(sys.argv) > 3 else bench["steps"]
chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 3  # ORBGPU_STREAMS default
name = bench["roofline"]["kernel"]
rows = [r for r in csv.DictReader(open(sys.argv[2])) if name in r["Kernel_Name"].replace("void ", "")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the headline steps launch the kernel on the chunk streams with the chunk grids (one grid per
# level and chunk size for a per-level kernel); the bench's serialized profiling pass (whole-batch
# grids) and the side-line configs (other grids) interrupt them: the timed region is the end of
# the longest run of launches whose grids occur among the first step's
grid = lambda r: (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
n_timed = bench["roofline"].get("timed_launches") or steps * chunks
per_chunk_step = max(1, n_timed // (steps * chunks))  # launches per chunk per step (levels)
first = {grid(r) for r in rows[:bench.get("warmup", 3) * chunks * per_chunk_step]}  # warm-up steps
runs, cur = [], []
for r in rows:
    if grid(r) in first:
        cur.append(r)
    else:
        if cur:
            runs.append(cur)
        cur = []
if cur:
    runs.append(cur)
head = max(runs, key=len)
# the serialized pass (whole-batch grids, the kernel alone on the GPU) is the first run of other
# grids after the warm-up steps
ser, cur, seen_head = [], [], False
for r in rows:
    if grid(r) in first:
        if cur:
            break
        continue
    cur.append(r)
ser = cur
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in head]
timed = d[-n_timed:]
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ser]
print(json.dumps({"kernel": name, "bench_avg_us": bench["roofline"]["avg_us"],
                  "rocprof_timed_region_avg_us": round(sum(timed) / len(timed), 2),
                  "rocprof_headline_launches_avg_us": round(sum(d) / len(d), 2), "launches": len(d),
                  "bench_serialized_avg_us": bench["roofline"].get("serialized_avg_us"),
                  "rocprof_serialized_avg_us": round(sum(ds) / len(ds), 2) if ds else None,
                  "serialized_launches": len(ds)}))
