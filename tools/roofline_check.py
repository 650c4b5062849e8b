"""Cross-check of bench.py's roofline kernel time against the rocprofv3 kernel trace of the same
bench command (tools/refresh_profiles.sh): the mean duration of the dominant kernel's launches in
the timed region (the first steps x chunks chunk-grid launches after the serialized pass), over
the whole chunk-grid run, and in the serialized pass.
Usage: python tools/roofline_check.py BENCH_JSON KERNEL_TRACE_CSV [steps] [chunks]
BENCH_JSON is best the line the profiled process itself printed: the concurrent launch time
depends on how the chunk streams' stages happen to line up in that run (a FAST launch that
meets another chunk's FAST takes ~2x as long as one beside the octree or descriptor stage)."""
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
# level and chunk size for a per-level kernel); the bench's serialized profiling pass uses
# whole-batch grids
grid = lambda r: (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
n_timed = bench["roofline"].get("timed_launches") or steps * chunks
per_chunk_step = max(1, n_timed // (steps * chunks))  # launches per chunk per step (levels)
first = {grid(r) for r in rows[:bench.get("warmup", 3) * chunks * per_chunk_step]}  # warm-up steps
# launch order: warm-up steps (chunk grids), the serialized profiled pass (whole-batch grids, the
# kernel alone on the GPU), then the timed region (chunk grids again).  The streaming-ingest loop
# that follows reuses the chunk grids, so the timed region is the first n_timed chunk-grid
# launches after the serialized pass -- not the last ones of the run.
i = 0
while i < len(rows) and grid(rows[i]) in first:
    i += 1
ser = []
while i < len(rows) and grid(rows[i]) not in first:
    ser.append(rows[i])
    i += 1
head = []
while i < len(rows) and grid(rows[i]) in first:
    head.append(rows[i])
    i += 1
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in head]
timed = d[:n_timed]
ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ser]
print(json.dumps({"kernel": name, "bench_avg_us": bench["roofline"]["avg_us"],
                  "rocprof_timed_region_avg_us": round(sum(timed) / len(timed), 2),
                  "rocprof_chunk_grid_run_avg_us": round(sum(d) / len(d), 2), "launches": len(d),
                  "timed_launches": len(timed),
                  "bench_serialized_avg_us": bench["roofline"].get("serialized_avg_us"),
                  "rocprof_serialized_avg_us": round(sum(ds) / len(ds), 2) if ds else None,
                  "serialized_launches": len(ds)}))
