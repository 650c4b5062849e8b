"""Cross-check of bench.py's roofline against the rocprofv3 kernel trace of the same bench command
(tools/refresh_profiles.sh).  The bench line's `roofline` is the dominant kernel alone on the GPU:
its launches in the bench's serialized pass (one whole-batch launch per step, per level for
k_blur_resize), timed with HIP events on the kernel's stream.  Here the same launches are located
in the trace and their mean duration gives frac = bytes_per_launch / mean / peak, which must agree
with the line's frac (within 10%).  The timed region's concurrent launches (chunk
grids, other chunks' stages beside them) are reported beside it.
Usage: python tools/roofline_check.py BENCH_JSON KERNEL_TRACE_CSV [chunks]
BENCH_JSON: the line the profiled process itself printed."""
import csv
import json
import re
import sys

bench = json.load(open(sys.argv[1]))
# chunk streams of the bench context: the runtime's default (orb_runtime.cpp orbgpu_create): 2 for
# contexts of >= 128 pairs, else 3, never more than the pairs
_imgs = bench.get("config", {}).get("images_per_gpu_per_step", 512)
chunks = int(sys.argv[3]) if len(sys.argv) > 3 else min(2 if _imgs >= 256 else 3, max(1, _imgs // 2))
roof = bench["roofline"]
name = roof["kernel"]
steps, warmup = bench["steps"], bench.get("warmup", 3)
def stage_of(kernel):
    """k_fast_cells<48, true> (and every instantiation's bool argument) -> k_fast_cells<48>."""
    k = kernel.split("(")[0].replace("void ", "").replace("orbgpu::", "").strip()
    return re.sub(r"^k_fast_cells<(\d+), (?:true|false)>$", r"k_fast_cells<\1>", k)


allrows = list(csv.DictReader(open(sys.argv[2])))
rows = [r for r in allrows if stage_of(r["Kernel_Name"]) == name or
        (name not in ("k_fast_cells<48>", "k_fast_cells<64>", "k_fast_cells<80>") and name in r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the overflow pass of the small-list FAST kernels runs right after the last FAST launch of a
# step on its stream (the 64-byte one): the stage the bench times (HIP events around its
# launches) ends with that pass, so it is added where it is the next kernel on the stream
by_stream = {}
for r in sorted(allrows, key=lambda r: int(r["Start_Timestamp"])):
    by_stream.setdefault(r["Stream_Id"], []).append(r)
nxt = {}
for lst in by_stream.values():
    for a, b in zip(lst, lst[1:]):
        nxt[id(a)] = b
grid = lambda r: (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])


def dur(r):
    end = int(r["End_Timestamp"])
    b = nxt.get(id(r))
    if b is not None and "k_fast_cells_ovf<" in b["Kernel_Name"]:
        end = int(b["End_Timestamp"])
    return (end - int(r["Start_Timestamp"])) / 1e3
n_ser = roof.get("launches") or 3  # serialized launches (3 steps x launches per step)
per_step = max(1, n_ser // 3)
# launch order: warm-up steps (chunk grids), the serialized pass (whole-batch grids, the kernel
# alone on the GPU), then the timed region (chunk grids again)
first = {grid(r) for r in rows[:warmup * chunks * per_step]}
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
ds = [dur(r) for r in ser]
dt = [dur(r) for r in head][:steps * chunks * per_step]
ser_avg = sum(ds) / len(ds) if ds else None
out = {"kernel": name, "peak_GBps": roof["peak"], "bytes_per_launch": roof.get("bytes_per_launch"),
       "bench_avg_us": roof["avg_us"], "rocprof_serialized_avg_us": round(ser_avg, 2) if ser_avg else None,
       "serialized_launches": len(ds), "bench_frac": roof["frac"]}
if ser_avg and roof.get("bytes_per_launch"):
    fr = roof["bytes_per_launch"] / (ser_avg * 1e-6) / 1e9 / roof["peak"]
    out["rocprof_frac"] = round(fr, 4)
    out["frac_agreement"] = round(fr / roof["frac"], 3) if roof["frac"] else None
    out["within_10pct"] = abs(fr / roof["frac"] - 1) <= 0.10 if roof["frac"] else None
conc = roof.get("concurrent") or {}
out["concurrent"] = {"bench_avg_us": conc.get("avg_us"),
                     "rocprof_timed_region_avg_us": round(sum(dt) / len(dt), 2) if dt else None,
                     "timed_launches": len(dt)}
print(json.dumps(out))
