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
# the headline batch's launches share the first launch's grid (the side-line configs differ)
rows = [r for r in rows if r["Grid_Size_X"] == rows[0]["Grid_Size_X"] and r["Grid_Size_Y"] == rows[0]["Grid_Size_Y"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
timed = d[-steps * chunks:]
print(json.dumps({"kernel": name, "bench_avg_us": bench["roofline"]["avg_us"],
                  "rocprof_timed_region_avg_us": round(sum(timed) / len(timed), 2),
                  "rocprof_all_launches_avg_us": round(sum(d) / len(d), 2), "launches": len(d)}))
