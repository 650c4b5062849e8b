"""Print the headline and the serialized per-stage table of a bench.py JSON line.
usage: python tools/stages.py gpurun_out/bench.json [more.json ...]"""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print("%s: %.1f Mfeatures/s, %.4f ms/step" % (path, d["value"], d["ms_per_step"]))
    tot = 0.0
    for k, v in d.get("stages", {}).items():
        tot += v.get("us_per_step", 0.0)
        print("  %-20s %8.1f us/step  avg %8.2f  frac %s  launches %s" % (
            k, v.get("us_per_step", 0.0), v.get("avg_us", 0.0), v.get("frac_hbm"), v.get("launches")))
    print("  serialized sum %.1f us" % tot)
    for key in ("roofline", "roofline_fast_pyramid", "roofline_knn2"):
        r = d.get(key) or {}
        print("  %-22s frac %s achieved %s %s" % (key, r.get("frac"), r.get("achieved"), r.get("unit")))
