"""Aggregate rocprofv3 --pmc CSVs (tools/pmc.sh output) into per-kernel averages per dispatch."""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
# the binary these counters describe (bench.py uses them only for the same liborbgpu.so)
import hashlib
lib = os.environ.get("ORBGPU_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "orbslam3lib_amd", "liborbgpu.so")
if os.path.exists(lib):
    print("# liborbgpu.so sha256 %s" % hashlib.sha256(open(lib, "rb").read()).hexdigest())
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    if k.startswith("__amd"):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-24s %14.4g" % (c, sum(v) / len(v)))
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        print("   VALU/wave %.0f  LDS/wave %.0f  SALU/wave %.0f" % (
            d["SQ_INSTS_VALU"] / d["SQ_WAVES"], d.get("SQ_INSTS_LDS", 0) / d["SQ_WAVES"],
            d.get("SQ_INSTS_SALU", 0) / d["SQ_WAVES"]))
    if "SQ_ACTIVE_INST_VALU" in d and "GRBM_GUI_ACTIVE" in d:
        pass
