"""Turns rocprofv3 PMC passes (tools/pmc.sh) into per-launch HBM traffic per kernel.

hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: MI355X_MICROARCH.md §HBM --
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced read (the x2 correction is
calibrated for 16 B/lane streams; narrower accesses are uncalibrated, so the figure is an upper
estimate for them), WRITE_SIZE is exact for streaming stores.
Usage: python tools/traffic.py gpurun_out/pmct profiles/traffic_r01.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main(src, dst):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("orbgpu::", "").replace("void ", "").strip()
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in acc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        out[k] = {"fetch_kb": round(fetch, 1), "write_kb": round(write, 1),
                  "hbm_bytes_per_launch": int((2 * fetch + write) * 1024),
                  "launches_sampled": len(c["FETCH_SIZE"])}
    out["_note"] = ("(2*FETCH_SIZE + WRITE_SIZE)*1024 per launch, tools/pmc.sh over tools/profile_batch.py "
                    "(128 stereo pairs, the bench batch; FAST launched once over the whole batch as in the bench); k_resize is per level launch (mean over levels)")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
