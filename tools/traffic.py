"""Turns the rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh over
tools/profile_batch.py, ORBGPU_STREAMS=1: every stage one whole-batch launch per step, as in the
bench's serialized pass) into HBM traffic per image and step, per bench stage name.

hbm bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: MI355X_MICROARCH.md §HBM -- on gfx950
FETCH_SIZE reads half the bytes of a wide coalesced read (the x2 correction is calibrated for
16 B/lane streams; narrower accesses are uncalibrated, so the figure is an upper estimate for
them), WRITE_SIZE is exact for streaming stores.  bench.py multiplies hbm_bytes_per_image_step by
the images of a launch and divides by the launches per step, like its algorithmic bytes.
Usage: python tools/traffic.py PMC_DIR OUT_JSON --images N --steps S --width W --height H
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def stage_name(kernel):
    """The bench stage a kernel belongs to: k_octree<NT> -> k_octree, k_knn2_mfma_pairs -> k_knn2,
    k_fast_cells<48, true> and its overflow pass k_fast_cells_ovf<48> -> k_fast_cells<48>."""
    k = kernel.split("(")[0].replace("orbgpu::", "").replace("void ", "").strip()
    k = re.sub(r"^k_octree<\d+>$", "k_octree", k)
    k = re.sub(r"^k_fast_cells(?:_ovf)?<(\d+)(?:, (?:true|false))?>$", r"k_fast_cells<\1>", k)
    return {"k_knn2_mfma_pairs": "k_knn2"}.get(k, k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--images", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(a.src, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            acc[stage_name(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"_config": {"images_per_launch": a.images, "steps": a.steps, "width": a.width, "height": a.height}}
    for k, c in acc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c or k.startswith("__"):
            continue
        fetch, write = sum(c["FETCH_SIZE"]), sum(c["WRITE_SIZE"])  # KiB over every launch
        per = (2 * fetch + write) * 1024 / (a.steps * a.images)
        out[k] = {"fetch_kb_total": round(fetch, 1), "write_kb_total": round(write, 1),
                  "launches": len(c["FETCH_SIZE"]), "hbm_bytes_per_image_step": round(per, 1)}
    out["_note"] = ("(2*FETCH_SIZE + WRITE_SIZE)*1024 summed over a step's launches, per image; "
                    "tools/pmc_traffic.sh over tools/profile_batch.py (ORBGPU_STREAMS=1: whole-batch launches)")
    json.dump(out, open(a.dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
