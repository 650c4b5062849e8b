"""Where the run-to-run differences of tools/determinism.py come from: the 1920x1080 / 12-level /
8200-feature frames of seed 60 and 61 under several launch shapes, each run R times, every image's
keypoints compared with the oracle per octave (same count? same (x, y) set? same order?) and the
candidate counts (keys into DistributeOctTree) with the first run.
Usage: python tools/race_probe.py [R]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from orbslam3lib_amd import synth  # noqa: E402


def diff_octaves(k, rk):
    out = []
    for o in range(12):
        a, b = k[k["octave"] == o], rk[rk["octave"] == o]
        if len(a) != len(b):
            out.append("L%d n %d/%d" % (o, len(a), len(b)))
            continue
        pa, pb = np.stack([a["x"], a["y"]], 1), np.stack([b["x"], b["y"]], 1)
        if np.array_equal(pa, pb) and np.array_equal(a["angle"], b["angle"]):
            continue
        same_set = set(map(tuple, pa.tolist())) == set(map(tuple, pb.tolist()))
        nd = int((pa != pb).any(1).sum())
        out.append("L%d %s %d/%d" % (o, "order" if same_set else "set", nd, len(a)))
    return out


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    os.environ["ORBGPU_DIAGNOSTICS"] = "1"
    import orbslam3lib_amd as og
    from oracle import oracle_py as oracle
    pairs = {s: synth.stereo_pair(1080, 1920, s) for s in (60, 61)}
    refs = {s: [oracle.extract(x, nfeatures=8200, nlevels=12) for x in pairs[s]] for s in pairs}
    shapes = [
        ("2 pairs, default", [60, 61], {}),
        ("2 pairs, 1 stream", [60, 61], {"ORBGPU_STREAMS": "1"}),
        ("2 pairs reversed", [61, 60], {}),
        ("1 pair 61", [61], {}),
        ("1 pair 61, no graph", [61], {"ORBGPU_GRAPH": "0"}),
        ("2 pairs, octree label passes", [60, 61], {"ORBGPU_OCT_PYR": "0"}),
    ]
    total = 0
    for name, seeds, env in shapes:
        for k, v in env.items():
            os.environ[k] = v
        imgs = np.stack([x for s in seeds for x in pairs[s]])
        be = og.BatchExtractor(8200, 1.2, 12, 20, 7, width=1920, height=1080, max_images=len(imgs))
        be.upload(imgs)
        first = None
        for rep in range(R):
            be.run()
            be.synchronize()
            cc = be.candidate_counts()
            if first is None:
                first = cc
            msgs = []
            if not np.array_equal(cc, first):
                msgs.append("candidates %s vs %s" % (cc.tolist(), first.tolist()))
            for i in range(len(imgs)):
                k, d, m = be.result(i)
                rk, rd, rm = refs[seeds[i // 2]][i % 2]
                dd = diff_octaves(k, rk)
                if dd or len(d) != len(rd) or not np.array_equal(d, rd):
                    msgs.append("img %d (seed %d): %s" % (i, seeds[i // 2], " ".join(dd) or "desc"))
            total += len(msgs)
            print("[%s] rep %d: %s" % (name, rep, "; ".join(msgs) if msgs else "ok"), flush=True)
        be.close()
        for k in env:
            del os.environ[k]
    print("race_probe: %d mismatching runs" % total)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
