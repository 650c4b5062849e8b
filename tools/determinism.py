"""Repeatability of the batch path on the 1920x1080 / 12-level / 8200-feature two-pair batch of
tests/test_batch_edges.py::test_batch_knn2_past_4096_train_rows: the same
uploaded batch is run + matched R times on one context and every image's keypoints, descriptors
and every pair's kNN2 are compared with the first run and with the oracle.  ORBGPU_LIB selects
the library (product or a variant build).  Usage: python tools/determinism.py [R]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from orbslam3lib_amd import synth  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    import orbslam3lib_amd as og
    from oracle import oracle_py as oracle
    pairs = [synth.stereo_pair(1080, 1920, 60 + i) for i in range(2)]
    imgs = np.stack([x for p in pairs for x in p])
    refs = [oracle.extract(imgs[i], nfeatures=8200, nlevels=12) for i in range(4)]
    be = og.BatchExtractor(8200, 1.2, 12, 20, 7, width=1920, height=1080, max_images=4)
    be.upload(imgs)
    first = None
    bad = 0
    for rep in range(R):
        be.run()
        be.match_stereo(False)
        be.synchronize()
        res = [be.result(i) for i in range(4)]
        mt = [be.matches(p) for p in range(2)]
        for i in range(4):
            k, d, m = res[i]
            rk, rd, rm = refs[i]
            fields = [f for f in ("x", "y", "size", "angle", "response", "octave")
                      if len(k) != len(rk) or not np.array_equal(k[f], rk[f])]
            dbad = len(d) != len(rd) or not np.array_equal(d, rd)
            if fields or dbad or m != rm:
                bad += 1
                nx = int((k["x"] != rk["x"]).sum()) if len(k) == len(rk) else -1
                print("rep %d image %d: fields %s desc %s mono %s/%s x-mismatch %d" % (rep, i, fields, dbad, m, rm, nx))
        if first is None:
            first = (res, mt)
        else:
            for p in range(2):
                for a, b in zip(mt[p], first[1][p]):
                    if not np.array_equal(a, b):
                        bad += 1
                        print("rep %d pair %d: kNN2 differs from run 0" % (rep, p))
    print("determinism: %d runs, %d mismatching items (lib %s)" % (R, bad, os.environ.get("ORBGPU_LIB", "product")))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
