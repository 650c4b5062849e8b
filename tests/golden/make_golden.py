"""Generates tests/golden/*.npz from the CPU oracle on seeded synthetic frames.

The reference ships no fixtures or tests for this path and its OpenCV is not
available, so these vectors pin the oracle's own outputs (regression fixtures) and let the GPU
tests check results without running the oracle.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle_py as O  # noqa: E402
from orbslam3lib_amd import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

CASES = [
    # name, (h, w), frame generator args, nfeatures, nlevels, lap
    ("c1_mono_640x480_n1000", (480, 640), ("frame", 0), 1000, 8, (0, 1000)),
    ("c2_left_640x480_n2000", (480, 640), ("left", 0), 2000, 8, (0, 0)),
    ("c2_right_640x480_n2000", (480, 640), ("right", 0), 2000, 8, (0, 0)),
    ("c3_euroc_752x480_n2000", (480, 752), ("frame", 1), 2000, 8, (0, 0)),
]


def make_image(shape, gen):
    h, w = shape
    kind, k = gen
    if kind == "frame":
        return synth.frame(h, w, k)
    L, R = synth.stereo_pair(h, w, k)
    return L if kind == "left" else R


def main():
    for name, shape, gen, nf, nl, lap in CASES:
        img = make_image(shape, gen)
        k, d, mono = O.extract(img, nfeatures=nf, nlevels=nl, lap=lap)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), img_sha256=hashlib.sha256(img.tobytes()).hexdigest(),
                            shape=np.array(shape), gen_kind=gen[0], gen_k=gen[1], nfeatures=nf, nlevels=nl,
                            lap=np.array(lap), mono=mono, kps=k, desc=d)
        print(name, len(k), mono)
    L = np.load(os.path.join(OUT, "c2_left_640x480_n2000.npz"))["desc"]
    R = np.load(os.path.join(OUT, "c2_right_640x480_n2000.npz"))["desc"]
    i1, d1, i2, d2 = O.knn2(L, R)
    np.savez_compressed(os.path.join(OUT, "c2_knn2_left_right.npz"), idx1=i1, dist1=d1, idx2=i2, dist2=d2)
    print("knn2", len(i1))


if __name__ == "__main__":
    main()
