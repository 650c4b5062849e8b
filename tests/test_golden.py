"""CPU: committed golden vectors (tests/golden/make_golden.py) reproduce bit-exactly from the
oracle on the regenerated synthetic frames -- pins the oracle against regressions."""
import glob
import hashlib
import os

import numpy as np
import pytest

from orbslam3lib_amd import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(p for p in glob.glob(os.path.join(GOLD, "c*_n*.npz")))


def load_case(path):
    z = np.load(path)
    h, w = (int(v) for v in z["shape"])
    kind, k = str(z["gen_kind"]), int(z["gen_k"])
    if kind == "frame":
        img = synth.frame(h, w, k)
    else:
        L, R = synth.stereo_pair(h, w, k)
        img = L if kind == "left" else R
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(z["img_sha256"]), "synthetic generator drifted"
    return img, z


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_oracle_reproduces_golden(oracle, path):
    img, z = load_case(path)
    k, d, mono = oracle.extract(img, nfeatures=int(z["nfeatures"]), nlevels=int(z["nlevels"]),
                                lap=tuple(int(v) for v in z["lap"]))
    assert mono == int(z["mono"])
    np.testing.assert_array_equal(k, z["kps"])
    np.testing.assert_array_equal(d, z["desc"])


def test_oracle_knn_golden(oracle):
    L = np.load(os.path.join(GOLD, "c2_left_640x480_n2000.npz"))["desc"]
    R = np.load(os.path.join(GOLD, "c2_right_640x480_n2000.npz"))["desc"]
    g = np.load(os.path.join(GOLD, "c2_knn2_left_right.npz"))
    for a, key in zip(oracle.knn2(L, R), ("idx1", "dist1", "idx2", "dist2")):
        np.testing.assert_array_equal(a, g[key])
