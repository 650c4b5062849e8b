"""GPU parity of the FAST stage over the threshold range (ORBextractor's iniThFAST / minThFAST,
ORBextractor_old.cc:828,847).  k_fast_cells' antipodal-pair pre-test (orb_fast_cell.h
fw_pretest4) is a necessary condition of a FAST corner at every threshold t, and its packed
arithmetic carries v -+ t in biased 16-bit halves: threshold 0 (strict p < v / p > v), small and
large thresholds, a minThFAST above iniThFAST (the rerun keeps the iniThFAST candidates) and the
255 edge, on seeded synthetic frames and on uniform noise, keypoints and descriptors bit-exact
against the oracle (oracle/orb_oracle.cpp, the checker; parity pinned as in test_golden.py)."""
import numpy as np
import pytest

from orbslam3lib_amd import synth

pytestmark = pytest.mark.gpu

H, W = 480, 640
THRESHOLDS = [(0, 0), (5, 2), (12, 4), (40, 15), (90, 30), (20, 25), (200, 100), (255, 254)]


def _frames():
    rng = np.random.default_rng(31)
    l, r = synth.stereo_pair(H, W, 9)
    return np.stack([l, r, rng.integers(0, 256, (H, W), dtype=np.uint8)])


@pytest.mark.parametrize("ini,mn", THRESHOLDS)
def test_fast_threshold_range(oracle, ini, mn):
    """k_fast_cells over the (iniThFAST, minThFAST) range."""
    import orbslam3lib_amd as og
    imgs = _frames()
    be = og.BatchExtractor(2000, 1.2, 8, ini, mn, width=W, height=H, max_images=len(imgs))
    be.upload(imgs)
    be.run()
    be.synchronize()
    for i in range(len(imgs)):
        k, d, m = be.result(i)
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000, ini_th=ini, min_th=mn)
        assert m == rm, (i, ini, mn)
        assert len(k) == len(rk), (i, ini, mn, len(k), len(rk))
        for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
            np.testing.assert_array_equal(k[f], rk[f], err_msg="image %d %s t=(%d,%d)" % (i, f, ini, mn))
        np.testing.assert_array_equal(d, rd, err_msg="image %d t=(%d,%d)" % (i, ini, mn))
