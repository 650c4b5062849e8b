"""SURVEY §8c secondary consistency check: the reference's own DSP FAST strength agrees with the
oracle's cornerScore<16>.

dsp/src/orbslam_dsp_fast.cpp:497-641 (calculate_fast_scores_stride) gathers the 16 ring pixels in
cyclic order (p1..p16 = (-3,0), (-3,1), (-2,2), (-1,3), (0,3), ... , (-3,-1), :517-548), then over
the 8 even start positions takes the min / max of the 8 pixels after the start, and folds
score_b = max(score_b, min(ring[s], a), min(ring[s + 9], a)) and
score_d = min(score_d, max(ring[s], b), max(ring[s + 9], b)), i.e. the best 9-arc minimum /
maximum over all 16 arcs; score = max(score_b - centre, centre - score_d, 0) (:605-641).
The oracle's cornerScore<16>(threshold) (OpenCV 4.2 fast_score.cpp) equals
max(threshold, m) - 1 for the threshold-independent strength m, so with threshold 0 the DSP score
is cornerScore<16>(0) + 1.  Restated below as written (a scalar loop per patch), checked on
>= 100k patches: uniform noise, smooth ramps and blobs (many corners), and the synthetic frames."""
import numpy as np

from orbslam3lib_amd import synth

# orbslam_dsp_fast.cpp:517-548, (dy, dx) of p1..p16
DSP_RING = [(-3, 0), (-3, 1), (-2, 2), (-1, 3), (0, 3), (1, 3), (2, 2), (3, 1),
            (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1)]


def dsp_strength(img, y, x):
    """calculate_fast_scores_stride for one pixel, in the DSP's operation order."""
    c = int(img[y, x])
    border = [int(img[y + dy, x + dx]) for dy, dx in DSP_RING]
    border += border[:8]                      # :597-600 (borderPixels[16 + i] = borderPixels[i])
    score_b, score_d = 0, 255
    for s in range(0, 16, 2):                 # :606
        a = min(border[s + 1], border[s + 2])
        b = max(border[s + 1], border[s + 2])
        for k in range(s + 3, s + 9):
            a = min(a, border[k])
            b = max(b, border[k])
        score_b = max(score_b, min(border[s], a))
        score_d = min(score_d, max(border[s], b))
        score_b = max(score_b, min(border[s + 9], a))
        score_d = min(score_d, max(border[s + 9], b))
    return max(score_b - c, c - score_d, 0)   # :636-638 (saturating halfword subtractions)


def _images():
    rng = np.random.default_rng(5)
    yield rng.integers(0, 256, (120, 160), dtype=np.uint8)
    yy, xx = np.mgrid[0:120, 0:160]
    ramp = (xx * 1.7 + yy * 0.9 + 40 * np.sin(xx / 7.0) * np.cos(yy / 5.0)) % 256
    yield ramp.astype(np.uint8)
    blobs = np.full((120, 160), 60, np.int32)
    for _ in range(60):
        cy, cx, r = rng.integers(0, 120), rng.integers(0, 160), rng.integers(2, 9)
        blobs[max(cy - r, 0):cy + r, max(cx - r, 0):cx + r] = rng.integers(0, 256)
    yield np.clip(blobs + rng.integers(-6, 7, blobs.shape), 0, 255).astype(np.uint8)
    for k in range(3):
        yield synth.frame(120, 160, 30 + k)


def test_dsp_fast_strength_equals_corner_score(oracle):
    n = corners = 0
    for img in _images():
        h, w = img.shape
        for y in range(3, h - 3):
            for x in range(3, w - 3):
                d = dsp_strength(img, y, x)
                assert d == oracle.corner_score(img, x, y, 0) + 1, (y, x)
                corners += d >= 20
                n += 1
    assert n >= 100_000
    assert corners > 1000  # the strong branch is exercised, not only flat patches
