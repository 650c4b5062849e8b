"""CPU: the dense, threshold-independent FAST formulation (round 4's k_fast_bands, measured slower
than k_fast_cells and removed from the library in round 5), restated in numpy and checked against the oracle's cell loop
(ComputeKeyPointsOctTree, ORBextractor_old.cc:807-871, with cv::FAST per cell ROI):

  m(p)   = max(v - min over 9-arcs of the arc maximum, max over 9-arcs of the arc minimum - v, 0)
           (corner at t <=> m > t; cornerScore = m - 1)
  R(p)   = m(p) if m(p) > m(q) for every 8-neighbour q in p's cell detection rectangle, else 0
  keys of a cell at t: pixels with R > max(t, 1), in row-major order,
           t = iniThFAST if the cell has one at iniThFAST, else minThFAST.

The keys (positions relative to minBorder, responses) must equal the oracle's vToDistributeKeys
cell by cell, on textures that force every branch: synthetic frames, uniform noise (dense
corners), salt and pepper (saturated strengths, ties), low-contrast noise (every cell falls back
to minThFAST) and a frame half flat, with several threshold pairs."""
import numpy as np
import pytest

from orbslam3lib_amd import synth

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
        (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
EDGE, MINB = 19, 16


def strength(lvl):
    """m for every pixel with a full ring (3-px border 0)."""
    im = lvl.astype(np.int32)
    h, w = im.shape
    v = im[3:h - 3, 3:w - 3]
    ring = np.stack([im[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in RING])
    amin = np.full(v.shape, 1 << 20, np.int32)
    bmax = np.full(v.shape, -1, np.int32)
    for s in range(16):
        arc = ring[[(s + k) % 16 for k in range(9)]]
        amin = np.minimum(amin, arc.max(0))
        bmax = np.maximum(bmax, arc.min(0))
    m = np.zeros(im.shape, np.int32)
    m[3:h - 3, 3:w - 3] = np.clip(np.maximum(v - amin, bmax - v), 0, 255)
    return m


def dense_level_keys(lvl, ini_th, min_th):
    """k_fast_bands' result for one level: the keys of every cell in cell order (x, y relative
    to minBorder, response), as the oracle's level candidates."""
    h, w = lvl.shape
    m = strength(lvl)
    maxBX, maxBY = w - EDGE + 3, h - EDGE + 3
    width, height = float(maxBX - MINB), float(maxBY - MINB)
    nCols, nRows = int(width / 35.0), int(height / 35.0)
    wCell, hCell = int(np.ceil(width / nCols)), int(np.ceil(height / nRows))
    out = []
    for i in range(nRows):
        iniY = MINB + i * hCell
        if iniY >= maxBY - 3:
            continue
        maxY = min(iniY + hCell + 6, maxBY)
        for j in range(nCols):
            iniX = MINB + j * wCell
            if iniX >= maxBX - 6:
                continue
            maxX = min(iniX + wCell + 6, maxBX)
            y0, y1, x0, x1 = iniY + 3, maxY - 3, iniX + 3, maxX - 3
            if y1 <= y0 or x1 <= x0:
                continue
            c = np.zeros((y1 - y0 + 2, x1 - x0 + 2), np.int32)  # the cell's m, 0 outside
            c[1:-1, 1:-1] = m[y0:y1, x0:x1]
            core = c[1:-1, 1:-1]
            nb = np.zeros_like(core)
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    if dx or dy:
                        nb = np.maximum(nb, c[1 + dy:c.shape[0] - 1 + dy, 1 + dx:c.shape[1] - 1 + dx])
            R = np.where(core > nb, core, 0)
            t = ini_th if (R > max(ini_th, 1)).any() else min_th
            ys, xs = np.nonzero(R > max(t, 1))  # row-major
            for yy, xx in zip(ys, xs):
                out.append((x0 + xx - MINB, y0 + yy - MINB, R[yy, xx] - 1))
    return out


def _frames():
    rng = np.random.default_rng(11)
    h, w = 240, 320
    half = synth.frame(h, w, 4)
    half[:, : w // 2] = 90
    return [synth.frame(h, w, 1), rng.integers(0, 256, (h, w), dtype=np.uint8),
            (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8),
            (128 + rng.integers(-6, 7, (h, w))).astype(np.uint8), half]


@pytest.mark.parametrize("th", [(20, 7), (0, 0), (7, 20), (40, 3)])
def test_dense_formulation_equals_cell_loop(oracle, th):
    ini, mn = th
    for img in _frames():
        for lvl in oracle.pyramid(img, 1.2, 3):
            ref = oracle.level_candidates(lvl, ini, mn)
            got = dense_level_keys(lvl, ini, mn)
            assert len(got) == len(ref)
            if got:
                g = np.array(got, np.float64)
                np.testing.assert_array_equal(g[:, 0], ref["x"])
                np.testing.assert_array_equal(g[:, 1], ref["y"])
                np.testing.assert_array_equal(g[:, 2], ref["response"])
