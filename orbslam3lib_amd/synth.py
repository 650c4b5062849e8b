"""Deterministic synthetic stereo frames — there is no dataset on the box.

Image = value-noise octaves (cells 64/16/4 px, weights .5/.3/.2, seed s) + 48 rectangles and
24 discs of random intensity (seed s+1) + a zero-mean 3-px texture octave (weight .35, seed s+7;
lifts the level-0 FAST candidate count at th=20 into the 5k-20k band SURVEY §8d asks for) +
Gaussian noise sigma=2 (seed s+2), clipped to u8.
The right eye is the clean left scene shifted by `disparity` px with its own noise (seed s+3).
Frame k uses s = 42 + 4k.  Pure numpy, so CPU tests and the GPU bench see identical pixels.
"""
from __future__ import annotations

import numpy as np

__all__ = ["scene", "frame", "stereo_pair", "stereo_batch"]


def _value_noise(rng, h, w, cell):
    gh, gw = h // cell + 2, w // cell + 2
    grid = rng.random((gh, gw), dtype=np.float64)
    ys = np.arange(h, dtype=np.float64) / cell
    xs = np.arange(w, dtype=np.float64) / cell
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    fy = fy * fy * (3 - 2 * fy)  # smoothstep
    fx = fx * fx * (3 - 2 * fx)
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    top = g00 * (1 - fx) + g01 * fx
    bot = g10 * (1 - fx) + g11 * fx
    return top * (1 - fy) + bot * fy


def scene(h: int, w: int, seed: int, pad: int = 0) -> np.ndarray:
    """Clean float scene of size h x (w + pad) (pad gives room for the stereo shift)."""
    W = w + pad
    rng = np.random.default_rng(seed)
    img = np.zeros((h, W), dtype=np.float64)
    for cell, wt in ((64, 0.5), (16, 0.3), (4, 0.2)):
        img += wt * 255.0 * _value_noise(rng, h, W, cell)
    rng2 = np.random.default_rng(seed + 1)
    yy, xx = np.mgrid[0:h, 0:W]
    for _ in range(48):
        x0, y0 = rng2.integers(0, W), rng2.integers(0, h)
        rw, rh = rng2.integers(8, max(9, W // 6)), rng2.integers(8, max(9, h // 6))
        val = rng2.integers(0, 256)
        img[y0:y0 + rh, x0:x0 + rw] = 0.35 * img[y0:y0 + rh, x0:x0 + rw] + 0.65 * val
    for _ in range(24):
        cx, cy = rng2.integers(0, W), rng2.integers(0, h)
        r = rng2.integers(5, max(6, min(h, W) // 10))
        val = rng2.integers(0, 256)
        m = (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r
        img[m] = 0.3 * img[m] + 0.7 * val
    rng3 = np.random.default_rng(seed + 7)
    img += 0.35 * 255.0 * (_value_noise(rng3, h, W, 3) - 0.5)
    return img


def _finish(img: np.ndarray, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    noisy = img + rng.normal(0.0, 2.0, size=img.shape)
    return np.clip(np.rint(noisy), 0, 255).astype(np.uint8)


def frame(h: int, w: int, k: int = 0) -> np.ndarray:
    """Mono frame k (h x w, uint8)."""
    s = 42 + 4 * k
    return _finish(scene(h, w, s), s + 2)


def stereo_pair(h: int, w: int, k: int = 0, disparity: int = 12):
    """(left, right) uint8 frames of pair k; right = left scene shifted by `disparity` px."""
    s = 42 + 4 * k
    sc = scene(h, w, s, pad=disparity)
    left = _finish(np.ascontiguousarray(sc[:, :w]), s + 2)
    right = _finish(np.ascontiguousarray(sc[:, disparity:disparity + w]), s + 3)
    return left, right


def stereo_batch(h: int, w: int, npairs: int, first: int = 0, disparity: int = 12) -> np.ndarray:
    """[2*npairs, h, w] uint8, images ordered L0, R0, L1, R1, ..."""
    out = np.empty((2 * npairs, h, w), dtype=np.uint8)
    for i in range(npairs):
        out[2 * i], out[2 * i + 1] = stereo_pair(h, w, first + i, disparity)
    return out


def map_points(xy_un, octave, desc, uright=None, n=2000, seed=0, nlevels=8, scale_factor=1.2):
    """Synthetic local-map points for ORBmatcher::SearchByProjection (a MAP_POINT_DTYPE array):
    projections near frame keypoints (several points per keypoint, so they compete), descriptors
    with 0..60 flipped bits (some unrelated), both RadiusByViewingCos branches, bad / not-in-view /
    observation-less / far points, and a few projections outside the image."""
    from . import MAP_POINT_DTYPE, MP_BAD, MP_HAS_OBS, MP_IN_VIEW
    rng = np.random.default_rng(seed)
    xy_un = np.asarray(xy_un, np.float32).reshape(-1, 2)
    octave = np.asarray(octave, np.int32)
    desc = np.asarray(desc, np.uint8).reshape(-1, 32)
    nk = len(octave)
    out = np.zeros(n, MAP_POINT_DTYPE)
    if nk == 0 or n == 0:
        return out
    scale = scale_factor ** np.arange(nlevels, dtype=np.float64)
    pool = rng.choice(nk, size=max(1, min(nk, n // 2)), replace=False)
    k = pool[rng.integers(0, len(pool), n)]
    lvl = np.clip(octave[k] + rng.choice([-1, 0, 0, 0, 1], n), 0, nlevels - 1)
    noise = rng.normal(0.0, 1.5, (n, 2)) * scale[octave[k]][:, None]
    p = xy_un[k] + noise
    outside = rng.random(n) < 0.03
    p[outside] = rng.uniform(-200, 1200, (int(outside.sum()), 2))
    out["proj_x"], out["proj_y"] = p[:, 0], p[:, 1]
    if uright is not None:
        ur = np.asarray(uright, np.float32)[k]
        out["proj_xr"] = np.where(ur > 0, ur + rng.normal(0, 2.0, n), p[:, 0] - 20)
    else:
        out["proj_xr"] = p[:, 0] - 20
    out["view_cos"] = rng.choice(np.array([0.9995, 0.999, 0.99, 0.95], np.float32), n)
    out["depth"] = rng.uniform(0.5, 80.0, n)
    out["level"] = lvl
    flags = np.where(rng.random(n) < 0.9, MP_IN_VIEW, 0) | np.where(rng.random(n) < 0.05, MP_BAD, 0) \
        | np.where(rng.random(n) < 0.9, MP_HAS_OBS, 0)
    out["flags"] = flags
    d = desc[k].copy()
    nflip = rng.choice([0, 2, 5, 10, 20, 35, 60], n)
    for i in range(n):
        if nflip[i]:
            b = np.unpackbits(d[i])
            b[rng.choice(256, nflip[i], replace=False)] ^= 1
            d[i] = np.packbits(b)
    unrelated = rng.random(n) < 0.05
    d[unrelated] = rng.integers(0, 256, (int(unrelated.sum()), 32), dtype=np.uint8)
    out["desc"] = d
    return out


def map_points_stereo(xyL, octL, descL, xyR, octR, l2r, n=2000, seed=0, nlevels=8, scale_factor=1.2):
    """Map points for the two-camera SearchByProjection: the left-window fields as map_points(),
    plus a right-camera projection next to the stereo partner of the source keypoint (or a random
    right keypoint), its own level / viewing cosine, and mbTrackInViewR on ~80% of the points."""
    from . import MP_IN_VIEW, MP_IN_VIEW_R
    rng = np.random.default_rng(seed + 1000)
    out = map_points(xyL, octL, descL, None, n=n, seed=seed, nlevels=nlevels, scale_factor=scale_factor)
    xyR = np.asarray(xyR, np.float32).reshape(-1, 2)
    octR = np.asarray(octR, np.int32)
    if len(octR) == 0 or n == 0:
        return out
    l2r = np.asarray(l2r, np.int32)
    scale = scale_factor ** np.arange(nlevels, dtype=np.float64)
    # the source keypoint map_points drew from is the closest left keypoint to the projection
    src = np.argmin(((xyL[None, :, :] - np.stack([out["proj_x"], out["proj_y"]], 1)[:, None, :]) ** 2).sum(2), 1) \
        if len(xyL) <= 4096 else rng.integers(0, len(xyL), n)
    partner = l2r[src]
    kr = np.where(partner >= 0, partner, rng.integers(0, len(octR), n))
    noise = rng.normal(0.0, 1.5, (n, 2)) * scale[octR[kr]][:, None]
    out["proj_xr"] = xyR[kr, 0] + noise[:, 0]
    out["proj_yr"] = xyR[kr, 1] + noise[:, 1]
    out["level_r"] = np.clip(octR[kr] + rng.choice([-1, 0, 0, 0, 1], n), 0, nlevels - 1)
    out["level_r"][rng.random(n) < 0.03] = -1
    out["view_cos_r"] = rng.choice(np.array([0.9995, 0.999, 0.99, 0.95], np.float32), n)
    inr = rng.random(n) < 0.8
    out["flags"] = (out["flags"] & ~MP_IN_VIEW_R) | np.where(inr, MP_IN_VIEW_R, 0)
    # some points only in the right view
    only_r = rng.random(n) < 0.05
    out["flags"] = np.where(only_r, (out["flags"] & ~MP_IN_VIEW) | MP_IN_VIEW_R, out["flags"])
    return out


def stereo_partners(descL, descR, seed=0, frac=0.6):
    """Synthetic mvLeftToRightMatch / mvRightToLeftMatch: a consistent one-to-one pairing of a
    fraction of the left keypoints with right keypoints (mutual best Hamming where possible)."""
    rng = np.random.default_rng(seed)
    nl, nr = len(descL), len(descR)
    l2r = np.full(nl, -1, np.int32)
    r2l = np.full(nr, -1, np.int32)
    if nl == 0 or nr == 0:
        return l2r, r2l
    cand = rng.permutation(nl)[:int(frac * nl)]
    free = np.ones(nr, bool)
    for i in cand:
        j = int(rng.integers(0, nr))
        if free[j]:
            l2r[i], r2l[j] = j, i
            free[j] = False
    return l2r, r2l
