"""ORBmatcher::SearchByProjection (cpp/src/ORBmatcher.cc:44-214, pinhole frames, with
Frame::GetFeaturesInArea, Frame.cc:673-735, and RadiusByViewingCos, :216-222).

CPU: the C oracle against an independent Python restatement on synthetic local maps.
GPU: k_sbp_candidates + k_sbp_resolve against the oracle, bit-exact on every keypoint's assigned
map point and on nmatches -- mono and stereo (mvuRight) frames, th != 1, far-point culling,
pre-occupied keypoints, many map points competing for the same keypoints.

Parity status: unpinned against the reference itself (ORBmatcher.cc needs the SLAM stack and
OpenCV; no fixtures ship for it) -- cross-checked restatements only."""
import math

import numpy as np
import pytest

from orbslam3lib_amd import synth

F32 = np.float32
K_ = (458.654, 457.296, 367.215, 248.375)
D_ = (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)


def _py_sbp(mps, xy, octv, desc, uright, bounds, cs, ci, blk, th, nnratio, far, th_far, scale):
    n = len(octv)
    blocked = np.zeros(n, bool) if blk is None else blk.astype(bool).copy()
    match = np.full(n, -1, np.int32)
    wi = F32(F32(64) / F32(bounds[1] - bounds[0]))
    hi = F32(F32(48) / F32(bounds[3] - bounds[2]))
    nm = 0
    for i, mp in enumerate(mps):
        if not (mp["flags"] & 1) or (far and mp["depth"] > F32(th_far)) or (mp["flags"] & 2):
            continue
        lvl = int(mp["level"])
        r = F32(2.5) if float(mp["view_cos"]) > 0.998 else F32(4.0)
        if F32(th) != 1.0:
            r = F32(r * F32(th))
        rs = F32(r * F32(scale[lvl]))
        x, y = F32(mp["proj_x"]), F32(mp["proj_y"])
        x0 = max(0, int(math.floor(F32(F32(F32(x - bounds[0]) - rs) * wi))))
        x1 = min(63, int(math.ceil(F32(F32(F32(x - bounds[0]) + rs) * wi))))
        y0 = max(0, int(math.floor(F32(F32(F32(y - bounds[2]) - rs) * hi))))
        y1 = min(47, int(math.ceil(F32(F32(F32(y - bounds[2]) + rs) * hi))))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        cand = []
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for k in ci[cs[ix * 48 + iy]:cs[ix * 48 + iy + 1]]:
                    if octv[k] < lvl - 1 or octv[k] > lvl:
                        continue
                    if abs(F32(xy[k, 0] - x)) < rs and abs(F32(xy[k, 1] - y)) < rs:
                        cand.append(k)
        best = (256, -1, -1)  # dist, level, idx
        second = (256, -1)
        for k in cand:
            if blocked[k]:
                continue
            if uright is not None and uright[k] > 0 and abs(F32(mp["proj_xr"] - uright[k])) > rs:
                continue
            dist = int(np.unpackbits(np.bitwise_xor(mp["desc"], desc[k])).sum())
            if dist < best[0]:
                second = best[:2]
                best = (dist, int(octv[k]), int(k))
            elif dist < second[0]:
                second = (dist, int(octv[k]))
        bd, bl, bi = best
        sd, sl = second
        if bd <= 100:
            if bl == sl and F32(bd) > F32(F32(nnratio) * F32(sd)):
                continue
            if bl != sl or F32(bd) <= F32(F32(nnratio) * F32(sd)):
                match[bi] = i
                blocked[bi] = bool(mp["flags"] & 4)
                nm += 1
    return match, nm


def _frame(oracle, seed, nf=1000):
    L, R = synth.stereo_pair(480, 640, seed)
    kl, dl, _ = oracle.extract(L, nfeatures=nf)
    kr, dr, _ = oracle.extract(R, nfeatures=nf)
    xy, b, cell, cs, ci = oracle.undistort_grid(kl, K_, D_, 640, 480)
    mbf, mb = 47.9, float(np.float32(47.9) / np.float32(435.2))
    ur, _, _ = oracle.stereo_matches(kl, dl, kr, dr, oracle.pyramid(L), oracle.pyramid(R), mbf, mb)
    return kl, dl.reshape(-1, 32), xy, b, cs, ci, ur


@pytest.mark.parametrize("th,far,stereo,blocked", [(1.0, False, True, False), (3.0, True, False, True),
                                                    (1.0, False, False, False)])
def test_oracle_matches_python_restatement(oracle, th, far, stereo, blocked):
    kl, dl, xy, b, cs, ci, ur = _frame(oracle, 5)
    mps = synth.map_points(xy, kl["octave"], dl, ur if stereo else None, n=400, seed=11)
    rng = np.random.default_rng(3)
    blk = (rng.random(len(kl)) < 0.1).astype(np.uint8) if blocked else None
    scale = oracle.scale_factors()[0]
    m, nm = oracle.search_by_projection(mps, xy, kl["octave"], dl, ur if stereo else None, b, cs, ci,
                                        blk, th, 0.8, far, 20.0)
    pm, pnm = _py_sbp(mps, xy, kl["octave"], dl, ur if stereo else None, b, cs, ci, blk, th, 0.8, far,
                      20.0, scale)
    np.testing.assert_array_equal(m, pm)
    assert nm == pnm
    assert nm > 50  # the synthetic map actually matches
    # competition happened: more in-view good points than matches
    assert (mps["flags"] & 1).sum() > nm


def _gpu_case(oracle, be, n_frames, stereo, th, far, th_far, blocked, n_mp, seed):
    rng = np.random.default_rng(seed)
    frames, mps_all, blks = [], [], []
    for f in range(n_frames):
        i = 2 * f  # the left eye of pair f
        kps, desc, _ = be.result(i)
        xy, _, _, _ = be.grid_result(i)
        ur = be.stereo_result(f)[0] if stereo else None
        mps_all.append(synth.map_points(xy, kps["octave"], desc, ur, n=n_mp, seed=seed + f))
        blks.append((rng.random(len(kps)) < 0.08).astype(np.uint8) if blocked else None)
        frames.append((kps, desc, xy, ur))
    be.search_by_projection(mps_all, image_step=2, use_uright=stereo,
                            kp_block=blks if blocked else None, th=th, nnratio=0.8, far_points=far,
                            th_far=th_far)
    be.synchronize()
    for f, (kps, desc, xy, ur) in enumerate(frames):
        _, b, _, cs, ci = oracle.undistort_grid(kps, K_, D_, 640, 480)
        m, nm = oracle.search_by_projection(mps_all[f], xy, kps["octave"], desc, ur, b, cs, ci, blks[f], th,
                                            0.8, far, th_far)
        gm, gnm = be.projection_matches(f)
        np.testing.assert_array_equal(gm, m, err_msg="frame %d" % f)
        assert gnm == nm, (f, gnm, nm)
    # the same call with the points already in the ABI's form (one array + offsets)
    off = np.concatenate([[0], np.cumsum([len(x) for x in mps_all])]).astype(np.int32)
    be.search_by_projection((np.concatenate(mps_all), off), image_step=2, use_uright=stereo,
                            kp_block=blks if blocked else None, th=th, nnratio=0.8, far_points=far,
                            th_far=th_far)
    be.synchronize()
    for f, (kps, desc, xy, ur) in enumerate(frames):
        _, b, _, cs, ci = oracle.undistort_grid(kps, K_, D_, 640, 480)
        m, nm = oracle.search_by_projection(mps_all[f], xy, kps["octave"], desc, ur, b, cs, ci, blks[f], th,
                                            0.8, far, th_far)
        gm, gnm = be.projection_matches(f)
        np.testing.assert_array_equal(gm, m, err_msg="frame %d (points + offsets)" % f)
        assert gnm == nm


def test_map_point_rows_forms():
    """The wrapper's two map-point forms give the ABI the same (points, offsets); malformed
    offsets are refused before any device call."""
    import orbslam3lib_amd as og
    rng = np.random.default_rng(3)
    parts = []
    for n in (5, 0, 7):
        a = np.zeros(n, og.MAP_POINT_DTYPE)
        a.view(np.uint8)[:] = rng.integers(0, 256, a.nbytes, dtype=np.uint8)
        parts.append(a)
    m1, o1, n1 = og.BatchExtractor._map_point_rows(parts)
    m2, o2, n2 = og.BatchExtractor._map_point_rows((np.concatenate(parts), np.array([0, 5, 5, 12])))
    assert n1 == n2 == 3 and o1.dtype == o2.dtype == np.int32
    np.testing.assert_array_equal(o1, o2)
    assert m1.tobytes() == m2.tobytes()
    for bad in ([1, 5, 5, 12], [0, 5, 4, 12], [0, 5, 5, 11]):
        with pytest.raises(ValueError):
            og.BatchExtractor._map_point_rows((np.concatenate(parts), np.array(bad)))


@pytest.mark.gpu
@pytest.mark.parametrize("stereo,th,far,blocked", [(True, 1.0, False, False), (True, 3.0, True, True),
                                                    (False, 1.0, False, True), (False, 5.0, False, False)])
def test_gpu_search_by_projection_bit_exact(oracle, stereo, th, far, blocked):
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(480, 640, 50 + s) for s in range(4)]
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=8)
    be.upload(np.stack([im for pr in pairs for im in pr]))
    be.run()
    be.undistort_grid(K_, D_)
    if stereo:
        be.stereo_matches(47.9, float(np.float32(47.9) / np.float32(435.2)))
    be.synchronize()
    _gpu_case(oracle, be, 4, stereo, th, far, 20.0, blocked, 3000, 100)


@pytest.mark.gpu
def test_gpu_search_by_projection_dense_conflicts(oracle):
    """8000 map points on one frame, most competing for a few hundred keypoints: the resolve
    pass's top-4 runs dry and re-walks windows."""
    import orbslam3lib_amd as og
    L, R = synth.stereo_pair(480, 640, 60)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
    be.upload(np.stack([L, R]))
    be.run()
    be.undistort_grid(K_, D_)
    be.synchronize()
    kps, desc, _ = be.result(0)
    xy, _, _, _ = be.grid_result(0)
    sub = np.random.default_rng(1).choice(len(kps), 200, replace=False)
    mps = synth.map_points(xy[sub], kps["octave"][sub], desc[sub], None, n=8000, seed=9)
    be.search_by_projection([mps], image_step=2, use_uright=False)
    _, b, _, cs, ci = oracle.undistort_grid(kps, K_, D_, 640, 480)
    m, nm = oracle.search_by_projection(mps, xy, kps["octave"], desc, None, b, cs, ci)
    gm, gnm = be.projection_matches(0)
    np.testing.assert_array_equal(gm, m)
    assert gnm == nm


@pytest.mark.gpu
def test_gpu_search_by_projection_empty_map(oracle):
    import orbslam3lib_amd as og
    L, R = synth.stereo_pair(480, 640, 61)
    be = og.BatchExtractor(500, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
    be.upload(np.stack([L, R]))
    be.run()
    be.undistort_grid(K_, ())
    be.search_by_projection([np.zeros(0, og.MAP_POINT_DTYPE)], image_step=2, use_uright=False)
    gm, gnm = be.projection_matches(0)
    assert gnm == 0 and (gm == -1).all()


# ---- two-camera frames (Nleft != -1, ORBmatcher.cc:59-214) -------------------------------------

def _py_window(xy, octv, cs, ci, bounds, x, y, rs, lvl):
    wi = F32(F32(64) / F32(bounds[1] - bounds[0]))
    hi = F32(F32(48) / F32(bounds[3] - bounds[2]))
    x0 = max(0, int(math.floor(F32(F32(F32(x - bounds[0]) - rs) * wi))))
    x1 = min(63, int(math.ceil(F32(F32(F32(x - bounds[0]) + rs) * wi))))
    y0 = max(0, int(math.floor(F32(F32(F32(y - bounds[2]) - rs) * hi))))
    y1 = min(47, int(math.ceil(F32(F32(F32(y - bounds[2]) + rs) * hi))))
    if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
        return []
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for k in ci[cs[ix * 48 + iy]:cs[ix * 48 + iy + 1]]:
                if lvl - 1 <= octv[k] <= lvl and abs(F32(xy[k, 0] - x)) < rs and abs(F32(xy[k, 1] - y)) < rs:
                    out.append(int(k))
    return out


def _py_best(mp_desc, cand, desc, octv, blocked):
    best, second = (256, -1, -1), (256, -1)
    for k in cand:
        if blocked(k):
            continue
        d = int(np.unpackbits(np.bitwise_xor(mp_desc, desc[k])).sum())
        if d < best[0]:
            second = best[:2]
            best = (d, int(octv[k]), k)
        elif d < second[0]:
            second = (d, int(octv[k]))
    return best, second


def _py_sbp2(mps, L, R, bounds, l2r, r2l, blk, th, nnratio, far, th_far, scale):
    (xyL, octL, dL, csL, ciL), (xyR, octR, dR, csR, ciR) = L, R
    nl, nr = len(octL), len(octR)
    blocked = np.zeros(nl + nr, bool) if blk is None else blk.astype(bool).copy()
    match = np.full(nl + nr, -1, np.int32)
    nm = 0

    def assign(k, i, mp):
        match[k] = i
        blocked[k] = bool(mp["flags"] & 4)
    for i, mp in enumerate(mps):
        if not (mp["flags"] & 9) or (far and mp["depth"] > F32(th_far)) or (mp["flags"] & 2):
            continue
        if mp["flags"] & 1:
            lvl = int(mp["level"])
            r = F32(2.5) if float(mp["view_cos"]) > 0.998 else F32(4.0)
            if F32(th) != 1.0:
                r = F32(r * F32(th))
            cand = _py_window(xyL, octL, csL, ciL, bounds, F32(mp["proj_x"]), F32(mp["proj_y"]),
                              F32(r * F32(scale[lvl])), lvl)
            if cand:
                (bd, bl, bi), (sd, sl) = _py_best(mp["desc"], cand, dL, octL, lambda k: blocked[k])
                if bd <= 100:
                    if bl == sl and F32(bd) > F32(F32(nnratio) * F32(sd)):
                        continue
                    if bl != sl or F32(bd) <= F32(F32(nnratio) * F32(sd)):
                        assign(bi, i, mp)
                        if l2r is not None and l2r[bi] != -1:
                            assign(nl + l2r[bi], i, mp)
                            nm += 1
                        nm += 1
        if mp["flags"] & 8:
            lvl = int(mp["level_r"])
            if lvl == -1:
                continue
            r = F32(2.5) if float(mp["view_cos_r"]) > 0.998 else F32(4.0)
            cand = _py_window(xyR, octR, csR, ciR, bounds, F32(mp["proj_xr"]), F32(mp["proj_yr"]),
                              F32(r * F32(scale[lvl])), lvl)
            if not cand:
                continue
            (bd, bl, bi), (sd, sl) = _py_best(mp["desc"], cand, dR, octR, lambda k: blocked[nl + k])
            if bd <= 100:
                if bl == sl and F32(bd) > F32(F32(nnratio) * F32(sd)):
                    continue
                if r2l is not None and r2l[bi] != -1:
                    assign(int(r2l[bi]), i, mp)
                    nm += 1
                assign(nl + bi, i, mp)
                nm += 1
    return match, nm


def _two_cam_frame(oracle, seed, nf=1000):
    Li, Ri = synth.stereo_pair(480, 640, seed)
    kl, dl, _ = oracle.extract(Li, nfeatures=nf)
    kr, dr, _ = oracle.extract(Ri, nfeatures=nf)
    xl, b, _, csl, cil = oracle.undistort_grid(kl, K_, (), 640, 480)
    xr, _, _, csr, cir = oracle.undistort_grid(kr, K_, (), 640, 480)
    return (xl, kl["octave"], dl.reshape(-1, 32), csl, cil), (xr, kr["octave"], dr.reshape(-1, 32), csr, cir), b


@pytest.mark.parametrize("th,far,blocked,partners", [(1.0, False, False, True), (3.0, True, True, True),
                                                      (1.0, False, True, False)])
def test_oracle_two_camera_matches_python_restatement(oracle, th, far, blocked, partners):
    L, R, b = _two_cam_frame(oracle, 7)
    l2r, r2l = synth.stereo_partners(L[2], R[2], seed=2) if partners else (None, None)
    mps = synth.map_points_stereo(L[0], L[1], L[2], R[0], R[1],
                                  l2r if l2r is not None else np.full(len(L[1]), -1), n=400, seed=13)
    blk = None
    if blocked:
        blk = (np.random.default_rng(4).random(len(L[1]) + len(R[1])) < 0.1).astype(np.uint8)
    m, nm = oracle.search_by_projection2(mps, L, R, b, l2r, r2l, blk, th, 0.8, far, 20.0)
    pm, pnm = _py_sbp2(mps, L, R, b, l2r, r2l, blk, th, 0.8, far, 20.0, oracle.scale_factors()[0])
    np.testing.assert_array_equal(m, pm)
    assert nm == pnm
    assert (m[len(L[1]):] >= 0).sum() > 20 and (m[:len(L[1])] >= 0).sum() > 20  # both windows match


def test_oracle_two_camera_left_only_equals_pinhole_without_uright(oracle):
    """With no right-camera points and no partners the two-camera form is the pinhole form
    without the mvuRight test."""
    L, R, b = _two_cam_frame(oracle, 8)
    mps = synth.map_points(L[0], L[1], L[2], None, n=300, seed=5)
    m2, nm2 = oracle.search_by_projection2(mps, L, R, b)
    m1, nm1 = oracle.search_by_projection(mps, L[0], L[1], L[2], None, b, L[3], L[4])
    np.testing.assert_array_equal(m2[:len(L[1])], m1)
    assert (m2[len(L[1]):] == -1).all() and nm1 == nm2


@pytest.mark.gpu
@pytest.mark.parametrize("th,far,blocked,partners,n_mp", [(1.0, False, False, True, 3000),
                                                           (3.0, True, True, True, 3000),
                                                           (1.0, False, True, False, 2000),
                                                           (1.0, False, True, True, 8000)])
def test_gpu_search_by_projection_two_camera_bit_exact(oracle, th, far, blocked, partners, n_mp):
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(480, 640, 70 + s) for s in range(3)]
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=6)
    be.upload(np.stack([im for pr in pairs for im in pr]))
    be.run()
    be.undistort_grid(K_, ())
    be.synchronize()
    rng = np.random.default_rng(21)
    sides, mps_all, l2rs, r2ls, blks = [], [], [], [], []
    for p in range(len(pairs)):
        side = []
        for e in range(2):
            kps, desc, _ = be.result(2 * p + e)
            xy, _, cs, ci = be.grid_result(2 * p + e)
            side.append((xy, kps["octave"], desc, cs, ci))
        L, R = side
        l2r, r2l = synth.stereo_partners(L[2], R[2], seed=p) if partners else (None, None)
        mps_all.append(synth.map_points_stereo(L[0], L[1], L[2], R[0], R[1],
                                               l2r if l2r is not None else np.full(len(L[1]), -1),
                                               n=n_mp, seed=40 + p))
        blks.append((rng.random(len(L[1]) + len(R[1])) < 0.08).astype(np.uint8) if blocked else None)
        sides.append(side)
        l2rs.append(l2r)
        r2ls.append(r2l)
    be.search_by_projection_stereo(mps_all, l2rs if partners else None, r2ls if partners else None,
                                   blks if blocked else None, th=th, nnratio=0.8, far_points=far, th_far=20.0)
    be.synchronize()
    b = np.array([0, 640, 0, 480], np.float32)
    for p, (L, R) in enumerate(sides):
        m, nm = oracle.search_by_projection2(mps_all[p], L, R, b, l2rs[p], r2ls[p], blks[p], th, 0.8, far, 20.0)
        gm, gnm = be.projection_matches(p)
        np.testing.assert_array_equal(gm, m, err_msg="pair %d" % p)
        assert gnm == nm, (p, gnm, nm)


@pytest.mark.gpu
def test_gpu_search_by_projection_1080p_large_lds(oracle):
    """C5 geometry (1920x1080, 12 levels, 5000 features): the resolve kernel's LDS tables exceed
    64 KB (two-camera: Nleft + Nright keypoints), the dynamic-LDS attribute path."""
    import orbslam3lib_amd as og
    L_, R_ = synth.stereo_pair(1080, 1920, 81)
    be = og.BatchExtractor(5000, 1.2, 12, 20, 7, width=1920, height=1080, max_images=2)
    be.upload(np.stack([L_, R_]))
    be.run()
    be.undistort_grid((1400.0, 1400.0, 960.0, 540.0), ())
    be.synchronize()
    side = []
    for e in range(2):
        kps, desc, _ = be.result(e)
        xy, _, cs, ci = be.grid_result(e)
        side.append((xy, kps["octave"], desc, cs, ci))
    Ls, Rs = side
    l2r, r2l = synth.stereo_partners(Ls[2], Rs[2], seed=3)
    mps = synth.map_points_stereo(Ls[0], Ls[1], Ls[2], Rs[0], Rs[1], l2r, n=6000, seed=17, nlevels=12)
    be.search_by_projection_stereo([mps], [l2r], [r2l])
    b = np.array([0, 1920, 0, 1080], np.float32)
    m, nm = oracle.search_by_projection2(mps, Ls, Rs, b, l2r, r2l, nlevels=12)
    gm, gnm = be.projection_matches(0)
    np.testing.assert_array_equal(gm, m)
    assert gnm == nm and nm > 100
    # the pinhole form on the left image of the same frame
    be.search_by_projection([mps], image_step=2, use_uright=False)
    m1, nm1 = oracle.search_by_projection(mps, Ls[0], Ls[1], Ls[2], None, b, Ls[3], Ls[4], nlevels=12)
    gm1, gnm1 = be.projection_matches(0)
    np.testing.assert_array_equal(gm1, m1)
    assert gnm1 == nm1
