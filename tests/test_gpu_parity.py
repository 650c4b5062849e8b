"""GPU parity: liborbgpu.so (HIP, gfx950) vs the CPU oracle, bit-exact, through the C ABI.

Bar (BASELINE.json north_star): keypoint indices/coordinates and 32-byte descriptors bit-exact;
angles (centroid) within 1e-4 deg -- here they are required bit-exact too, since the descriptor
sampling depends on them.
"""
import numpy as np
import pytest

from orbslam3lib_amd import synth

pytestmark = pytest.mark.gpu


def _extractor(nf=2000, L=8, w=640, h=480, imgs=2, sf=1.2):
    import orbslam3lib_amd as og
    return og.ORBextractor(nf, sf, L, 20, 7, max_width=w, max_height=h, max_images=imgs)


def _same_kps(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


@pytest.fixture(scope="module")
def frame0():
    return synth.stereo_pair(480, 640, 0)


def test_pyramid_and_blur_bit_exact(oracle, frame0):
    L, _ = frame0
    ex = _extractor()
    ex(L)
    ref = oracle.pyramid(L)
    for l in range(8):
        g = ex.pyramid_level(0, l)
        np.testing.assert_array_equal(g, ref[l], err_msg="level %d" % l)
        np.testing.assert_array_equal(ex.pyramid_level(0, l, blurred=True), oracle.blur(ref[l]),
                                      err_msg="blur level %d" % l)


def test_level_keypoints_and_descriptors(oracle, frame0):
    L, _ = frame0
    ex = _extractor()
    ex(L)
    got = ex.level_keypoints(0)
    ref = oracle.extract_levels(L, nfeatures=2000)
    for l in range(8):
        (gk, gd), (rk, rd) = got[l], ref[l]
        _same_kps(gk, rk)
        np.testing.assert_array_equal(gd, rd, err_msg="desc level %d" % l)


@pytest.mark.parametrize("lap", [(0, 0), (0, 1000), (200, 420)])
def test_extract_matches_oracle(oracle, frame0, lap):
    L, R = frame0
    ex = _extractor()
    for img in (L, R):
        k, d, m = ex(img, None, lap)
        rk, rd, rm = oracle.extract(img, nfeatures=2000, lap=lap)
        assert m == rm
        _same_kps(k, rk)
        np.testing.assert_array_equal(d, rd)


def test_mono_config_c1(oracle):
    img = synth.frame(480, 640, 3)
    ex = _extractor(nf=1000)
    k, d, m = ex(img, None, (0, 1000))
    rk, rd, rm = oracle.extract(img, nfeatures=1000, lap=(0, 1000))
    assert m == rm == 0
    _same_kps(k, rk)
    np.testing.assert_array_equal(d, rd)


def test_stereo_entry_point(oracle, frame0):
    L, R = frame0
    ex = _extractor()
    (kl, dl, ml), (kr, dr, mr) = ex.extract_stereo(L, R, (0, 0), (100, 639))
    for (k, d, m), img, lap in (((kl, dl, ml), L, (0, 0)), ((kr, dr, mr), R, (100, 639))):
        rk, rd, rm = oracle.extract(img, nfeatures=2000, lap=lap)
        assert m == rm
        _same_kps(k, rk)
        np.testing.assert_array_equal(d, rd)


def test_batch_path_matches_oracle(oracle):
    import orbslam3lib_amd as og
    imgs = synth.stereo_batch(480, 640, 4, first=5)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=8)
    be.upload(imgs)
    laps = np.array([[0, 0], [50, 600]] * 4, np.int32)
    be.run(laps)
    be.match_stereo(False)
    be.synchronize()
    for i in range(8):
        k, d, m = be.result(i)
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000, lap=tuple(laps[i]))
        assert m == rm
        _same_kps(k, rk)
        np.testing.assert_array_equal(d, rd)
    for p in range(4):
        i1, d1, i2, d2 = be.matches(p)
        _, ql, _ = be.result(2 * p)
        _, tr, _ = be.result(2 * p + 1)
        r = oracle.knn2(ql, tr)
        for a, b in zip((i1, d1, i2, d2), r):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("pairs,rows_only", [(1, True), (1, False), (3, False)])
def test_run_batch_match_one_submission(oracle, pairs, rows_only):
    """orbgpu_run_batch_match: one pair runs extraction + kNN2 as ONE captured graph (replayed for
    the next frames, the graph keyed on the match too); three pairs take the chunked path (the two
    calls).  Keypoints, descriptors and every pair's kNN2 (all rows or the stereo rows [mono, n)
    of both eyes, Frame.cc:1142-1148) against the oracle, over three different frames."""
    import orbslam3lib_amd as og
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2 * pairs)
    laps = np.array([[0, 0], [60, 600]] * pairs if not rows_only else [[120, 640], [0, 520]] * pairs, np.int32)
    for f in range(3):
        imgs = synth.stereo_batch(480, 640, pairs, first=20 + 7 * f)
        be.upload(imgs)
        be.run_match(laps=laps, stereo_rows_only=rows_only)
        be.synchronize()
        res = [be.result(i) for i in range(2 * pairs)]
        for i in range(2 * pairs):
            rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000, lap=tuple(laps[i]))
            k, d, m = res[i]
            assert m == rm
            _same_kps(k, rk)
            np.testing.assert_array_equal(d, rd)
        for p in range(pairs):
            _, ql, ml = res[2 * p]
            _, tr, mr = res[2 * p + 1]
            q, t = (ql[ml:], tr[mr:]) if rows_only else (ql, tr)
            assert len(q) > 0 and len(t) > 0
            r = oracle.knn2(q, t)
            got = be.matches(p)
            for a, b in zip(got, r):
                np.testing.assert_array_equal(a, b)


def test_knn2_ties_and_edges(oracle):
    import orbslam3lib_amd as og
    ex = _extractor()
    bf = og.BFMatcher(ex)
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    t = np.concatenate([base, base, base[:7]])          # exact duplicates -> ties
    q = np.concatenate([base[:13], rng.integers(0, 256, (1200, 32), dtype=np.uint8)])
    for tt in (t, t[:1], t[:0], rng.integers(0, 256, (1700, 32), dtype=np.uint8)):
        got = bf.knnMatch(q, tt, 2)
        ref = oracle.knn2(q, tt)
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)


def test_euroc_size_and_other_frames(oracle):
    ex = _extractor(w=752, h=480)
    for k in (1, 7):
        img = synth.frame(480, 752, k)
        g = ex(img, None, (0, 0))
        r = oracle.extract(img, nfeatures=2000, lap=(0, 0))
        assert g[2] == r[2]
        _same_kps(g[0], r[0])
        np.testing.assert_array_equal(g[1], r[1])


def test_c5_1080p_12_levels(oracle):
    """C5's frame: 1920x1080, 12 levels, 5000 features."""
    img = synth.frame(1080, 1920, 2)
    ex = _extractor(nf=5000, L=12, w=1920, h=1080)
    g = ex(img, None, (0, 0))
    r = oracle.extract(img, nfeatures=5000, nlevels=12, lap=(0, 0))
    assert g[2] == r[2]
    _same_kps(g[0], r[0])
    np.testing.assert_array_equal(g[1], r[1])


@pytest.mark.parametrize("sf,L", [(2.5, 4), (3.0, 3)])
def test_scale_factor_above_2(oracle, sf, L):
    """Scale factors above 2 (ORBextractor accepts any value above 1; ORB-SLAM3's settings use
    1.2): the pyramid takes k_level_linear per level from HBM and k_blur per level, since
    k_blur_resize's staged window holds a resize step's taps only up to 2.  1920x1080, the
    levels kept above the 42-px minimum: pyramid, blur, keypoints and descriptors equal the
    oracle, through the single-image and the batch entry points."""
    import orbslam3lib_amd as og
    img = synth.frame(1080, 1920, 9)
    ex = _extractor(nf=3000, L=L, w=1920, h=1080, sf=sf)
    g = ex(img, None, (0, 0))
    r = oracle.extract(img, nfeatures=3000, scale_factor=sf, nlevels=L, lap=(0, 0))
    assert g[2] == r[2]
    _same_kps(g[0], r[0])
    np.testing.assert_array_equal(g[1], r[1])
    ref = oracle.pyramid(img, scale_factor=sf, nlevels=L)
    for l in range(L):
        np.testing.assert_array_equal(ex.pyramid_level(0, l), ref[l], err_msg="level %d" % l)
        np.testing.assert_array_equal(ex.pyramid_level(0, l, blurred=True), oracle.blur(ref[l]),
                                      err_msg="blur level %d" % l)
    be = og.BatchExtractor(3000, sf, L, 20, 7, width=1920, height=1080, max_images=2)
    be.upload(np.stack([img, img[::-1].copy()]))
    be.run()
    be.synchronize()
    k, d, m = be.result(0)
    assert m == r[2]
    _same_kps(k, r[0])
    np.testing.assert_array_equal(d, r[1])


def test_flat_and_empty_images(oracle):
    ex = _extractor()
    flat = np.full((480, 640), 128, np.uint8)
    k, d, m = ex(flat)
    rk, rd, rm = oracle.extract(flat, nfeatures=2000)
    assert len(k) == len(rk) == 0 and m == rm == 0
    k, d, m = ex(np.zeros((0, 0), np.uint8))
    assert m == -1 and len(k) == 0


def _two_sided_frames():
    """Frames where most pixels pass the compass pre-test on BOTH sides (a steep diagonal ramp:
    ring points 0/4 brighter, 8/12 darker: 77% of pixels), a mix of ramp and noise inside one
    cell (23%), and a 3-px checkerboard where every pixel is a one-sided candidate -- the densest
    candidate lists k_fast_cells builds."""
    h, w = 480, 640
    y, x = np.mgrid[0:h, 0:w]
    ramp = (((x + y) * 10) & 255).astype(np.uint8)
    noise = synth.frame(h, w, 4)
    mixed = noise.copy()
    mixed[:, ::70] = ramp[:, ::70]
    band = (x // 17 + y // 13) % 2 == 0
    mixed[band] = ramp[band]
    checker = (((x // 3 + y // 3) % 2) * 200 + 20).astype(np.uint8)
    return ramp, mixed, checker


def test_fast_two_sided_candidates(oracle):
    ex = _extractor()
    for img in _two_sided_frames():
        for lap in ((0, 0), (0, 1000)):
            k, d, m = ex(img, None, lap)
            rk, rd, rm = oracle.extract(img, nfeatures=2000, lap=lap)
            assert m == rm
            _same_kps(k, rk)
            np.testing.assert_array_equal(d, rd)


def test_descriptor_distance_matches_reference(oracle):
    import orbslam3lib_amd as og
    rng = np.random.default_rng(3)
    for _ in range(200):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert og.ORBmatcher.DescriptorDistance(a, b) == oracle.descriptor_distance(a, b)


@pytest.mark.parametrize("w,h", [(640, 480), (640, 400)])
def test_cpp_facade(w, h):
    """The C++ ORB_SLAM3::ORBextractor facade (what an ORB-SLAM3 build links) vs the oracle: mono
    operator(), the side-by-side / two-image / AHardwareBuffer stereo forms and BFMatchORB, at
    640x480 and at the headset's 640x400 eyes (1280x400 side-by-side AHB,
    LynxHardwareAccelerator.h:20-21, ORBextractor.cc:136-143)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "cpp", "build", "facade_test")
    assert os.path.exists(exe), "run make (builds tests/cpp/build/facade_test)"
    r = subprocess.run([exe, os.path.join(root, "oracle", "build", "liborb_oracle.so"), str(w), str(h)],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FACADE OK" in r.stdout


def test_gpu_matches_golden_fixtures():
    """GPU output equals the committed golden vectors (no oracle call on the box)."""
    import glob
    import os

    import orbslam3lib_amd as og
    from tests.test_golden import CASES, load_case
    assert CASES
    for path in CASES:
        img, z = load_case(path)
        h, w = img.shape
        ex = og.ORBextractor(int(z["nfeatures"]), 1.2, int(z["nlevels"]), 20, 7, max_width=w,
                             max_height=h, max_images=2)
        k, d, mono = ex(img, None, tuple(int(v) for v in z["lap"]))
        assert mono == int(z["mono"]), path
        _same_kps(k, z["kps"])
        np.testing.assert_array_equal(d, z["desc"])
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    L = np.load(os.path.join(gold, "c2_left_640x480_n2000.npz"))["desc"]
    R = np.load(os.path.join(gold, "c2_right_640x480_n2000.npz"))["desc"]
    g = np.load(os.path.join(gold, "c2_knn2_left_right.npz"))
    got = og.BFMatcher(ex).knnMatch(L, R, 2)
    for a, key in zip(got, ("idx1", "dist1", "idx2", "dist2")):
        np.testing.assert_array_equal(a, g[key])


@pytest.mark.parametrize("env", [{"ORBGPU_OCT_SPLIT": "0"}, {"ORBGPU_OCT_SPLIT": "3"},
                                 {"ORBGPU_OCT_SPLIT": "0", "ORBGPU_OCT_SMALL_THREADS": "128"},
                                 {"ORBGPU_OCT_SMALL_LDS": "65536", "ORBGPU_OCT_SPLIT": "1"}])
def test_octree_launch_shapes(oracle, monkeypatch, env):
    """k_octree's two launch shapes: 512-thread workgroups with the full LDS layout for levels
    [0, split) and 256/128-thread workgroups with the small layout for the rest (default: every
    level small for 640x480-class launches of >= 32 images, most labels in the global workspace;
    the 128-pair bench batch of test_batch_edges runs that).  Forced splits on a 4-frame batch,
    both small workgroup sizes and a layout with all labels in LDS give the oracle's keypoints."""
    import orbslam3lib_amd as og
    for k, v in env.items():
        monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
        monkeypatch.setenv(k, v)
    imgs = synth.stereo_batch(480, 640, 2, first=11)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=4)
    be.upload(imgs)
    be.run()
    be.synchronize()
    for i in range(4):
        k, d, m = be.result(i)
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000)
        assert m == rm
        _same_kps(k, rk)
        np.testing.assert_array_equal(d, rd)


@pytest.mark.parametrize("pitch", ["64", "80"])
def test_forced_fast_tile(oracle, frame0, monkeypatch, pitch):
    """The 64- and 80-byte-pitch FAST tiles (the runtime uses 48 bytes for the leading levels of
    a 640x480 pyramid, 64 for its top levels and 80 for cells wider than 55 px) on every level
    of the 640x480 frame, forced through ORBGPU_FAST_PITCH."""
    L, _ = frame0
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_FAST_PITCH", pitch)
    ex = _extractor()
    k, d, m = ex(L)
    rk, rd, rm = oracle.extract(L, nfeatures=2000)
    _same_kps(k, rk)
    np.testing.assert_array_equal(d, rd)


def test_general_fast_tile_small_frame(oracle):
    """A small frame (cells wider than 55 px on its top levels): k_fast_cells picks its 80-byte
    tile by itself there."""
    img = synth.frame(120, 160, 5)
    ex = _extractor(nf=300, L=4, w=160, h=120)
    k, d, m = ex(img)
    rk, rd, rm = oracle.extract(img, nfeatures=300, nlevels=4)
    _same_kps(k, rk)
    np.testing.assert_array_equal(d, rd)


def test_octree_generic_instantiation(oracle, frame0, monkeypatch):
    """Every level through k_octree_retry (generic pointers, the path taken by levels with
    more candidates than the LDS label capacity), forced with ORBGPU_OCT_GENERIC."""
    L, _ = frame0
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_OCT_GENERIC", "1")
    ex = _extractor()
    k, d, m = ex(L)
    rk, rd, rm = oracle.extract(L, nfeatures=2000)
    _same_kps(k, rk)
    np.testing.assert_array_equal(d, rd)


def _check_pyramid(ex, oracle, imgs, sf=1.2, L=8):
    for i, img in enumerate(imgs):
        ref = oracle.pyramid(img, sf, L)
        for l in range(L):
            np.testing.assert_array_equal(ex.pyramid_level(i, l), ref[l], err_msg="img %d level %d" % (i, l))
            np.testing.assert_array_equal(ex.pyramid_level(i, l, blurred=True), oracle.blur(ref[l]),
                                          err_msg="img %d blur level %d" % (i, l))


@pytest.mark.parametrize("tail", [True, False])
def test_pyramid_per_level_path(oracle, monkeypatch, tail):
    """The per-level k_blur_resize launches then k_pyr_tail (levels 5-7 and the blurs of 4-7 of
    a 640x480 pyramid in one launch; forced with ORBGPU_TAIL_MIN=0, since the product takes the
    tail only for launches of >= 128 images) -- or, with the tail off (ORBGPU_NO_TAIL, the path a
    pair takes by default), k_blur_resize for every level and k_blur for the last: pyramid and
    blurred levels of a stereo pair."""
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_TAIL_MIN" if tail else "ORBGPU_NO_TAIL", "0" if tail else "1")
    L, R = synth.stereo_pair(480, 640, 3)
    ex = _extractor()
    ex.extract_stereo(L, R)
    _check_pyramid(ex, oracle, [L, R])


@pytest.mark.parametrize("tail", [True, False])
def test_pyramid_exact_2x_area_path(oracle, monkeypatch, tail):
    """Scale factor 2 on a 640x480 frame: every level is an exact 2x downscale, which OpenCV
    serves with INTER_AREA (2x2 mean) instead of INTER_LINEAR (the area path of k_blur_resize
    for level 1 and of k_pyr_tail for level 2, forced with ORBGPU_TAIL_MIN=0; with the tail off,
    k_blur_resize's for both)."""
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_TAIL_MIN" if tail else "ORBGPU_NO_TAIL", "0" if tail else "1")
    img = synth.frame(480, 640, 6)
    ex = _extractor(nf=500, L=3, sf=2.0)
    k, d, m = ex(img)
    _check_pyramid(ex, oracle, [img], sf=2.0, L=3)
    rk, rd, rm = oracle.extract(img, nfeatures=500, scale_factor=2.0, nlevels=3)
    _same_kps(k, rk)
    np.testing.assert_array_equal(d, rd)
