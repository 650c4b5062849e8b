"""GPU parity at the geometries the reference itself runs and at odd sizes (bit-exact vs the
oracle, through the C ABI):

* the headset: 640x400 per eye, delivered as a 1280x400 side-by-side Y8 frame
  (cpp/include/LynxHardwareAcceleration/LynxHardwareAccelerator.h:20-21,
  cpp/src/ORBextractor.cc:136-143).  368/35 -> 10 cell rows of 37 px at level 0, level heights
  400, 333, 278, 231, 193, 161, 134, 112 -- a different cell grid and pyramid than 640x480;
* odd level-0 widths and heights (641x401 ...): unaligned rows in every kernel, odd resize
  tables, lapping areas that end inside the frame;
* the one-stream single-pair context (max_images = 2, the facade / C4 shape) fed by the async
  upload, alternating run / run_match and both match variants: every combination replays its
  own captured graph (orb_runtime.cpp graph cache) and must still read the right input slot;
* C5's cross-camera exchange kernels on real C5 cameras: orbgpu_export_descriptors then
  orbgpu_match_knn2_device on two 1920x1080 / 12-level / 5000-feature cameras.
"""
import ctypes as C

import numpy as np
import pytest

from orbslam3lib_amd import synth

pytestmark = pytest.mark.gpu


def _check_image(oracle, be, i, img, lap=(0, 0), nf=2000, L=8):
    rk, rd, rm = oracle.extract(img, nfeatures=nf, nlevels=L, lap=tuple(int(v) for v in lap))
    k, d, m = be.result(i)
    assert m == rm, (i, m, rm)
    np.testing.assert_array_equal(k.view(np.uint8), rk.view(np.uint8), err_msg="image %d keypoints" % i)
    np.testing.assert_array_equal(d, rd.reshape(-1, 32), err_msg="image %d descriptors" % i)
    return k, d, m


def _check_knn(oracle, be, p, q, t):
    ref = oracle.knn2(q, t)
    got = be.matches(p)
    for a, b, name in zip(got, ref, ("idx1", "dist1", "idx2", "dist2")):
        np.testing.assert_array_equal(a, b, err_msg="pair %d %s" % (p, name))


def _force_tail(monkeypatch, tail):
    """tail="forced": k_pyr_tail even for these few-image launches (the product takes it from 128
    images per launch on), so both pyramid paths see the geometry."""
    if tail == "forced":
        monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
        monkeypatch.setenv("ORBGPU_TAIL_MIN", "0")


@pytest.mark.parametrize("tail", ["default", "forced"])
def test_headset_sbs_1280x400(oracle, monkeypatch, tail):
    """Three 1280x400 side-by-side frames -> split on the device -> extraction of every eye and
    the stereo-row kNN2 (BFMatchORB, Frame.cc:1164) of every pair; pyramid and blurred levels of
    one eye as well."""
    import orbslam3lib_amd as og
    _force_tail(monkeypatch, tail)
    W, H = 640, 400
    pairs = [synth.stereo_pair(H, W, 300 + s) for s in range(3)]
    frames = np.ascontiguousarray(np.stack([np.concatenate([L, R], 1) for L, R in pairs]))
    assert frames.shape == (3, 400, 1280)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=6)
    be.upload_sbs(frames, width=W)
    assert be.n == 6 and (be.width, be.height) == (W, H)
    laps = np.array([[100, 639], [0, 540]] * 3, np.int32)
    be.run_match(laps=laps, stereo_rows_only=True)
    be.synchronize()
    for p, (L, R) in enumerate(pairs):
        _, dl, ml = _check_image(oracle, be, 2 * p, L, laps[2 * p])
        _, dr, mr = _check_image(oracle, be, 2 * p + 1, R, laps[2 * p + 1])
        assert len(dl) > ml and len(dr) > mr
        _check_knn(oracle, be, p, dl[ml:], dr[mr:])
    ex = og.ORBextractor(2000, 1.2, 8, 20, 7, max_width=W, max_height=H)
    ex(pairs[0][1])
    ref = oracle.pyramid(pairs[0][1])
    assert [r.shape for r in ref] == [(400, 640), (333, 533), (278, 444), (231, 370), (193, 309),
                                      (161, 257), (134, 214), (112, 179)]
    for l in range(8):
        np.testing.assert_array_equal(ex.pyramid_level(0, l), ref[l], err_msg="level %d" % l)
        np.testing.assert_array_equal(ex.pyramid_level(0, l, blurred=True), oracle.blur(ref[l]),
                                      err_msg="blurred level %d" % l)


@pytest.mark.parametrize("tail", ["default", "forced"])
@pytest.mark.parametrize("w,h", [(641, 401), (643, 479), (753, 481), (637, 403)])
def test_odd_level0_sizes(oracle, monkeypatch, w, h, tail):
    """Odd / non-multiple-of-4 level-0 sizes through the single-image path and the chunked batch
    path (chunk streams), with lapping areas ending inside the frame."""
    import orbslam3lib_amd as og
    _force_tail(monkeypatch, tail)
    ex = og.ORBextractor(2000, 1.2, 8, 20, 7, max_width=w, max_height=h)
    img = synth.frame(h, w, 40 + w)
    for lap in ((0, 0), (101, w - 37)):
        k, d, m = ex(img, None, lap)
        rk, rd, rm = oracle.extract(img, nfeatures=2000, lap=lap)
        assert m == rm
        np.testing.assert_array_equal(k.view(np.uint8), rk.view(np.uint8))
        np.testing.assert_array_equal(d, rd.reshape(-1, 32))
    imgs = synth.stereo_batch(h, w, 3, first=50 + h)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=w, height=h, max_images=6)
    be.upload(imgs)
    laps = np.array([[0, 0], [17, w - 3]] * 3, np.int32)
    be.run(laps)
    be.match_stereo(False)
    be.synchronize()
    for i in range(6):
        _check_image(oracle, be, i, imgs[i], laps[i])
    for p in range(3):
        _check_knn(oracle, be, p, be.result(2 * p)[1], be.result(2 * p + 1)[1])


def test_single_pair_context_async_upload_graphs(oracle):
    """max_images = 2 (one stream, every batch a captured graph): async uploads flip the input
    slot each frame, and run / run_match(all rows) / run_match(stereo rows) alternate, so six
    graph keys are live; each frame's results must be that frame's."""
    import orbslam3lib_amd as og
    W, H = 640, 480
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2)
    pin = be.pinned((2, H, W))
    laps = np.array([[60, 639], [0, 580]], np.int32)
    modes = ["run_match_all", "run", "run_match_rows", "run_match_all", "run_match_rows", "run",
             "run_match_all", "run"]
    try:
        for f, mode in enumerate(modes):
            L, R = synth.stereo_pair(H, W, 400 + f)
            be.synchronize()  # the previous frame's copy has read `pin`
            pin[0], pin[1] = L, R
            be.upload_async(pin)
            if mode == "run":
                be.run(laps)
                be.match_stereo(False)
            else:
                be.run_match(laps=laps, stereo_rows_only=(mode == "run_match_rows"))
            be.synchronize()
            _, dl, ml = _check_image(oracle, be, 0, L, laps[0])
            _, dr, mr = _check_image(oracle, be, 1, R, laps[1])
            if mode == "run_match_rows":
                _check_knn(oracle, be, 0, dl[ml:], dr[mr:])
            else:
                _check_knn(oracle, be, 0, dl, dr)
    finally:
        be.free_pinned()


def test_c5_cross_camera_device_exchange(oracle):
    """The C5 exchange step's kernels (dist.cross_camera_match_device) on C5 cameras: two
    1920x1080 frames (two ranks' cameras), 12 levels, 5000 features; each camera's rows exported
    device to device, then the device kNN2 of camera 0 against camera 1 and back, vs the oracle."""
    import orbslam3lib_amd as og
    hip_malloc = og.hip_function("hipMalloc")
    hip_malloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip_memcpy = og.hip_function("hipMemcpy")
    hip_memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip_free = og.hip_function("hipFree")
    hip_free.argtypes = [C.c_void_p]
    hip_sync = og.hip_function("hipDeviceSynchronize")
    W, H = 1920, 1080
    cams = [synth.stereo_pair(H, W, 500 + 100000 * r)[0] for r in range(2)]  # bench.py's rank seeds
    be = og.BatchExtractor(5000, 1.2, 12, 20, 7, width=W, height=H, max_images=2)
    be.upload(np.stack(cams))
    be.run()
    be.synchronize()
    descs = []
    for i in range(2):
        _, d, _ = _check_image(oracle, be, i, cams[i], nf=5000, L=12)
        assert len(d) > 4500
        descs.append(d)
    bufs = []
    try:
        cap = 5200
        for _ in range(4):
            p = C.c_void_p()
            assert hip_malloc(C.byref(p), cap * 32) == 0
            bufs.append(p)
        n = [be.export_descriptors(i, bufs[i].value, cap) for i in range(2)]
        assert n == [len(descs[0]), len(descs[1])]
        for q, t, o in ((0, 1, 2), (1, 0, 3)):
            be.match_knn2_device(bufs[q].value, n[q], bufs[t].value, n[t], bufs[o].value)
        assert hip_sync() == 0
        for q, t, o in ((0, 1, 2), (1, 0, 3)):
            out = np.zeros((4, n[q]), np.int32)
            assert hip_memcpy(out.ctypes.data, bufs[o].value, out.nbytes, 2) == 0
            ref = oracle.knn2(descs[q], descs[t])
            for a, b in zip(out, ref):
                np.testing.assert_array_equal(a, b)
    finally:
        be.synchronize()
        for p in bufs:
            hip_free(p)
