"""Wire formats either side of the hot path: side-by-side stereo Y8 ingest
(ORBextractor.cc:131-143, orbslam_dsp.cpp:643-648) and the orbslam3.idl:15-19 SoA egress
(X / Y / encoded angle / level int32 arrays, N x 32 B descriptors, int16 kNN indices and
distances), plus the one-call orbslam3_extractFeatures equivalent.

CPU: the oracle's SoA packing against a numpy restatement, and the reference host decode
(LynxHardwareAccelerator.cpp:174-178) of the angle encoding within a degree of the exact angle.
GPU: the split kernel, the pack kernel and the one-call ABI against the oracle, bit-exact.

Parity status: the keypoints / descriptors / matches are the oracle's (pinned as in
test_golden.py); the SoA encoding itself has no reference fixture (the DSP's own angle LUT is
HVX-specific) -- it is defined here so the reference host decode reads it, and cross-checked."""
import ctypes as C

import numpy as np
import pytest

from orbslam3lib_amd import synth

NF = 2000


def _sbs(pairs, pad=0):
    """Side-by-side frames [n, H, 2W + pad]: left half, right half, optional row padding."""
    fr = [np.concatenate([L, R] + ([np.full((L.shape[0], pad), 77, np.uint8)] if pad else []), 1)
          for L, R in pairs]
    return np.ascontiguousarray(np.stack(fr))


def _np_soa(kps):
    # the descriptor's std::cos(float) / std::sin(float) (ORBextractor_old.cc:114-115): libm cosf
    libm = C.CDLL("libm.so.6")
    libm.cosf.restype = libm.sinf.restype = C.c_float
    libm.cosf.argtypes = libm.sinf.argtypes = [C.c_float]
    rad = (kps["angle"].astype(np.float32) * np.float32(np.pi / 180.0)).astype(np.float32)
    a = np.array([libm.cosf(float(r)) for r in rad], np.float32)
    b = np.array([libm.sinf(float(r)) for r in rad], np.float32)
    c8 = np.rint(np.float32(64) * a).astype(np.int32)
    s8 = np.rint(np.float32(64) * b).astype(np.int32)
    return {"x": kps["x"].astype(np.int32), "y": kps["y"].astype(np.int32),
            "angle": (c8 & 0xFF) | ((s8 & 0xFF) << 8), "level": kps["octave"].astype(np.int32)}


def test_oracle_soa_matches_numpy_and_host_decode(oracle):
    L = synth.frame(480, 640, 3)
    kps, _, _ = oracle.extract(L, nfeatures=NF)
    soa = oracle.pack_soa(kps)
    ref = _np_soa(kps)
    for k in ("x", "y", "angle", "level"):
        np.testing.assert_array_equal(soa[k], ref[k], err_msg=k)
    # the reference host's decode lands within a degree of the exact angle (circularly)
    dec = oracle.decode_angle(soa["angle"])
    diff = np.abs((dec - kps["angle"] + 180.0) % 360.0 - 180.0)
    assert diff.max() < 1.0, diff.max()
    assert (soa["x"] >= 0).all() and (soa["y"] >= 0).all()


def test_oracle_soa_empty(oracle):
    soa = oracle.pack_soa(np.zeros(0, oracle.KP_DTYPE))
    assert all(len(v) == 0 for v in soa.values())


def _check_image(oracle, be, i, img, lap=(0, 0)):
    kps, desc, mono = oracle.extract(img, nfeatures=NF, lap=lap)
    gk, gd, gm = be.result(i)
    np.testing.assert_array_equal(gk.view(np.uint8), kps.view(np.uint8), err_msg="image %d kps" % i)
    np.testing.assert_array_equal(gd, desc.reshape(-1, 32) if desc is not None else gd,
                                  err_msg="image %d desc" % i)
    assert gm == mono
    return kps, desc, mono


@pytest.mark.gpu
@pytest.mark.parametrize("w,pad", [(640, 0), (640, 64), (750, 4)])
def test_gpu_sbs_ingest_bit_exact(oracle, w, pad):
    """Split kernel (16 B path for w % 16 == 0 with an aligned stride, byte path otherwise)
    followed by the full extraction: every eye equals the oracle's extraction of that eye."""
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(480, w, s) for s in range(3)]
    be = og.BatchExtractor(NF, 1.2, 8, 20, 7, width=w, height=480, max_images=6)
    be.upload_sbs(_sbs(pairs, pad), width=w)
    assert be.n == 6 and be.width == w
    be.run()
    be.synchronize()
    for p, (L, R) in enumerate(pairs):
        _check_image(oracle, be, 2 * p, L)
        _check_image(oracle, be, 2 * p + 1, R)
        lv = be.pyramid_level(2 * p + 1, 0) if hasattr(be, "pyramid_level") else None
        if lv is not None:
            np.testing.assert_array_equal(lv, R)


@pytest.mark.gpu
def test_gpu_sbs_ingest_from_device_memory(oracle):
    """Zero-copy ingest: a producer (the camera DMA, here a hipMemcpy) writes side-by-side frames
    straight into the context's device staging buffer; the split runs on the device."""
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(480, 640, 20 + s) for s in range(2)]
    frames = _sbs(pairs)
    be = og.BatchExtractor(NF, 1.2, 8, 20, 7, width=640, height=480, max_images=4)
    lib = og.load_library()
    dptr = lib.orbgpu_device_sbs_input(be.ctx.handle)
    assert dptr
    memcpy = og.hip_function("hipMemcpy")  # the runtime liborbgpu.so is bound to
    memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert memcpy(dptr, frames.ctypes.data, frames.nbytes, 1) == 0  # hipMemcpyHostToDevice
    be.ingest_sbs(dptr, 2, 1280)
    be.run()
    be.synchronize()
    for p, (L, R) in enumerate(pairs):
        _check_image(oracle, be, 2 * p, L)
        _check_image(oracle, be, 2 * p + 1, R)


def _knn_ref(oracle, dq, dt):
    i1, d1, i2, d2 = oracle.knn2(dq, dt)
    return i1.astype(np.int16), np.minimum(d1, 32767).astype(np.int16), np.minimum(d2, 32767).astype(np.int16)


@pytest.mark.gpu
def test_gpu_soa_egress_and_stereo_rows(oracle):
    """pack_soa over a batch with lapping areas: SoA == oracle.pack_soa of the oracle keypoints,
    descriptors verbatim, and the int16 kNN of the stereo rows ([mono, n) of each eye)."""
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(480, 640, 30 + s) for s in range(3)]
    laps = [(0, 0), (0, 0), (400, 640), (0, 240), (120, 520), (100, 500)]
    be = og.BatchExtractor(NF, 1.2, 8, 20, 7, width=640, height=480, max_images=6)
    be.upload_sbs(_sbs(pairs))
    be.run(laps=np.array(laps, np.int32))
    be.match_stereo(stereo_rows_only=True)
    be.pack_soa()
    be.synchronize()
    for p, (L, R) in enumerate(pairs):
        res = []
        for e, img in enumerate((L, R)):
            i = 2 * p + e
            kps, desc, mono = _check_image(oracle, be, i, img, laps[i])
            soa = be.soa_result(i)
            ref = oracle.pack_soa(kps)
            for k in ("x", "y", "angle", "level"):
                np.testing.assert_array_equal(soa[k], ref[k], err_msg="image %d %s" % (i, k))
            np.testing.assert_array_equal(soa["orb"], desc.reshape(-1, 32))
            assert soa["mono"] == mono
            res.append((desc.reshape(-1, 32), mono))
        (dl, ml), (dr, mr) = res
        gi, g1, g2 = be.matches16(p)
        ri, r1, r2 = _knn_ref(oracle, dl[ml:], dr[mr:])
        np.testing.assert_array_equal(gi, ri, err_msg="pair %d indices" % p)
        np.testing.assert_array_equal(g1, r1, err_msg="pair %d dist1" % p)
        np.testing.assert_array_equal(g2, r2, err_msg="pair %d dist2" % p)


@pytest.mark.gpu
def test_gpu_extract_features_one_call(oracle):
    """orbslam3_extractFeatures-shaped call: one side-by-side frame in, SoA + matches out."""
    import orbslam3lib_amd as og
    lib = og.load_library()
    L, R = synth.stereo_pair(480, 640, 40)
    frame = _sbs([(L, R)])[0]
    ctx = og._Context(NF, 1.2, 8, 20, 7, 0, 640, 480, 2)
    cap = 20000
    arr = {k: np.zeros(cap, np.int32) for k in ("xl", "yl", "al", "ll", "xr", "yr", "ar", "lr")}
    orb_l = np.zeros((cap, 32), np.uint8)
    orb_r = np.zeros((cap, 32), np.uint8)
    idx, d1, d2 = (np.zeros(cap, np.int16) for _ in range(3))
    nl, nr, ml, mr = (C.c_int(0) for _ in range(4))
    P = og._p
    lapL, lapR = (300, 640), (0, 340)
    rc = lib.orbgpu_extract_features(
        ctx.handle, P(frame), frame.size, 640, 480, 1280, 20, lapL[0], lapL[1], lapR[0], lapR[1],
        C.byref(nl), P(arr["xl"]), P(arr["yl"]), P(arr["al"]), P(arr["ll"]), P(orb_l),
        C.byref(nr), P(arr["xr"]), P(arr["yr"]), P(arr["ar"]), P(arr["lr"]), P(orb_r), cap,
        C.byref(ml), C.byref(mr), P(idx), P(d1), P(d2), cap)
    assert rc == 0, lib.orbgpu_last_error()
    kl, dl, mono_l = oracle.extract(L, nfeatures=NF, lap=lapL)
    kr, dr, mono_r = oracle.extract(R, nfeatures=NF, lap=lapR)
    assert (nl.value, ml.value, nr.value, mr.value) == (len(kl), mono_l, len(kr), mono_r)
    for kps, desc, n, xs, ys, angs, lvls, orb in ((kl, dl, nl.value, "xl", "yl", "al", "ll", orb_l),
                                                  (kr, dr, nr.value, "xr", "yr", "ar", "lr", orb_r)):
        ref = oracle.pack_soa(kps)
        np.testing.assert_array_equal(arr[xs][:n], ref["x"])
        np.testing.assert_array_equal(arr[ys][:n], ref["y"])
        np.testing.assert_array_equal(arr[angs][:n], ref["angle"])
        np.testing.assert_array_equal(arr[lvls][:n], ref["level"])
        np.testing.assert_array_equal(orb[:n], desc.reshape(-1, 32))
    ri, r1, r2 = _knn_ref(oracle, dl.reshape(-1, 32)[mono_l:], dr.reshape(-1, 32)[mono_r:])
    nq = len(ri)
    np.testing.assert_array_equal(idx[:nq], ri)
    np.testing.assert_array_equal(d1[:nq], r1)
    np.testing.assert_array_equal(d2[:nq], r2)
    # too small a buffer for the frame: refused, nothing read out of bounds
    assert lib.orbgpu_extract_features(
        ctx.handle, P(frame), 1000, 640, 480, 1280, 20, 0, 0, 0, 0, C.byref(nl), None, None, None,
        None, None, C.byref(nr), None, None, None, None, None, cap, C.byref(ml), C.byref(mr), None,
        None, None, cap) == -3
    ctx.close()


def _fnv(arrs):
    h = 1469598103934665603
    for a in arrs:
        for b in np.ascontiguousarray(a).view(np.uint8).ravel().tolist():
            h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.gpu
def test_gpu_extract_features_from_plain_c(oracle, tmp_path):
    """tests/c/idl_test.c (gcc, C99) calls orbgpu_extract_features as the FastRPC host wrapper
    would; its outputs (hashed) equal the oracle's SoA + stereo-row kNN."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "c", "build", "idl_test")
    assert os.path.exists(exe), "built by `make` (idl_test target)"
    W, H = 640, 480
    L, R = synth.stereo_pair(H, W, 44)
    frame = _sbs([(L, R)])[0]
    path = tmp_path / "sbs.y8"
    frame.tofile(path)
    out = subprocess.run([exe, str(path), str(W), str(H)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.split("\n")
    laps = [(300, W), (0, W - 300)]
    descs = []
    for e, img in enumerate((L, R)):
        kps, desc, mono = oracle.extract(img, nfeatures=NF, lap=laps[e])
        soa = oracle.pack_soa(kps)
        h = _fnv([soa["x"], soa["y"], soa["angle"], soa["level"], desc.reshape(-1, 32)])
        assert lines[e] == "eye %d n %d mono %d hash %016x" % (e, len(kps), mono, h), lines[e]
        descs.append((desc.reshape(-1, 32), mono))
    (dl, ml), (dr, mr) = descs
    ri, r1, r2 = _knn_ref(oracle, dl[ml:], dr[mr:])
    assert lines[2] == "matches %d hash %016x" % (len(ri), _fnv([ri, r1, r2])), lines[2]
