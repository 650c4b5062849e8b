"""GPU parity on the configurations the headline numbers run, and on the matcher's segment edges.

* kNN2 past one 4096-row train segment (k_knn2_mfma walks train rows in 4096-row segments with a
  12-bit local index, orb_kernels.hip knn2_mfma_block): nt in {4095, 4096, 4097, 5000, 8193} with
  exact-duplicate rows on both sides of every segment boundary, so the cross-segment tie rule
  (lowest index wins, cv::BFMatcher k=2 / SURVEY §8 a10) is exercised.
* The batch matcher (orbgpu_match_stereo_batch) with more than 4096 train rows per pair, and the
  C5 batch the bench's side line runs (1920x1080, 12 levels, 5000 features, 16 pairs).
* The exact bench batch (bench.py: 256 pairs tiled from the distinct seeded pairs, 2 chunk
  streams (the default; 3 forced too), staggered first step, then the steady state), sampled
  against the oracle.
* Consumers given an explicit stream right after a multi-stream batch (they must wait
  for the chunk streams), and the IDL one-call entry with a padded stride and a buffer that ends
  at the last pixel.

Oracle: oracle/orb_oracle.cpp (the checker), parity pinned as in test_golden.py."""
import ctypes as C

import numpy as np
import pytest

from orbslam3lib_amd import synth

pytestmark = pytest.mark.gpu


def _same_kps(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


def _same_knn(got, ref, msg=""):
    for a, b, name in zip(got, ref, ("idx1", "dist1", "idx2", "dist2")):
        np.testing.assert_array_equal(a, b, err_msg="%s %s" % (msg, name))


@pytest.mark.parametrize("nt", [4095, 4096, 4097, 5000, 8193])
def test_knn2_train_segments(oracle, nt):
    import orbslam3lib_amd as og
    ex = og.ORBextractor(500, 1.2, 4, 20, 7, max_width=160, max_height=120, max_images=1)
    bf = og.BFMatcher(ex)
    rng = np.random.default_rng(nt)
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    # duplicates straddling each segment boundary (and the ends): the same row at b-2 .. b+1
    for b in range(4096, nt + 1, 4096):
        src = t[(b * 7) % 1000].copy()
        for r in (b - 2, b - 1, b, b + 1):
            if 0 <= r < nt:
                t[r] = src
    t[nt - 1] = t[3]
    probes = [t[r] for r in range(nt) if r % 4096 in (4094, 4095, 0, 1)] + [t[3], t[nt - 1]]
    # near-duplicates (one bit flipped) compete with exact ones across segments
    near = []
    for p in probes[:8]:
        x = p.copy()
        x[5] ^= 0x10
        near.append(x)
    q = np.concatenate([np.stack(probes + near), rng.integers(0, 256, (700, 32), dtype=np.uint8)])
    got = bf.knnMatch(q, t, 2)
    _same_knn(got, oracle.knn2(q, t), "nt=%d" % nt)
    # every probe finds itself at distance 0, and its twin (if any) second
    assert (got[1][:len(probes)] == 0).all()


def _batch(og, w, h, L, nf, imgs):
    be = og.BatchExtractor(nf, 1.2, L, 20, 7, width=w, height=h, max_images=len(imgs))
    be.upload(imgs)
    return be


def test_batch_knn2_past_4096_train_rows(oracle):
    """orbgpu_match_stereo_batch with > 4096 keypoints per eye (1920x1080, 12 levels, 8200
    features): the pair's kNN2 crosses a train segment."""
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(1080, 1920, 60 + i) for i in range(2)]
    imgs = np.stack([x for p in pairs for x in p])
    be = _batch(og, 1920, 1080, 12, 8200, imgs)
    be.run()
    be.match_stereo(False)
    be.synchronize()
    for p in range(2):
        _, dl, _ = be.result(2 * p)
        _, dr, _ = be.result(2 * p + 1)
        assert len(dr) > 4096 and len(dl) > 4096, (len(dl), len(dr))
        _same_knn(be.matches(p), oracle.knn2(dl, dr), "pair %d" % p)
    k, d, m = be.result(3)
    rk, rd, rm = oracle.extract(imgs[3], nfeatures=8200, nlevels=12)
    assert m == rm
    _same_kps(k, rk)
    np.testing.assert_array_equal(d, rd)


@pytest.mark.parametrize("pyr", [None, "0"])
def test_batch_1080p_8200_repeatable(oracle, monkeypatch, pyr):
    """Levels 0-2 of a 1920x1080 / 12-level / 8200-feature frame hold more than 1024 octree nodes,
    so k_octree_retry keeps their node state in the global workspace.  Until round 6 that region
    was sized for 78 B per node while the carve uses 86 (orb_kernels.h oct_layout), so level l
    wrote into level l + 1's keys while another workgroup was using them: with two chunk streams
    the level-1 / level-2 keypoint sets changed from run to run (tools/race_probe.py).  Every image
    of both pairs against the oracle on three runs of one context, with the count pyramid and with
    the label passes only (ORBGPU_OCT_PYR=0)."""
    import orbslam3lib_amd as og
    if pyr is not None:
        monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
        monkeypatch.setenv("ORBGPU_OCT_PYR", pyr)
    pairs = [synth.stereo_pair(1080, 1920, 60 + i) for i in range(2)]
    imgs = np.stack([x for p in pairs for x in p])
    refs = [oracle.extract(x, nfeatures=8200, nlevels=12) for x in imgs]
    be = _batch(og, 1920, 1080, 12, 8200, imgs)
    for rep in range(3):
        be.run()
        be.synchronize()
        for i in range(4):
            k, d, m = be.result(i)
            rk, rd, rm = refs[i]
            assert m == rm, (rep, i)
            _same_kps(k, rk)
            np.testing.assert_array_equal(d, rd, err_msg="run %d image %d" % (rep, i))


def test_split_knn2_one_pair_past_4096_rows(oracle, monkeypatch):
    """A one-pair batch (the C4 shape) matches with the train rows split over 8 workgroups per
    query block, the last of which merges the partial lists (orb_kernels.hip k_knn2_mfma_pairs'
    counter hand-off); at 1920x1080 with 8200 features the splits straddle the 4096-row key
    segments.  Equal to the oracle on three launches in a row (the arrival counters reset
    themselves), and to the unsplit launch (ORBGPU_KNN_NOSPLIT)."""
    import orbslam3lib_amd as og
    imgs = np.stack(synth.stereo_pair(1080, 1920, 61))
    be = _batch(og, 1920, 1080, 12, 8200, imgs)
    be.run()
    be.match_stereo(False)
    be.synchronize()
    _, dl, _ = be.result(0)
    _, dr, _ = be.result(1)
    assert len(dr) > 4096 and len(dl) > 4096, (len(dl), len(dr))
    split = be.matches(0)
    _same_knn(split, oracle.knn2(dl, dr), "split")
    for rep in range(2):
        be.match_stereo(False)
        be.synchronize()
        _same_knn(be.matches(0), split, "split, launch %d" % (rep + 2))
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_KNN_NOSPLIT", "1")
    be.match_stereo(False)
    be.synchronize()
    _same_knn(be.matches(0), split, "unsplit vs split")


def test_small_batch_on_large_context(oracle):
    """A context sized for the bench batch (512 images) running 2 pairs: the chunk count follows
    the batch (orb_runtime.cpp kChunksFor), the one-pair split matcher and the 1024-thread
    finalize take the small launches; keypoints, descriptors and matches equal the oracle."""
    import orbslam3lib_amd as og
    pairs = [synth.stereo_pair(480, 640, 70 + i) for i in range(2)]
    imgs = np.stack([pairs[i // 2][i % 2] for i in range(4)])
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=512)
    be.upload(imgs)
    for n in (4, 2):  # two pairs, then one pair on the same large context
        be.n = n  # the first n uploaded images (orbgpu_run_batch reads images [0, n))
        be.run()
        be.match_stereo(False)
        be.synchronize()
        res = [be.result(i) for i in range(n)]
        for i in range(n):
            rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000)
            assert res[i][2] == rm
            _same_kps(res[i][0], rk)
            np.testing.assert_array_equal(res[i][1], rd)
        for p in range(n // 2):
            _same_knn(be.matches(p), oracle.knn2(res[2 * p][1], res[2 * p + 1][1]), "n %d pair %d" % (n, p))


def test_c5_batch_16_pairs(oracle):
    """The C5 side line's batch (bench.py other_configs: 1920x1080, 12 levels, 5000 features,
    16 pairs tiled from 4 seeded pairs, on the context's chunk streams): every pair's 5000 x 5000 kNN2 against
    the oracle matcher, sampled images against the oracle extractor."""
    import orbslam3lib_amd as og
    cu = [synth.stereo_pair(1080, 1920, 500 + i) for i in range(4)]
    imgs = np.stack([cu[(i // 2) % 4][i % 2] for i in range(32)])
    be = _batch(og, 1920, 1080, 12, 5000, imgs)
    for _ in range(2):
        be.run()
        be.match_stereo(False)
    be.synchronize()
    res = [be.result(i) for i in range(32)]
    for i in (0, 3):
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=5000, nlevels=12)
        assert res[i][2] == rm
        _same_kps(res[i][0], rk)
        np.testing.assert_array_equal(res[i][1], rd)
    for i in range(4, 32):  # tiled copies extract identically on every stream
        _same_kps(res[i][0], res[i % 8][0])
        np.testing.assert_array_equal(res[i][1], res[i % 8][1])
    assert max(len(r[1]) for r in res) > 4096
    for p in range(16):
        _same_knn(be.matches(p), oracle.knn2(res[2 * p][1], res[2 * p + 1][1]), "pair %d" % p)


@pytest.mark.parametrize("P,streams", [(128, None), (256, None), (256, 3)])
def test_bench_batch_pairs(oracle, monkeypatch, P, streams):
    """bench.py's headline batch exactly (256 pairs since round 2; 128 in round 1): 16 distinct
    seeded pairs tiled, 2 chunk streams (the default since round 4; 3 before, forced through
    ORBGPU_STREAMS), the staggered first step and the steady state after it."""
    if streams:
        monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
        monkeypatch.setenv("ORBGPU_STREAMS", str(streams))
    import orbslam3lib_amd as og
    from orbslam3lib_amd.dist import pair_seed_base
    U, W, H = 16, 640, 480
    uniq = [synth.stereo_pair(H, W, pair_seed_base(0) + i) for i in range(U)]
    imgs = np.empty((2 * P, H, W), np.uint8)
    for p in range(P):
        imgs[2 * p], imgs[2 * p + 1] = uniq[p % U]
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2 * P)
    be.upload(imgs)
    laps = np.zeros((2 * P, 2), np.int32)
    ref = {}
    for u in range(U):
        for e in range(2):
            ref[2 * u + e] = oracle.extract(uniq[u][e], nfeatures=2000, lap=(0, 0))
    sample = sorted(set(list(range(2 * U)) + list(range(2 * U, 2 * P, 13)) + [2 * P - 2, 2 * P - 1]))
    for step in range(3):  # step 0: staggered layout; then the steady state
        be.run(laps)
        be.match_stereo(stereo_rows_only=False)
        be.synchronize()
        if step == 1:
            continue
        for i in sample:
            k, d, m = be.result(i)
            rk, rd, rm = ref[i % (2 * U)]
            assert m == rm, (step, i)
            _same_kps(k, rk)
            np.testing.assert_array_equal(d, rd, err_msg="step %d image %d" % (step, i))
        for p in sorted(set(list(range(0, P, 9)) + [P - 1])):
            u = p % U
            _same_knn(be.matches(p), oracle.knn2(ref[2 * u][1], ref[2 * u + 1][1]), "step %d pair %d" % (step, p))


class _Hip:
    """HIP runtime entry points from the runtime liborbgpu.so is bound to (og.hip_function)."""

    def __getattr__(self, name):
        import orbslam3lib_amd as og
        f = og.hip_function(name)
        setattr(self, name, f)
        return f


def _hip():
    lib = _Hip()
    lib.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    lib.hipStreamDestroy.argtypes = [C.c_void_p]
    return lib


def test_explicit_stream_after_chunked_batch(oracle):
    """A 256-image batch runs on the context's chunk streams; kNN2, stereo matching and the grid are
    then launched on a caller stream without synchronising first: they must wait for the chunks
    (orbgpu_match_stereo_batch / stereo_matches_batch / undistort_grid_batch join the context's
    streams), and the next batch must wait for them."""
    import orbslam3lib_amd as og
    P, U, W, H = 128, 8, 640, 480
    uniq = [synth.stereo_pair(H, W, 900 + i) for i in range(U)]
    imgs = np.stack([uniq[(i // 2) % U][i % 2] for i in range(2 * P)])
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2 * P)
    be.upload(imgs)
    hip = _hip()
    s = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(s)) == 0
    mbf = 47.9
    mb = float(np.float32(mbf) / np.float32(435.2))
    K = (458.654, 457.296, 367.215, 248.375)
    try:
        for _ in range(2):
            be.run()
            be.match_stereo(False, stream=s.value)
            be.stereo_matches(mbf, mb, stream=s.value)
            be.undistort_grid(K, (), stream=s.value)
        be.synchronize()
        for p in (0, 5, P - 1):
            u = p % U
            kl, dl, _ = be.result(2 * p)
            kr, dr, _ = be.result(2 * p + 1)
            rk, rd, _ = oracle.extract(uniq[u][0], nfeatures=2000)
            _same_kps(kl, rk)
            _same_knn(be.matches(p), oracle.knn2(dl, dr), "pair %d" % p)
            ur, dep, _ = be.stereo_result(p)
            rur, rdep, _ = oracle.stereo_matches(kl, dl, kr, dr, oracle.pyramid(uniq[u][0]),
                                                 oracle.pyramid(uniq[u][1]), mbf, mb)
            np.testing.assert_array_equal(ur, rur)
            np.testing.assert_array_equal(dep, rdep)
            xy, cell, cs, ci = be.grid_result(2 * p)
            rxy, _, rcell, rcs, rci = oracle.undistort_grid(kl, K, (), W, H)
            np.testing.assert_array_equal(cell, rcell)
            np.testing.assert_array_equal(ci, rci)
    finally:
        be.synchronize()
        hip.hipStreamDestroy(s)


def test_extract_features_padded_stride_exact_buffer(oracle):
    """orbgpu_extract_features with stride > 2W and a buffer that ends at the last row's last
    pixel (image_len = stride * (H - 1) + 2W): accepted, nothing past it is read (the upload
    copies 2W bytes per row), results equal the unpadded call's."""
    import orbslam3lib_amd as og
    lib = og.load_library()
    W, H, pad = 640, 480, 96
    L, R = synth.stereo_pair(H, W, 41)
    stride = 2 * W + pad
    n = stride * (H - 1) + 2 * W
    buf = np.full(n, 255, np.uint8)  # an exactly-sized buffer, padding bytes 255
    for y in range(H):
        buf[y * stride:y * stride + W] = L[y]
        buf[y * stride + W:y * stride + 2 * W] = R[y]
    ctx = og._Context(2000, 1.2, 8, 20, 7, 0, W, H, 2)
    cap = 20000
    outs = {k: np.zeros(cap, np.int32) for k in ("xl", "yl", "al", "ll", "xr", "yr", "ar", "lr")}
    orb_l, orb_r = np.zeros((cap, 32), np.uint8), np.zeros((cap, 32), np.uint8)
    idx, d1, d2 = (np.zeros(cap, np.int16) for _ in range(3))
    nl, nr, ml, mr = (C.c_int(0) for _ in range(4))
    P = og._p
    rc = lib.orbgpu_extract_features(
        ctx.handle, P(buf), n, W, H, stride, 20, 0, 0, 0, 0,
        C.byref(nl), P(outs["xl"]), P(outs["yl"]), P(outs["al"]), P(outs["ll"]), P(orb_l),
        C.byref(nr), P(outs["xr"]), P(outs["yr"]), P(outs["ar"]), P(outs["lr"]), P(orb_r), cap,
        C.byref(ml), C.byref(mr), P(idx), P(d1), P(d2), cap)
    assert rc == 0, lib.orbgpu_last_error()
    kl, dl, _ = oracle.extract(L, nfeatures=2000)
    kr, dr, _ = oracle.extract(R, nfeatures=2000)
    assert (nl.value, nr.value) == (len(kl), len(kr))
    np.testing.assert_array_equal(orb_l[:nl.value], dl)
    np.testing.assert_array_equal(orb_r[:nr.value], dr)
    np.testing.assert_array_equal(outs["xl"][:nl.value], oracle.pack_soa(kl)["x"])
    # one byte short of the last pixel: refused
    assert lib.orbgpu_extract_features(
        ctx.handle, P(buf), n - 1, W, H, stride, 20, 0, 0, 0, 0, C.byref(nl), None, None, None,
        None, None, C.byref(nr), None, None, None, None, None, cap, C.byref(ml), C.byref(mr), None,
        None, None, cap) == -3
    ctx.close()


def test_async_upload_pipeline(oracle):
    """orbgpu_upload_images_async: batch k + 1's pixels are copied into the second input buffer
    while batch k computes; three batches of different frames through both slots, every batch's
    results (and its level-0 pyramid / stereo consumers) equal the oracle's for its own frames."""
    import orbslam3lib_amd as og
    P, W, H = 8, 640, 480
    sets = [np.stack([x for i in range(P) for x in synth.stereo_pair(H, W, 700 + 20 * b + i)]) for b in range(3)]
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2 * P)
    pin = [be.pinned(s.shape) for s in sets]
    for p_, s_ in zip(pin, sets):
        p_[:] = s_
    be.upload(sets[0])
    try:
        for b in range(3):
            be.run()
            be.match_stereo(False)
            if b + 1 < 3:
                be.upload_async(pin[b + 1])   # overlaps this batch's kernels
            be.synchronize()
            for i in (0, 5, 2 * P - 1):
                k, d, m = be.result(i)
                rk, rd, rm = oracle.extract(sets[b][i], nfeatures=2000)
                _same_kps(k, rk)
                np.testing.assert_array_equal(d, rd, err_msg="batch %d image %d" % (b, i))
            _, dl, _ = be.result(2)
            _, dr, _ = be.result(3)
            _same_knn(be.matches(1), oracle.knn2(dl, dr), "batch %d" % b)
        # a staged upload must be consumed before another is staged
        be.upload_async(pin[0])
        with pytest.raises(og.OrbGpuError):
            be.upload_async(pin[1])
        be.run()
        be.synchronize()
        k, d, _ = be.result(1)
        rk, rd, _ = oracle.extract(sets[0][1], nfeatures=2000)
        np.testing.assert_array_equal(d, rd)
    finally:
        be.synchronize()
        be.free_pinned()


def test_device_descriptor_export_and_knn2(oracle):
    """The C5 exchange's device path (dist.cross_camera_match_device): orbgpu_export_descriptors
    copies an image's rows [row0, n) device to device, orbgpu_match_knn2_device matches device
    buffers; checked against the oracle matcher on the downloaded descriptors (raw HIP buffers
    here: the multi-rank RCCL exchange around them runs in bench.py on 8-GPU nodes, its gloo
    rehearsal in test_distributed.py)."""
    import orbslam3lib_amd as og
    hip = _hip()
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    P, W, H = 2, 640, 480
    imgs = np.stack([x for i in range(P) for x in synth.stereo_pair(H, W, 70 + i)])
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2 * P)
    be.upload(imgs)
    be.run()
    bufs = []
    try:
        cap = 4096
        for _ in range(3):
            p = C.c_void_p()
            assert hip.hipMalloc(C.byref(p), cap * 32) == 0
            bufs.append(p)
        na = be.export_descriptors(0, bufs[0].value, cap)
        nb = be.export_descriptors(3, bufs[1].value, cap, row0=100)
        _, da, _ = be.result(0)
        _, db, _ = be.result(3)
        assert na == len(da) and nb == len(db) - 100
        ref = oracle.knn2(da, db[100:])
        be.match_knn2_device(bufs[0].value, na, bufs[1].value, nb, bufs[2].value)
        assert hip.hipDeviceSynchronize() == 0
        out = np.zeros((4, na), np.int32)
        assert hip.hipMemcpy(out.ctypes.data, bufs[2].value, out.nbytes, 2) == 0
        for a, b in zip(out, ref):
            np.testing.assert_array_equal(a, b)
        # the exported rows are the image's descriptors byte for byte
        back = np.zeros((na, 32), np.uint8)
        assert hip.hipMemcpy(back.ctypes.data, bufs[0].value, back.nbytes, 2) == 0
        np.testing.assert_array_equal(back, da)
        with pytest.raises(og.OrbGpuError):
            be.export_descriptors(0, bufs[0].value, 10)  # capacity too small
    finally:
        be.synchronize()
        for p in bufs:
            hip.hipFree(p)


def test_device_entry_points_refuse_host_pointers():
    """orbgpu_export_descriptors / orbgpu_match_knn2_device take device memory only: a host
    address is refused with ORBGPU_ERR_INVALID instead of being written by a device copy or
    read by a kernel (the gloo branch of the C5 exchange once passed host tensors)."""
    import orbslam3lib_amd as og
    imgs = np.stack(synth.stereo_pair(480, 640, 71))
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
    be.upload(imgs)
    be.run()
    host = np.zeros((4096, 32), np.uint8)
    with pytest.raises(og.OrbGpuError) as e:
        be.export_descriptors(0, host.ctypes.data, 4096)
    assert e.value.code == -3
    out = np.zeros((4, 16), np.int32)
    with pytest.raises(og.OrbGpuError) as e:
        be.match_knn2_device(host.ctypes.data, 16, host.ctypes.data, 16, out.ctypes.data)
    assert e.value.code == -3
    # the context stays usable, and no stale HIP error leaks into the next launch
    be.run()
    be.synchronize()
    assert be.counts()[0].min() > 0


def test_caller_stream_batches_with_async_upload(oracle):
    """orbgpu_run_batch on a caller's stream interleaved with orbgpu_upload_images_async through
    both input slots: the batch on the caller's stream is rejoined into the
    context's streams, so the copy that refills its input slot two batches later waits for it.
    Every batch's results equal the oracle's for its own frames."""
    import orbslam3lib_amd as og
    P, W, H = 16, 640, 480
    sets = [np.stack([x for i in range(P) for x in synth.stereo_pair(H, W, 1300 + 40 * b + i)]) for b in range(4)]
    refs = {}
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2 * P)
    pin = [be.pinned(s_.shape) for s_ in sets]
    for p_, s_ in zip(pin, sets):
        p_[:] = s_
    hip = _hip()
    s = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(s)) == 0
    try:
        be.upload(sets[0])
        for b in range(4):
            be.run(stream=s.value)
            be.match_stereo(False, stream=s.value)
            if b + 1 < 4:
                be.upload_async(pin[b + 1])  # slot of batch b - 1, which ran on the caller's stream
            be.synchronize()
            for i in (0, 2 * P - 1):
                key = (b, i)
                if key not in refs:
                    refs[key] = oracle.extract(sets[b][i], nfeatures=2000)
                k, d, m = be.result(i)
                rk, rd, rm = refs[key]
                _same_kps(k, rk)
                np.testing.assert_array_equal(d, rd, err_msg="batch %d image %d" % (b, i))
            _, dl, _ = be.result(2 * P - 2)
            _, dr, _ = be.result(2 * P - 1)
            _same_knn(be.matches(P - 1), oracle.knn2(dl, dr), "batch %d" % b)
    finally:
        be.synchronize()
        be.close()
        hip.hipStreamDestroy(s)


def test_two_contexts_do_not_wait_for_each_other():
    """One extractor per eye from two threads (Frame.cc:142-145): a context's synchronous calls
    wait for its own stream only.  Context A (a one-pair context: one stream) queues ~100 ms of
    single-pair batches without synchronising; context B's blocking stereo extraction must return
    long before A's queue drains (with a device-wide synchronize it would wait for all of A's
    work), with results equal to its unloaded run."""
    import time

    import orbslam3lib_amd as og
    W, H = 640, 480
    L, R = synth.stereo_pair(H, W, 77)
    a = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2)
    a.upload(np.stack([L, R]))
    ex = og.ORBextractor(2000, 1.2, 8, 20, 7, max_width=W, max_height=H, max_images=2)
    (k0, d0, m0), _ = ex.extract_stereo(L, R)  # warm: code objects loaded, buffers sized
    t0 = time.perf_counter()
    for _ in range(20):
        a.run()
    a.synchronize()
    t_one = (time.perf_counter() - t0) / 20
    nb = max(100, int(0.1 / max(t_one, 1e-5)))  # >= ~100 ms of queued work
    t0 = time.perf_counter()
    for _ in range(nb):
        a.run()
    tb0 = time.perf_counter()
    (kl, dl, ml), _ = ex.extract_stereo(L, R)
    t_b = time.perf_counter() - tb0
    a.synchronize()
    t_a = time.perf_counter() - t0
    np.testing.assert_array_equal(dl, d0)
    assert t_b < 0.3 * t_a, (t_b, t_a, nb, t_one)


def test_two_threads_two_contexts_concurrently(oracle):
    """One context per eye, driven from two threads at the same time (the headset's per-eye
    threads, Frame.cc:142-145): every call enters the library's per-call runtime check and the
    launch sequence concurrently (ctypes releases the GIL), and each thread's results stay equal
    to the oracle on its own frames."""
    import threading

    import orbslam3lib_amd as og
    W, H = 640, 480
    frames = [synth.frame(H, W, 900 + k) for k in range(2)]
    refs = [oracle.extract(f, nfeatures=2000) for f in frames]
    errors = []

    def worker(k):
        try:
            ex = og.ORBextractor(2000, 1.2, 8, 20, 7, max_width=W, max_height=H, max_images=2)
            for _ in range(12):
                kp, d, m = ex(frames[k])
                rk, rd, rm = refs[k]
                assert m == rm and len(kp) == len(rk)
                np.testing.assert_array_equal(d, rd.reshape(-1, 32))
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors


@pytest.mark.parametrize("stereo_rows_only", [False, True])
def test_device_ingest_and_batch_export(oracle, stereo_rows_only):
    """The C4 ingest-rank path's two entry points (dist.ingest_scatter_gather): frames already
    in device memory (a padded stride, as a collective's receive buffer may have) go in through
    orbgpu_ingest_images, and orbgpu_export_batch packs the batch's counts and its produced
    keypoints, descriptors and kNN2 rows into one device buffer of exactly that size; decoded, it
    equals result() / matches() and the oracle, bit for bit."""
    import orbslam3lib_amd as og
    hip = _hip()
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    P, W, H, S = 2, 640, 480, 704
    imgs = np.stack([x for i in range(P) for x in synth.stereo_pair(H, W, 140 + i)])
    padded = np.zeros((2 * P, H, S), np.uint8)
    padded[:, :, :W] = imgs
    padded[:, :, W:] = 255  # bytes past the width must not leak into the images
    laps = np.array([[0, 0], [60, 590]] * P, np.int32)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=W, height=H, max_images=2 * P)
    bufs = []
    try:
        src, dst = C.c_void_p(), C.c_void_p()
        assert hip.hipMalloc(C.byref(src), padded.nbytes) == 0
        bufs.append(src)
        assert hip.hipMemcpy(src.value, padded.ctypes.data, padded.nbytes, 1) == 0
        be.ingest_images(src.value, 2 * P, stride=S)
        be.run_match(laps=laps, stereo_rows_only=stereo_rows_only)
        nbytes = be.export_batch_size(2 * P, P)
        # only the produced rows: the header plus 60 B per keypoint and 16 B per query row
        ks = [be.result(i) for i in range(2 * P)]
        assert nbytes == 4 * (4 * P + P) + sum(60 * len(k) for k, _, _ in ks) + \
            sum(16 * len(be.matches(p)[0]) for p in range(P))
        assert nbytes < be.export_batch_bytes(2 * P, P)
        assert hip.hipMalloc(C.byref(dst), nbytes) == 0
        bufs.append(dst)
        used = be.export_batch(dst.value, 2 * P, P, nbytes)
        assert used == nbytes
        be.synchronize()
        host = np.zeros(nbytes, np.uint8)
        assert hip.hipMemcpy(host.ctypes.data, dst.value, nbytes, 2) == 0
        images, pairs = og.BatchExtractor.decode_export(host, 2 * P, P)
        for i in range(2 * P):
            k, d, m = ks[i]
            ek, ed, em = images[i]
            assert em == m
            np.testing.assert_array_equal(ek.view(np.uint8), k.view(np.uint8))
            np.testing.assert_array_equal(ed, d)
            rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000, lap=tuple(laps[i]))
            assert rm == m
            np.testing.assert_array_equal(ed, rd.reshape(-1, 32))
        for p in range(P):
            for a, b in zip(pairs[p], be.matches(p)):
                np.testing.assert_array_equal(a, b)
        with pytest.raises(og.OrbGpuError):
            be.export_batch(dst.value, 2 * P, P, nbytes - 1)  # buffer too small
        with pytest.raises(og.OrbGpuError):
            be.ingest_images(padded.ctypes.data, 2 * P, stride=S)  # host pointer refused
    finally:
        be.synchronize()
        for p in bufs:
            hip.hipFree(p)


def test_context_on_current_device():
    """the drop-in facades build their context on the caller's current HIP
    device (ORBGPU_DEVICE_CURRENT) instead of ordinal 0, so a multi-camera process can place an
    extractor on the GPU it selected (LynxHardwareAccelerator.cpp:146-204 runs one session per
    process).  Through the C ABI: ORBGPU_DEVICE_CURRENT resolves to hipGetDevice()'s ordinal and
    orbgpu_get_device reports it; an ordinal past the device count is ORBGPU_ERR_NO_DEVICE.  (The
    facade side is checked by tests/cpp/facade_test.cpp.)"""
    import orbslam3lib_amd as og
    hip = _hip()
    cur = C.c_int(-1)
    assert hip.hipGetDevice(C.byref(cur)) == 0
    be = og.BatchExtractor(500, 1.2, 4, 20, 7, device=og.DEVICE_CURRENT, width=160, height=120, max_images=2)
    assert be.ctx.device() == cur.value
    be.close()
    ndev = C.c_int(0)
    assert hip.hipGetDeviceCount(C.byref(ndev)) == 0
    with pytest.raises(og.OrbGpuError) as ei:
        og.BatchExtractor(500, 1.2, 4, 20, 7, device=ndev.value, width=160, height=120, max_images=2)
    assert ei.value.code == -6


def test_fused_assembly_equals_finalize(oracle, monkeypatch):
    """Batches with no lapping area (every keypoint mono) are assembled by k_orient_desc itself
    (BatchArgs.fuse_out: rows off[l] + j, pt *= mvScaleFactor[l], ORBextractor_old.cc:1130-1190)
    and k_finalize does not run; a lapping area anywhere in the batch, or ORBGPU_NO_FUSE_OUT,
    takes k_finalize.  The two give the same counts, keypoints and descriptors, the level
    keypoints (orbgpu_get_level_keypoints, read from the assembled rows when fused) agree, and
    a later batch with lapping areas on the same context still matches the oracle."""
    import orbslam3lib_amd as og
    imgs = np.stack([x for i in range(3) for x in synth.stereo_pair(480, 640, 190 + i)])
    be = _batch(og, 640, 480, 8, 2000, imgs)
    be.run()
    be.synchronize()
    fused = [be.result(i) for i in range(len(imgs))]
    laps = np.array([[0, 0], [60, 590]] * 3, np.int32)
    be.run(laps=laps)  # k_finalize path on the same context
    be.synchronize()
    for i in range(len(imgs)):
        k, d, m = be.result(i)
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000, lap=tuple(laps[i]))
        assert m == rm
        np.testing.assert_array_equal(d, rd.reshape(-1, 32))
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_NO_FUSE_OUT", "1")
    be2 = _batch(og, 640, 480, 8, 2000, imgs)
    be2.run()
    be2.synchronize()
    for i in range(len(imgs)):
        k, d, m = be2.result(i)
        fk, fd, fm = fused[i]
        assert m == fm == len(fk)
        np.testing.assert_array_equal(k.view(np.uint8), fk.view(np.uint8))
        np.testing.assert_array_equal(d, fd)
    monkeypatch.delenv("ORBGPU_NO_FUSE_OUT")
    ex = og.ORBextractor(2000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_images=1)
    kp, d, m = ex(imgs[0])
    lk = ex.level_keypoints(0)
    rk, rd, rm = oracle.extract(imgs[0], nfeatures=2000)
    np.testing.assert_array_equal(d, rd.reshape(-1, 32))
    # all mono: the level keypoints in level order are the output rows (level coordinates)
    np.testing.assert_array_equal(np.concatenate([x[1] for x in lk]), d)
    np.testing.assert_array_equal(np.concatenate([x[0]["angle"] for x in lk]), kp["angle"])
    np.testing.assert_array_equal(np.concatenate([x[0]["octave"] for x in lk]), kp["octave"])


def test_fast_small_list_and_overflow_pass(oracle, monkeypatch):
    """k_fast_cells<48>'s small-list form (512 candidates, the batch shape's FAST) and the
    full-list pass over the cells it queues (k_fast_cells_ovf).  Forced on for a small batch
    (ORBGPU_FAST_SMALL=1), including frames of uniform noise whose cells pass far more than 512
    pixels of the pre-test, and with every cell sent through the overflow pass
    (ORBGPU_FAST_OVF_ALL=1): the same keypoints and descriptors as the full-list kernel, on
    repeated batches of one context (the queue counters reset themselves), and the oracle's."""
    import orbslam3lib_amd as og
    rng = np.random.default_rng(77)
    noise = [rng.integers(0, 256, (480, 640), dtype=np.uint8) for _ in range(2)]
    imgs = np.stack([x for i in range(2) for x in synth.stereo_pair(480, 640, 400 + i)] + noise)

    def run_all(be):
        out = []
        for _ in range(2):  # twice on one context
            be.run()
            be.synchronize()
            out.append([be.result(i) for i in range(len(imgs))])
        return out

    ref = run_all(_batch(og, 640, 480, 8, 2000, imgs))
    for i in (0, len(imgs) - 1):
        k, d, m = ref[0][i]
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000)
        assert m == rm
        np.testing.assert_array_equal(d, rd.reshape(-1, 32))
    monkeypatch.setenv("ORBGPU_DIAGNOSTICS", "1")
    monkeypatch.setenv("ORBGPU_FAST_SMALL", "1")
    for ovf_all in (False, True):
        if ovf_all:
            monkeypatch.setenv("ORBGPU_FAST_OVF_ALL", "1")
        got = run_all(_batch(og, 640, 480, 8, 2000, imgs))
        for rep in range(2):
            for i in range(len(imgs)):
                k, d, m = got[rep][i]
                fk, fd, fm = ref[0][i]
                assert m == fm, (ovf_all, rep, i)
                np.testing.assert_array_equal(k.view(np.uint8), fk.view(np.uint8))
                np.testing.assert_array_equal(d, fd)
