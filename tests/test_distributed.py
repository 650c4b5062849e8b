"""CPU: the multi-process path of bench.py (gloo, world_size 2): sharding without overlap, and
max/sum reductions of the timing and feature counts across ranks."""
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from orbslam3lib_amd import dist as od
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = od.shard_range(130, rank, world)
    t = od.reduce_scalar(dist, 1.5 + rank, "max")
    s = od.reduce_scalar(dist, hi - lo, "sum")
    dist.barrier()
    q.put((rank, lo, hi, t, s, od.pair_seed_base(rank)))
    dist.destroy_process_group()


def test_gloo_world2_sharding_and_reductions():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, t0, s0, b0), (r1, lo1, hi1, t1, s1, b1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 65, 65, 130)
    assert t0 == t1 == 2.5 and s0 == s1 == 130
    assert b0 != b1


def _cross_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist

    from oracle import oracle_py as O
    from orbslam3lib_amd import dist as od
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cams = [np.random.default_rng(50 + r).integers(0, 256, (37 + 11 * r, 32), dtype=np.uint8)
            for r in range(world)]
    got = od.cross_camera_match(dist, cams[rank], O.knn2)
    ok = sorted(got) == [r for r in range(world) if r != rank]
    for r, res in got.items():
        ref = O.knn2(cams[rank], cams[r])
        ok &= all(np.array_equal(a, b) for a, b in zip(res, ref))
    dist.barrier()
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_gloo_cross_camera_match_world3():
    """C5's exchange step: each rank's camera descriptors (ragged counts) reach every other rank
    intact and are matched there (the oracle kNN2 stands in for the GPU matcher on the CPU)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cross_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


@pytest.mark.parametrize("total,world", [(7, 3), (128, 8), (1, 4)])
def test_shard_range_partitions(total, world):
    from orbslam3lib_amd import dist as od
    spans = [od.shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and b >= a


class _HostExtractor:
    """Stands in for BatchExtractor on the CPU: the same pointer-based calls
    (export_descriptors / match_knn2_device) over host addresses, the oracle as the matcher."""

    def __init__(self, desc):
        import numpy as np
        self.desc = np.ascontiguousarray(desc, dtype=np.uint8)

    def counts(self):
        import numpy as np
        return np.array([len(self.desc)], np.int32), np.zeros(1, np.int32)

    def export_descriptors(self, image, ptr, cap, row0=0, stream=None):
        import ctypes
        n = max(len(self.desc) - row0, 0)
        assert n <= cap and stream is None
        ctypes.memmove(ptr, self.desc[row0:].ctypes.data, 32 * n)
        return n

    def match_knn2_device(self, dq, nq, dt, nt, dout, stream=None):
        import ctypes

        import numpy as np

        from oracle import oracle_py as O
        q = np.ctypeslib.as_array((ctypes.c_uint8 * (32 * nq)).from_address(dq)).reshape(nq, 32)
        t = np.ctypeslib.as_array((ctypes.c_uint8 * (32 * max(nt, 1))).from_address(dt))[:32 * nt].reshape(nt, 32)
        res = np.stack(O.knn2(q, t)).astype(np.int32)
        ctypes.memmove(dout, res.ctypes.data, res.nbytes)


def _cross_dev_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist

    from oracle import oracle_py as O
    from orbslam3lib_amd import dist as od
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cams = [np.random.default_rng(80 + r).integers(0, 256, (40 + 9 * r, 32), dtype=np.uint8)
            for r in range(world)]
    row0 = 3
    got = od.cross_camera_match_device(dist, _HostExtractor(cams[rank]), 0, row0)
    ok = sorted(got) == [r for r in range(world) if r != rank]
    for r, res in got.items():
        ref = O.knn2(cams[rank][row0:], cams[r][row0:])
        ok &= all(np.array_equal(a.numpy(), b) for a, b in zip(res, ref))
    dist.barrier()
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_gloo_cross_camera_match_device_path_world2():
    """dist.cross_camera_match_device (the RCCL path of bench.py on 8-GPU nodes) under gloo: the
    counts exchange, the padded all_gather of exported rows and the per-camera matcher calls,
    with host tensors and a host stand-in for the extractor's device entry points."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cross_dev_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


class _HostBatch:
    """Stands in for BatchExtractor on the CPU for ingest_scatter_gather: ingest_images /
    run_match / export_batch over host addresses (the oracle as the extractor and matcher),
    writing the packed orbgpu_export_batch layout (orbslam3lib_amd.encode_export) that
    decode_export reads."""

    device_resident = False

    def __init__(self, h, w, nfeatures=300, nlevels=4):
        self.height, self.width, self.nf, self.nl = h, w, nfeatures, nlevels
        self.out_cap = 512

    def ingest_images(self, ptr, n, stride=None, stream=None):
        import ctypes

        import numpy as np
        stride = stride or self.width
        a = np.ctypeslib.as_array((ctypes.c_uint8 * (n * self.height * stride)).from_address(ptr))
        self.imgs = a.reshape(n, self.height, stride)[:, :, :self.width].copy()

    def run_match(self, stereo_rows_only=False):
        from oracle import oracle_py as O
        self.res = [O.extract(im, nfeatures=self.nf, nlevels=self.nl) for im in self.imgs]
        self.m = [O.knn2(self.res[2 * p][1], self.res[2 * p + 1][1]) for p in range(len(self.imgs) // 2)]

    def _export(self, n_img, n_pairs):
        from orbslam3lib_amd import encode_export
        return encode_export(self.res[:n_img], self.m[:n_pairs])

    def export_batch_bytes(self, n_img, n_pairs):
        return self._export(n_img, n_pairs).nbytes

    def export_batch_size(self, n_img, n_pairs, stream=None):
        return self._export(n_img, n_pairs).nbytes

    def export_batch(self, ptr, n_img, n_pairs, nbytes, stream=None):
        import ctypes
        buf = self._export(n_img, n_pairs)
        assert buf.nbytes <= nbytes
        ctypes.memmove(ptr, buf.ctypes.data, buf.nbytes)
        return buf.nbytes

    @staticmethod
    def decode_export(buf, n_images, n_pairs):
        from orbslam3lib_amd import decode_export
        return decode_export(buf, n_images, n_pairs)


def _frames_for(world, pairs, h, w):
    from orbslam3lib_amd import synth
    import numpy as np
    return np.stack([synth.frame(h, w, 300 + i) for i in range(world * 2 * pairs)])


def _ingest_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist

    from oracle import oracle_py as O
    from orbslam3lib_amd import dist as od
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    h, w, P = 120, 160, 1
    frames = _frames_for(world, P, h, w) if rank == 0 else None
    got = od.ingest_scatter_gather(dist, _HostBatch(h, w), frames, pairs_per_rank=P, src=0)
    ok = True
    if rank == 0:
        ok = len(got) == world
        for r, (images, pairs) in enumerate(got):
            for i, (k, d, m) in enumerate(images):
                rk, rd, rm = O.extract(frames[r * 2 * P + i], nfeatures=300, nlevels=4)
                ok &= m == rm and np.array_equal(k, rk) and np.array_equal(d, rd.reshape(-1, 32))
            for p, res in enumerate(pairs):
                ref = O.knn2(images[2 * p][1], images[2 * p + 1][1])
                ok &= all(np.array_equal(a, b) for a, b in zip(res, ref))
    else:
        ok = got is None
    dist.barrier()
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_gloo_ingest_scatter_gather_world2():
    """The C4 ingest-rank path (dist.ingest_scatter_gather): rank 0's frames scattered one stereo
    pair per rank, each rank's extraction + kNN2 results gathered back to rank 0 in the
    orbgpu_export_batch layout, decoded and equal to the oracle on the frames that rank got."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ingest_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


class _FailingHostBatch(_HostBatch):
    """_HostBatch whose extraction raises (a device error on that rank)."""

    def run_match(self, stereo_rows_only=False):
        raise RuntimeError("injected extraction failure")


def _ingest_fail_worker(rank, world, port, q):
    import torch.distributed as dist

    from orbslam3lib_amd import dist as od
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    h, w, P = 120, 160, 1
    frames = _frames_for(world, P, h, w) if rank == 0 else None
    be = _FailingHostBatch(h, w) if rank == 1 else _HostBatch(h, w)
    msg = None
    try:
        od.ingest_scatter_gather(dist, be, frames, pairs_per_rank=P, src=0)
    except RuntimeError as e:
        msg = str(e)
    dist.barrier()  # both ranks got here: nobody is left in the gather
    q.put((rank, msg))
    dist.destroy_process_group()


def test_gloo_ingest_rank_failure_world2():
    """a rank whose extraction raises between the scatter and the gather must not leave
    the others waiting in the gather.  ingest_scatter_gather agrees on a failure flag (max
    all_reduce) first: rank 1 raises its own error, rank 0 (src) raises "another rank failed", and
    both return to the caller."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ingest_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] == "injected extraction failure"
    assert res[0] is not None and "another rank failed" in res[0]


def test_export_layout_roundtrip_and_status_counts():
    """The packed orbgpu_export_batch layout (include/orbgpu.h): encode_export (the host
    restatement) -> decode_export returns the same rows; trailing padding (the gather pads every
    rank to the largest size) is ignored; a count holding a device status word (-5 octree
    overflow, -2 capacity) raises OrbGpuError with that code instead of returning stale rows."""
    import numpy as np

    import orbslam3lib_amd as og
    rng = np.random.default_rng(5)
    images = []
    for n in (7, 0, 12, 3):
        k = np.zeros(n, og.KEYPOINT_DTYPE)
        k["x"] = rng.random(n) * 600
        k["octave"] = rng.integers(0, 8, n)
        images.append((k, rng.integers(0, 256, (n, 32), dtype=np.uint8), n // 2))
    pairs = [tuple(rng.integers(-1, 300, 7, dtype=np.int32) for _ in range(4)),
             tuple(np.zeros(12, np.int32) for _ in range(4))]
    pairs[1] = tuple(rng.integers(-1, 300, 12, dtype=np.int32) for _ in range(4))
    buf = og.encode_export(images, pairs)
    assert buf.nbytes == 4 * (2 * 4 + 2) + 60 * 22 + 16 * 19
    for padded in (buf, np.concatenate([buf, np.full(100, 0xAB, np.uint8)])):
        got_i, got_p = og.decode_export(padded, 4, 2)
        for (k, d, m), (ek, ed, em) in zip(images, got_i):
            assert m == em
            np.testing.assert_array_equal(k.view(np.uint8), ek.view(np.uint8))
            np.testing.assert_array_equal(d, ed)
        for a, b in zip(pairs, got_p):
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
    for status in (-5, -2):
        bad = buf.copy()
        bad[4:8] = np.array([status], np.int32).view(np.uint8)  # image 1's count
        with pytest.raises(og.OrbGpuError) as ei:
            og.decode_export(bad, 4, 2)
        assert ei.value.code == status
    with pytest.raises(og.OrbGpuError):
        og.decode_export(buf[:-1], 4, 2)  # truncated
