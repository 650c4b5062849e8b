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
