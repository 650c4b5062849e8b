"""Multi-GPU plumbing for the batch path: one process per GPU (torch.distributed, RCCL on the
GPU box, gloo on CPU).  Stereo pairs are independent, so the hot path shards them with no
data-path collective; only the timing barrier and the max/sum reductions of bench.py cross
ranks ("replicas only").  The exchange steps of §8e: the cross-camera BFMatch of C5
(one camera per GPU, cross_camera_match / cross_camera_match_device) and, for frames ingested
on one GPU, the C4 scatter of frames and gather of results (ingest_scatter_gather)."""
from __future__ import annotations


def shard_range(total: int, rank: int, world: int):
    """Contiguous [lo, hi) slice of `total` units owned by `rank` (balanced to within 1)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def pair_seed_base(rank: int) -> int:
    """Synthetic frame index offset of a rank's shard (ranks never share frames)."""
    return rank * 100000


def cross_camera_match(dist, desc, matcher, device=None):
    """C5 cross-camera BFMatch: each rank holds one camera's descriptors (uint8
    [n, 32]); one exchange step -- an all_gather of the counts, then of the rows padded to the
    largest count (RCCL over xGMI on the GPU box, gloo on the CPU) -- after which every rank
    matches its own rows against every other camera's rows with matcher(query, train) ->
    (idx1, dist1, idx2, dist2).  Returns {rank: matcher result} for the other ranks."""
    import numpy as np
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = device or ("cuda" if dist.get_backend() == "nccl" else "cpu")
    desc = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
    n = torch.tensor([desc.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    buf = torch.zeros((max(max(counts), 1), 32), dtype=torch.uint8, device=dev)
    buf[:desc.shape[0]] = torch.from_numpy(desc).to(dev)
    rows = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(rows, buf)
    return {r: matcher(desc, rows[r][:counts[r]].cpu().numpy()) for r in range(world) if r != rank}


def cross_camera_match_device(dist, be, image=0, row0=0):
    """C5 cross-camera BFMatch with the descriptors kept on the GPUs: this rank's
    camera = batch image `image` of BatchExtractor `be` (rows [row0, n)).  The rows go from the
    extractor's HBM straight into a torch buffer (orbgpu_export_descriptors, device to device),
    one RCCL all_gather moves every camera's rows over xGMI, and every other camera is matched on
    this GPU from device memory (orbgpu_match_knn2_device) on torch's current stream.  Only the
    per-camera row counts (one int each) pass through the host.  Returns {rank: int32 device
    tensor [4, n] (idx1, dist1, idx2, dist2)} for the other ranks.

    Under gloo (the ranks share fewer GPUs than there are ranks, e.g. the one-GPU rehearsal) the
    export and the matcher still run on device buffers; only the all_gather is staged through
    host tensors.  An extractor that is not device-resident (the CPU tests' stand-in) gets host
    buffers throughout; liborbgpu refuses host pointers in its device entry points."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    nccl = dist.get_backend() == "nccl"
    on_device = nccl or (bool(getattr(be, "device_resident", False)) and torch.cuda.is_available())
    if on_device:
        dev = torch.device("cuda", torch.cuda.current_device())
        stream = torch.cuda.current_stream().cuda_stream
    else:  # host stand-in (tests): `be` works on host addresses
        dev, stream = torch.device("cpu"), None
    comm = dev if nccl else torch.device("cpu")  # where the collectives' tensors live
    nk, _ = be.counts()
    n_local = max(int(nk[image]) - int(row0), 0)
    n = torch.tensor([n_local], dtype=torch.int64, device=comm)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    maxn = max(max(counts), 1)
    buf = torch.zeros((maxn, 32), dtype=torch.uint8, device=dev)
    be.export_descriptors(image, buf.data_ptr(), maxn, row0, stream)
    if comm == dev:
        rows = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(rows, buf)
    else:  # gloo between device buffers: host staging around the collective only
        if dev.type == "cuda":
            torch.cuda.current_stream().synchronize()
        hb = buf.cpu()
        hrows = [torch.empty_like(hb) for _ in range(world)]
        dist.all_gather(hrows, hb)
        rows = [h.to(dev) for h in hrows]
    out = {}
    for r in range(world):
        if r == rank:
            continue
        res = torch.empty((4, max(n_local, 1)), dtype=torch.int32, device=dev)
        be.match_knn2_device(buf.data_ptr(), n_local, rows[r].data_ptr(), counts[r], res.data_ptr(), stream)
        out[r] = res[:, :n_local]
    return out


def ingest_scatter_gather(dist, be, frames=None, pairs_per_rank=1, src=0, stereo_rows_only=False, stats=None):
    """The C4 ingest-rank path ("if frames are ingested on one GPU"): rank `src` holds
    the frames of every rank's stereo pairs, uint8 [world * 2P, H, W] (pair p = images 2p, 2p + 1;
    rank r owns pairs [rP, (r + 1)P)).  One scatter hands each rank its 2P images, each rank runs
    extraction + stereo kNN2 on its own GPU (BatchExtractor `be`: ingest_images -> run_match), and
    one gather brings every rank's results back to `src` -- the reference hands each frame's
    keypoints, descriptors and matches back to its one caller
    (cpp/src/LynxHardwareAcceleration/LynxHardwareAccelerator.cpp:146-204).
    Only the rows produced travel: each rank packs its batch with orbgpu_export_batch (counts,
    then the keypoints, descriptors and match rows it made), the ranks agree on the largest packed
    size and on whether every rank got that far (one max all_reduce of [failed, bytes]), and the
    gather moves that many bytes per rank.  A rank whose ingest / extraction / export raised makes
    every rank skip the gather and raise, so no rank is left waiting in it.  Under RCCL the frames
    and results move device to device over xGMI; under gloo the collectives are staged through host
    tensors (the extractor still ingests from / exports to device memory when it is
    device-resident).  Returns, on `src`, one (images, pairs) per rank as decode_export gives them;
    None on the other ranks.  `stats` (a dict, optional) receives the bytes each rank sent
    (`gathered_bytes_per_rank`) and what the capacity layout would have sent
    (`capacity_bytes_per_rank`)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    nccl = dist.get_backend() == "nccl"
    on_device = nccl or (bool(getattr(be, "device_resident", False)) and torch.cuda.is_available())
    dev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
    comm = dev if nccl else torch.device("cpu")
    stream = torch.cuda.current_stream().cuda_stream if on_device else None
    n_img, h, w = 2 * pairs_per_rank, be.height, be.width
    recv = torch.empty((n_img, h, w), dtype=torch.uint8, device=comm)
    parts = None
    if rank == src:
        ft = torch.as_tensor(frames).reshape(world * n_img, h, w).to(comm)
        parts = list(ft.chunk(world))
    dist.scatter(recv, parts, src=src)
    err, local, used = None, None, 0
    try:
        img = recv if recv.device == dev else recv.to(dev)
        be.ingest_images(img.data_ptr(), n_img, w, stream)
        be.run_match(stereo_rows_only=stereo_rows_only)
        used = be.export_batch_size(n_img, pairs_per_rank, stream)
        local = torch.empty(max(used, 4), dtype=torch.uint8, device=dev)
        used = be.export_batch(local.data_ptr(), n_img, pairs_per_rank, local.numel(), stream)
    except Exception as e:  # noqa: BLE001 -- agreed on below, then re-raised
        err = e
    flag = torch.tensor([1 if err is not None else 0, used], dtype=torch.int64, device=comm)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag[0]) != 0:
        if err is not None:
            raise err
        raise RuntimeError("ingest_scatter_gather: another rank failed before the gather")
    nbytes = max(int(flag[1]), 4)
    if stats is not None:
        stats["gathered_bytes_per_rank"] = nbytes
        cap = getattr(be, "export_batch_bytes", None)
        stats["capacity_bytes_per_rank"] = int(cap(n_img, pairs_per_rank)) if cap else None
    out = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    out[:local.numel()] = local
    if out.device != comm:
        if out.device.type == "cuda":
            torch.cuda.current_stream().synchronize()
        out = out.to(comm)
    bufs = [torch.empty_like(out) for _ in range(world)] if rank == src else None
    dist.gather(out, bufs, dst=src)
    if rank != src:
        return None
    return [be.decode_export(b.cpu().numpy(), n_img, pairs_per_rank) for b in bufs]


def reduce_scalar(dist, x: float, op: str = "max") -> float:
    if dist is None:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())
