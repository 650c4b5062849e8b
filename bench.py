#!/usr/bin/env python3
"""bench.py -- Mfeatures/s (ORB extract) + Mmatches/s (Hamming kNN2) on MI355X.

Workload (BASELINE.json configs[1], C2): 640x480 stereo pairs, 8-level pyramid (scale 1.2),
2000 features per frame, FAST 20/7; each pair's left descriptors are matched against all its
right descriptors (2000 x 2000 kNN2, the C3 matcher step).  A "step" = one pass of the hot path
over a device-resident batch of `--pairs` stereo pairs per GPU (inputs already in HBM).

Multi-GPU: one process per GPU; every rank extracts its own shard of pairs (frames are
independent -> weak scaling, no data-path collective); barrier + max over ranks bracket the timed
region.  Launched either by torch.distributed.run (RANK / WORLD_SIZE in the environment) or as
`python bench.py --gpus N`, which starts the N ranks itself (spawn_ranks) before this process
touches torch or the GPU.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 256 CU x 4 SIMD32 x 32 lanes x 2.4 GHz, int32 ops
# dense int8 MFMA: 2x the BF16 rate per clock (MI355X_MICROARCH.md, matrix-core table: I8 32x32x32
# takes the cycles of BF16 32x32x16), BF16 dense ~2.5 PF -> ~5.0 POPS
MFMA_I8_PEAK_TOPS = 5000.0
# dense block-scaled FP4 MFMA (the unit k_knn2 runs on since round 6): 4x the BF16 rate per clock
# (32x32x64 takes the cycles of BF16 32x32x16), ~10 PF dense
MFMA_FP4_PEAK_TOPS = 10000.0


def level_sizes(w, h, sf=1.2, L=8):
    """ComputePyramid sizes (ORBextractor_old.cc:1336) with the float math of the ctor."""
    scale = [np.float32(1.0)]
    for _ in range(1, L):
        scale.append(np.float32(np.float64(scale[-1]) * np.float64(np.float32(sf))))
    out = []
    for s in scale:
        inv = np.float32(1.0) / s
        out.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return out


def fast_tiers(w, h, sf=1.2, L=8):
    """FAST LDS tile per level (orb_runtime.cpp rule: the smallest of 48 / 64 / 80 bytes with
    wCell + 9 <= tile and hCell + 6 <= tile, chosen per level)."""
    out = []
    for lw, lh in level_sizes(w, h, sf, L):
        W, H = np.float32(lw - 32), np.float32(lh - 32)
        nc, nr = int(W / np.float32(35)), int(H / np.float32(35))
        wc, hc = int(np.ceil(W / np.float32(nc))), int(np.ceil(H / np.float32(nr)))
        out.append(next((t for t in (48, 64) if wc + 9 <= t and hc + 6 <= t), 80))
    return out


def algorithmic_bytes(w, h, L, nkp, sf=1.2, ncand=0.0, tail0=None):
    """Per-image bytes by stage: pyramid sum(A_{l-1}+A_l), FAST sum(A_l) (split
    between the 48-, 64- and 80-byte tile launches), blur 2*sum(A_l), 48 B per output keypoint
    (16 B keypoint + 32 B descriptor) for orientation + descriptor; the octree reads its 4-byte
    candidate keys and writes 4 bytes per kept keypoint; the assembly reads the level keypoint
    (key, angle, descriptor: 40 B) and writes the cv::KeyPoint and the descriptor (60 B).
    tail0: first level k_pyr_tail makes (it reads level tail0 - 1 once and writes the blurs of
    levels tail0 - 1 .. L-1 and levels tail0 .. L-1); None: k_blur_resize for every level and
    k_blur for the last level's blur."""
    A = [a * b for a, b in level_sizes(w, h, sf, L)]
    tier = fast_tiers(w, h, sf, L)
    t = tail0 if tail0 is not None else L + 1
    last_br = t if t <= L else L
    return {
        # one pass over level l-1 per launch: read it, write its blur and level l
        "k_blur_resize": sum(2 * A[l - 1] + A[l] for l in range(1, last_br)),
        "k_pyr_tail": (A[t - 1] + sum(A[t - 1:]) + sum(A[t:])) if t <= L else 0,
        "k_fast_cells<48>": sum(a for a, t in zip(A, tier) if t == 48),
        "k_fast_cells<64>": sum(a for a, t in zip(A, tier) if t == 64),
        "k_fast_cells<80>": sum(a for a, t in zip(A, tier) if t == 80),
        "k_blur": 2 * A[L - 1] if t > L else 0,  # the last level's blur (the others ride in k_blur_resize)
        "k_orient_desc": 48 * nkp,
        "k_octree": 4 * ncand + 4 * nkp,
        "k_finalize": 100 * nkp,
    }


def fast_pyramid_bytes(w, h, L, sf=1.2):
    """B_fp per image: pyramid sum_{l>=1}(A_{l-1}+A_l) + FAST sum_l A_l."""
    A = [a * b for a, b in level_sizes(w, h, sf, L)]
    return sum(A[l - 1] + A[l] for l in range(1, L)) + sum(A)


def pmc_valu_table(root):
    """Per-kernel VALU issue from the latest committed PMC summary (profiles/r*/pmc_summary.txt,
    written by tools/refresh_profiles.sh from separate rocprofv3 --pmc passes of the same
    whole-batch launches): instructions per launch and the fraction of SIMD cycles the VALU was
    issuing, SQ_ACTIVE_INST_VALU quad-cycles x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).
    Keys are the bench's stage names (k_fast_cells<48>, k_knn2, k_octree, ...)."""
    import re
    paths = sorted(glob.glob(os.path.join(root, "profiles", "r*", "pmc_summary.txt")))
    if not paths:
        return {}, None
    out = {}
    try:
        txt = open(paths[-1]).read()
    except OSError:
        return {}, None
    # the counters describe one binary; use them only for the library loaded now
    import hashlib
    m = re.search(r"^# liborbgpu.so sha256 ([0-9a-f]{64})", txt, re.M)
    lib = os.environ.get("ORBGPU_LIB") or os.path.join(root, "orbslam3lib_amd", "liborbgpu.so")
    try:
        cur = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    except OSError:
        cur = None
    if not m or m.group(1) != cur:
        return {}, "%s (stale: recorded for %s, loaded %s)" % (
            os.path.relpath(paths[-1], root), m.group(1)[:12] if m else "no library hash", (cur or "?")[:12])
    acc = {}
    for block in re.split(r"\n(?=\S)", txt):
        lines = block.strip().split("\n")
        name = lines[0].replace("void ", "").replace("orbgpu::", "").strip()
        c = {}
        for ln in lines[1:]:
            m = re.match(r"\s+(\w+)\s+([-\d.e+]+)$", ln)
            if m:
                c[m.group(1)] = float(m.group(2))
        if "SQ_ACTIVE_INST_VALU" not in c or not c.get("GRBM_GUI_ACTIVE"):
            continue
        stage = name
        for pre, st in (("k_knn2", "k_knn2"), ("k_octree", "k_octree"), ("k_finalize", "k_finalize")):
            if name.startswith(pre):
                stage = st
        # the small-list FAST kernel and its overflow pass make one stage (k_fast_cells<48>)
        stage = re.sub(r"^k_fast_cells(?:_ovf)?<(\d+)(?:, (?:true|false))?>$", r"k_fast_cells<\1>", stage)
        tot = acc.setdefault(stage, {})
        for k, v in c.items():
            tot[k] = tot.get(k, 0.0) + v
    for stage, c in acc.items():
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        out[stage] = {"valu_busy": round(c["SQ_ACTIVE_INST_VALU"] * 4.0 / 1024.0 / cyc, 3),
                      "valu_instr_per_launch": c.get("SQ_INSTS_VALU")}
    return out, os.path.relpath(paths[-1], root)


def spawn_ranks(n):
    """`bench.py --gpus N` with no launcher: start N ranks of this script (rank r on GPU r,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in each child's environment, the
    rendezvous on 127.0.0.1).  This process never imports torch or liborbgpu: the children are
    started before anything touches the GPU.  Rank 0 prints the JSON line (its stdout is this
    process's); a rank that fails ends the others (their rendezvous would wait for it).  Returns
    the worst exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    codes = [None] * n
    while any(c is None for c in codes):
        for r, p in enumerate(procs):
            if codes[r] is None:
                codes[r] = p.poll()
        if any(c not in (None, 0) for c in codes):
            for r, p in enumerate(procs):
                if codes[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                if codes[r] is None:
                    try:
                        codes[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[r] = p.wait()
            break
        time.sleep(0.2)
    bad = [c for c in codes if c]
    return max(bad, key=abs) if bad else 0


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        # device_count() does not initialise the GPU (torch reads it from the driver); RCCL needs
        # one device per rank, so fewer devices than ranks (the one-GPU rehearsal) run gloo with
        # the ranks sharing the devices; ORBGPU_BENCH_BACKEND / ORBGPU_BENCH_DEVICE override
        ndev = torch.cuda.device_count()
        backend = os.environ.get("ORBGPU_BENCH_BACKEND") or ("nccl" if ndev >= world else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        else:
            local = int(os.environ.get("ORBGPU_BENCH_DEVICE", local % max(ndev, 1)))
        # the process group's own connection messages (gloo prints to stdout) go to stderr:
        # rank 0's stdout carries exactly one line, the JSON result
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            td.init_process_group(backend=backend)
            td.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        dist = td
    return world, rank, local, dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x):
    if dist is None:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


EUROC_K = (458.654, 457.296, 367.215, 248.375)  # EuRoC cam0 fx fy cx cy
EUROC_D = (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)


def cpu_baseline(w, h, nfeatures, seconds, map_points=3000):
    """The oracle (scalar C++ restatement of the reference CPU ORBextractor + BFMatcher), one
    thread, on a bounded sample of the same workload: pairs until `seconds` elapse."""
    from oracle import oracle_py as O
    from orbslam3lib_amd import synth
    native = O.use_native()  # -O3 -march=native -ffp-contract=off, built on this host
    O.lib()
    pairs = [synth.stereo_pair(h, w, 1000 + i) for i in range(4)]
    stereo_pyr = [(O.pyramid(L), O.pyramid(R)) for L, R in pairs]
    t_st = [0.0]
    t_gr = t_sbp = 0.0
    pair_times = []
    maps = []
    n_mp = 0
    nfeat = nq = 0
    t_ex = t_bf = 0.0
    i = 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or i == 0:
        L, R = pairs[i % len(pairs)]
        t0 = time.perf_counter()
        kl, dl, _ = O.extract(L, nfeatures=nfeatures, lap=(0, 0))
        kr, dr, _ = O.extract(R, nfeatures=nfeatures, lap=(0, 0))
        t1 = time.perf_counter()
        if i >= 3:  # after 3 warm-up pairs
            pair_times.append(t1 - t0)
        O.knn2(dl, dr)
        t2 = time.perf_counter()
        if stereo_pyr is not None:
            O.stereo_matches(kl, dl, kr, dr, stereo_pyr[i % len(pairs)][0], stereo_pyr[i % len(pairs)][1],
                             47.9, float(np.float32(47.9) / np.float32(435.2)))
            t_st[0] += time.perf_counter() - t2
        t3 = time.perf_counter()
        xy, b, _, cs, ci = O.undistort_grid(kl, EUROC_K, EUROC_D, w, h)
        O.undistort_grid(kr, EUROC_K, EUROC_D, w, h)
        t4 = time.perf_counter()
        t_gr += t4 - t3
        if i < len(pairs):  # synthetic maps are generated once per distinct pair
            maps.append(synth.map_points(xy, kl["octave"], dl, None, n=map_points, seed=7 + i))
        t4 = time.perf_counter()
        O.search_by_projection(maps[i % len(pairs)], xy, kl["octave"], dl, None, b, cs, ci)
        t_sbp += time.perf_counter() - t4
        n_mp += map_points
        nfeat += len(kl) + len(kr)
        nq += len(dl)
        t_ex += t1 - t0
        t_bf += t2 - t1
        i += 1
    # SURVEY §8d modes 2 and 3, inside the oracle (std::thread, no Python in the loop): both eyes of
    # a pair on two threads (Frame.cc:142-145), and a frames-parallel pool over every core this
    # process may run on (and over 16, the box's CPU share per GPU, as a second figure)
    def pool_rate(nthreads, nimg, secs):
        batch = np.stack([pairs[(k // 2) % len(pairs)][k % 2] for k in range(nimg)])
        nf_, t0, reps = 0, time.perf_counter(), 0
        while time.perf_counter() - t0 < secs or reps == 0:
            nf_ += O.extract_many(batch, nthreads, nfeatures)
            reps += 1
        return nf_ / (time.perf_counter() - t0) / 1e6
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    # the cores this process can actually use: its affinity mask, capped by its cgroup CPU quota
    # (the GPU box gives each GPU's job 16 CPUs of a 256-thread host: 256 threads there run at
    # the speed of 16, and slower than 16 threads)
    cores = avail if quota is None else max(1, min(avail, int(quota)))
    mode2 = pool_rate(2, 2, max(2.0, seconds / 6))
    mode3 = pool_rate(cores, max(4 * cores, 32), max(3.0, seconds / 3))
    mode3_all = pool_rate(avail, 4 * avail, 2.0) if avail != cores else mode3
    return {"pairs": i, "mfeat_s": nfeat / t_ex / 1e6, "mmatch_s": nq / t_bf / 1e6,
            "mfeat_s_2threads_per_pair": mode2, "mfeat_s_pool": mode3, "pool_threads": cores,
            "affinity": avail, "mfeat_s_pool_affinity": mode3_all, "cgroup_cpu_quota": quota,
            "native": native is not None,
            "median_pair_ms": 1e3 * float(np.median(pair_times)) if pair_times else None,
            "stereo_mkp_s": nq / t_st[0] / 1e6 if t_st[0] > 0 else None,
            "grid_mkp_s": nfeat / t_gr / 1e6 if t_gr > 0 else None,
            "sbp_mmp_s": n_mp / t_sbp / 1e6 if t_sbp > 0 else None,
            "mfeat_s_pipeline": nfeat / (t_ex + t_bf) / 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=256, help="stereo pairs per GPU per step")
    ap.add_argument("--unique-pairs", type=int, default=16,
                    help="distinct synthetic pairs generated per rank (tiled to --pairs)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--nlevels", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stereo", action="store_true", help="skip the ComputeStereoMatches leg")
    ap.add_argument("--no-grid", action="store_true", help="skip the UndistortKeyPoints + grid leg")
    ap.add_argument("--no-wire", action="store_true", help="skip the side-by-side ingest / SoA egress leg")
    ap.add_argument("--no-sbp", action="store_true", help="skip the SearchByProjection leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the C3 / C5 side lines")
    ap.add_argument("--map-points", type=int, default=3000, help="local-map points per frame (SBP leg)")
    ap.add_argument("--no-profile", action="store_true",
                    help="do not bracket launches with HIP events in the timed region")
    ap.add_argument("--stub-gpu", action="store_true",
                    help="CPU test of the launch / rendezvous / reduction path only: a host stand-in "
                         "(tests/bench_stub.py) replaces liborbgpu; the line says data: stub")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)
    world, rank, local, dist = dist_setup()
    if args.gpus != world and rank == 0:
        print("bench: --gpus %d but %d rank(s) launched; reporting the launched ranks" % (args.gpus, world),
              file=sys.stderr)
    # torch before liborbgpu: both then share one HIP runtime (torch bundles its own with the
    # same soname), so torch.cuda.synchronize() below brackets the same device queues
    try:
        import torch
        has_cuda = torch.cuda.is_available() and not args.stub_gpu
    except Exception:
        torch, has_cuda = None, False
    if args.stub_gpu:
        from tests import bench_stub as og
    else:
        import orbslam3lib_amd as og
    from orbslam3lib_amd import synth
    # where every rank runs (rank, device, host pid): the line shows that all ranks joined
    placement = [(rank, local, os.getpid())]
    if dist is not None:
        allp = [None] * world
        dist.all_gather_object(allp, placement[0])
        placement = allp

    P, W, H = args.pairs, args.width, args.height
    U = max(1, min(args.unique_pairs, P))
    from orbslam3lib_amd.dist import pair_seed_base
    base = pair_seed_base(rank)  # each rank extracts its own shard of the stream (weak scaling)
    uniq = [synth.stereo_pair(H, W, base + i) for i in range(U)]
    imgs = np.empty((2 * P, H, W), np.uint8)
    for p in range(P):
        imgs[2 * p], imgs[2 * p + 1] = uniq[p % U]

    be = og.BatchExtractor(args.nfeatures, 1.2, args.nlevels, 20, 7, device=local, width=W,
                           height=H, max_images=2 * P)
    be.upload(imgs)  # PCIe upload: outside the timed region (inputs resident in HBM)
    be.synchronize()
    h0 = time.perf_counter()  # the same upload timed alone, for the H2D-inclusive rate
    be.upload(imgs)
    be.synchronize()
    h2d_s = time.perf_counter() - h0
    laps = np.zeros((2 * P, 2), np.int32)

    def step():
        be.run(laps)
        be.match_stereo(stereo_rows_only=False)

    for _ in range(args.warmup):
        step()
    be.synchronize()
    nk, _ = be.counts()
    cand_per_img = float(be.candidate_counts().mean())
    feats_per_step = int(nk.sum())
    nq_per_step = int(sum(nk[2 * p] for p in range(P)))
    pairs_per_step = int(sum(int(nk[2 * p]) * int(nk[2 * p + 1]) for p in range(P)))

    # 1. short untimed pass, every stage one whole-batch launch bracketed by HIP events -> per-stage
    #    table and the dominant kernel; 2. the timed region (production sub-batch streams, one
    #    launch per stream and stage) brackets only that kernel's launches, so event cost stays
    #    small; their durations include whatever the other streams run beside them
    be.set_profiling(True, serialize=True)
    be.reset_stage_times()
    for _ in range(3):
        step()
    be.synchronize()
    stages_all = be.stage_times()
    dom_name = max(stages_all, key=lambda k: stages_all[k][0]) if stages_all else None
    if args.no_profile or dom_name is None:
        be.set_profiling(False)
    else:
        be.set_profiling(True, stages=[dom_name])
    be.reset_stage_times()
    barrier(dist)
    be.synchronize()
    if has_cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    be.synchronize()
    if has_cuda:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(dist)
    elapsed = max_over_ranks(dist, t1 - t0)
    stages_timed = be.stage_times()
    be.set_profiling(False)

    # streaming ingest (C3's shape: every batch arrives from the host): each step's 2P frames are
    # copied from pinned host memory on the copy stream while the previous step computes
    # (orbgpu_upload_images_async); K uploads + K steps in the timed loop, the first upload exposed
    pin = be.pinned(imgs.shape)
    pin[:] = imgs
    for _ in range(2):  # warm-up: creates the copy stream, touches both input buffers
        be.upload_async(pin)
        step()
    be.synchronize()
    barrier(dist)
    p0 = time.perf_counter()
    be.upload_async(pin)
    for k in range(args.steps):
        step()
        if k + 1 < args.steps:
            be.upload_async(pin)
    be.synchronize()
    p_el = max_over_ranks(dist, time.perf_counter() - p0)
    be.free_pinned()

    total_feats = sum_over_ranks(dist, feats_per_step * args.steps)
    total_q = sum_over_ranks(dist, nq_per_step * args.steps)
    total_pairs = sum_over_ranks(dist, pairs_per_step * args.steps)
    mfeat = total_feats / elapsed / 1e6
    # the PCIe-inclusive rate beside the resident one (never `value`)
    h2d_max = max_over_ranks(dist, h2d_s)
    h2d_serial = sum_over_ranks(dist, feats_per_step) / (elapsed / args.steps + h2d_max) / 1e6
    h2d_incl = total_feats / p_el / 1e6
    mmatch = total_q / elapsed / 1e6

    # per-stage table from the serialized pass: each stage one whole-batch launch per step (one per
    # level for k_blur_resize), alone on the GPU, so its duration is the kernel's own and the
    # rocprofv3 trace of the same command reproduces it (tools/roofline_check.py).  Bytes are
    # SURVEY §8d's algorithmic bytes per launch; `traffic` is the counter-measured HBM bytes per
    # launch of the same whole-batch launch (profiles/traffic_r*.json, per image and step there)
    n_img = 2 * P
    nser = 3
    # k_pyr_tail's first level from the serialized pass: k_blur_resize runs once per level below it
    tail0 = None
    if "k_pyr_tail" in stages_all and "k_blur_resize" in stages_all:
        tail0 = int(round(stages_all["k_blur_resize"][1] / nser)) + 1
    per_img = algorithmic_bytes(W, H, args.nlevels, feats_per_step / n_img, ncand=cand_per_img, tail0=tail0)
    traffic_tab, traffic_src = {}, None
    tps = sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json")))
    if tps:
        try:
            tt = json.load(open(tps[-1]))
            if tt.get("_config", {}).get("width") == W and tt.get("_config", {}).get("height") == H:
                traffic_tab = {k: v for k, v in tt.items() if isinstance(v, dict) and "hbm_bytes_per_image_step" in v}
                traffic_src = os.path.relpath(tps[-1], ROOT)
        except Exception:
            traffic_tab = {}
    stage_rows = {}
    for name, (ms, cnt) in stages_all.items():
        if cnt == 0:
            continue
        avg_ms = ms / cnt
        launches_per_step = cnt / nser
        row = {"avg_us": round(avg_ms * 1e3, 2), "launches": cnt, "total_ms": round(ms, 3),
               "us_per_step": round(ms / nser * 1e3, 1), "source": "serialized pass (kernel alone)"}
        if name in per_img:
            bytes_launch = per_img[name] * n_img / launches_per_step
            row["bytes_per_launch"] = int(bytes_launch)
            row["GBps"] = round(bytes_launch / (avg_ms * 1e-3) / 1e9, 1)
            row["frac_hbm"] = round(row["GBps"] / HBM_PEAK_GBS, 4)
            if name in traffic_tab:
                tb = traffic_tab[name]["hbm_bytes_per_image_step"] * n_img / launches_per_step
                row["traffic_per_launch"] = int(tb)
                row["traffic_over_algorithmic"] = round(tb / bytes_launch, 2) if bytes_launch else None
        if name == "k_knn2":
            # the kernel runs on the block-scaled FP4 matrix cores: 2 x 256 ops per
            # (query, train) pair (one MAC per descriptor bit) are what it issues.  Priced against the
            # dense FP4 peak; the fraction of the i8 peak (the unit of rounds 2-5) and the 16-op VALU
            # popcount figure sit beside it
            pairs_launch = pairs_per_step / launches_per_step
            row["Tops_mfma"] = round(512.0 * pairs_launch / (avg_ms * 1e-3) / 1e12, 1)
            row["frac_mfma_fp4"] = round(row["Tops_mfma"] / MFMA_FP4_PEAK_TOPS, 4)
            row["frac_of_i8_peak"] = round(row["Tops_mfma"] / MFMA_I8_PEAK_TOPS, 4)
            row["Tops"] = round(16.0 * pairs_launch / (avg_ms * 1e-3) / 1e12, 2)
            row["frac_valu"] = round(row["Tops"] / VALU_PEAK_TOPS, 4)
        stage_rows[name] = row
    # the dominant kernel: the largest serialized total; its timed-region (concurrent) launches
    # were bracketed with HIP events on their own streams and sit beside the kernel-alone figure
    dom = dom_name if dom_name in stage_rows else None
    if dom is not None and stages_timed.get(dom, (0, 0))[1] > 0 and "bytes_per_launch" in stage_rows[dom]:
        tms, tcnt = stages_timed[dom]
        tb = per_img[dom] * n_img / (tcnt / args.steps)
        stage_rows[dom]["concurrent"] = {
            "source": "timed region, HIP events on the chunk streams (other chunks' stages run beside it)",
            "avg_us": round(tms / tcnt * 1e3, 2), "launches": tcnt, "bytes_per_launch": int(tb),
            "GBps": round(tb / (tms / tcnt * 1e-3) / 1e9, 1),
            "frac_hbm": round(tb / (tms / tcnt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    roof = None
    if dom is not None:
        r = stage_rows[dom]
        if "GBps" in r:
            roof = {"kernel": dom, "bound": "hbm", "achieved": r["GBps"], "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": r["frac_hbm"], "traffic": r.get("traffic_per_launch"),
                    "traffic_over_algorithmic": r.get("traffic_over_algorithmic"), "traffic_source": traffic_src,
                    "bytes_per_launch": r["bytes_per_launch"], "avg_us": r["avg_us"],
                    "launch": "whole batch (%d images), serialized pass, kernel alone" % n_img,
                    "launches": r["launches"], "concurrent": r.get("concurrent")}
        elif "Tops_mfma" in r:
            roof = {"kernel": dom, "bound": "mfma_fp4", "achieved": r["Tops_mfma"], "peak": MFMA_FP4_PEAK_TOPS,
                    "unit": "Tops/s", "frac": r["frac_mfma_fp4"], "traffic": r.get("traffic_per_launch"),
                    "avg_us": r["avg_us"]}
        else:
            roof = {"kernel": dom, "bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": None, "traffic": r.get("traffic_per_launch"), "avg_us": r["avg_us"]}
        if dom == "k_octree":
            roof["note"] = ("DistributeOctTree is barrier/LDS-latency bound (serial list rounds per "
                            "(image, level)); its HBM bytes are the 4-B keys in and out")

    # the north_star's named pair, FAST + pyramid, as one figure over the summed per-step time of
    # the serialized pass.  The pyramid kernel also writes each level's blur (k_blur_resize reads
    # level l-1 once for both), so its time carries the blur: the bytes are SURVEY §8d's B_fp plus
    # the blur's 2 sum(A_l) (B_extract without the 48 B per keypoint)
    fp_names = [k for k in stages_all if k in ("k_blur_resize", "k_blur", "k_pyr_tail")
                or k.startswith("k_fast_cells")]
    fp_ms = sum(stages_all[k][0] for k in fp_names) / 3.0  # 3 serialized steps
    roof_fp = None
    if fp_ms > 0:
        A_ = [a_ * b_ for a_, b_ in level_sizes(W, H, 1.2, args.nlevels)]
        fp_bytes = (fast_pyramid_bytes(W, H, args.nlevels) + 2 * sum(A_)) * n_img
        ach = fp_bytes / (fp_ms * 1e-3) / 1e9
        roof_fp = {"kernels": fp_names, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_step": int(fp_bytes),
                   "includes": "pyramid + blur (fused) + FAST; bytes = B_fp + 2 sum(A_l)",
                   "us_per_step": round(fp_ms * 1e3, 1)}

    # the bound that applies to the dominant kernel: VALU issue.  The busy
    # fraction comes from the committed PMC passes; the instruction rate uses this run's time
    roof_valu = None
    try:
        vt, vsrc = pmc_valu_table(ROOT)
    except Exception:
        vt, vsrc = {}, None
    if dom is not None and not vt and vsrc:
        roof_valu = {"kernel": dom, "bound": "valu", "stale": True, "source": vsrc}
    if dom is not None and dom in vt:
        v = vt[dom]
        roof_valu = {"kernel": dom, "bound": "valu", "busy": v["valu_busy"],
                     "valu_instr_per_launch": v["valu_instr_per_launch"],
                     "achieved_wave_instr_per_us": (round(v["valu_instr_per_launch"] / stage_rows[dom]["avg_us"], 1)
                                                    if v["valu_instr_per_launch"] else None),
                     "source": vsrc, "busy_by_kernel": {k: x["valu_busy"] for k, x in sorted(vt.items())},
                     "definition": "SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), "
                                   "whole-batch launches, kernel alone"}

    # the matcher's own roofline (north_star: "Hamming BFMatch"): it runs on the FP4 matrix cores
    kr = stage_rows.get("k_knn2")
    roof_knn = None
    if kr and "Tops_mfma" in kr:
        roof_knn = {"kernel": "k_knn2", "bound": "mfma_fp4", "achieved": kr["Tops_mfma"], "peak": MFMA_FP4_PEAK_TOPS,
                    "unit": "Tops/s", "frac": kr["frac_mfma_fp4"], "avg_us": kr["avg_us"],
                    "ops_per_pair": 512, "frac_of_i8_peak": kr["frac_of_i8_peak"], "i8_peak": MFMA_I8_PEAK_TOPS,
                    "valu_equivalent_Tops": kr["Tops"], "frac_valu_int32": kr["frac_valu"]}

    # Frame::ComputeStereoMatches on the same resident batch, timed on its own
    # (not part of the headline step): EuRoC-like rig, baseline 0.11 m, fx 435.2
    stereo = None
    if not args.no_stereo:
        mbf = 47.9
        mb = float(np.float32(mbf) / np.float32(435.2))
        be.stereo_matches(mbf, mb)
        be.synchronize()
        be.set_profiling(True, stages=["k_stereo"])
        be.reset_stage_times()
        barrier(dist)
        be.synchronize()
        s0 = time.perf_counter()
        for _ in range(args.steps):
            be.stereo_matches(mbf, mb)
        be.synchronize()
        s1 = time.perf_counter()
        st_el = max_over_ranks(dist, s1 - s0)
        st = be.stage_times().get("k_stereo", (0.0, 0))
        be.set_profiling(False)
        ur, _, _ = be.stereo_result(0)
        stereo = {"metric": "left keypoints stereo-matched per second (Frame::ComputeStereoMatches)",
                  "value": round(sum_over_ranks(dist, nq_per_step * args.steps) / st_el / 1e6, 3),
                  "unit": "Mkeypoints/s", "ms_per_step": round(st_el / args.steps * 1e3, 4),
                  "kernel_ms_per_launch": round(st[0] / st[1], 4) if st[1] else None,
                  "pairs_per_step": P, "matched_frac_pair0": round(float((ur >= 0).mean()), 3) if len(ur) else 0.0}

    # Frame::UndistortKeyPoints + AssignFeaturesToGrid over every image of the
    # resident batch, timed on its own: EuRoC cam0 calibration (k1 k2 p1 p2)
    grid = None
    if not args.no_grid:
        be.undistort_grid(EUROC_K, EUROC_D)
        be.synchronize()
        be.set_profiling(True, stages=["k_undistort_grid"])
        be.reset_stage_times()
        barrier(dist)
        be.synchronize()
        g0 = time.perf_counter()
        for _ in range(args.steps):
            be.undistort_grid(EUROC_K, EUROC_D)
        be.synchronize()
        g1 = time.perf_counter()
        g_el = max_over_ranks(dist, g1 - g0)
        gt = be.stage_times().get("k_undistort_grid", (0.0, 0))
        be.set_profiling(False)
        grid = {"metric": "keypoints undistorted + gridded per second (Frame::UndistortKeyPoints + "
                          "AssignFeaturesToGrid)",
                "value": round(sum_over_ranks(dist, feats_per_step * args.steps) / g_el / 1e6, 3),
                "unit": "Mkeypoints/s", "ms_per_step": round(g_el / args.steps * 1e3, 4),
                "kernel_ms_per_launch": round(gt[0] / gt[1], 4) if gt[1] else None,
                "images_per_step": 2 * P}

    # ORBmatcher::SearchByProjection on every pair's left frame: a synthetic
    # local map of --map-points points per frame (projections near the frame's keypoints, several
    # per keypoint), mvuRight from the stereo leg.  Kernel time from the stage timer; the call
    # time includes uploading the map points (PCIe, they come from the host each frame).
    sbp = None
    if not args.no_sbp and grid is not None:
        uniq_mps = []
        for u in range(U):
            kl_u, dl_u, _ = be.result(2 * u)
            xy_u, _, _, _ = be.grid_result(2 * u)
            ur_u = be.stereo_result(u)[0] if stereo is not None else None
            uniq_mps.append(synth.map_points(xy_u, kl_u["octave"], dl_u, ur_u, n=args.map_points, seed=7 + u))
        mp_list = [uniq_mps[p % U] for p in range(P)]
        # the timed calls pass the points in the ABI's form (one array + offsets, as a caller that
        # keeps its local map packed would); the list form adds a host concatenation per call
        mp_rows = (np.concatenate(mp_list), np.concatenate([[0], np.cumsum([len(m) for m in mp_list])]))
        use_ur = stereo is not None
        be.undistort_grid(EUROC_K, EUROC_D)
        be.search_by_projection(mp_list, image_step=2, use_uright=use_ur)
        be.synchronize()
        t_l0 = time.perf_counter()
        be.search_by_projection(mp_list, image_step=2, use_uright=use_ur)
        be.synchronize()
        t_list = time.perf_counter() - t_l0
        be.set_profiling(True, stages=["k_sbp"])
        be.reset_stage_times()
        barrier(dist)
        q0 = time.perf_counter()
        for _ in range(args.steps):
            be.search_by_projection(mp_rows, image_step=2, use_uright=use_ur)
        be.synchronize()
        q1 = time.perf_counter()
        q_el = max_over_ranks(dist, q1 - q0)
        qt = be.stage_times().get("k_sbp", (0.0, 0))
        be.set_profiling(False)
        _, nm0 = be.projection_matches(0)
        n_mp = P * args.map_points
        k_ms = qt[0] / qt[1] if qt[1] else None
        sbp = {"metric": "map points searched per second (ORBmatcher::SearchByProjection, pinhole)",
               "value": round(sum_over_ranks(dist, n_mp) / (k_ms * 1e-3) / 1e6, 3) if k_ms else None,
               "unit": "Mmappoints/s", "kernel_ms_per_step": round(k_ms, 4) if k_ms else None,
               "call_ms_per_step": round(q_el / args.steps * 1e3, 4),
               "call_ms_list_form": round(t_list * 1e3, 4),
               "map_points_per_frame": args.map_points, "frames_per_step": P, "nmatches_frame0": nm0}
        # the two-camera form (Nleft != -1, the fisheye rig): grids on the raw positions, both
        # windows per point, stereo partners from a synthetic one-to-one pairing
        uniq2, lr = [], []
        be.undistort_grid(EUROC_K, ())
        for u in range(U):
            sides = []
            for e in range(2):
                k_, d_, _ = be.result(2 * u + e)
                xy_, _, _, _ = be.grid_result(2 * u + e)
                sides.append((xy_, k_["octave"], d_))
            l2r_, r2l_ = synth.stereo_partners(sides[0][2], sides[1][2], seed=u)
            lr.append((l2r_, r2l_))
            uniq2.append(synth.map_points_stereo(sides[0][0], sides[0][1], sides[0][2], sides[1][0],
                                                 sides[1][1], l2r_, n=args.map_points, seed=7 + u))
        mp2 = [uniq2[p % U] for p in range(P)]
        l2rs, r2ls = [lr[p % U][0] for p in range(P)], [lr[p % U][1] for p in range(P)]
        be.search_by_projection_stereo(mp2, l2rs, r2ls)
        be.synchronize()
        be.set_profiling(True, stages=["k_sbp"])
        be.reset_stage_times()
        for _ in range(args.steps):
            be.search_by_projection_stereo(mp2, l2rs, r2ls)
        be.synchronize()
        qt2 = be.stage_times().get("k_sbp", (0.0, 0))
        be.set_profiling(False)
        k2 = qt2[0] / qt2[1] if qt2[1] else None
        sbp["two_camera"] = {"value": round(sum_over_ranks(dist, n_mp) / (k2 * 1e-3) / 1e6, 3) if k2 else None,
                             "unit": "Mmappoints/s", "kernel_ms_per_step": round(k2, 4) if k2 else None,
                             "nmatches_pair0": be.projection_matches(0)[1]}

    # Wire formats: the P side-by-side frames of a step split from the device
    # staging buffer into the batch layout, and the step's results packed to the IDL SoA layout.
    # Timed on their own (HBM-bound copies; 4 B/px moved by the split, 2 x 28 B read + 16 B
    # written per keypoint and 3 x (4 + 2) B per match by the pack).
    wire = None
    if not args.no_wire:
        lib = og.load_library()
        dptr = lib.orbgpu_device_sbs_input(be.ctx.handle)
        if dptr and be.ctx.max_images >= 2:
            # fill the staging buffer from the resident batch (device to device, untimed) through
            # the HIP runtime liborbgpu.so itself is bound to
            memcpy2d = og.hip_function("hipMemcpy2D")
            vp, sz = ctypes.c_void_p, ctypes.c_size_t
            memcpy2d.argtypes = [vp, sz, vp, sz, sz, sz, ctypes.c_int]
            src = lib.orbgpu_device_input(be.ctx.handle)
            for p in range(P):
                for e in range(2):
                    memcpy2d(dptr + p * H * 2 * W + e * W, 2 * W, src + (2 * p + e) * H * W, W, W, H, 3)
            be.ingest_sbs(dptr, P, 2 * W)
            be.run()
            be.match_stereo(stereo_rows_only=False)
            be.pack_soa()
            be.synchronize()
            be.set_profiling(True, stages=["k_sbs_split", "k_pack_soa"])
            be.reset_stage_times()
            for _ in range(args.steps):
                be.ingest_sbs(dptr, P, 2 * W)
                be.pack_soa()
            be.synchronize()
            wt = be.stage_times()
            be.set_profiling(False)
            sp, pk = wt.get("k_sbs_split", (0.0, 0)), wt.get("k_pack_soa", (0.0, 0))
            split_b = 4.0 * H * W * P
            pack_b = 72.0 * feats_per_step + 18.0 * nq_per_step
            wire = {"sbs_split_us": round(sp[0] / sp[1] * 1e3, 2) if sp[1] else None,
                    "sbs_split_GBps": round(split_b / (sp[0] / sp[1] * 1e-3) / 1e9, 1) if sp[1] else None,
                    "pack_soa_us": round(pk[0] / pk[1] * 1e3, 2) if pk[1] else None,
                    "pack_soa_GBps": round(pack_b / (pk[0] / pk[1] * 1e-3) / 1e9, 1) if pk[1] else None,
                    "frames_per_step": P, "hbm_peak_GBps": HBM_PEAK_GBS}

    # Frame::ComputeStereoFishEyeMatches (Frame.cc:1142-1201) on the same resident images, timed on
    # its own: stereo-row kNN2 + KannalaBrandt8 triangulation, TUM-VI-like fisheye rig (0.1 m).
    # The batch is re-extracted first (untimed) with lapping areas over the whole frame, so every
    # keypoint is a stereo row (the headline's zero lapping areas leave none).
    fisheye = None
    if not args.no_stereo:
        kb = [250.0, 249.9, 320.5, 240.2, 0.0034823894, 0.00071503485, -0.0020532361, 0.00020293674]
        rig = og.KB8Rig.make(kb, kb, None, (0.101, 0.0, 0.0))
        be.run(np.tile(np.array([0, W], np.int32), (2 * P, 1)))
        be.fisheye_stereo(rig)
        be.synchronize()
        be.set_profiling(True, stages=["k_fisheye_stereo", "k_knn2"])
        be.reset_stage_times()
        barrier(dist)
        be.synchronize()
        f0 = time.perf_counter()
        for _ in range(args.steps):
            be.fisheye_stereo(rig)
        be.synchronize()
        f1 = time.perf_counter()
        fe_el = max_over_ranks(dist, f1 - f0)
        times = be.stage_times()
        fk = times.get("k_fisheye_stereo", (0.0, 0))
        kk = times.get("k_knn2", (0.0, 0))
        be.set_profiling(False)
        r0 = be.fisheye_result(0)
        fisheye = {"metric": "left keypoints through ComputeStereoFishEyeMatches per second (stereo-row kNN2 + "
                             "KannalaBrandt8 triangulation)",
                   "value": round(sum_over_ranks(dist, nq_per_step * args.steps) / fe_el / 1e6, 3),
                   "unit": "Mkeypoints/s", "ms_per_step": round(fe_el / args.steps * 1e3, 4),
                   "triangulation_ms_per_launch": round(fk[0] / fk[1], 4) if fk[1] else None,
                   "knn2_ms_per_launch": round(kk[0] / kk[1], 4) if kk[1] else None,
                   "pairs_per_step": P, "n_matches_pair0": r0["n_matches"]}

    # the other BASELINE configs as side lines (the headline stays C2): C3's 752x480 stream
    # (synthetic, EuRoC geometry) and C5's 1920x1080 / 12 levels / 5000 features, each with its
    # per-pair kNN2 (left -> right, all rows), resident batches, a few steps
    configs = None
    if not args.no_configs:
        configs = {}
        # C4 (BASELINE configs[3]): 8 stereo pairs sharded one pair per GPU -- each rank extracts
        # and matches ONE pair per step (the latency-bound shape; the headline batch is the
        # throughput shape).  Steps timed back to back, max over ranks.
        c4 = og.BatchExtractor(args.nfeatures, 1.2, args.nlevels, 20, 7, device=local, width=W, height=H, max_images=2)
        c4.upload(np.stack(uniq[0]))
        for _ in range(5):
            c4.run_match(stereo_rows_only=False)
        c4.synchronize()
        barrier(dist)
        k0 = time.perf_counter()
        n4 = 50
        for _ in range(n4):
            c4.run_match(stereo_rows_only=False)  # extraction + kNN2 as one graph submission
        c4.synchronize()
        k_el = max_over_ranks(dist, time.perf_counter() - k0)
        c4n, _ = c4.counts()
        configs["C4"] = {"workload": "1 stereo pair (640x480, 8 levels, 2000 feat/frame) + kNN2 per GPU per step",
                         "pairs_per_gpu_per_step": 1, "gpus": world,
                         "mfeatures_s": round(sum_over_ranks(dist, float(c4n.sum()) * n4) / k_el / 1e6, 3),
                         "ms_per_step": round(k_el / n4 * 1e3, 3), "data": "synthetic"}
        del c4
        for name, (cw, ch, cl, cn, cp) in {"C3": (752, 480, 8, 2000, 64), "C5": (1920, 1080, 12, 5000, 16)}.items():
            cu = [synth.stereo_pair(ch, cw, 500 + base + i) for i in range(4)]
            cimg = np.stack([cu[(i // 2) % 4][i % 2] for i in range(2 * cp)])
            cb_ = og.BatchExtractor(cn, 1.2, cl, 20, 7, device=local, width=cw, height=ch, max_images=2 * cp)
            cb_.upload(cimg)
            for _ in range(2):
                cb_.run()
                cb_.match_stereo(stereo_rows_only=False)
            cb_.synchronize()
            barrier(dist)
            c0_ = time.perf_counter()
            for _ in range(5):
                cb_.run()
                cb_.match_stereo(stereo_rows_only=False)
            cb_.synchronize()
            c_el = max_over_ranks(dist, time.perf_counter() - c0_)
            cnk, _ = cb_.counts()
            configs[name] = {"workload": "%dx%d stereo, %d levels, %d feat/frame + per-pair kNN2" % (cw, ch, cl, cn),
                             "pairs_per_gpu_per_step": cp,
                             "mfeatures_s": round(sum_over_ranks(dist, float(cnk.sum()) * 5) / c_el / 1e6, 3),
                             "mmatches_s": round(sum_over_ranks(dist, float(cnk[0::2].sum()) * 5) / c_el / 1e6, 3),
                             "ms_per_step": round(c_el / 5 * 1e3, 3), "data": "synthetic"}
            cb_.close() if hasattr(cb_, "close") else None
            del cb_

    # C5's exchange step (BASELINE configs[4]) when several GPUs run: every rank
    # contributes one C5 camera -- its own 1920x1080 frame, 12 levels, 5000 features, extracted on
    # its GPU -- one RCCL all_gather moves the descriptors (5000 x 32 B per camera), and each rank
    # matches its camera against every other camera on its GPU.  Reported beside the headline,
    # never part of it.
    cross = None
    if world > 1:
        try:
            from orbslam3lib_amd.dist import cross_camera_match, cross_camera_match_device
            C5W, C5H, C5L, C5N = 1920, 1080, 12, 5000
            c5, setup_err = None, None
            try:  # local setup first; every rank agrees on it before any collective of the leg
                c5 = og.BatchExtractor(C5N, 1.2, C5L, 20, 7, device=local, width=C5W, height=C5H, max_images=2)
                c5.upload(np.stack(synth.stereo_pair(C5H, C5W, 500 + base)))  # this rank's camera = image 0
                c5.run()
                c5.synchronize()
                kl0, dl0, _ = c5.result(0)
            except Exception as e:
                setup_err = e
            if -max_over_ranks(dist, -(0.0 if setup_err else 1.0)) < 1.0:
                raise RuntimeError("cross-camera setup failed on a rank: %r" % (setup_err,))
            device_path = has_cuda
            res = None
            for _ in range(2):  # the first exchange sets up the communicator and buffers
                barrier(dist)
                c0 = time.perf_counter()
                if device_path:
                    # descriptors stay in HBM: export -> all_gather (RCCL over xGMI; under gloo
                    # staged through the host) -> device kNN2 on every other camera
                    res = cross_camera_match_device(dist, c5, 0)
                    torch.cuda.synchronize()
                else:  # no GPU (the stub test): the host exchange
                    res = cross_camera_match(dist, dl0, c5.knn_match)
                c1 = time.perf_counter()
            cel = max_over_ranks(dist, c1 - c0)
            nqm = sum_over_ranks(dist, len(dl0) * len(res))
            # every rank checks its device results against the host matcher on the same rows
            ok = 1.0
            if device_path:
                from orbslam3lib_amd.dist import cross_camera_match as host_x
                ref = host_x(dist, dl0, c5.knn_match)
                for r_, got in res.items():
                    g = got.cpu().numpy()
                    ok = min(ok, float(all(np.array_equal(g[k], ref[r_][k]) for k in range(4))))
            ok = -max_over_ranks(dist, -ok)
            cross = {"workload": "C5 camera per rank: %dx%d, %d levels, %d feat/frame (BASELINE configs[4])"
                                 % (C5W, C5H, C5L, C5N),
                     "cameras": world, "queries_per_camera": len(dl0), "ms": round(cel * 1e3, 3),
                     "mmatches_s": round(nqm / cel / 1e6, 3),
                     "device_matches_equal_host_matcher": bool(ok == 1.0) if device_path else None,
                     "exchange": "all_gather (%s%s)" % (dist.get_backend(), ", device-resident rows"
                                                        if device_path else ", host rows")}
            c5.close()
            del c5
        except Exception as e:  # reported, never fatal to the headline line
            cross = {"error": repr(e)[:200]}

    # The C4 ingest-rank path (BASELINE configs[3]) when several GPUs run: rank 0 holds
    # one 640x480 stereo pair per rank, one scatter hands each rank its pair, each rank extracts
    # and matches it on its GPU, one gather brings every rank's results (counts, then the
    # keypoints, descriptors and kNN2 rows produced; orbgpu_export_batch) back to rank 0.  Reported beside the headline,
    # never part of it.
    ingest = None
    if world > 1:
        try:
            from orbslam3lib_amd.dist import ingest_scatter_gather
            ib, frames, setup_err = None, None, None
            try:  # local setup first; every rank agrees on it before any collective of the leg
                ib = og.BatchExtractor(args.nfeatures, 1.2, args.nlevels, 20, 7, device=local, width=W, height=H,
                                       max_images=2)
                frames = (np.stack([x for r_ in range(world) for x in synth.stereo_pair(H, W, 700 + r_)])
                          if rank == 0 else None)
            except Exception as e:
                setup_err = e
            if -max_over_ranks(dist, -(0.0 if setup_err else 1.0)) < 1.0:
                raise RuntimeError("ingest setup failed on a rank: %r" % (setup_err,))
            got = None
            istats = {}
            for _ in range(4):  # the first exchanges set up the communicators and buffers
                barrier(dist)
                i0 = time.perf_counter()
                got = ingest_scatter_gather(dist, ib, frames, pairs_per_rank=1, src=0, stats=istats)
                if has_cuda:
                    torch.cuda.synchronize()
                i1 = time.perf_counter()
            iel = max_over_ranks(dist, i1 - i0)
            ok = 1.0
            nfe = 0.0
            if rank == 0:
                for r_images, _ in got:
                    nfe += sum(len(k) for k, _, _ in r_images)
                for i, (k, d, m) in enumerate(got[0][0]):  # rank 0's own pair: equal to its local results
                    lk, ld, lm = ib.result(i)
                    ok = min(ok, float(m == lm and np.array_equal(d, ld)))
            ingest = {"workload": "C4: one 640x480 stereo pair per rank per step, frames on rank 0 "
                                  "(BASELINE configs[3]); extraction + kNN2 on every rank's GPU",
                      "ranks": world, "ms_per_step": round(iel * 1e3, 3),
                      "mfeatures_s": round(nfe / iel / 1e6, 3) if rank == 0 else None,
                      "exchange": "scatter of frames + gather of results (%s%s)"
                                  % (dist.get_backend(), ", device-resident" if has_cuda else ", host"),
                      # the gather moves the produced rows only (orbgpu_export_batch, packed)
                      "gathered_bytes_per_rank": istats.get("gathered_bytes_per_rank"),
                      "capacity_layout_bytes_per_rank": istats.get("capacity_bytes_per_rank"),
                      "rank0_results_equal_local": bool(ok == 1.0) if rank == 0 else None}
            ib.close()
            del ib
        except Exception as e:  # reported, never fatal to the headline line
            ingest = {"error": repr(e)[:200]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(W, H, args.nfeatures, args.cpu_seconds, args.map_points)
        cpu_model = ""
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        cpu = {"value": round(cb["mfeat_s_pool"], 4), "unit": "Mfeatures/s", "cores": cb["pool_threads"],
               "kind": "port",
               "label": "oracle restatement, scalar C++ (-O3%s -ffp-contract=off, no fast-math), not OpenCV-SIMD; "
                        "frames-parallel pool of %d std::threads = every CPU this process may use (affinity %d "
                        "threads, cgroup quota %s CPUs)" % (" -march=native" if cb["native"] else "",
                                                            cb["pool_threads"], cb["affinity"], cb["cgroup_cpu_quota"]),
               "host": {"nproc": os.cpu_count(), "affinity": cb["affinity"], "cgroup_cpu_quota": cb["cgroup_cpu_quota"],
                        "model": cpu_model},
               "mfeatures_s_1thread": round(cb["mfeat_s"], 5),
               "median_pair_ms_1thread": round(cb["median_pair_ms"], 2) if cb["median_pair_ms"] else None,
               "mfeatures_s_2threads_per_pair": round(cb["mfeat_s_2threads_per_pair"], 5),
               "mfeatures_s_pool_all_affinity_threads": round(cb["mfeat_s_pool_affinity"], 4),
               "mfeatures_s_whole_host_linear_estimate": round(cb["mfeat_s_pool"] / cb["pool_threads"] *
                                                               (os.cpu_count() or 1), 3),
               "sample": "4 synthetic 640x480 stereo pairs: %d pairs extracted on 1 thread (both eyes) + BF kNN2, "
                         "then the pool over >= 32 frames for >= %.0f s" % (cb["pairs"], max(3.0, args.cpu_seconds / 3)),
               "mmatches_s_1thread": round(cb["mmatch_s"], 5),
               "stereo_mkeypoints_s": round(cb["stereo_mkp_s"], 5) if cb["stereo_mkp_s"] else None,
               "undistort_grid_mkeypoints_s": round(cb["grid_mkp_s"], 5) if cb["grid_mkp_s"] else None,
               "search_by_projection_mmappoints_s": round(cb["sbp_mmp_s"], 5) if cb["sbp_mmp_s"] else None}

    if rank == 0:
        out = {
            "metric": "Mfeatures/s extract + Mmatches/s BFMatch, 640x480 stereo 8-level pyr, 1/2/4/8 GPU",
            "value": round(mfeat, 3),
            "unit": "Mfeatures/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("stub (CPU test of the multi-rank path, no GPU work)" if args.stub_gpu else
                     "synthetic seeded stereo frames (SURVEY §8d generator), resident in HBM"),
            "ranks": [{"rank": r_, "device": d_, "pid": p_} for r_, d_, p_ in placement],
            "backend": dist.get_backend() if dist is not None else None,
            "config": {"workload": "C2 640x480 stereo, 8 levels x1.2, 2000 feat/frame, FAST 20/7, "
                                   "+ per-pair 2000x2000 Hamming kNN2 (left->right, all rows)",
                       "pairs_per_gpu_per_step": P, "images_per_gpu_per_step": 2 * P,
                       "parallelism": "frames sharded across %d GPU(s), replicas" % world},
            "matches": {"value": round(mmatch, 3), "unit": "Mmatches/s",
                        "gpairs_s": round(total_pairs / elapsed / 1e9, 3)},
            "features_per_step_per_gpu": feats_per_step,
            "h2d": {"ms_per_batch_upload": round(h2d_max * 1e3, 3),
                    "GBps": round(imgs.nbytes / h2d_max / 1e9, 2) if h2d_max > 0 else None,
                    "mfeatures_s_incl_upload": round(h2d_incl, 3),
                    "ms_per_step_incl_upload": round(p_el / args.steps * 1e3, 4),
                    "mode": "pinned host batch, async copy stream, upload of step k+1 beside step k",
                    "mfeatures_s_upload_then_compute": round(h2d_serial, 3)},
            "roofline": roof,
            "roofline_fast_pyramid": roof_fp,
            "roofline_knn2": roof_knn,
            "roofline_valu": roof_valu,
            "stages": stage_rows,
            "cpu_baseline": cpu,
            "stereo_matches": stereo,
            "fisheye_stereo_matches": fisheye,
            "undistort_grid": grid,
            "search_by_projection": sbp,
            "other_configs": configs,
            "wire": wire,
            "cross_camera": cross,
            "ingest_c4": ingest,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
