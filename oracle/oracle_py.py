"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline
leg.  The product path (orbslam3lib_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborb_oracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class OracleKP(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _load(LIB_PATH)
    return _lib


def use_native():
    """Switch to the -march=native build (bench.py's CPU baseline); builds it if needed.  Returns
    the library path, or None when it cannot be built (the default build stays in use)."""
    global _lib
    path = os.path.join(HERE, "build", "liborb_oracle_native.so")
    try:
        subprocess.check_call(["make", "-s", "-C", HERE, "native"])
    except (OSError, subprocess.CalledProcessError):
        return None
    _lib = None
    _load(path)
    return path


def _load(path):
    global _lib
    _lib = C.CDLL(path)
    _lib.oracle_fast_atan2.restype = C.c_float
    _lib.oracle_fast_atan2.argtypes = [C.c_float, C.c_float]
    _lib.oracle_ic_angle.restype = C.c_float
    _lib.oracle_extract_many.restype = C.c_longlong
    return _lib


def extract_many(imgs, nthreads, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    """Frames-parallel pool inside the oracle (std::thread): imgs [n, h, w] -> total keypoints."""
    imgs = np.ascontiguousarray(imgs, dtype=np.uint8)
    n, h, w = imgs.shape
    r = lib().oracle_extract_many(nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th, _p(imgs), n, w, h,
                                  int(nthreads), None)
    if r < 0:
        raise RuntimeError("oracle_extract_many failed: %d" % r)
    return int(r)


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def level_sizes(w, h, scale_factor=1.2, nlevels=8):
    lw = np.zeros(nlevels, np.int32)
    lh = np.zeros(nlevels, np.int32)
    lib().oracle_level_sizes(C.c_float(scale_factor), nlevels, w, h, _p(lw), _p(lh))
    return list(zip(lw.tolist(), lh.tolist()))


def pyramid(img, scale_factor=1.2, nlevels=8):
    h, w = img.shape
    img = np.ascontiguousarray(img, dtype=np.uint8)
    sizes = level_sizes(w, h, scale_factor, nlevels)
    out = np.zeros(sum(a * b for a, b in sizes), np.uint8)
    lib().oracle_pyramid(C.c_float(scale_factor), nlevels, _p(img), w, h, w, _p(out))
    levels, off = [], 0
    for lw_, lh_ in sizes:
        levels.append(out[off:off + lw_ * lh_].reshape(lh_, lw_))
        off += lw_ * lh_
    return levels


def resize(src, dw, dh):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(dst), dw, dh, dw)
    return dst


def blur(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.zeros_like(img)
    lib().oracle_gaussian_blur(_p(img), img.shape[1], img.shape[0], _p(out))
    return out


def blur_kernel():
    k = np.zeros(7, np.int32)
    lib().oracle_blur_kernel(_p(k))
    return k.tolist()


def resize_simd_end(width):
    return lib().oracle_resize_simd_end(width)


def fast(img, th, roi=None):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    x0, y0, cols, rows = roi if roi else (0, 0, w, h)
    cap = max(16, cols * rows // 2)
    out = np.zeros(cap, KP_DTYPE)
    n = lib().oracle_fast(_p(img), w, x0, y0, cols, rows, th, _p(out), cap)
    return out[:n]


def corner_score(img, x, y, th):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return lib().oracle_corner_score(_p(img), img.shape[1], x, y, th)


def level_candidates(lvl, ini_th=20, min_th=7):
    lvl = np.ascontiguousarray(lvl, dtype=np.uint8)
    cap = lvl.size // 2 + 16
    out = np.zeros(cap, KP_DTYPE)
    n = lib().oracle_level_candidates(_p(lvl), lvl.shape[1], lvl.shape[0], ini_th, min_th,
                                      _p(out), cap)
    return out[:n]


def distribute_octree(keys, minX, maxX, minY, maxY, N):
    keys = np.ascontiguousarray(keys, dtype=KP_DTYPE)
    cap = max(16, 4 * max(N, 1) + len(keys))
    out = np.zeros(cap, KP_DTYPE)
    m = lib().oracle_distribute_octree(_p(keys), len(keys), minX, maxX, minY, maxY, N, _p(out), cap)
    return out[:m]


def fast_atan2(y, x):
    return lib().oracle_fast_atan2(float(y), float(x))


def ic_angle(img, x, y):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return lib().oracle_ic_angle(_p(img), img.shape[1], int(x), int(y))


def orb_descriptor(blurred, x, y, angle):
    blurred = np.ascontiguousarray(blurred, dtype=np.uint8)
    d = np.zeros(32, np.uint8)
    lib().oracle_orb_descriptor(_p(blurred), blurred.shape[1], C.c_float(x), C.c_float(y),
                                C.c_float(angle), _p(d))
    return d


def umax():
    u = np.zeros(16, np.int32)
    lib().oracle_umax(_p(u))
    return u.tolist()


def features_per_level(nfeatures, scale_factor=1.2, nlevels=8):
    o = np.zeros(nlevels, np.int32)
    lib().oracle_features_per_level(nfeatures, C.c_float(scale_factor), nlevels, _p(o))
    return o.tolist()


def scale_factors(scale_factor=1.2, nlevels=8):
    arr = [np.zeros(nlevels, np.float32) for _ in range(4)]
    lib().oracle_scale_factors(C.c_float(scale_factor), nlevels, *[_p(a) for a in arr])
    return arr


def extract(img, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, lap=(0, 0)):
    """ORBextractor::operator() -> (keypoints[KP_DTYPE], descriptors[N,32], monoIndex)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = 4 * nfeatures + 64 * nlevels
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    mono = lib().oracle_extract(nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th,
                                _p(img), w, h, w, int(lap[0]), int(lap[1]), _p(kps), _p(desc),
                                cap, C.byref(n))
    if mono < 0:
        raise RuntimeError("oracle_extract failed: %d" % mono)
    return kps[:n.value], desc[:n.value], mono


def extract_levels(img, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = 4 * nfeatures + 64 * nlevels
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    cnt = np.zeros(nlevels, np.int32)
    n = lib().oracle_extract_levels(nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th,
                                    _p(img), w, h, w, _p(kps), _p(desc), cap, _p(cnt))
    if n < 0:
        raise RuntimeError("oracle_extract_levels failed: %d" % n)
    out, off = [], 0
    for c in cnt.tolist():
        out.append((kps[off:off + c], desc[off:off + c]))
        off += c
    return out


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return lib().oracle_descriptor_distance(_p(a), _p(b))


def knn2(q, t):
    q = np.ascontiguousarray(q, dtype=np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(t, dtype=np.uint8).reshape(-1, 32)
    nq = q.shape[0]
    i1, d1, i2, d2 = (np.zeros(nq, np.int32) for _ in range(4))
    lib().oracle_knn2(_p(q), nq, _p(t), t.shape[0], _p(i1), _p(d1), _p(i2), _p(d2))
    return i1, d1, i2, d2


def sort_nodes(size, ulx):
    size = np.ascontiguousarray(size, dtype=np.int32)
    ulx = np.ascontiguousarray(ulx, dtype=np.int32)
    perm = np.zeros(len(size), np.int32)
    lib().oracle_sort_nodes(_p(size), _p(ulx), len(size), _p(perm))
    return perm


def stereo_matches(kps_l, desc_l, kps_r, desc_r, pyr_l, pyr_r, mbf, mb, scale_factor=1.2):
    """Frame::ComputeStereoMatches (Frame.cc:827-997) -> (mvuRight, mvDepth, sad) float32/int32.
    pyr_l / pyr_r: the unblurred pyramids (lists of levels, as pyramid() returns)."""
    nlevels = len(pyr_l)
    kl = np.ascontiguousarray(kps_l, dtype=KP_DTYPE)
    kr = np.ascontiguousarray(kps_r, dtype=KP_DTYPE)
    dl = np.ascontiguousarray(desc_l, dtype=np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(desc_r, dtype=np.uint8).reshape(-1, 32)
    pl = [np.ascontiguousarray(p, dtype=np.uint8) for p in pyr_l]
    pr = [np.ascontiguousarray(p, dtype=np.uint8) for p in pyr_r]
    PL = (C.c_void_p * nlevels)(*[p.ctypes.data for p in pl])
    PR = (C.c_void_p * nlevels)(*[p.ctypes.data for p in pr])
    lw = np.array([p.shape[1] for p in pl], np.int32)
    lh = np.array([p.shape[0] for p in pl], np.int32)
    scale, inv_scale, _, _ = scale_factors(scale_factor, nlevels)
    n = len(kl)
    ur = np.zeros(n, np.float32)
    dep = np.zeros(n, np.float32)
    sad = np.zeros(n, np.int32)
    lib().oracle_stereo_matches(_p(kl), n, _p(dl), _p(kr), len(kr), _p(dr), PL, PR, _p(lw), _p(lh),
                                nlevels, _p(scale), _p(inv_scale), C.c_float(mbf), C.c_float(mb),
                                _p(ur), _p(dep), _p(sad))
    return ur, dep, sad


def fisheye_stereo(kps_l, mono_l, kps_r, mono_r, idx1, dist1, rig, sigma2):
    """Frame::ComputeStereoFishEyeMatches (Frame.cc:1142-1201) on one frame's stereo-row kNN2
    (idx1 / dist1 from knn2(desc_l[mono_l:], desc_r[mono_r:])).  rig: dict with cam_left /
    cam_right (8 KannalaBrandt8 parameters), precision_left / precision_right, R12 (3x3), t12.
    Returns dict: l2r, r2l, depth, p3d, code, margins, n_matches (parity unpinned: see
    orb_fisheye.cpp)."""
    kl = np.ascontiguousarray(kps_l, dtype=KP_DTYPE)
    kr = np.ascontiguousarray(kps_r, dtype=KP_DTYPE)
    nl, nr = len(kl), len(kr)
    nq = max(nl - mono_l, 0)
    i1 = np.ascontiguousarray(idx1[:nq], dtype=np.int32)
    d1 = np.ascontiguousarray(dist1[:nq], dtype=np.int32)
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).ravel()
    cl, cr = f32(rig["cam_left"]), f32(rig["cam_right"])
    R, t, s2 = f32(rig["R12"]), f32(rig["t12"]), f32(sigma2)
    out = dict(l2r=np.zeros(nl, np.int32), r2l=np.zeros(nr, np.int32), depth=np.zeros(nl, np.float32),
               p3d=np.zeros((nl, 3), np.float32), code=np.zeros(nq, np.int32),
               margins=np.zeros((nq, 5), np.float64))
    out["n_matches"] = lib().oracle_fisheye_stereo(
        _p(kl), nl, mono_l, _p(kr), nr, mono_r, _p(i1), _p(d1), _p(cl), _p(cr),
        C.c_float(rig.get("precision_left", 1e-6)), C.c_float(rig.get("precision_right", 1e-6)),
        _p(R), _p(t), _p(s2), _p(out["l2r"]), _p(out["r2l"]), _p(out["depth"]), _p(out["p3d"]),
        _p(out["code"]), _p(out["margins"]))
    return out


def undistort_grid(kps, K, dist, cols, rows):
    """Frame::UndistortKeyPoints + ComputeImageBounds + AssignFeaturesToGrid (Frame.cc:405-436,
    741-825) -> (xy_un [n,2] f32, bounds [4] f32, cell [n] i32, cell_start [3073], cell_idx)."""
    kps = np.ascontiguousarray(kps, dtype=KP_DTYPE)
    n = len(kps)
    xy = np.ascontiguousarray(np.stack([kps["x"], kps["y"]], 1).astype(np.float32))
    Kf = np.ascontiguousarray(K, dtype=np.float32)
    d = np.ascontiguousarray(dist, dtype=np.float32)
    out = np.zeros((n, 2), np.float32)
    lib().oracle_undistort_points(_p(xy), n, _p(Kf), _p(d), len(d), _p(out))
    bounds = np.zeros(4, np.float32)
    lib().oracle_image_bounds(int(cols), int(rows), _p(Kf), _p(d), len(d), _p(bounds))
    cell = np.zeros(n, np.int32)
    cs = np.zeros(64 * 48 + 1, np.int32)
    ci = np.zeros(max(n, 1), np.int32)
    lib().oracle_assign_grid(_p(out), n, _p(bounds), _p(cell), _p(cs), _p(ci))
    return out, bounds, cell, cs, ci[:cs[-1]]


def pack_soa(kps):
    """orbslam3.idl SoA of keypoints: dict of int32 x, y, angle (cos8 | sin8 << 8), level."""
    kps = np.ascontiguousarray(kps, dtype=KP_DTYPE)
    n = len(kps)
    out = {k: np.zeros(max(n, 1), np.int32) for k in ("x", "y", "angle", "level")}
    lib().oracle_pack_soa(_p(kps), n, _p(out["x"]), _p(out["y"]), _p(out["angle"]), _p(out["level"]))
    return {k: v[:n] for k, v in out.items()}


def decode_angle(enc):
    """LynxHardwareAccelerator.cpp:174-178: int8 cos / sin -> degrees."""
    enc = np.asarray(enc, np.int32)
    c = (enc & 0xFF).astype(np.uint8).view(np.int8).astype(np.float32)
    s = ((enc >> 8) & 0xFF).astype(np.uint8).view(np.int8).astype(np.float32)
    return np.degrees(np.arctan2(s / 64.0, c / 64.0))


MP_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                     ("depth", "<f4"), ("level", "<i4"), ("flags", "<i4"), ("desc", "u1", (32,)),
                     ("proj_yr", "<f4"), ("view_cos_r", "<f4"), ("level_r", "<i4")])


def search_by_projection(mps, xy_un, octave, desc, uright, bounds, cell_start, cell_idx, kp_block=None,
                         th=1.0, nnratio=0.8, far_points=False, th_far=50.0, scale_factor=1.2, nlevels=8):
    """ORBmatcher::SearchByProjection (ORBmatcher.cc:44-214), pinhole -> (match [n], nmatches)."""
    mps = np.ascontiguousarray(mps, dtype=MP_DTYPE)
    n = len(octave)
    xy = np.ascontiguousarray(xy_un, dtype=np.float32).reshape(-1, 2)
    octv = np.ascontiguousarray(octave, dtype=np.int32)
    d = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
    ur = None if uright is None else np.ascontiguousarray(uright, dtype=np.float32)
    b = np.ascontiguousarray(bounds, dtype=np.float32)
    cs = np.ascontiguousarray(cell_start, dtype=np.int32)
    ci = np.ascontiguousarray(cell_idx, dtype=np.int32)
    if len(ci) == 0:
        ci = np.zeros(1, np.int32)
    blk = None if kp_block is None else np.ascontiguousarray(kp_block, dtype=np.uint8)
    scale = scale_factors(scale_factor, nlevels)[0]
    match = np.zeros(max(n, 1), np.int32)
    nm = lib().oracle_search_by_projection(
        _p(mps) if len(mps) else None, len(mps), _p(xy) if n else None, _p(octv) if n else None,
        _p(d) if n else None, _p(ur) if ur is not None else None, n, _p(b), _p(cs), _p(ci), _p(scale), nlevels,
        _p(blk) if blk is not None else None, C.c_float(th), C.c_float(nnratio), int(far_points),
        C.c_float(th_far), _p(match))
    return match[:n], nm


def search_by_projection2(mps, left, right, bounds, l2r=None, r2l=None, kp_block=None, th=1.0, nnratio=0.8,
                          far_points=False, th_far=50.0, scale_factor=1.2, nlevels=8):
    """Two-camera SearchByProjection (Nleft != -1).  left / right = (xy [n,2], octave [n],
    desc [n,32], cell_start, cell_idx) -> (match [nl + nr], nmatches)."""
    mps = np.ascontiguousarray(mps, dtype=MP_DTYPE)

    def prep(side):
        xy, octv, d, cs, ci = side
        xy = np.ascontiguousarray(xy, dtype=np.float32).reshape(-1, 2)
        octv = np.ascontiguousarray(octv, dtype=np.int32)
        d = np.ascontiguousarray(d, dtype=np.uint8).reshape(-1, 32)
        cs = np.ascontiguousarray(cs, dtype=np.int32)
        ci = np.ascontiguousarray(ci if len(ci) else np.zeros(1), dtype=np.int32)
        return xy, octv, d, cs, ci
    L, R = prep(left), prep(right)
    nl, nr = len(L[1]), len(R[1])
    arr = lambda a, dt: None if a is None else np.ascontiguousarray(a, dtype=dt)
    l2r, r2l, blk = arr(l2r, np.int32), arr(r2l, np.int32), arr(kp_block, np.uint8)
    scale = scale_factors(scale_factor, nlevels)[0]
    match = np.zeros(max(nl + nr, 1), np.int32)
    pp = lambda a: _p(a) if a is not None and a.size else None
    nm = lib().oracle_search_by_projection2(
        pp(mps), len(mps), pp(L[0]), pp(L[1]), pp(L[2]), nl, _p(L[3]), _p(L[4]),
        pp(R[0]), pp(R[1]), pp(R[2]), nr, _p(R[3]), _p(R[4]), _p(np.ascontiguousarray(bounds, np.float32)),
        pp(l2r), pp(r2l), _p(scale), nlevels, pp(blk), C.c_float(th), C.c_float(nnratio), int(far_points),
        C.c_float(th_far), _p(match))
    return match[:nl + nr], nm
