"""orbslam3lib_amd -- MI355X-native ORB front-end (Python mirror of the reference interface).

The compute path is liborbgpu.so (HIP kernels for gfx950 behind the C ABI in
include/orbgpu.h).  This module mirrors the reference's operator surface so the parity tests
read like the reference's own call sites:

  ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
      cpp/include/ORBextractor_old.h:51-59; operator() :56-59; getters :62-84; mvImagePyramid :86
  ORBmatcher.DescriptorDistance(a, b)        cpp/include/ORBmatcher.h:44
  BFMatcher(NORM_HAMMING).knnMatch(q, t, 2)  cpp/src/Frame.cc:45,1227

There is no CPU fallback: if liborbgpu.so or a gfx950 device is missing, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

__all__ = ["ORBextractor", "ORBmatcher", "BFMatcher", "BatchExtractor", "KEYPOINT_DTYPE", "MAP_POINT_DTYPE",
           "OrbGpuError", "load_library", "LIB_PATH"]

HERE = os.path.dirname(os.path.abspath(__file__))
# ORBGPU_LIB names another build of the same library (measurement variants under tools/)
LIB_PATH = os.environ.get("ORBGPU_LIB") or os.path.join(HERE, "liborbgpu.so")

# orbgpu_map_point (60 B): the MapPoint state ORBmatcher::SearchByProjection reads
MAP_POINT_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                            ("depth", "<f4"), ("level", "<i4"), ("flags", "<i4"), ("desc", "u1", (32,)),
                            ("proj_yr", "<f4"), ("view_cos_r", "<f4"), ("level_r", "<i4")])
MP_IN_VIEW, MP_BAD, MP_HAS_OBS, MP_IN_VIEW_R = 1, 2, 4, 8

# cv::KeyPoint layout (28 B)
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

EXPORTED = [
    "orbgpu_create", "orbgpu_destroy", "orbgpu_get_scale_tables", "orbgpu_extract",
    "orbgpu_extract_stereo", "orbgpu_upload_images", "orbgpu_device_input", "orbgpu_run_batch",
    "orbgpu_download_result", "orbgpu_download_counts", "orbgpu_synchronize",
    "orbgpu_get_pyramid_level", "orbgpu_get_level_keypoints", "orbgpu_match_knn2",
    "orbgpu_match_stereo_batch", "orbgpu_download_matches", "orbgpu_descriptor_distance",
    "orbgpu_stereo_matches_batch", "orbgpu_download_stereo", "orbgpu_candidate_counts",
    "orbgpu_image_bounds", "orbgpu_undistort_grid_batch", "orbgpu_download_grid",
    "orbgpu_device_sbs_input", "orbgpu_upload_sbs", "orbgpu_ingest_sbs", "orbgpu_pack_soa",
    "orbgpu_download_soa", "orbgpu_download_matches16", "orbgpu_extract_features",
    "orbgpu_search_by_projection_batch", "orbgpu_search_by_projection_stereo",
    "orbgpu_download_projection_matches", "orbgpu_upload_images_async", "orbgpu_host_alloc",
    "orbgpu_host_free", "orbgpu_export_descriptors", "orbgpu_match_knn2_device",
    "orbgpu_set_profiling", "orbgpu_num_stages", "orbgpu_stage_name", "orbgpu_stage_times",
    "orbgpu_reset_stage_times", "orbgpu_last_error", "orbgpu_abi_version",
    "orbgpu_fisheye_stereo_batch", "orbgpu_download_fisheye", "orbgpu_run_batch_match",
    "orbgpu_diagnostic_knobs", "orbgpu_ingest_images", "orbgpu_export_batch_bytes", "orbgpu_export_batch",
    "orbgpu_get_device",
]

DEVICE_CURRENT = -1  # ORBGPU_DEVICE_CURRENT: the calling thread's current HIP device


class KB8Rig(C.Structure):
    """orbgpu_kb8_rig: the two KannalaBrandt8 cameras and Frame::mRlr / mtlr."""
    _fields_ = [("cam_left", C.c_float * 8), ("cam_right", C.c_float * 8), ("precision_left", C.c_float),
                ("precision_right", C.c_float), ("R12", C.c_float * 9), ("t12", C.c_float * 3)]

    @classmethod
    def make(cls, cam_left, cam_right, R12=None, t12=(0.0, 0.0, 0.0), precision_left=1e-6,
             precision_right=1e-6):
        r = cls()
        r.cam_left[:] = [float(v) for v in cam_left]
        r.cam_right[:] = [float(v) for v in cam_right]
        r.precision_left, r.precision_right = precision_left, precision_right
        R = np.eye(3, dtype=np.float32) if R12 is None else np.asarray(R12, np.float32).reshape(9)
        r.R12[:] = [float(v) for v in np.ravel(R)]
        r.t12[:] = [float(v) for v in t12]
        return r

    def as_dict(self):
        return dict(cam_left=list(self.cam_left), cam_right=list(self.cam_right),
                    precision_left=self.precision_left, precision_right=self.precision_right,
                    R12=np.array(list(self.R12), np.float32).reshape(3, 3), t12=list(self.t12))


class OrbGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("orbgpu error %d: %s" % (code, msg))
        self.code = code


class _Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load liborbgpu.so (raises if it has not been built -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OrbGpuError(-6, "liborbgpu.so not built (run `make` or __graft_entry__.build())")
    lib = C.CDLL(path)
    lib.orbgpu_last_error.restype = C.c_char_p
    lib.orbgpu_stage_name.restype = C.c_char_p
    lib.orbgpu_device_input.restype = C.c_void_p
    lib.orbgpu_device_input.argtypes = [C.c_void_p]
    lib.orbgpu_device_sbs_input.restype = C.c_void_p
    lib.orbgpu_device_sbs_input.argtypes = [C.c_void_p]
    lib.orbgpu_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
    lib.orbgpu_host_free.argtypes = [C.c_void_p]
    lib.orbgpu_diagnostic_knobs.argtypes = [C.c_char_p, C.c_size_t]
    lib.orbgpu_export_descriptors.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                              C.POINTER(C.c_int), C.c_void_p]
    lib.orbgpu_match_knn2_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int] + \
        [C.c_void_p] * 5
    lib.orbgpu_ingest_images.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    lib.orbgpu_export_batch_bytes.restype = C.c_size_t
    lib.orbgpu_export_batch_bytes.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.orbgpu_export_batch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                        C.POINTER(C.c_size_t), C.c_void_p]
    lib.orbgpu_get_device.argtypes = [C.c_void_p]
    for name in ("orbgpu_destroy", "orbgpu_synchronize", "orbgpu_set_profiling",
                 "orbgpu_reset_stage_times"):
        getattr(lib, name).argtypes = [C.c_void_p] + ([C.c_int] if name == "orbgpu_set_profiling" else [])
    _lib = lib
    return lib


def hip_function(name: str):
    """A HIP runtime entry point (e.g. "hipMemcpy2D") from the runtime liborbgpu.so is bound to.
    ctypes looks the name up with dlsym on the library's handle, which searches liborbgpu.so and
    then its dependencies in load order, i.e. the libamdhip64 it actually mapped (torch's bundled
    copy when torch was imported first) -- no soname is hard-coded.  Test / bench plumbing."""
    return getattr(load_library(), name)


def diagnostic_knobs() -> dict:
    """The measurement knobs liborbgpu.so honours right now (orbgpu_diagnostic_knobs): empty
    unless ORBGPU_DIAGNOSTICS=1 is set beside them."""
    buf = C.create_string_buffer(4096)
    load_library().orbgpu_diagnostic_knobs(buf, len(buf))
    txt = buf.value.decode()
    return dict(kv.split("=", 1) for kv in txt.split(";")) if txt else {}


def _check(code):
    if code < 0:
        raise OrbGpuError(code, _lib.orbgpu_last_error().decode())
    return code


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


_COUNT_STATUS = {-5: "device workspace overflow (octree)", -2: "context output capacity exceeded"}


def decode_export(buf, n_images, n_pairs):
    """The packed orbgpu_export_batch layout (include/orbgpu.h) -> ([(kps, desc, mono)] per image,
    [(idx1, dist1, idx2, dist2)] per pair).  Raises OrbGpuError on a status word in a count."""
    b = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    hdr = 4 * (2 * n_images + n_pairs)
    if b.size < hdr:
        raise OrbGpuError(-2, "export buffer shorter than its header")
    h = b[:hdr].view(np.int32)
    counts, mono, nq = h[:n_images], h[n_images:2 * n_images], h[2 * n_images:]
    for c in list(counts) + list(nq):
        if c < 0:
            code = int(c) if int(c) in _COUNT_STATUS else -2
            raise OrbGpuError(code, _COUNT_STATUS.get(int(c), "negative row count in export"))
    if b.size < hdr + 60 * int(counts.sum()) + 16 * int(nq.sum()):
        raise OrbGpuError(-2, "export buffer shorter than its counts say")
    o = hdr
    images = []
    for i in range(n_images):
        n = int(counts[i])
        kps = b[o:o + 28 * n].copy().view(KEYPOINT_DTYPE); o += 28 * n
        desc = b[o:o + 32 * n].copy().reshape(n, 32); o += 32 * n
        images.append((kps, desc, int(mono[i])))
    pairs = []
    for p in range(n_pairs):
        n = int(nq[p])
        m = b[o:o + 16 * n].copy().view(np.int32).reshape(4, n); o += 16 * n
        pairs.append(tuple(m[k] for k in range(4)))
    return images, pairs


def encode_export(images, pairs):
    """Host restatement of the packed layout (what orbgpu_export_batch writes) from per-image
    (kps, desc, mono) and per-pair (idx1, dist1, idx2, dist2): the CPU stand-ins' export."""
    parts = [np.array([len(k) for k, _, _ in images], np.int32), np.array([m for _, _, m in images], np.int32),
             np.array([len(p[0]) for p in pairs], np.int32)]
    for k, d, _ in images:
        parts.append(np.ascontiguousarray(k, KEYPOINT_DTYPE).view(np.uint8).reshape(-1))
        parts.append(np.ascontiguousarray(d, np.uint8).reshape(-1))
    for p in pairs:
        parts.append(np.stack([np.asarray(a, np.int32) for a in p]).reshape(-1))
    return np.concatenate([x.view(np.uint8).reshape(-1) for x in parts])


class _Context:
    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device, max_width,
                 max_height, max_images):
        lib = load_library()
        self.params = _Params(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST),
                              int(minThFAST))
        self.handle = C.c_void_p()
        _check(lib.orbgpu_create(C.byref(self.params), int(device), int(max_width),
                                 int(max_height), int(max_images), C.byref(self.handle)))
        self.nlevels = int(nlevels)
        self.max_images = int(max_images)

    def device(self):
        """The HIP ordinal the context runs on (orbgpu_get_device)."""
        return _check(_lib.orbgpu_get_device(self.handle))

    def close(self):
        if self.handle:
            _lib.orbgpu_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ORBextractor:
    """ORB_SLAM3::ORBextractor on the GPU (cpp/src/ORBextractor_old.cc:411-1191).

    __call__(image, mask=None, vLappingArea=(0, 0)) -> (keypoints, descriptors, monoIndex)
      keypoints: structured array with cv::KeyPoint fields; descriptors: uint8 [N, 32];
      monoIndex: number of keypoints outside the lapping area (written first).
      Returns (empty, None, -1) for an empty image, like the reference (:1092-1093).
    """

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device=0,
                 max_width=1920, max_height=1080, max_images=2):
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(scaleFactor)
        self.nlevels = int(nlevels)
        self.iniThFAST = int(iniThFAST)
        self.minThFAST = int(minThFAST)
        self._ctx = _Context(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device,
                             max_width, max_height, max_images)
        L = self.nlevels
        self.mvScaleFactor = np.zeros(L, np.float32)
        self.mvInvScaleFactor = np.zeros(L, np.float32)
        self.mvLevelSigma2 = np.zeros(L, np.float32)
        self.mvInvLevelSigma2 = np.zeros(L, np.float32)
        self.mnFeaturesPerLevel = np.zeros(L, np.int32)
        _check(_lib.orbgpu_get_scale_tables(self._ctx.handle, _p(self.mvScaleFactor),
                                            _p(self.mvInvScaleFactor), _p(self.mvLevelSigma2),
                                            _p(self.mvInvLevelSigma2), _p(self.mnFeaturesPerLevel)))
        self._cap = 4 * max(self.nfeatures, 1) * 2 + 64 * L + 4096
        self._last_n_images = 0

    # getters (ORBextractor_old.h:62-84)
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.scaleFactor

    def GetScaleFactors(self):
        return self.mvScaleFactor.tolist()

    def GetInverseScaleFactors(self):
        return self.mvInvScaleFactor.tolist()

    def GetScaleSigmaSquares(self):
        return self.mvLevelSigma2.tolist()

    def GetInverseScaleSigmaSquares(self):
        return self.mvInvLevelSigma2.tolist()

    def __call__(self, image, mask=None, vLappingArea=(0, 0)):
        img = np.asarray(image)
        if img.size == 0:
            return np.zeros(0, KEYPOINT_DTYPE), None, -1
        if img.dtype != np.uint8 or img.ndim != 2:
            raise OrbGpuError(-3, "image must be CV_8UC1 (2-D uint8)")  # assert :1096
        img = np.ascontiguousarray(img)
        h, w = img.shape
        kps = np.zeros(self._cap, KEYPOINT_DTYPE)
        desc = np.zeros((self._cap, 32), np.uint8)
        n, mono = C.c_int(0), C.c_int(0)
        _check(_lib.orbgpu_extract(self._ctx.handle, _p(img), w, h, w, int(vLappingArea[0]),
                                   int(vLappingArea[1]), _p(kps), _p(desc), self._cap,
                                   C.byref(n), C.byref(mono)))
        self._last_n_images = 1
        return kps[:n.value], (desc[:n.value] if n.value else None), mono.value

    def extract_stereo(self, left, right, lapLeft=(0, 0), lapRight=(0, 0)):
        """Stereo operator() (cpp/include/ORBextractor.h:52-57): both eyes in one device pass."""
        left = np.ascontiguousarray(left, dtype=np.uint8)
        right = np.ascontiguousarray(right, dtype=np.uint8)
        h, w = left.shape
        out = []
        bufs = [(np.zeros(self._cap, KEYPOINT_DTYPE), np.zeros((self._cap, 32), np.uint8),
                 C.c_int(0), C.c_int(0)) for _ in range(2)]
        la = (C.c_int * 2)(*lapLeft)
        ra = (C.c_int * 2)(*lapRight)
        (kl, dl, nl, ml), (kr, dr, nr, mr) = bufs
        _check(_lib.orbgpu_extract_stereo(self._ctx.handle, _p(left), _p(right), w, h, w, la, ra,
                                          _p(kl), _p(dl), C.byref(nl), C.byref(ml), _p(kr), _p(dr),
                                          C.byref(nr), C.byref(mr), self._cap))
        self._last_n_images = 2
        for k, d, n, m in bufs:
            out.append((k[:n.value], d[:n.value], m.value))
        return out

    @property
    def mvImagePyramid(self):
        """Levels of the last extracted image (public member, ORBextractor_old.h:86)."""
        return [self.pyramid_level(0, l) for l in range(self.nlevels)]

    def pyramid_level(self, image, level, blurred=False):
        w, h = C.c_int(0), C.c_int(0)
        _check(_lib.orbgpu_get_pyramid_level(self._ctx.handle, image, level, int(blurred), None, 0,
                                             C.byref(w), C.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        _check(_lib.orbgpu_get_pyramid_level(self._ctx.handle, image, level, int(blurred), _p(out),
                                             w.value, None, None))
        return out

    def level_keypoints(self, image=0):
        """Per-level keypoints (level coords, octree order, with angle) + descriptors."""
        kps = np.zeros(self._cap, KEYPOINT_DTYPE)
        desc = np.zeros((self._cap, 32), np.uint8)
        cnt = np.zeros(self.nlevels, np.int32)
        _check(_lib.orbgpu_get_level_keypoints(self._ctx.handle, image, _p(kps), _p(desc), self._cap,
                                               _p(cnt)))
        out, off = [], 0
        for c in cnt.tolist():
            out.append((kps[off:off + c], desc[off:off + c]))
            off += c
        return out


class ORBmatcher:
    @staticmethod
    def DescriptorDistance(a, b):
        """Hamming distance of two 32-byte descriptors (cpp/src/ORBmatcher.cc:2107-2123)."""
        lib = load_library()
        a = np.ascontiguousarray(a, dtype=np.uint8).reshape(32)
        b = np.ascontiguousarray(b, dtype=np.uint8).reshape(32)
        return lib.orbgpu_descriptor_distance(_p(a), _p(b))


class BFMatcher:
    """cv::BFMatcher(NORM_HAMMING) with knnMatch(k=2) on the GPU."""

    def __init__(self, extractor: ORBextractor):
        self._ctx = extractor._ctx

    def knnMatch(self, query, train, k=2):
        """Returns (idx1, dist1, idx2, dist2) int32 arrays; idx = -1 where absent."""
        if k != 2:
            raise OrbGpuError(-3, "only k=2 is implemented (the reference uses k=2)")
        q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 32)
        nq = q.shape[0]
        out = [np.zeros(nq, np.int32) for _ in range(4)]
        _check(_lib.orbgpu_match_knn2(self._ctx.handle, _p(q), nq, _p(t), t.shape[0],
                                      *[_p(o) for o in out]))
        return tuple(out)


class BatchExtractor:
    """Device-resident batch path (the throughput path used by bench.py).

    upload(images[n,h,w]) -> run(laps) -> results stay in HBM; match_stereo() pairs 2p/2p+1.
    """

    device_resident = True  # results live in HBM (dist.cross_camera_match_device)

    def __init__(self, nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7,
                 device=0, width=640, height=480, max_images=128):
        self.ctx = _Context(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device, width,
                            height, max_images)
        self.width, self.height = int(width), int(height)
        self.n = 0
        self._staged = None  # (n, h, w) of the batch upload_async staged for the next run()
        self._pinned = []

    def close(self):
        """Frees the pinned host buffers of pinned() and the device context."""
        self.free_pinned()
        self.ctx.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, images):
        imgs = np.ascontiguousarray(images, dtype=np.uint8)
        n, h, w = imgs.shape
        _check(_lib.orbgpu_upload_images(self.ctx.handle, _p(imgs), n, w, h, w))
        self.n, self.height, self.width = n, h, w
        self._staged = None  # the synchronous upload replaces a staged one (orbgpu_upload_images)
        _check(_lib.orbgpu_synchronize(self.ctx.handle))

    def knn_match(self, query, train):
        """BFMatcher(NORM_HAMMING).knnMatch(query, train, 2) on this context's device, host arrays
        in and out: (idx1, dist1, idx2, dist2) int32."""
        q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 32)
        out = [np.zeros(q.shape[0], np.int32) for _ in range(4)]
        _check(_lib.orbgpu_match_knn2(self.ctx.handle, _p(q), q.shape[0], _p(t), t.shape[0], *[_p(o) for o in out]))
        return tuple(out)

    def export_descriptors(self, image, device_ptr, cap_rows, row0=0, stream=None):
        """Rows [row0, n) of image's descriptors into device memory (device-to-device);
        returns the row count."""
        n = C.c_int(0)
        _check(_lib.orbgpu_export_descriptors(self.ctx.handle, int(image), int(row0), C.c_void_p(device_ptr),
                                              int(cap_rows), C.byref(n), C.c_void_p(stream) if stream else None))
        return n.value

    def match_knn2_device(self, d_query, nq, d_train, nt, d_out, stream=None):
        """kNN2 on device buffers; d_out: device int32 [4, nq] (idx1, dist1, idx2, dist2)."""
        _check(_lib.orbgpu_match_knn2_device(self.ctx.handle, C.c_void_p(d_query), int(nq), C.c_void_p(d_train),
                                             int(nt), C.c_void_p(d_out), C.c_void_p(d_out + 4 * nq),
                                             C.c_void_p(d_out + 8 * nq), C.c_void_p(d_out + 12 * nq),
                                             C.c_void_p(stream) if stream else None))

    def ingest_images(self, device_ptr, n, stride=None, stream=None):
        """n images of this context's size already in device memory (rows of `stride` bytes,
        e.g. a collective's receive buffer) -> the input buffer, device to device
        (orbgpu_ingest_images); the next run() / run_match() reads them."""
        _check(_lib.orbgpu_ingest_images(self.ctx.handle, C.c_void_p(device_ptr), int(n), self.width, self.height,
                                         int(stride or self.width), C.c_void_p(stream) if stream else None))
        self.n = int(n)
        self._staged = None

    def export_batch_bytes(self, n_images, n_pairs):
        """The largest orbgpu_export_batch layout (every image at the context's row capacity)."""
        return int(_lib.orbgpu_export_batch_bytes(self.ctx.handle, int(n_images), int(n_pairs)))

    def export_batch_size(self, n_images, n_pairs, stream=None):
        """The exact size of the packed orbgpu_export_batch layout of the last batch (waits for it)."""
        used = C.c_size_t(0)
        _check(_lib.orbgpu_export_batch(self.ctx.handle, int(n_images), int(n_pairs), None, 0, C.byref(used),
                                        C.c_void_p(stream) if stream else None))
        return used.value

    def export_batch(self, device_ptr, n_images, n_pairs, nbytes, stream=None):
        """The last batch's produced rows of images [0, n_images) and pairs [0, n_pairs) packed into
        one device buffer (orbgpu_export_batch, device to device); returns the bytes written."""
        used = C.c_size_t(0)
        _check(_lib.orbgpu_export_batch(self.ctx.handle, int(n_images), int(n_pairs), C.c_void_p(device_ptr),
                                        int(nbytes), C.byref(used), C.c_void_p(stream) if stream else None))
        return used.value

    @staticmethod
    def decode_export(buf, n_images, n_pairs):
        """Host view of an orbgpu_export_batch buffer (uint8 array, trailing padding allowed): per
        image (keypoints in the cv::KeyPoint layout, descriptors [n, 32], mono index) and per pair
        (idx1, dist1, idx2, dist2) over the pair's query rows -- what result() / matches() return.
        A negative count is a device status word (-5 octree workspace overflow, -2 capacity), not
        rows: raised as OrbGpuError, as every download path does."""
        return decode_export(buf, n_images, n_pairs)

    def upload_async(self, images):
        """Stage the NEXT batch (orbgpu_upload_images_async): the copy runs beside the current
        batch's kernels; the next run() reads it.  `images` should come from pinned()."""
        imgs = np.ascontiguousarray(images, dtype=np.uint8)
        n, h, w = imgs.shape
        _check(_lib.orbgpu_upload_images_async(self.ctx.handle, _p(imgs), n, w, h, w))
        # the current batch keeps its size until run() switches to the staged one: counts(),
        # match_stereo() etc. issued before that still refer to the current batch
        self._staged = (n, h, w)

    def pinned(self, shape):
        """A uint8 numpy array over page-locked host memory.  The memory is freed by free_pinned()
        or close() (or when the extractor is collected); the array must not be used after that."""
        nbytes = int(np.prod(shape))
        ptr = C.c_void_p()
        _check(_lib.orbgpu_host_alloc(nbytes, C.byref(ptr)))
        self._pinned.append(ptr)
        buf = (C.c_uint8 * nbytes).from_address(ptr.value)
        return np.frombuffer(buf, np.uint8).reshape(shape)

    def free_pinned(self):
        """Frees every pinned() buffer (after the staged uploads that read them have landed)."""
        if self._pinned and self.ctx.handle:
            _check(_lib.orbgpu_synchronize(self.ctx.handle))
        for ptr in self._pinned:
            _lib.orbgpu_host_free(ptr)
        self._pinned = []

    def run(self, laps=None, stream=None):
        if self._staged is not None:  # the batch upload_async staged becomes the current one
            self.n, self.height, self.width = self._staged
            self._staged = None
        n = self.n
        lp = None
        if laps is not None:
            lp = np.ascontiguousarray(laps, dtype=np.int32).reshape(n, 2)
        _check(_lib.orbgpu_run_batch(self.ctx.handle, n, self.width, self.height,
                                     _p(lp) if lp is not None else None,
                                     C.c_void_p(stream) if stream else None))

    def run_match(self, laps=None, stereo_rows_only=False, stream=None):
        """run() then match_stereo() over every pair as one submission when the batch is one
        captured graph (orbgpu_run_batch_match; the latency shape)."""
        if self._staged is not None:
            self.n, self.height, self.width = self._staged
            self._staged = None
        n = self.n
        lp = None
        if laps is not None:
            lp = np.ascontiguousarray(laps, dtype=np.int32).reshape(n, 2)
        _check(_lib.orbgpu_run_batch_match(self.ctx.handle, n, self.width, self.height,
                                           _p(lp) if lp is not None else None, int(stereo_rows_only),
                                           C.c_void_p(stream) if stream else None))

    def match_stereo(self, stereo_rows_only=False, stream=None):
        _check(_lib.orbgpu_match_stereo_batch(self.ctx.handle, self.n // 2, int(stereo_rows_only),
                                              C.c_void_p(stream) if stream else None))

    def synchronize(self):
        _check(_lib.orbgpu_synchronize(self.ctx.handle))

    def counts(self):
        n = np.zeros(self.n, np.int32)
        m = np.zeros(self.n, np.int32)
        _check(_lib.orbgpu_download_counts(self.ctx.handle, self.n, _p(n), _p(m)))
        return n, m

    def candidate_counts(self):
        """Keys that entered DistributeOctTree per image (all levels) in the last run()."""
        c = np.zeros(self.n, np.int32)
        _check(_lib.orbgpu_candidate_counts(self.ctx.handle, self.n, _p(c)))
        return c

    def result(self, i, cap=65536):
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n, m = C.c_int(0), C.c_int(0)
        _check(_lib.orbgpu_download_result(self.ctx.handle, i, _p(kps), _p(desc), cap, C.byref(n),
                                           C.byref(m)))
        return kps[:n.value], desc[:n.value], m.value

    def matches(self, pair, cap=65536):
        out = [np.zeros(cap, np.int32) for _ in range(4)]
        nq = C.c_int(0)
        _check(_lib.orbgpu_download_matches(self.ctx.handle, pair, *[_p(o) for o in out], cap,
                                            C.byref(nq)))
        return tuple(o[:nq.value] for o in out)

    def stereo_matches(self, mbf, mb, stream=None):
        """Frame::ComputeStereoMatches (Frame.cc:827-997) for every pair 2p / 2p+1 of the last
        run(); results stay in HBM (stereo_result)."""
        _check(_lib.orbgpu_stereo_matches_batch(self.ctx.handle, self.n // 2, C.c_float(mbf),
                                                C.c_float(mb), C.c_void_p(stream) if stream else None))

    def stereo_result(self, pair, cap=65536):
        """(mvuRight, mvDepth, sad) of pair `pair`: float32, float32, int32 per left keypoint."""
        ur = np.zeros(cap, np.float32)
        dp = np.zeros(cap, np.float32)
        sad = np.zeros(cap, np.int32)
        n = C.c_int(0)
        _check(_lib.orbgpu_download_stereo(self.ctx.handle, pair, _p(ur), _p(dp), _p(sad), cap,
                                           C.byref(n)))
        return ur[:n.value], dp[:n.value], sad[:n.value]

    def fisheye_stereo(self, rig, stream=None):
        """Frame::ComputeStereoFishEyeMatches (Frame.cc:1142-1201) for every pair 2p / 2p+1 of the
        last run(): the stereo-row kNN2 (matches() returns it afterwards) and the KannalaBrandt8
        triangulation (rig: KB8Rig); results stay in HBM (fisheye_result)."""
        _check(_lib.orbgpu_fisheye_stereo_batch(self.ctx.handle, self.n // 2, C.byref(rig),
                                                C.c_void_p(stream) if stream else None))

    def fisheye_result(self, pair, cap=65536):
        """dict(l2r, r2l, depth, p3d, n_matches) of pair `pair` (mvLeftToRightMatch,
        mvRightToLeftMatch, mvDepth, mvStereo3Dpoints)."""
        l2r = np.zeros(cap, np.int32)
        r2l = np.zeros(cap, np.int32)
        dp = np.zeros(cap, np.float32)
        p3 = np.zeros((cap, 3), np.float32)
        nl, nr, nm = C.c_int(0), C.c_int(0), C.c_int(0)
        _check(_lib.orbgpu_download_fisheye(self.ctx.handle, pair, _p(l2r), _p(r2l), _p(dp), _p(p3), cap,
                                            C.byref(nl), C.byref(nr), C.byref(nm)))
        return dict(l2r=l2r[:nl.value], r2l=r2l[:nr.value], depth=dp[:nl.value], p3d=p3[:nl.value],
                    n_matches=nm.value)

    def upload_sbs(self, frames, width=None):
        """Side-by-side stereo Y8 frames [n, H, S] (row stride S >= 2W; W = S // 2 by default) ->
        images 2f (left half) and 2f + 1 (right half) of the batch (ORBextractor.cc:131-143)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        n, h, stride = frames.shape
        w = stride // 2 if width is None else int(width)
        _check(_lib.orbgpu_upload_sbs(self.ctx.handle, _p(frames), n, w, h, stride))
        self.n, self.height, self.width = 2 * n, h, w
        self._staged = None

    def ingest_sbs(self, device_ptr, n_frames, stride, stream=None):
        """Split side-by-side frames already in device memory (zero-copy ingest)."""
        _check(_lib.orbgpu_ingest_sbs(self.ctx.handle, C.c_void_p(device_ptr), int(n_frames), self.width,
                                      self.height, int(stride), C.c_void_p(stream) if stream else None))
        self.n = 2 * int(n_frames)
        self._staged = None

    def pack_soa(self, n_pairs=None, stream=None):
        """The orbslam3.idl SoA layout for every image (and n_pairs stereo pairs' matches)."""
        npairs = self.n // 2 if n_pairs is None else int(n_pairs)
        _check(_lib.orbgpu_pack_soa(self.ctx.handle, self.n, npairs, C.c_void_p(stream) if stream else None))

    def soa_result(self, image, cap=65536):
        """dict(x, y, angle, level: int32 [n], orb: uint8 [n, 32], mono: int)."""
        a = {k: np.zeros(cap, np.int32) for k in ("x", "y", "angle", "level")}
        orb = np.zeros((cap, 32), np.uint8)
        n, m = C.c_int(0), C.c_int(0)
        _check(_lib.orbgpu_download_soa(self.ctx.handle, image, _p(a["x"]), _p(a["y"]), _p(a["angle"]),
                                        _p(a["level"]), _p(orb), cap, C.byref(n), C.byref(m)))
        out = {k: v[:n.value] for k, v in a.items()}
        out["orb"] = orb[:n.value]
        out["mono"] = m.value
        return out

    def matches16(self, pair, cap=65536):
        """(indices, distances1, distances2) int16 of stereo pair `pair` after pack_soa."""
        r = [np.zeros(cap, np.int16) for _ in range(3)]
        n = C.c_int(0)
        _check(_lib.orbgpu_download_matches16(self.ctx.handle, pair, _p(r[0]), _p(r[1]), _p(r[2]), cap,
                                              C.byref(n)))
        return tuple(a[:n.value] for a in r)

    @staticmethod
    def _map_point_rows(map_points):
        """(points, offsets, n_frames) for the C ABI: map_points is either a list (one per frame)
        of MAP_POINT_DTYPE arrays, concatenated here, or a tuple (points, offsets) already in the
        ABI's form -- every frame's points in one MAP_POINT_DTYPE array and int32 offsets [n + 1] --
        which is passed through without a host copy."""
        if isinstance(map_points, tuple):
            mps, off = map_points
            mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
            off = np.ascontiguousarray(off, np.int32)
            if off.ndim != 1 or len(off) < 1 or off[0] != 0 or off[-1] != len(mps) or np.any(np.diff(off) < 0):
                raise ValueError("map point offsets must start at 0, not decrease and end at len(points)")
            return mps, off, len(off) - 1
        nf = len(map_points)
        mps = np.ascontiguousarray(np.concatenate([np.asarray(m, MAP_POINT_DTYPE) for m in map_points])
                                   if nf else np.zeros(0, MAP_POINT_DTYPE))
        off = np.zeros(nf + 1, np.int32)
        off[1:] = np.cumsum([len(m) for m in map_points])
        return mps, off, nf

    def search_by_projection(self, map_points, image_step=2, use_uright=True, kp_block=None, th=1.0,
                             nnratio=0.8, far_points=False, th_far=50.0, stream=None):
        """ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints)
        (ORBmatcher.cc:44-214) for frames f = images f * image_step after undistort_grid();
        map_points: list (one per frame) of MAP_POINT_DTYPE arrays, or (points, offsets) with every
        frame's points in one array (_map_point_rows); kp_block: optional list of u8 arrays (1 =
        keypoint already holds a map point with observations)."""
        mps, off, nf = self._map_point_rows(map_points)
        blk, stride = None, 0
        if kp_block is not None:
            stride = max(1, max(len(b) for b in kp_block))
            blk = np.zeros((nf, stride), np.uint8)
            for f, b in enumerate(kp_block):
                blk[f, :len(b)] = b
        _check(_lib.orbgpu_search_by_projection_batch(
            self.ctx.handle, nf, int(image_step), int(use_uright), _p(mps) if len(mps) else None, _p(off),
            _p(blk) if blk is not None else None, stride, C.c_float(th), C.c_float(nnratio),
            int(far_points), C.c_float(th_far), C.c_void_p(stream) if stream else None))

    def search_by_projection_stereo(self, map_points, left_to_right=None, right_to_left=None, kp_block=None,
                                    th=1.0, nnratio=0.8, far_points=False, th_far=50.0, stream=None):
        """The two-camera SearchByProjection (Nleft != -1, ORBmatcher.cc:59-214) on every stereo
        pair of the last run() (grids from undistort_grid(K, ())); left_to_right / right_to_left:
        per pair int32 arrays (mvLeftToRightMatch / mvRightToLeftMatch); kp_block per pair over
        Nleft + Nright keypoints; map_points as for search_by_projection."""
        mps, off, nf = self._map_point_rows(map_points)

        def rows(lst, dtype, fill):
            if lst is None:
                return None, 0
            stride = max(1, max(len(x) for x in lst))
            out = np.full((nf, stride), fill, dtype)
            for f, x in enumerate(lst):
                out[f, :len(x)] = x
            return out, stride
        l2r, lrs = rows(left_to_right, np.int32, -1)
        r2l, lrs2 = rows(right_to_left, np.int32, -1)
        if l2r is not None and r2l is not None and lrs != lrs2:
            w = max(lrs, lrs2)
            l2r = np.pad(l2r, ((0, 0), (0, w - lrs)), constant_values=-1)
            r2l = np.pad(r2l, ((0, 0), (0, w - lrs2)), constant_values=-1)
            lrs = w
        lrs = lrs or lrs2
        blk, bst = rows(kp_block, np.uint8, 0)
        _check(_lib.orbgpu_search_by_projection_stereo(
            self.ctx.handle, nf, _p(mps) if len(mps) else None, _p(off),
            _p(l2r) if l2r is not None else None, _p(r2l) if r2l is not None else None, lrs,
            _p(blk) if blk is not None else None, bst, C.c_float(th), C.c_float(nnratio), int(far_points),
            C.c_float(th_far), C.c_void_p(stream) if stream else None))

    def projection_matches(self, frame, cap=65536):
        """(match [n_kp] int32: map point index or -1, nmatches) of frame `frame`."""
        m = np.zeros(cap, np.int32)
        n, nm = C.c_int(0), C.c_int(0)
        _check(_lib.orbgpu_download_projection_matches(self.ctx.handle, frame, _p(m), cap, C.byref(n),
                                                       C.byref(nm)))
        return m[:n.value], nm.value

    def undistort_grid(self, K, dist=(), stream=None):
        """Frame::UndistortKeyPoints + AssignFeaturesToGrid (Frame.cc:405-436, 741-825) for every
        image of the last run(); K = (fx, fy, cx, cy), dist = (k1, k2, p1, p2[, k3])."""
        Kf = np.ascontiguousarray(K, dtype=np.float32)
        d = np.ascontiguousarray(dist, dtype=np.float32)
        _check(_lib.orbgpu_undistort_grid_batch(self.ctx.handle, self.n, _p(Kf), _p(d) if len(d) else None,
                                                len(d), C.c_void_p(stream) if stream else None))

    def grid_result(self, image, cap=65536):
        """(xy_un [n,2], cell [n], cell_start [3073], cell_idx) of image `image`."""
        xy = np.zeros((cap, 2), np.float32)
        cell = np.zeros(cap, np.int32)
        cs = np.zeros(64 * 48 + 1, np.int32)
        ci = np.zeros(cap, np.int32)
        n = C.c_int(0)
        _check(_lib.orbgpu_download_grid(self.ctx.handle, image, _p(xy), _p(cell), _p(cs), _p(ci), cap,
                                         C.byref(n)))
        return xy[:n.value], cell[:n.value], cs, ci[:cs[-1]]

    def set_profiling(self, on=True, stages=None, serialize=False):
        """on: bracket every stage's launches with HIP events; stages: only these stage names;
        serialize: launch each stage once over the whole batch (clean per-kernel durations)."""
        names = [_lib.orbgpu_stage_name(i).decode() for i in range(_lib.orbgpu_num_stages())]
        if not on:
            arg = C.c_int(0)
        elif stages is None and not serialize:
            arg = C.c_int(1)
        else:
            mask = 0
            for st in (names if stages is None else stages):
                mask |= 1 << names.index(st)
            word = (1 << 31) | (1 << 30 if serialize else 0) | mask
            arg = C.c_int(word - (1 << 32))  # the flag word as a signed int
        _check(_lib.orbgpu_set_profiling(self.ctx.handle, arg))

    def reset_stage_times(self):
        _check(_lib.orbgpu_reset_stage_times(self.ctx.handle))

    def stage_times(self):
        ns = _lib.orbgpu_num_stages()
        ms = np.zeros(ns, np.float64)
        cnt = np.zeros(ns, np.int64)
        _check(_lib.orbgpu_stage_times(self.ctx.handle, _p(ms), _p(cnt), ns))
        return {_lib.orbgpu_stage_name(i).decode(): (float(ms[i]), int(cnt[i])) for i in range(ns)}
