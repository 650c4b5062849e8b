"""Host stand-in for the parts of orbslam3lib_amd that bench.py's headline leg calls, for the CPU
test of `bench.py --gpus N --stub-gpu` (tests/test_bench_multirank.py): the rank launch, the
rendezvous, the barrier-bracketed timing, the max / sum reductions and the C5 exchange run for
real; the extraction is replaced by fixed per-image counts and seeded random descriptors.  Never
imported by the product path; bench.py labels its line data: "stub"."""
from __future__ import annotations

import numpy as np

_STAGE = "k_fast_cells<48>"


class BatchExtractor:
    device_resident = False  # dist.cross_camera_match_device keeps host buffers for this one

    def __init__(self, nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7, device=0,
                 width=640, height=480, max_images=128):
        self.nfeatures, self.device = int(nfeatures), int(device)
        self.width, self.height, self.max_images = int(width), int(height), int(max_images)
        self.n = 0
        self._prof, self._serial, self._times = False, False, {}

    def upload(self, images):
        self.n, self.height, self.width = images.shape
        self._seed = int(images[:, ::37, ::41].sum()) % 100000

    def upload_async(self, images):
        self.upload(images)

    def pinned(self, shape):
        return np.zeros(shape, np.uint8)

    def free_pinned(self):
        pass

    def close(self):
        pass

    def _count(self, i):
        return 40 + (self._seed + 7 * i) % 13

    def run(self, laps=None, stream=None):
        if self._prof:
            ms, cnt = self._times.get(_STAGE, (0.0, 0))
            self._times[_STAGE] = (ms + 0.01, cnt + (1 if self._serial else 3))

    def match_stereo(self, stereo_rows_only=False, stream=None):
        pass

    def run_match(self, laps=None, stereo_rows_only=False, stream=None):
        self.run(laps, stream)
        self.match_stereo(stereo_rows_only, stream)

    def synchronize(self):
        pass

    def counts(self):
        n = np.array([self._count(i) for i in range(self.n)], np.int32)
        return n, np.zeros(self.n, np.int32)

    def candidate_counts(self):
        return 5 * self.counts()[0]

    def result(self, i, cap=65536):
        n = self._count(i)
        desc = np.random.default_rng(self._seed + i).integers(0, 256, (n, 32), dtype=np.uint8)
        return np.zeros(n), desc, n

    def knn_match(self, query, train):
        q = np.unpackbits(np.asarray(query, np.uint8).reshape(-1, 32), axis=1).astype(np.int32)
        t = np.unpackbits(np.asarray(train, np.uint8).reshape(-1, 32), axis=1).astype(np.int32)
        d = q @ (1 - t).T + (1 - q) @ t.T  # Hamming distances [nq, nt]
        key = d.astype(np.int64) * (1 << 16) + np.arange(t.shape[0])[None, :]
        order = np.argsort(key, axis=1, kind="stable")[:, :2]
        i1, i2 = order[:, 0], (order[:, 1] if t.shape[0] > 1 else np.full(len(q), -1))
        r = np.arange(len(q))
        d1 = d[r, i1]
        d2 = d[r, i2] if t.shape[0] > 1 else np.full(len(q), 0x7FFFFFFF)
        return (i1.astype(np.int32), d1.astype(np.int32), np.asarray(i2, np.int32), np.asarray(d2, np.int32))

    def ingest_images(self, ptr, n, stride=None, stream=None):
        import ctypes
        stride = stride or self.width
        a = np.ctypeslib.as_array((ctypes.c_uint8 * (n * self.height * stride)).from_address(ptr))
        self.upload(a.reshape(n, self.height, stride)[:, :, :self.width].copy())

    def _export(self, n_img, n_pairs):
        """The packed orbgpu_export_batch layout over the stub's results (zero keypoints)."""
        from orbslam3lib_amd import KEYPOINT_DTYPE, encode_export
        images = []
        for i in range(n_img):
            d = self.result(i)[1]
            images.append((np.zeros(len(d), KEYPOINT_DTYPE), d, len(d)))  # mono = n, as result()
        pairs = [self.knn_match(images[2 * p][1], images[2 * p + 1][1]) for p in range(n_pairs)]
        return encode_export(images, pairs)

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

    def set_profiling(self, on=True, stages=None, serialize=False):
        self._prof, self._serial = bool(on), bool(serialize)

    def reset_stage_times(self):
        self._times = {}

    def stage_times(self):
        return dict(self._times)
