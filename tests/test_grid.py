"""Frame::UndistortKeyPoints + ComputeImageBounds + AssignFeaturesToGrid (cpp/src/Frame.cc:405-436,
741-825): the CPU oracle against an independent Python restatement of cv::undistortPoints
(OpenCV 4.2 cvUndistortPointsInternal: 5 fixed iterations in double, P = K) and of the 64 x 48
grid (CPU), and the gfx950 kernel (orb_frame.hip) against the oracle, bit-exact on the
undistorted positions, cell ids and per-cell keypoint lists (GPU tests).

Parity status: unpinned against the reference itself (Frame.cc needs OpenCV + the SLAM stack; the
reference ships no fixtures for these functions) -- cross-checked restatements only."""
import math

import numpy as np
import pytest

from orbslam3lib_amd import synth

F32 = np.float32
# EuRoC cam0 (the reference's stereo-inertial example calibration): fx, fy, cx, cy; k1 k2 p1 p2
EUROC_K = (458.654, 457.296, 367.215, 248.375)
EUROC_D = (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)


def _py_undistort(u, v, K, d):
    fx, fy, cx, cy = (float(F32(a)) for a in K)
    k = [0.0] * 14
    for i, a in enumerate(d):
        k[i] = float(F32(a))
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = (float(F32(u)) - cx) * ifx
    y = (float(F32(v)) - cy) * ify
    x0, y0 = x, y
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        if icdist < 0:
            x = (float(F32(u)) - cx) * ifx
            y = (float(F32(v)) - cy) * ify
            break
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    return F32(fx * x + cx), F32(fy * y + cy)


def _py_frame(kps, K, d, cols, rows):
    dist_on = len(d) > 0 and F32(d[0]) != 0
    if dist_on:
        xy = np.array([_py_undistort(a, b, K, d) for a, b in zip(kps["x"], kps["y"])], np.float32)
        c = [_py_undistort(a, b, K, d) for a, b in ((0, 0), (cols, 0), (0, rows), (cols, rows))]
        bounds = np.array([min(c[0][0], c[2][0]), max(c[1][0], c[3][0]),
                           min(c[0][1], c[1][1]), max(c[2][1], c[3][1])], np.float32)
    else:
        xy = np.stack([kps["x"], kps["y"]], 1).astype(np.float32)
        bounds = np.array([0, cols, 0, rows], np.float32)
    wi = F32(F32(64) / F32(bounds[1] - bounds[0]))
    hi = F32(F32(48) / F32(bounds[3] - bounds[2]))
    rnd = lambda v: int(math.floor(abs(float(v)) + 0.5)) * (1 if v >= 0 else -1)  # std::round
    cells = [[] for _ in range(64 * 48)]
    cell = np.full(len(kps), -1, np.int32)
    for i, (x, y) in enumerate(xy):
        px, py = rnd(F32(F32(x - bounds[0]) * wi)), rnd(F32(F32(y - bounds[2]) * hi))
        if 0 <= px < 64 and 0 <= py < 48:
            cell[i] = px * 48 + py
            cells[px * 48 + py].append(i)
    cs = np.cumsum([0] + [len(c) for c in cells]).astype(np.int32)
    ci = np.array([i for c in cells for i in c], np.int32)
    return xy, bounds, cell, cs, ci


CASES = [
    (EUROC_K, EUROC_D),                                   # barrel: bounds wider than the image
    (EUROC_K, (0.6, 0.2, 0.001, -0.0008)),               # pincushion: border keypoints leave the grid
    (EUROC_K, (-0.28, 0.07, 0.0, 0.0, 0.012)),            # 5 coefficients (k3)
    (EUROC_K, (-2.0, 0.0, 0.0, 0.0)),                     # icdist < 0 at the corners: the break branch
    (EUROC_K, (0.0, 0.1, 0.01, 0.01)),                    # k1 == 0: no undistortion at all (:765)
    (EUROC_K, ()),                                        # no coefficients
]


@pytest.mark.parametrize("K,d", CASES)
def test_oracle_matches_python_restatement(oracle, K, d):
    img = synth.frame(480, 640, 4)
    kps, _, _ = oracle.extract(img, nfeatures=1500)
    xy, b, cell, cs, ci = oracle.undistort_grid(kps, K, d, 640, 480)
    pxy, pb, pcell, pcs, pci = _py_frame(kps, K, d, 640, 480)
    np.testing.assert_array_equal(b, pb)
    np.testing.assert_array_equal(xy, pxy)
    np.testing.assert_array_equal(cell, pcell)
    np.testing.assert_array_equal(cs, pcs)
    np.testing.assert_array_equal(ci, pci)
    if d == EUROC_D:
        assert b[0] < 0 and b[1] > 640 and (cell >= 0).all()
    if d and d[0] > 0:
        assert (cell < 0).any()


def _gpu_vs_oracle(oracle, imgs, K, d, w=640, h=480, L=8, nf=2000):
    import orbslam3lib_amd as og
    be = og.BatchExtractor(nf, 1.2, L, 20, 7, width=w, height=h, max_images=len(imgs))
    be.upload(np.stack(imgs))
    be.run()
    be.undistort_grid(K, d)
    be.synchronize()
    for i in range(len(imgs)):
        kps, _, _ = be.result(i)
        xy, b, cell, cs, ci = oracle.undistort_grid(kps, K, d, w, h)
        gxy, gcell, gcs, gci = be.grid_result(i)
        np.testing.assert_array_equal(gxy, xy, err_msg="image %d xy_un" % i)
        np.testing.assert_array_equal(gcell, cell, err_msg="image %d cell" % i)
        np.testing.assert_array_equal(gcs, cs, err_msg="image %d cell_start" % i)
        np.testing.assert_array_equal(gci, ci, err_msg="image %d cell_idx" % i)


@pytest.mark.gpu
@pytest.mark.parametrize("K,d", CASES)
def test_gpu_undistort_grid_bit_exact(oracle, K, d):
    imgs = [synth.frame(480, 640, s) for s in range(3)] + [np.zeros((480, 640), np.uint8)]
    _gpu_vs_oracle(oracle, imgs, K, d)


@pytest.mark.gpu
def test_gpu_undistort_grid_1080p_dense(oracle):
    # 5000 features in one image: many keypoints per cell, the chunked stable scatter
    K = (1400.0, 1400.0, 960.0, 540.0)
    _gpu_vs_oracle(oracle, [synth.frame(1080, 1920, 11)], K, (-0.1, 0.02, 0.0005, -0.0003),
                   w=1920, h=1080, L=12, nf=5000)


def test_image_bounds_abi_matches_oracle(oracle):
    """orbgpu_image_bounds is host-only: callable without a device."""
    import ctypes as C

    import orbslam3lib_amd as og
    lib = og.load_library()
    for K, d in CASES:
        Kf = np.ascontiguousarray(K, np.float32)
        df = np.ascontiguousarray(d, np.float32)
        out = np.zeros(4, np.float32)
        assert lib.orbgpu_image_bounds(640, 480, Kf.ctypes.data_as(C.c_void_p),
                                       df.ctypes.data_as(C.c_void_p) if len(df) else None, len(df),
                                       out.ctypes.data_as(C.c_void_p)) == 0
        _, b, _, _, _ = oracle.undistort_grid(np.zeros(0, oracle.KP_DTYPE), K, d, 640, 480)
        np.testing.assert_array_equal(out, b)
