"""Frame::ComputeStereoFishEyeMatches (Frame.cc:1142-1201) with KannalaBrandt8::TriangulateMatches
(CameraModels/KannalaBrandt8.cpp:300-366).

PARITY UNPINNED (against the reference): the reference triangulates with Eigen::JacobiSVD
(external dependency, not in /root/reference) built by the Android NDK (FMA contraction, Eigen's
evaluation order) and uses the Android libm's atan2f / tanf.  The oracle (oracle/orb_fisheye.cpp)
restates Eigen's JacobiSVD and the camera model in IEEE single without contraction, calling the
host libm (glibc) for atan2f / tanf / cosf / sinf.  The GPU kernel follows the same operation order
and evaluates those four functions with orb_math.h's restatements of glibc's algorithms, which
equal the host libm on their whole domains here (tests/test_host_harness.py,
tools/libm_fisheye_exhaustive.py).  So:
  * CPU: the oracle is checked against float64 ground truth (points projected through the
    KannalaBrandt8 model: depths recovered to 1e-4 relative) and against the reference's control
    flow (dist1 == 0 skipped, dist1 < 70, index checks, last accepted left row per right row).
  * GPU: bit-exact with the oracle -- every decision, mvLeftToRightMatch / mvRightToLeftMatch,
    mvDepth and mvStereo3Dpoints.
"""
import numpy as np
import pytest

from orbslam3lib_amd import synth

# TUM-VI-like KannalaBrandt8 intrinsics re-centred on a 640x480 frame
CAM_L = [250.0, 249.9, 320.5, 240.2, 0.00348238940225, 0.000715034845216, -0.00205323614187, 0.000202936735918]
CAM_R = [249.6, 249.7, 318.9, 241.0, 0.00341, 0.00069, -0.00201, 0.00019]


def _rot(ax, ay, az):
    cx, sx, cy, sy, cz, sz = np.cos(ax), np.sin(ax), np.cos(ay), np.sin(ay), np.cos(az), np.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _project64(cam, X):
    fx, fy, cx, cy, k0, k1, k2, k3 = cam
    r = np.sqrt(X[:, 0] ** 2 + X[:, 1] ** 2)
    th = np.arctan2(r, X[:, 2])
    psi = np.arctan2(X[:, 1], X[:, 0])
    rd = th + k0 * th ** 3 + k1 * th ** 5 + k2 * th ** 7 + k3 * th ** 9
    return np.stack([fx * rd * np.cos(psi) + cx, fy * rd * np.sin(psi) + cy], 1)


def _kps(uv, octave=0):
    from oracle.oracle_py import KP_DTYPE
    k = np.zeros(len(uv), KP_DTYPE)
    k["x"], k["y"] = uv[:, 0], uv[:, 1]
    k["octave"] = octave
    k["size"] = 31.0
    return k


def _rig_dict(R12, t12):
    return dict(cam_left=CAM_L, cam_right=CAM_R, R12=np.asarray(R12, np.float32), t12=list(t12),
                precision_left=1e-6, precision_right=1e-6)


def _sigma2(n=8, f=1.2):
    s = np.ones(n, np.float32)
    for i in range(1, n):
        s[i] = np.float32(s[i - 1] * np.float32(f))
    return (s * s).astype(np.float32)


def test_oracle_recovers_depth_of_projected_points(oracle):
    rng = np.random.default_rng(5)
    R12 = _rot(0.01, -0.02, 0.005)
    t12 = np.array([0.11, 0.002, -0.003])
    n = 400
    Z = rng.uniform(1.0, 5.0, n)  # parallax above the 0.99998 cosine bound for this baseline
    X = np.stack([rng.uniform(-0.9, 0.9, n) * Z, rng.uniform(-0.7, 0.7, n) * Z, Z], 1)
    uv1 = _project64(CAM_L, X).astype(np.float32)
    X2 = (R12.T @ (X - t12).T).T  # camera-2 coordinates: R21 (p - t12)
    uv2 = _project64(CAM_R, X2).astype(np.float32)
    mono = 5  # the first rows are monocular (no stereo search)
    kl = _kps(np.concatenate([np.zeros((mono, 2), np.float32), uv1]))
    kr = _kps(np.concatenate([np.zeros((3, 2), np.float32), uv2]))
    idx1 = np.arange(n, dtype=np.int32)
    dist1 = np.full(n, 17, np.int32)
    r = oracle.fisheye_stereo(kl, mono, kr, 3, idx1, dist1, _rig_dict(R12, t12), _sigma2())
    assert r["n_matches"] == n, np.bincount(r["code"])
    np.testing.assert_array_equal(r["l2r"][:mono], -1)
    np.testing.assert_array_equal(r["l2r"][mono:], np.arange(n) + 3)
    np.testing.assert_array_equal(r["r2l"][3:], np.arange(n) + mono)
    np.testing.assert_allclose(r["depth"][mono:], Z, rtol=1e-4)
    np.testing.assert_allclose(r["p3d"][mono:], X, rtol=1e-4, atol=1e-5)


def test_oracle_control_flow(oracle):
    """dist1 == 0 -> skipped, dist1 >= 70 -> no match, out-of-range index -> skipped, several left
    rows on one right row -> mvRightToLeftMatch keeps the last accepted one, parallax /
    z / reprojection rejections coded."""
    R12 = np.eye(3)
    t12 = np.array([0.1, 0.0, 0.0])
    Z = np.array([2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 500000.0])
    X = np.stack([np.linspace(-1, 1, len(Z)) * 0.3 * Z, np.linspace(0.5, -0.5, len(Z)) * 0.2 * Z, Z], 1)
    uv1 = _project64(CAM_L, X).astype(np.float32)
    uv2 = _project64(CAM_R, X - t12).astype(np.float32)
    kl, kr = _kps(uv1), _kps(uv2)
    idx1 = np.array([0, 1, 2, 3, 9, 2, 6], np.int32)
    dist1 = np.array([0, 69, 70, 12, 12, 30, 5], np.int32)
    r = oracle.fisheye_stereo(kl, 0, kr, 0, idx1, dist1, _rig_dict(R12, t12), _sigma2())
    code = r["code"]
    assert code[0] == 1 and code[2] == 2 and code[4] == 3  # dist 0, dist >= 70, index
    assert code[1] == 10 and code[3] == 10
    assert code[5] == 7  # row 5 against right row 2: reprojection error
    assert code[6] == 4  # point at 500 km: no parallax
    np.testing.assert_array_equal(r["l2r"], [-1, 1, -1, 3, -1, -1, -1])
    assert r["n_matches"] == 2
    # two accepted rows on one right row: the later one wins
    idx1 = np.array([1, 1, 1, 3, 3, 5, 6], np.int32)
    dist1 = np.full(7, 20, np.int32)
    uv2b = uv2.copy()
    kr2 = _kps(uv2b)
    r = oracle.fisheye_stereo(kl, 0, kr2, 0, idx1, dist1, _rig_dict(R12, t12), _sigma2())
    acc = np.flatnonzero(r["code"] == 10)
    for j in np.unique(idx1[acc]):
        assert r["r2l"][j] == acc[idx1[acc] == j].max()


def _near(m, code, eps=1e-4):
    """Is the oracle row's decision within eps of a threshold (cos parallax 0.99998, z > 0,
    reprojection bounds, depth 1e-4)?"""
    c, z1, z2, e1, e2 = m
    near = abs(c - 0.99998) < eps
    near |= np.isfinite(z1) and abs(z1) < eps
    near |= np.isfinite(z2) and abs(z2) < eps
    near |= np.isfinite(e1) and abs(e1) < 1e-2
    near |= np.isfinite(e2) and abs(e2) < 1e-2
    return bool(near)


@pytest.mark.gpu
@pytest.mark.parametrize("rig_kind", ["rectified", "rotated"])
def test_fisheye_stereo_batch_matches_oracle(oracle, rig_kind):
    """The batch path (extraction -> stereo-row kNN2 -> triangulation, 4 pairs) against the
    oracle on the device's own keypoints and kNN2 (both already bit-exact with the oracle)."""
    import orbslam3lib_amd as og
    imgs = synth.stereo_batch(480, 640, 4, first=21)
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=8)
    be.upload(imgs)
    laps = np.array([[0, 640], [0, 640]] * 4, np.int32)  # every keypoint in the stereo rows
    laps[2:4] = [[0, 0], [100, 639]]  # one pair with monocular rows on both sides
    be.run(laps)
    if rig_kind == "rectified":
        R12, t12 = np.eye(3), (0.12, 0.0, 0.0)
    else:
        R12, t12 = _rot(0.004, -0.006, 0.002), (0.12, 0.003, -0.002)
    rig = og.KB8Rig.make(CAM_L, CAM_R, R12, t12)
    be.fisheye_stereo(rig)
    be.synchronize()
    total_acc = total_rej = 0
    for p in range(4):
        g = be.fisheye_result(p)
        kl, dl, ml = be.result(2 * p)
        kr, dr, mr = be.result(2 * p + 1)
        i1, d1, _, _ = be.matches(p)
        ref_knn = oracle.knn2(dl[ml:], dr[mr:])
        np.testing.assert_array_equal(i1, ref_knn[0])
        np.testing.assert_array_equal(d1, ref_knn[1])
        r = oracle.fisheye_stereo(kl, ml, kr, mr, i1, d1, rig.as_dict(), _sigma2())
        # bit-exact: decisions, matches both ways, depths and 3-D points
        np.testing.assert_array_equal(g["l2r"], r["l2r"], err_msg="pair %d l2r" % p)
        np.testing.assert_array_equal(g["r2l"], r["r2l"], err_msg="pair %d r2l" % p)
        np.testing.assert_array_equal(g["depth"].view(np.uint32), r["depth"].view(np.uint32),
                                      err_msg="pair %d depth" % p)
        np.testing.assert_array_equal(g["p3d"].view(np.uint32), r["p3d"].view(np.uint32),
                                      err_msg="pair %d p3d" % p)
        assert g["n_matches"] == r["n_matches"]
        np.testing.assert_array_equal(g["l2r"][:ml], -1)
        total_acc += int((r["code"] == 10).sum())
        total_rej += int(((r["code"] >= 4) & (r["code"] <= 9)).sum())
    print("fisheye %s: accepted %d rejected %d, bit-exact" % (rig_kind, total_acc, total_rej))
    assert total_acc > 100 and total_rej > 0, (total_acc, total_rej)
