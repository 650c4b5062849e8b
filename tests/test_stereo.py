"""Frame::ComputeStereoMatches (cpp/src/Frame.cc:827-997): the CPU oracle against an independent
pure-Python restatement (CPU), and the gfx950 kernels (orb_stereo.hip) against the oracle,
bit-exact on mvuRight / mvDepth / SAD (GPU tests).

Parity status: unpinned against the reference itself (Frame.cc needs OpenCV + the SLAM stack and
cannot be built here; the reference ships no fixtures for it) -- the oracle restates the
function line by line and is cross-checked by the Python restatement below."""
import math

import numpy as np
import pytest

from orbslam3lib_amd import synth

F32 = np.float32


def _py_stereo(kl, dl, kr, dr, pl, pr, mbf, mb, scale, inv_scale):
    """Independent restatement in numpy float32 scalars (no FMA: one rounding per op)."""
    nL = len(kl)
    ur = np.full(nL, -1, np.float32)
    dep = np.full(nL, -1, np.float32)
    nrows = pl[0].shape[0]
    rows = [[] for _ in range(nrows)]
    for iR in range(len(kr)):
        r = F32(2.0) * F32(scale[kr["octave"][iR]])
        y = F32(kr["y"][iR])
        for yi in range(int(math.floor(F32(y - r))), int(math.ceil(F32(y + r))) + 1):
            if 0 <= yi < nrows:
                rows[yi].append(iR)
    maxD = F32(F32(mbf) / F32(mb))
    pairs = []
    for iL in range(nL):
        uL, vL, oct_ = F32(kl["x"][iL]), F32(kl["y"][iL]), int(kl["octave"][iL])
        cands = rows[int(vL)]
        if not cands:
            continue
        minU, maxU = F32(uL - maxD), F32(uL - F32(0))
        if maxU < 0:
            continue
        best, bi = 100, 0
        for iR in cands:
            if not (oct_ - 1 <= kr["octave"][iR] <= oct_ + 1):
                continue
            if minU <= kr["x"][iR] <= maxU:
                d = int(np.unpackbits(np.bitwise_xor(dl[iL], dr[iR])).sum())
                if d < best:
                    best, bi = d, iR
        if best >= 75:
            continue
        sf = F32(inv_scale[oct_])
        rnd = lambda v: F32(math.floor(abs(v) + 0.5) * (1 if v >= 0 else -1))  # std::round
        suL, svL, suR0 = rnd(F32(uL * sf)), rnd(F32(vL * sf)), rnd(F32(F32(kr["x"][bi]) * sf))
        W = pl[oct_].shape[1]
        if suR0 < 0 or suR0 + 11 >= W:
            continue
        IL = pl[oct_][int(svL) - 5:int(svL) + 6, int(suL) - 5:int(suL) + 6].astype(np.int32)
        dists = []
        for inc in range(-5, 6):
            c = int(suR0) + inc
            IR = pr[oct_][int(svL) - 5:int(svL) + 6, c - 5:c + 6].astype(np.int32)
            dists.append(F32(np.abs(IL - IR).sum()))
        bestinc = int(np.argmin(dists)) - 5  # first minimum
        if abs(bestinc) == 5:
            continue
        d1, d2, d3 = dists[bestinc + 4], dists[bestinc + 5], dists[bestinc + 6]
        deltaR = F32(F32(d1 - d3) / F32(F32(2.0) * F32(F32(d1 + d3) - F32(F32(2.0) * d2))))
        if deltaR < -1 or deltaR > 1:
            continue
        buR = F32(F32(scale[oct_]) * F32(F32(suR0 + F32(bestinc)) + deltaR))
        disp = F32(uL - buR)
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp = F32(0.01)
                buR = F32(float(uL) - 0.01)
            dep[iL] = F32(F32(mbf) / disp)
            ur[iL] = buR
            pairs.append((int(d2), iL))
    if pairs:
        pairs.sort()
        th = F32(F32(F32(1.5) * F32(1.4)) * F32(pairs[len(pairs) // 2][0]))
        for d, i in pairs:
            if not (F32(d) < th):
                ur[i] = dep[i] = -1
    return ur, dep


def _frame(oracle, seed, shift=12, h=480, w=640, nf=2000):
    L, R = synth.stereo_pair(h, w, seed)
    if shift != 12:  # re-shift the right eye (synth uses 12 px)
        R = np.roll(L, -shift, axis=1)
    kl, dl, _ = oracle.extract(L, nfeatures=nf)
    kr, dr, _ = oracle.extract(R, nfeatures=nf)
    return L, R, kl, dl, kr, dr


def test_oracle_matches_python_restatement(oracle):
    L, R, kl, dl, kr, dr = _frame(oracle, 2)
    pl, pr = oracle.pyramid(L), oracle.pyramid(R)
    mbf, mb = 47.9, float(np.float32(47.9) / np.float32(435.2))
    ur, dep, sad = oracle.stereo_matches(kl, dl, kr, dr, pl, pr, mbf, mb)
    scale, inv_scale, _, _ = oracle.scale_factors()
    pur, pdep = _py_stereo(kl, dl, kr, dr, pl, pr, mbf, mb, scale, inv_scale)
    np.testing.assert_array_equal(ur, pur)
    np.testing.assert_array_equal(dep, pdep)
    assert (ur >= 0).sum() > len(kl) // 3  # the 12 px disparity is found for most keypoints
    ok = ur >= 0
    assert np.abs((kl["x"][ok] - ur[ok]) - 12).max() < 1.0


def _gpu_vs_oracle(oracle, imgs_pairs, mbf, mb, w=640, h=480, L=8, nf=2000):
    import orbslam3lib_amd as og
    n = 2 * len(imgs_pairs)
    be = og.BatchExtractor(nf, 1.2, L, 20, 7, width=w, height=h, max_images=n)
    be.upload(np.stack([im for pr in imgs_pairs for im in pr]))
    be.run()
    be.stereo_matches(mbf, mb)
    be.synchronize()
    for p, (Li, Ri) in enumerate(imgs_pairs):
        kl, dl, _ = be.result(2 * p)
        kr, dr, _ = be.result(2 * p + 1)
        ur, dep, sad = oracle.stereo_matches(kl, dl, kr, dr, oracle.pyramid(Li, 1.2, L),
                                             oracle.pyramid(Ri, 1.2, L), mbf, mb)
        gur, gdep, gsad = be.stereo_result(p)
        np.testing.assert_array_equal(gsad, sad, err_msg="pair %d sad" % p)
        np.testing.assert_array_equal(gur, ur, err_msg="pair %d uRight" % p)
        np.testing.assert_array_equal(gdep, dep, err_msg="pair %d depth" % p)


@pytest.mark.gpu
def test_gpu_stereo_matches_bit_exact(oracle):
    pairs = [synth.stereo_pair(480, 640, s) for s in range(4)]
    L0 = pairs[0][0]
    pairs.append((L0, L0.copy()))                 # zero disparity: the disparity <= 0 branch
    pairs.append((L0, np.roll(L0, -3, axis=1)))   # 3 px disparity
    pairs.append((L0, np.zeros_like(L0)))         # empty right image: no candidates at all
    pairs.append((synth.frame(480, 640, 9), synth.frame(480, 640, 10)))  # unrelated views
    _gpu_vs_oracle(oracle, pairs, 47.9, float(np.float32(47.9) / np.float32(435.2)))


@pytest.mark.gpu
def test_gpu_stereo_matches_narrow_disparity_range(oracle):
    # maxD = mbf / mb = 8 px: the 12 px matches fall outside [minU, maxU] or [minD, maxD)
    pairs = [synth.stereo_pair(480, 640, s) for s in (5, 6)]
    _gpu_vs_oracle(oracle, pairs, 8.0, 1.0)


@pytest.mark.gpu
def test_gpu_stereo_matches_euroc_and_1080p(oracle):
    _gpu_vs_oracle(oracle, [synth.stereo_pair(480, 752, 7)], 47.9, 0.11, w=752, h=480)
    _gpu_vs_oracle(oracle, [synth.stereo_pair(1080, 1920, 8)], 47.9, 0.11, w=1920, h=1080, L=12, nf=5000)
