"""CPU model of the matrix-core blur (orb_kernels.hip blur_tile_compute_mfma).

The kernel computes the 7x7 GaussianBlur of a 128 x 32 tile (ORBextractor_old.cc:1146-1147,
OpenCV 8U fixed point: 7-tap kernel {18, 34, 48, 56, 48, 34, 18} / 256 per axis, one rounding
(S + 2^15) >> 16 at the end) as two int8 GEMMs on v_mfma_i32_32x32x32_i8.  This test replays its
arithmetic on the CPU with the MFMA operand / result layouts of cdna_hip_programming.md §3
(A: lane (row l & 31, half h) holds K = 16h .. 16h+15; B likewise per column; D: lane holds column
l & 31, rows (g & 3) + 8 (g >> 2) + 4h) and the same constant tables, and checks the output against
the direct integer blur: the bias / plane-split bookkeeping (pixel ^ 0x80, hi / lo planes, the
+2^16 carried in a spare K slot, the bit-7 flip) is exact, not just close.
"""
import numpy as np

G7 = [18, 34, 48, 56, 48, 34, 18]
IW, IH = 160, 40


def _tables():
    b1 = np.zeros((2, 64, 16), np.int64)
    b2 = np.zeros((2, 64, 16), np.int64)
    for k in range(2):
        for l in range(64):
            n, h = l & 31, l >> 5
            for j in range(16):
                d1 = 32 * k + 16 * h + j - (n + 13)
                rho = 32 * k + (j & 3) + 8 * (j >> 2) + 4 * h
                d2 = rho - (n + 1)
                b1[k, l, j] = G7[d1] if 0 <= d1 < 7 else 0
                b2[k, l, j] = G7[d2] if 0 <= d2 < 7 else 0
                if k == 1 and j == 4:
                    b2[k, l, j] = -128
    return b1, b2


def _mfma(a, b, c):
    """v_mfma_i32_32x32x32_i8 on per-lane operands a, b [64][16] and accumulators c [64][16]."""
    am = np.zeros((32, 32), np.int64)
    bm = np.zeros((32, 32), np.int64)
    lanes = np.arange(64)
    for j in range(16):
        am[lanes & 31, 16 * (lanes >> 5) + j] = a[:, j]
        bm[16 * (lanes >> 5) + j, lanes & 31] = b[:, j]
    d = am @ bm
    out = c.copy()
    for g in range(16):
        out[:, g] += d[(g & 3) + 8 * (g >> 2) + 4 * (lanes >> 5), lanes & 31]
    return out


def _i8(x):
    x = np.asarray(x, np.int64) & 255
    return np.where(x >= 128, x - 256, x)


def _mfma_blur(win):
    b1, b2 = _tables()
    lanes = np.arange(64)
    out = np.zeros((32, 128), np.int64)
    for w in range(4):
        planes = []
        for mb in range(2):
            acc = np.zeros((64, 16), np.int64)
            rows = np.minimum(32 * mb + (lanes & 31), IH - 1)
            for k in range(2):
                cols = 32 * w + 32 * k + 16 * (lanes >> 5)
                a = np.stack([_i8(win[rows, cols + j] ^ 0x80) for j in range(16)], axis=1)
                acc = _mfma(a, b1[k], acc)
            u = acc & 0xFFFFFFFF
            hi, lo = _i8(u >> 8), _i8((u & 255) ^ 0x80)
            if mb == 1:  # rows >= 40: unused; slot 4 carries the + 2^16
                hi[:, 4:] = 0
                lo[:, 4:] = 0
                hi[:, 4] = -1
            planes.append((hi, lo))
        ah = np.zeros((64, 16), np.int64)
        al = np.zeros((64, 16), np.int64)
        for mb in range(2):
            ah = _mfma(planes[mb][0], b2[mb], ah)
            al = _mfma(planes[mb][1], b2[mb], al)
        t = ((ah << 8) + al) & 0xFFFFFFFF
        res = ((t >> 16) & 255) ^ 0x80
        for g in range(16):
            x = 32 * w + 8 * (g >> 2) + 4 * (lanes >> 5) + (g & 3)
            out[lanes & 31, x] = res[:, g]
    return out


def _direct_blur(win):
    h = np.zeros((IH, 128), np.int64)
    for dx in range(7):
        h += G7[dx] * win[:, 13 + dx:13 + dx + 128]
    s = np.zeros((32, 128), np.int64)
    for dy in range(7):
        s += G7[dy] * h[1 + dy:1 + dy + 32]
    return (s + (1 << 15)) >> 16


def test_mfma_blur_model_is_exact():
    rng = np.random.default_rng(7)
    for win in (rng.integers(0, 256, (IH, IW)), np.full((IH, IW), 255), np.zeros((IH, IW), np.int64),
                (np.indices((IH, IW)).sum(0) % 2) * 255):
        win = np.asarray(win, np.int64)
        assert np.array_equal(_mfma_blur(win), _direct_blur(win))
