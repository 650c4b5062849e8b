"""LDS bank-conflict model of k_fast_cells' two read patterns (orb_fast_cell.h), for choosing the
tile pitch: the pre-test's dword reads (11 per 4-pixel item) and the strength phase's ring-byte
reads (16 per candidate), on level 0 of the SURVEY §8d synthetic 640x480 frames at iniThFAST.

Bank model (MI355X_MICROARCH.md §LDS, ds_read_b32 / ds_read_u8): a wave instruction is served in
two 32-lane groups, bank = (byte address / 4) mod 32, lanes reading the same dword broadcast,
and a group costs as many cycles as the most-loaded bank has distinct dwords.

    python tools/lds_bank_sim.py [pitch ...]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from orbslam3lib_amd import synth  # noqa: E402

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
        (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def group_cycles(dwords, active):
    """cycles of one wave instruction: two 32-lane groups"""
    cyc = 0
    for g in range(2):
        d = dwords[32 * g:32 * g + 32][active[32 * g:32 * g + 32]]
        if d.size == 0:
            continue
        u = np.unique(d)
        cyc += np.bincount(u % 32, minlength=32).max()
        IDEAL[0] += 1
    return cyc


IDEAL = [0]


def cells(w=640, h=480):
    maxbx, maxby = w - 16, h - 16
    width, height = maxbx - 16, maxby - 16
    ncols, nrows = width // 35, height // 35
    wc, hc = -(-width // ncols), -(-height // nrows)
    for i in range(nrows):
        for j in range(ncols):
            iy, ix = 16 + i * hc, 16 + j * wc
            if iy >= maxby - 3 or ix >= maxbx - 6:
                continue
            yield ix, iy, min(iy + hc + 6, maxby) - iy, min(ix + wc + 6, maxbx) - ix


def pretest(img, t):
    im = img.astype(np.int32)
    H, W = im.shape
    pad = np.pad(im, 3)
    def at(dx, dy):
        return pad[3 + dy:3 + dy + H, 3 + dx:3 + dx + W]
    dark = np.ones_like(im, bool)
    bright = np.ones_like(im, bool)
    for k in (0, 2, 4, 6):
        a, b = at(*RING[k]), at(*RING[k + 8])
        dark &= (a < im - t) | (b < im - t)
        bright &= (a > im + t) | (b > im + t)
    return dark | bright


def simulate(pitch, frames, t=20, swz=0):
    pre = strength = 0
    rw = pitch // 4
    for img in frames:
        cand = pretest(img, t)
        for ix, iy, rows, cols in cells():
            sh = ix & 3
            dr, dc = rows - 6, cols - 6
            xs = 3 + sh
            g0 = xs >> 2
            ng = ((xs + dc - 1) >> 2) - g0 + 1
            items = dr * ng
            for wv in range(2):
                j0, j1 = wv * items // 2, (wv + 1) * items // 2
                for base in range(j0, j1, 64):
                    i = np.arange(base, base + 64)
                    act = i < j1
                    r, q = i // ng, i % ng
                    dw = (r + 3) * rw + g0 + q
                    for off in (0, -1, 1, -3 * rw, 3 * rw, -2 * rw - 1, -2 * rw, -2 * rw + 1, 2 * rw - 1, 2 * rw,
                                2 * rw + 1):
                        pre += group_cycles(dw + off, act)
                # this wave's candidates in row-major order (tile byte offsets)
                lst = []
                for j in range(j0, j1):
                    r, q = j // ng, j % ng
                    for b in range(4):
                        c = 4 * (g0 + q) + b  # tile column
                        if c < xs or c >= xs + dc:
                            continue
                        y, x = iy + 3 + r, ix + (c - sh)
                        if cand[y, x]:
                            lst.append((3 + r) * pitch + c)
                lst = np.array(lst, np.int64)
                for b0 in range(0, len(lst), 64):
                    o = lst[b0:b0 + 64]
                    o = np.pad(o, (0, 64 - len(o)))
                    act = np.arange(64) < len(lst) - b0
                    for dx, dy in RING:
                        a = o + dx + dy * pitch
                        dwd = a >> 2
                        if swz:
                            dwd = dwd ^ ((a // pitch) >> swz & 7) * 4
                        strength += group_cycles(dwd, act)
    return pre, strength


def main():
    pitches = [int(p) for p in sys.argv[1:]] or [48, 52, 56, 60, 64, 68, 72, 76, 80]
    frames = [synth.frame(480, 640, k) for k in range(2)]
    for p in pitches:
        IDEAL[0] = 0
        pre, st = simulate(p, frames)
        print("pitch %3d  pre-test %9d cycles  strength %9d cycles  total %9d  (conflict-free %d)"
              % (p, pre, st, pre + st, IDEAL[0]))


if __name__ == "__main__":
    main()
