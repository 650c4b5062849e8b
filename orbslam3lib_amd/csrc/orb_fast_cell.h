// orb_fast_cell.h -- one FAST cell of ComputeKeyPointsOctTree as a data-parallel program.
//
// Restates cpp/src/ORBextractor_old.cc:807-871 with cv::FAST(cell, kps, th, nonmax=true)
// (OpenCV FAST_t<16>): detection on [3,rows-3)x[3,cols-3) of the cell ROI, 3x3 nonmax that
// sees only this cell's corners, iniThFAST first and minThFAST if the cell kept nothing, keys
// emitted in row-major order relative to (minBorderX, minBorderY).
//
// Work is narrowed in three ordered passes so that lanes stay busy:
//   A. compass pre-test at t_low = min(ini, min) (two cyclically adjacent points of {0,4,8,12}
//      beyond t_low, necessary for any 9-arc),
//   B. exact 9-contiguous-arc test at t_low on the 16-bit dark/bright masks,
//   C. exact strength m (orb_math.h) for the survivors only.
// Every pixel not in the final list has m <= t_low <= t, which the nonmax rule treats exactly
// like m = 0, so NMS and compaction only visit the list.  Policy-templated like orb_octree.h so
// the host harness runs the same code on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_math.h"
#include "orb_octree.h"

namespace orbgpu {

constexpr int kCellMax = 80;    // wCell, hCell < 70 (nCols = floor(W/35)) plus the 6-px overlap
constexpr int kCellList = 4900; // >= detection pixels of a cell (<= 69 x 69)

struct CellGeom {
    int iniX, iniY;   // cell ROI origin in level coordinates
    int rows, cols;   // ROI size (already clipped to maxBorder)
    int minBorder;
};

// M holds the exact strength for listed pixels, 0 elsewhere (pitch kCellMax).
__host__ __device__ inline bool fast_kept(const uint8_t* M, int off, int t) {
    const uint8_t* m = &M[off];
    const int v = m[0];
    if (v <= t || v < 2) return false;
    const int nb[8] = {-kCellMax - 1, -kCellMax, -kCellMax + 1, -1, 1,
                       kCellMax - 1,  kCellMax,  kCellMax + 1};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int q = m[nb[k]];
        if (q > t && v <= q) return false;
    }
    return true;
}

__host__ __device__ inline bool fast_compass(const uint8_t* c, int t) {
    const int v = c[0];
    const int p0 = c[3 * kCellMax], p4 = c[3], p8 = c[-3 * kCellMax], p12 = c[-3];
    const int dm = ((v - p0 > t) << 0) | ((v - p4 > t) << 1) | ((v - p8 > t) << 2) | ((v - p12 > t) << 3);
    const int bm = ((p0 - v > t) << 0) | ((p4 - v > t) << 1) | ((p8 - v > t) << 2) | ((p12 - v > t) << 3);
    const int dr = ((dm << 1) | (dm >> 3)) & 15, br = ((bm << 1) | (bm >> 3)) & 15;
    return (dm & dr) || (bm & br);
}

__host__ __device__ inline bool arc9(uint32_t mask16) {
    const uint32_t m = mask16 | (mask16 << 16);
    uint32_t a = m & (m >> 1);
    a &= a >> 2;
    a &= a >> 4;        // 8 consecutive from each bit
    a &= m >> 8;        // 9 consecutive
    return (a & 0xFFFFu) != 0;
}

__host__ __device__ inline bool fast_corner(const uint8_t* c, int t) {
    const int v = c[0];
    uint32_t dm = 0, bm = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int p = c[ring_dx(k) + ring_dy(k) * kCellMax];
        dm |= (uint32_t)(v - p > t) << k;
        bm |= (uint32_t)(p - v > t) << k;
    }
    return arc9(dm) || arc9(bm);
}

// src points at the ROI's first row, at column x_al = iniX & ~3 when dword loads are allowed
// (`sh` = iniX - x_al), else at iniX (sh = 0).  T and M are kCellMax^2 scratch arrays, `list`
// holds kCellList u16 (LDS on the GPU); cnt is a shared counter.  Returns the key count.
template <class P>
__host__ __device__ int fast_cell_run(P& p, const uint8_t* src, long long pitch, int sh,
                                      bool dword_ok, const CellGeom& g, int ini_th, int min_th,
                                      uint8_t* T, uint8_t* M, uint16_t* list, int* cnt,
                                      uint32_t* keys_out) {
    const int tid = p.tid(), NT = p.nthreads();
    const int rows = g.rows, cols = g.cols;
    if (dword_ok) {
        const int ndw = (sh + cols + 3) >> 2;
        uint32_t* T32 = reinterpret_cast<uint32_t*>(T);
        uint32_t* M32 = reinterpret_cast<uint32_t*>(M);
        for (int i = tid; i < rows * ndw; i += NT) {
            const int r = i / ndw, d = i % ndw;
            uint32_t v;
            const uint8_t* s = src + (long long)r * pitch + 4 * d;
            v = *reinterpret_cast<const uint32_t*>(s);
            T32[r * (kCellMax / 4) + d] = v;
            M32[r * (kCellMax / 4) + d] = 0;
        }
    } else {
        for (int i = tid; i < rows * cols; i += NT) {
            const int r = i / cols, c = i % cols;
            T[r * kCellMax + c + sh] = src[(long long)r * pitch + c];
            M[r * kCellMax + c + sh] = 0;
        }
    }
    if (tid == 0) *cnt = 0;
    p.sync();
    const int dr = rows - 6 > 0 ? rows - 6 : 0;
    const int dc = cols - 6 > 0 ? cols - 6 : 0;
    const int nd = dr * dc;
    const int tini = ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th);
    const int tmin = min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th);
    const int tlow = tini < tmin ? tini : tmin;
    auto off_of = [&](int i) { return (3 + i / dc) * kCellMax + 3 + sh + i % dc; };
    // A: compass pre-test over the whole detection region (ordered compaction)
    int na = 0;
    for (int base = 0; base < nd; base += NT) {
        const int i = base + tid;
        const bool f = i < nd && fast_compass(&T[off_of(i)], tlow);
        int tot;
        const int ex = p.scan_excl(f ? 1 : 0, &tot);
        if (f) list[na + ex] = (uint16_t)i;
        na += tot;
    }
    p.sync();
    // B: exact 9-arc test at t_low, compacted in place (writes never pass the reads)
    int nb = 0;
    for (int base = 0; base < na; base += NT) {
        const int j = base + tid;
        int i = 0;
        bool f = false;
        if (j < na) {
            i = list[j];
            f = fast_corner(&T[off_of(i)], tlow);
        }
        int tot;
        const int ex = p.scan_excl(f ? 1 : 0, &tot);
        if (f) list[nb + ex] = (uint16_t)i;
        nb += tot;
    }
    p.sync();
    // C: exact strength of the corners
    for (int j = tid; j < nb; j += NT) {
        const int o = off_of(list[j]);
        M[o] = (uint8_t)fast_strength(&T[o], kCellMax, -1);
    }
    p.sync();
    int mine = 0;
    for (int j = tid; j < nb; j += NT) mine += fast_kept(M, off_of(list[j]), tini);
    if (mine) p.atomic_add(cnt, mine);
    p.sync();
    const int t = *cnt > 0 ? tini : tmin;
    int carry = 0;
    for (int base = 0; base < nb; base += NT) {
        const int j = base + tid;
        int i = 0;
        bool k = false;
        if (j < nb) {
            i = list[j];
            k = fast_kept(M, off_of(i), t);
        }
        int tot;
        const int ex = p.scan_excl(k ? 1 : 0, &tot);
        if (k) {
            const int r = 3 + i / dc, c = 3 + i % dc;
            const int resp = M[off_of(i)] - 1;  // cornerScore<16> = m - 1
            keys_out[carry + ex] = make_key(g.iniX + c - g.minBorder, g.iniY + r - g.minBorder, resp);
        }
        carry += tot;
    }
    return carry;
}

}  // namespace orbgpu
