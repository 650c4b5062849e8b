// orb_fast_cell.h -- one FAST cell of ComputeKeyPointsOctTree as a data-parallel program.
//
// Restates cpp/src/ORBextractor_old.cc:807-871 with cv::FAST(cell, kps, th, nonmax=true)
// (OpenCV FAST_t<16>): detection on [3,rows-3)x[3,cols-3) of the cell ROI, 3x3 nonmax that
// sees only this cell's corners, iniThFAST first and minThFAST if the cell kept nothing, keys
// emitted in row-major order relative to (minBorderX, minBorderY).  Policy-templated like
// orb_octree.h so the host harness runs the same code on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_math.h"
#include "orb_octree.h"

namespace orbgpu {

constexpr int kCellMax = 80;  // wCell, hCell < 70 (nCols = floor(W/35)) plus the 6-px overlap

struct CellGeom {
    int iniX, iniY;   // cell ROI origin in level coordinates
    int rows, cols;   // ROI size (already clipped to maxBorder)
    int minBorder;
};

// m[] holds fast_strength over the detection region, 0 elsewhere (pitch kCellMax).
__host__ __device__ inline bool fast_kept(const uint8_t* M, int r, int c, int t) {
    const uint8_t* m = &M[r * kCellMax + c];
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

// src points at the ROI origin with row pitch `pitch`; T and M are kCellMax^2 scratch arrays
// (LDS on the GPU); cnt is a shared counter.  Returns the number of keys written to keys_out.
template <class P>
__host__ __device__ int fast_cell_run(P& p, const uint8_t* src, long long pitch, const CellGeom& g,
                                      int ini_th, int min_th, uint8_t* T, uint8_t* M, int* cnt,
                                      uint32_t* keys_out) {
    const int tid = p.tid(), NT = p.nthreads();
    const int rows = g.rows, cols = g.cols;
    for (int i = tid; i < rows * cols; i += NT) {
        const int r = i / cols, c = i % cols;
        T[r * kCellMax + c] = src[(long long)r * pitch + c];
        M[r * kCellMax + c] = 0;
    }
    if (tid == 0) *cnt = 0;
    p.sync();
    const int dr = rows - 6 > 0 ? rows - 6 : 0;
    const int dc = cols - 6 > 0 ? cols - 6 : 0;
    const int nd = dr * dc;
    const int tini = ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th);
    const int tmin = min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th);
    const int tlow = tini < tmin ? tini : tmin;
    for (int i = tid; i < nd; i += NT) {
        const int r = 3 + i / dc, c = 3 + i % dc;
        M[r * kCellMax + c] = (uint8_t)fast_strength(&T[r * kCellMax + c], kCellMax, tlow);
    }
    p.sync();
    int mine = 0;
    for (int i = tid; i < nd; i += NT) mine += fast_kept(M, 3 + i / dc, 3 + i % dc, tini);
    if (mine) p.atomic_add(cnt, mine);
    p.sync();
    const int t = *cnt > 0 ? tini : tmin;
    int carry = 0;
    for (int base = 0; base < nd; base += NT) {
        const int i = base + tid;
        const bool k = i < nd && fast_kept(M, 3 + i / dc, 3 + i % dc, t);
        int tot;
        const int ex = p.scan_excl(k ? 1 : 0, &tot);
        if (k) {
            const int r = 3 + i / dc, c = 3 + i % dc;
            const int resp = M[r * kCellMax + c] - 1;  // cornerScore<16> = m - 1
            keys_out[carry + ex] = make_key(g.iniX + c - g.minBorder, g.iniY + r - g.minBorder, resp);
        }
        carry += tot;
    }
    return carry;
}

}  // namespace orbgpu
