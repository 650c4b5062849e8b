// orb_fast_cell.h -- one FAST cell of ComputeKeyPointsOctTree as a data-parallel program.
//
// Restates cpp/src/ORBextractor_old.cc:807-871 with cv::FAST(cell, kps, th, nonmax=true)
// (OpenCV FAST_t<16>): detection on [3,rows-3)x[3,cols-3) of the cell ROI, 3x3 nonmax that
// sees only this cell's corners, iniThFAST first and minThFAST if the cell kept nothing, keys
// emitted in row-major order relative to (minBorderX, minBorderY).
//
// Layout: the ROI (<= 76 x 78 bytes) is staged in LDS; "lanes" own columns and "row groups"
// own rows (no integer division anywhere).  m = exact FAST strength (orb_math.h) is computed for
// pixels passing the compass pre-test at t_low = min(ini, min), 0 elsewhere (exact for every
// t >= t_low).  Keys are compacted per row (a 64-bit keep mask per row and its popcount), then
// one scan over <= 70 row counts gives every row's output offset.  Policy-templated like
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

// M holds m for pixels passing the pre-test, 0 elsewhere (pitch kCellMax).
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
    a &= a >> 4;  // 8 consecutive from each bit
    a &= m >> 8;  // 9 consecutive
    return (a & 0xFFFFu) != 0;
}

// cv::FAST segment test at threshold t (strict > / <), exact.
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

// Per-cell scratch (LDS on the GPU).
struct CellScratch {
    uint8_t* T;        // [kCellMax * kCellMax], 4-byte aligned
    uint8_t* M;        // [kCellMax * kCellMax], 4-byte aligned
    uint16_t* list;    // [kCellList] wave-private candidate lists (LDS offsets into T/M)
    int32_t* wcnt;     // [waves]
};

constexpr int kCellList = 4900;  // >= detection pixels of a cell (<= 69 x 69)

// The detection pixels are split into one contiguous row-major range per wave, so the wave
// lists concatenated in wave order are row-major: ordered output needs only a prefix over waves.
template <class P>
__host__ __device__ int fast_cell_run(P& p, const uint8_t* src, long long pitch, int sh,
                                      bool dword_ok, const CellGeom& g, int ini_th, int min_th,
                                      const CellScratch& cs, uint32_t* keys_out) {
    const int tid = p.tid(), NT = p.nthreads();
    const int rows = g.rows, cols = g.cols;
    uint8_t* T = cs.T;
    uint8_t* M = cs.M;
    constexpr int RW = kCellMax / 4;  // dwords per LDS row (constant divisors only)
    if (dword_ok) {
        const int ndw = (sh + cols + 3) >> 2;
        uint32_t* T32 = reinterpret_cast<uint32_t*>(T);
        uint32_t* M32 = reinterpret_cast<uint32_t*>(M);
        for (int i = tid; i < rows * RW; i += NT) {
            const int r = i / RW, d = i % RW;
            if (d < ndw) {
                T32[i] = *reinterpret_cast<const uint32_t*>(src + (long long)r * pitch + 4 * d);
                M32[i] = 0;
            }
        }
    } else {
        for (int i = tid; i < rows * kCellMax; i += NT) {
            const int r = i / kCellMax, c = i % kCellMax;
            if (c < cols) {
                T[r * kCellMax + c + sh] = src[(long long)r * pitch + c];
                M[r * kCellMax + c + sh] = 0;
            }
        }
    }
    p.sync();
    const int dr = rows - 6 > 0 ? rows - 6 : 0;
    const int dc = cols - 6 > 0 ? cols - 6 : 0;
    const int nd = dr * dc;
    const int tini = ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th);
    const int tmin = min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th);
    const int W = p.nwaves(), w = p.wave(), L = p.wave_width(), lane = p.lane();
    const uint64_t lt = p.lanemask_lt();
    const int i0 = (int)((long long)w * nd / W), i1 = (int)((long long)(w + 1) * nd / W);
    uint16_t* list = cs.list + i0;
    const float inv_dc = dc > 0 ? 1.f / (float)dc : 0.f;
    auto off_of = [&](int i) {
        const int r = (int)(((float)i + 0.5f) * inv_dc);  // exact: i < 4900, dc < 70
        return (3 + r) * kCellMax + 3 + sh + (i - r * dc);
    };
    // candidates -> corners at t -> exact strength; returns this wave's corner count
    auto build = [&](int t) {
        int na = 0;
        for (int base = i0; base < i1; base += L) {
            const int i = base + lane;
            const int o = i < i1 ? off_of(i) : 0;
            const bool f = i < i1 && fast_compass(&T[o], t);
            const uint64_t m = p.ballot(f);
            if (f) list[na + p.popc64(m & lt)] = (uint16_t)o;
            na += p.popc64(m);
        }
        int nb = 0;
        for (int base = 0; base < na; base += L) {
            const int j = base + lane;
            const int o = j < na ? list[j] : 0;
            const bool f = j < na && fast_corner(&T[o], t);
            const uint64_t m = p.ballot(f);
            if (f) list[nb + p.popc64(m & lt)] = (uint16_t)o;  // in place: never passes the reads
            nb += p.popc64(m);
        }
        for (int j = lane; j < nb; j += L) {
            const int o = list[j];
            M[o] = (uint8_t)fast_strength(&T[o], kCellMax, -1);
        }
        return nb;
    };
    auto count_kept = [&](int nb, int t) {
        int c = 0;
        for (int base = 0; base < nb; base += L) {
            const int j = base + lane;
            const bool k = j < nb && fast_kept(M, list[j], t);
            c += p.popc64(p.ballot(k));
        }
        if (lane == 0) cs.wcnt[w] = c;
        p.sync();
        int tot = 0, before = 0;
        for (int v = 0; v < W; ++v) {
            tot += cs.wcnt[v];
            before += v < w ? cs.wcnt[v] : 0;
        }
        return make_int2(tot, before);
    };
    int nb = build(tini);
    p.sync();  // M complete: nonmax reads neighbours owned by other waves
    int2 cb = count_kept(nb, tini);
    int t = tini;
    if (cb.x == 0) {  // the cell kept nothing at iniThFAST: rerun at minThFAST (:845-861)
        t = tmin;
        p.sync();
        if (tmin < tini) {
            nb = build(tmin);
            p.sync();
        }
        cb = count_kept(nb, t);
    }
    int run = 0;
    for (int base = 0; base < nb; base += L) {
        const int j = base + lane;
        const int o = j < nb ? list[j] : 0;
        const bool k = j < nb && fast_kept(M, o, t);
        const uint64_t m = p.ballot(k);
        if (k) {
            const int r = o / kCellMax, c = o % kCellMax - sh;
            const int resp = M[o] - 1;  // cornerScore<16> = m - 1
            keys_out[cb.y + run + p.popc64(m & lt)] =
                make_key(g.iniX + c - g.minBorder, g.iniY + r - g.minBorder, resp);
        }
        run += p.popc64(m);
    }
    return cb.x;
}

}  // namespace orbgpu
