// orb_fast_tile.h -- FAST-9 of one 128 x 32 pyramid tile while its window is in LDS (device only).
//
// The pyramid kernels (k_blur_resize, and k_blur for the last level) stage a 160 x 40 window of
// level s around each 128 x 32 tile to blur it (and resize level s + 1 from it).  The cell loop of
// ComputeKeyPointsOctTree (cpp/src/ORBextractor_old.cc:807-871, cv::FAST(cell, kps, iniThFAST,
// true)) is restated per pixel on that same window, so the level is not read again:
//   * every pixel of the level's detection area [19, w - 19) x [19, h - 19) (the union of the
//     cells' detection regions [iniX + 3, iniX + cols - 3), EDGE_THRESHOLD = 19) gets the
//     threshold-independent FAST strength m (orb_math.h: corner at t <=> m > t, cornerScore =
//     m - 1), computed only for pixels that pass the compass pre-test at iniThFAST;
//   * the 3x3 nonmax of FAST_t<16> at iniThFAST runs on the tile core: a corner is kept when
//     m >= 2 and m exceeds every 8-neighbour that is a corner of the SAME cell (cv::FAST sees
//     only the cell's own pixels: neighbours across a cell border count as 0).  Cell borders are
//     where (x - 19) mod wCell == 0 / (y - 19) mod hCell == 0 (the cells' detection regions tile
//     the detection area); the one-pixel ring around the core gets its strength too, so the
//     nonmax at the tile edge sees its neighbours;
//   * the tile writes KS(x, y) = m for kept corners, 0 elsewhere, into the level's KS plane.
// k_fast_gather then walks each cell's detection region of KS in row-major order (the emission
// order of cv::FAST) and writes the cell's keys; a cell that kept nothing at iniThFAST is redone
// at minThFAST by k_fast_cells (:845-861), the per-cell kernel of orb_fast_cell.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_fast_cell.h"
#include "orb_kernels.h"
#include "orb_math.h"

namespace orbgpu {

constexpr int kFtW = 128, kFtH = 32;             // tile core (= the blur tile)
constexpr int kFtPitch = 160;                    // window pitch: columns tx0 - 16 .. tx0 + 143
constexpr int kFtPitchDw = kFtPitch / 4;
constexpr int kFtRow0 = 4, kFtCol0 = 16;         // core (0, 0) in the window
// strength tile: the core and a one-pixel ring, window pitch; S(r, c) at (r + 1) * 160 + c + 4
constexpr int kFtSRows = kFtH + 2;
constexpr int kFtSOff = (kFtRow0 - 1) * kFtPitch + kFtCol0 - 4;  // window offset - S offset
// compass items: dword groups q in [-1, 33) of rows r in [-1, 33) (the core and its ring)
constexpr int kFtItemsX = kFtW / 4 + 2, kFtItemsY = kFtH + 2;
constexpr int kFtItems = kFtItemsX * kFtItemsY;
constexpr int kFtIters = (kFtItems + 255) / 256;        // per thread (256-thread workgroups)
constexpr int kFtListPerWave = kFtIters * 64 * 4;        // candidate capacity of a wave's list
constexpr int kFtListBytes = 4 * kFtListPerWave * 2;     // 4 waves, u16 entries
static_assert(kFtSOff == 492, "strength tile offset");

struct FastTileSmem {
    uint8_t S[kFtSRows * kFtPitch];  // strength m of corners at iniThFAST, 0 elsewhere
    uint8_t colf[kFtW];              // bit 0: first column of a cell, bit 1: last column
    uint8_t rowf[kFtH];              // bit 0: first row of a cell, bit 1: last row
};

// FAST of tile (tx0, ty0) of level G.  win: the staged window (160 x 40 bytes, row 0 = ty0 - 4,
// column 0 = tx0 - 16); list: kFtListBytes of LDS free for the whole call (the blur's row-pair
// buffer); the window is free for reuse once the strengths are in (the KS tile is built in it).
// ks: this image's KS plane of level G (pitch G.bpitch).  Call with all 256 threads, after the
// last use of `list`'s memory by the caller (the function begins with writes to fs, then a
// barrier); ends after its last LDS access with every thread's global stores issued.
__device__ inline void fast_tile(const LevelGeom& G, int tx0, int ty0, int t, uint8_t* win, uint16_t* list,
                                 FastTileSmem& fs, uint8_t* ks) {
    const int tid = (int)threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // (a) cell borders of the core's columns / rows, and a zero strength tile
    if (tid < kFtW) {
        const int b = (tx0 + tid - 19 + G.wCell) % G.wCell;  // x >= 0 > 19 - wCell
        fs.colf[tid] = (uint8_t)((b == 0 ? 1 : 0) | (b == G.wCell - 1 ? 2 : 0));
    } else if (tid < kFtW + kFtH) {
        const int b = (ty0 + tid - kFtW - 19 + G.hCell) % G.hCell;
        fs.rowf[tid - kFtW] = (uint8_t)((b == 0 ? 1 : 0) | (b == G.hCell - 1 ? 2 : 0));
    }
    for (int i = tid; i < kFtSRows * kFtPitch / 16; i += 256) reinterpret_cast<uint4*>(fs.S)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // (b) compass pre-test at t, 4 pixels per lane, candidates into this wave's list (any order)
    const uint32_t* W32 = reinterpret_cast<const uint32_t*>(win);
    uint16_t* L = list + w * kFtListPerWave;
    const uint32_t tt = (uint32_t)t * 0x00010001u;
    const int xlo = 19, xhi = G.w - 19, ylo = 19, yhi = G.h - 19;
    auto rank = [](uint64_t b) {
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    };
    int na = 0;
#pragma unroll
    for (int k = 0; k < kFtIters; ++k) {
        const int i = w * 64 + lane + 256 * k;
        uint32_t m4 = 0;
        int o = 0;
        if (i < kFtItems) {
            const int ir = (int)(((float)i + 0.5f) * (1.0f / (float)kFtItemsX));  // exact: i < 1156
            const int r = ir - 1, q = i - ir * kFtItemsX - 1;
            const int dw = (r + kFtRow0) * kFtPitchDw + q + kFtCol0 / 4;
            const int x0 = tx0 + 4 * q, y = ty0 + r;
            // pixels of the core and its ring inside the detection area
            const int lo = max(max(xlo - x0, 0), q < 0 ? 3 : 0);
            const int hi = min(min(xhi - x0, 4), q >= kFtW / 4 ? 1 : 4);
            if (y >= ylo && y < yhi && hi > lo) {
                m4 = fw_compass4(W32[dw], W32[dw - 1], W32[dw + 1], W32[dw - 3 * kFtPitchDw], W32[dw + 3 * kFtPitchDw], tt);
                m4 &= ((1u << hi) - 1u) & ~((1u << lo) - 1u);
            }
            o = 4 * dw;
        }
        const int c = __builtin_popcount(m4);
        const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
        int pos = na + rank(b0) + 2 * rank(b1) + 4 * rank(b2);
        // unconditional stores: the slots past this lane's candidates go to a sink, the wave's
        // last entry (no exec-mask juggling per pixel).  A wave's items hold at most 320 x 4
        // pixels less the ring items' (one pixel each, at least 18 of them), so no candidate
        // ever lands on the sink
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool on = (m4 >> j) & 1u;
            L[on ? pos : kFtListPerWave - 1] = (uint16_t)(o + j);
            pos += on ? 1 : 0;
        }
        na += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the list is read by other lanes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (c) exact strength of every candidate; corners (m > t) into the strength tile and, in
    // place, to the front of the list
    const uint64_t lt = (1ull << lane) - 1ull;
    int nb = 0;
    for (int base = 0; base < na; base += 64) {
        const int j = base + lane;
        const int o = L[j < na ? j : 0];
        const int m = fast_strength_packed<kFtPitch>(win + o);
        const bool f = j < na && m > t;
        const uint64_t bm = __ballot(f);
        if (f) {
            L[nb + __popcll(bm & lt)] = (uint16_t)o;
            fs.S[o - kFtSOff] = (uint8_t)m;
        }
        nb += __popcll(bm);
    }
    __syncthreads();  // every strength in the tile; the window is free
    // (d) the KS tile (core, pitch 128) in the window's memory: zero, then the kept corners
    uint8_t* kst = win;
    reinterpret_cast<uint4*>(kst)[tid] = make_uint4(0, 0, 0, 0);  // 256 x 16 B = 128 x 32
    __syncthreads();
    for (int base = 0; base < nb; base += 64) {
        const int j = base + lane;
        if (j < nb) {
            const int s = (int)L[j] - kFtSOff;  // strength-tile offset
            const int r1 = (int)(((float)s + 0.5f) * (1.0f / (float)kFtPitch));  // exact: s < 5440
            const int r = r1 - 1, c = s - r1 * kFtPitch - 4;
            if (r >= 0 && r < kFtH && c >= 0 && c < kFtW) {
                const uint8_t* S = fs.S + s;
                const int v = S[0];
                const int cf = fs.colf[c], rf = fs.rowf[r];
                // neighbours across a cell border are not in the cell's FAST image: 0
                const int lm = (cf & 1) ? 0 : 255, rm = (cf & 2) ? 0 : 255;
                const int um = (rf & 1) ? 0 : 255, dm = (rf & 2) ? 0 : 255;
                const int q0 = S[-kFtPitch - 1] & lm & um, q1 = S[-kFtPitch] & um, q2 = S[-kFtPitch + 1] & rm & um;
                const int q3 = S[-1] & lm, q4 = S[1] & rm;
                const int q5 = S[kFtPitch - 1] & lm & dm, q6 = S[kFtPitch] & dm, q7 = S[kFtPitch + 1] & rm & dm;
                const int mx = imax(imax(imax(q0, q1), imax(q2, q3)), imax(imax(q4, q5), imax(q6, q7)));
                if (v >= 2 && v > mx) kst[r * kFtW + c] = (uint8_t)v;
            }
        }
    }
    __syncthreads();
    // (e) the KS tile to the plane (16-byte stores; rows past the level, chunks past the pitch
    // are not stored)
    const int rr = tid >> 3, cc = tid & 7;
    if (ty0 + rr < G.h && tx0 + 16 * cc < G.bpitch)
        *reinterpret_cast<uint4*>(ks + (long long)(ty0 + rr) * G.bpitch + tx0 + 16 * cc) =
            reinterpret_cast<const uint4*>(kst)[tid];
}

}  // namespace orbgpu
