// orb_fast_wave.h -- one FAST cell per wave (gfx950 device code).
//
// Same contract as fast_cell_detect (orb_fast_cell.h): cv::FAST(cell, kps, th, nonmax=true) on
// the cell ROI of ComputeKeyPointsOctTree (cpp/src/ORBextractor_old.cc:807-871), iniThFAST
// first and minThFAST when the cell kept nothing, keys in row-major order.  What changes is the
// compass pre-test: every lane takes 4 horizontally adjacent pixels (one LDS dword) and tests
// them with packed u16 arithmetic (pixels 0/2 and 1/3 in the two halves of a word, built with
// v_perm), so one pass of a wave tests 256 pixels instead of 64; the candidates are compacted in
// row-major order by an exclusive prefix of the per-lane counts (bit-sliced ballots).  The exact
// strength (fast_strength_packed) and the 3x3 nonmax (fast_kept) are those of orb_fast_cell.h.
// A wave owns its cell from staging to output, so no workgroup barrier is involved.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_fast_cell.h"

namespace orbgpu {

// LDS written by some lanes of this wave is read by other lanes after this point.
__device__ inline void fw_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Detection on a staged ROI: T = ROI (pitch CP, ROI column c at LDS column c + sh), M = zeroed
// strength plane, list = candidate list.  Writes the kept keys in row-major order to keys_out
// and returns their count.
template <int CP>
__device__ int fast_cell_wave(const uint8_t* T, uint8_t* M, uint16_t* list, int sh, const CellGeom& g,
                              int ini_th, int min_th, uint32_t* keys_out) {
    constexpr int RW = CP / 4;  // dwords per LDS row
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t lt = (1ull << lane) - 1ull;
    const int rows = g.rows, cols = g.cols;
    const int dr = rows - 6 > 0 ? rows - 6 : 0;
    const int dc = cols - 6 > 0 ? cols - 6 : 0;
    const int tini = ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th);
    const int tmin = min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th);
    // detection LDS columns [xs, xe) of rows 3 .. 3 + dr, covered by dword groups g0 .. g0 + ng
    const int xs = 3 + sh, xe = 3 + sh + dc;
    const int g0 = xs >> 2;
    const int ng = dc > 0 ? ((xe - 1) >> 2) - g0 + 1 : 0;
    const int items = dr * ng;
    const float inv_ng = ng > 0 ? 1.f / (float)ng : 0.f;
    const uint32_t* T32 = reinterpret_cast<const uint32_t*>(T);
    // candidates (row-major) -> corners at t (exact strength, kept in order); returns corners
    auto build = [&](int t) {
        const uint32_t tt = (uint32_t)t * 0x00010001u;
        int na = 0;
        for (int base = 0; base < items; base += 64) {
            const int i = base + lane;
            uint32_t m4 = 0;
            int o = 0;
            if (i < items) {
                const int r = (int)(((float)i + 0.5f) * inv_ng);  // exact: i < 69 * 19, ng <= 19
                const int gg = g0 + (i - r * ng);
                const int dw = (r + 3) * RW + gg;
                m4 = fw_compass4(T32[dw], T32[dw - 1], T32[dw + 1], T32[dw - 3 * RW], T32[dw + 3 * RW], tt);
                const int x0 = 4 * gg;
                const int lo_cut = xs - x0 > 0 ? xs - x0 : 0;
                const int hi_cut = xe - x0 < 4 ? xe - x0 : 4;
                m4 &= ((1u << hi_cut) - 1u) & ~((1u << lo_cut) - 1u);
                o = (r + 3) * CP + x0;
            }
            const int c = __builtin_popcount(m4);
            const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
            int pos = na + __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((m4 >> k) & 1u) list[pos++] = (uint16_t)(o + k);
            na += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        }
        fw_wave_sync();
        int nb = 0;
        for (int base = 0; base < na; base += 64) {
            const int j = base + lane;
            const int o = list[j < na ? j : 0];
            const int sm = fast_strength_packed<CP>(&T[o]);
            const bool f = j < na && sm > t;
            const uint64_t m = __ballot(f);
            if (f) {
                list[nb + __popcll(m & lt)] = (uint16_t)o;  // in place: never passes the reads
                M[o] = (uint8_t)sm;
            }
            nb += __popcll(m);
        }
        fw_wave_sync();  // M complete: the nonmax reads the neighbours other lanes wrote
        return nb;
    };
    // nonmax at t; the verdict goes to bit 15 of the entry (LDS offsets < 6400 use 13 bits)
    auto count_kept = [&](int nb, int t) {
        int cnt = 0;
        for (int base = 0; base < nb; base += 64) {
            const int j = base + lane;
            const bool in = j < nb;
            const int o = list[in ? j : nb - 1] & 0x1FFF;
            const bool k = in && fast_kept<CP>(M, o, t);
            if (in) list[j] = (uint16_t)(o | (k ? 0x8000 : 0));
            cnt += __popcll(__ballot(k));
        }
        fw_wave_sync();
        return cnt;
    };
    int nb = build(tini);
    int cnt = count_kept(nb, tini);
    int t = tini;
    if (cnt == 0) {  // the cell kept nothing at iniThFAST: rerun at minThFAST (:845-861)
        t = tmin;
        if (tmin < tini) nb = build(tmin);
        cnt = count_kept(nb, t);
    }
    int run = 0;
    for (int base = 0; base < nb; base += 64) {
        const int j = base + lane;
        const int e = j < nb ? list[j] : 0;
        const bool k = (e & 0x8000) != 0;
        const uint64_t m = __ballot(k);
        if (k) {
            const int o = e & 0x1FFF;
            const int r = o / CP, c = o % CP - sh;
            const int resp = M[o] - 1;  // cornerScore<16> = m - 1
            keys_out[run + __popcll(m & lt)] = make_key(g.iniX + c - g.minBorder, g.iniY + r - g.minBorder, resp);
        }
        run += __popcll(m);
    }
    return cnt;
}

}  // namespace orbgpu
