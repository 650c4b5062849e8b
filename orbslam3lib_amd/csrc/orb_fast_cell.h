// orb_fast_cell.h -- one FAST cell of ComputeKeyPointsOctTree as a data-parallel program.
//
// Restates cpp/src/ORBextractor_old.cc:807-871 with cv::FAST(cell, kps, th, nonmax=true)
// (OpenCV FAST_t<16>): detection on [3,rows-3)x[3,cols-3) of the cell ROI, 3x3 nonmax that
// sees only this cell's corners, iniThFAST first and minThFAST if the cell kept nothing, keys
// emitted in row-major order relative to (minBorderX, minBorderY).
//
// Layout: the ROI is staged in LDS with a compile-time pitch P (64 when every level's cells fit,
// kCellMax = 80 otherwise).  On the GPU one wave runs one cell (no workgroup barriers); the
// code also accepts several waves per cell: each wave owns one contiguous row-major range of
// detection pixels and keeps a private candidate list, so the wave lists concatenated in wave
// order are row-major and ordered output needs only a prefix over waves.  Per threshold t:
// (1) the antipodal-pair pre-test (fw_pretest4) on 4 pixels per lane, passing pixels compacted
// into the wave list; (2) the exact strength m (orb_math.h fast_strength_packed) of every
// candidate, m > t being the segment test itself; (3) the 3x3 nonmax over the corners.
// Policy-templated like orb_octree.h so the host harness runs the same code on the CPU.
#pragma once
#ifndef FAST_THREADS
// k_fast_cells workgroup: one wave per cell.  Round 5 (single stream, 512 images, k_fast_cells<48>):
// 2 waves per cell 678-684 us, 1 wave 648-664 us, 1 wave with the fixed-size policy 652-654 us
#define FAST_THREADS 64
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_math.h"
#include "orb_octree.h"

namespace orbgpu {

constexpr int kCellMax = 80;  // wCell, hCell < 70 (nCols = floor(W/35)) plus the 6-px overlap
constexpr int kCellPitchSmall = 64;  // 640x480-class pyramids: every level's cells <= 55 x 58
constexpr int kCellPitchTiny = 48;   // the leading levels of 640x480-class pyramids (cells <= 39 x 42)
#ifndef FAST_THREADS_64
// k_fast_cells<64>: two waves per cell.  Its cells are the largest of 640x480-class pyramids
// (up to 55 x 58) and its launch is short, so one wave per cell left it latency-bound (0.54
// VALU busy).  Round 5, single stream, 512 images: 1 wave 107.3 us, 2 waves 94.1, 4 waves 99.3;
// headline +0.9% (bench A/B, 3 rounds).
#define FAST_THREADS_64 128
#endif
// k_fast_cells<CP> workgroup size
template <int CP>
__host__ __device__ constexpr int fast_threads() { return CP == kCellPitchSmall ? FAST_THREADS_64 : FAST_THREADS; }
// candidate list capacity for pitch P: the detection area, (P-6)^2 for the 64-byte tile, 69^2
// for the general one (wCell, hCell <= 69: nCols = floor(W/35) >= 1)
template <int P>
constexpr int cell_list_cap() { return P == kCellMax ? 69 * 69 : (P - 6) * (P - 6); }

struct CellGeom {
    int iniX, iniY;   // cell ROI origin in level coordinates
    int rows, cols;   // ROI size (already clipped to maxBorder)
    int minBorder;
};

// M holds m for corners, 0 elsewhere (pitch P).  Nonmax at t: kept <=> m > t, m >= 2 and no
// neighbour q with q > t and q >= m; given m > t, q >= m already implies q > t, so the
// neighbour test is max(q) < m -- nine loads issued together, no short-circuit chain.
template <int P>
__host__ __device__ inline bool fast_kept(const uint8_t* M, int off, int t) {
    const uint8_t* m = &M[off];
    const int v = m[0];
    const int q0 = m[-P - 1], q1 = m[-P], q2 = m[-P + 1], q3 = m[-1];
    const int q4 = m[1], q5 = m[P - 1], q6 = m[P], q7 = m[P + 1];
    const int a = imax(imax(q0, q1), imax(q2, q3)), b = imax(imax(q4, q5), imax(q6, q7));
    return (v > t) & (v >= 2) & (imax(a, b) < v);
}

typedef unsigned short fw_u16x2 __attribute__((ext_vector_type(2)));

__device__ inline fw_u16x2 fw_as16(uint32_t x) { return __builtin_bit_cast(fw_u16x2, x); }
__device__ inline uint32_t fw_as32(fw_u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// Pre-test of the 4 pixels of LDS dword C, device only: byte k of the result is 0x80 when, for
// each of the four antipodal pairs of ring points {0,8}, {2,10}, {4,12}, {6,14}, one point of the
// pair is darker than v-t (or, for all four pairs, one point is brighter than v+t), 0 otherwise.
// Any 9-arc of the 16-point ring holds one point of every antipodal pair, so a FAST corner at t
// passes (a necessary condition; the exact strength decides).  On the SURVEY 8d frames 26% of
// the detection pixels pass at iniThFAST (the 4-point compass {0,8} x {4,12} of rounds 1-3
// passed 43%; corners 14%).
// Inputs: row 0 (C and the dwords left / right of it: Cm, Cp), rows -3 / +3 (U3, D3: the same
// column only), rows -2 / +2 with both neighbours (U2m, U2, U2p; D2m, D2, D2p); kt = 255 - t and
// tt = t in both u16 halves.
// All four pixels are compared at once, one byte each (SWAR): v_lerp_u8 averages bytes, so with
// nlo = ~lo, lo = sat(v - t):  (p + nlo + 1) >> 1 >= 128  <=>  p >= lo  (not darker), and with
// nhi = ~hi, hi = sat(v + t):  (p + nhi) >> 1 >= 128  <=>  p > hi  (brighter): one instruction
// per ring point and side, bit 7 of each byte.  lo / hi come from 16-bit halves (v_perm split,
// clamped v_pk_sub_u16) -- 40 VALU per 4 pixels where the packed-16-bit form took ~62.
// Returns {dark, bright}: 0x80 in the bytes whose pixel passed on that side.
__device__ inline uint2 fw_pretest4(uint32_t C, uint32_t Cm, uint32_t Cp, uint32_t U3, uint32_t D3,
                                    uint32_t U2m, uint32_t U2, uint32_t U2p, uint32_t D2m, uint32_t D2,
                                    uint32_t D2p, uint32_t tt, uint32_t kt) {
    const uint32_t L3 = __builtin_amdgcn_alignbyte(C, Cm, 1);    // (-3, 0): ring 12
    const uint32_t R3 = __builtin_amdgcn_alignbyte(Cp, C, 3);    // (+3, 0): ring 4
    const uint32_t UL = __builtin_amdgcn_alignbyte(U2, U2m, 2);  // (-2, -2): ring 10
    const uint32_t UR = __builtin_amdgcn_alignbyte(U2p, U2, 2);  // (+2, -2): ring 6
    const uint32_t DL = __builtin_amdgcn_alignbyte(D2, D2m, 2);  // (-2, +2): ring 14
    const uint32_t DR = __builtin_amdgcn_alignbyte(D2p, D2, 2);  // (+2, +2): ring 2
    // bytes 0, 2 and 1, 3 of C as u16 halves
    const fw_u16x2 E = fw_as16(__builtin_amdgcn_perm(0u, C, 0x0c020c00u));
    const fw_u16x2 O = fw_as16(__builtin_amdgcn_perm(0u, C, 0x0c030c01u));
    const fw_u16x2 T2 = fw_as16(tt), K2 = fw_as16(kt);
    // lo = sat(v - t); nhi = ~sat(v + t) = sat(255 - t - v); both repacked to bytes
    const uint32_t loE = fw_as32(__builtin_elementwise_sub_sat(E, T2)), loO = fw_as32(__builtin_elementwise_sub_sat(O, T2));
    const uint32_t nhE = fw_as32(__builtin_elementwise_sub_sat(K2, E)), nhO = fw_as32(__builtin_elementwise_sub_sat(K2, O));
    const uint32_t nlo = ~__builtin_amdgcn_perm(loO, loE, 0x06020400u);
    const uint32_t nhi = __builtin_amdgcn_perm(nhO, nhE, 0x06020400u);
    auto nd = [&](uint32_t p) { return __builtin_amdgcn_lerp(p, nlo, 0x01010101u); };  // bit 7: p >= lo
    auto br = [&](uint32_t p) { return __builtin_amdgcn_lerp(p, nhi, 0u); };          // bit 7: p > hi
    // dark: every pair has a point < lo  <=>  no pair has both points >= lo (the 3-input OR as
    // v_bitop3_b32, a full-rate op, where the compiler's v_or3_b32 issues at the slow rate:
    // profiles/r06/valu_rates.json)
    const uint32_t x = __builtin_amdgcn_bitop3_b32(nd(R3) & nd(L3), nd(D3) & nd(U3), nd(DR) & nd(UL), 0xfe) |
                       (nd(UR) & nd(DL));
    // bright: every pair has a point > hi
    uint32_t y = br(R3) | br(L3);
    y = (br(D3) | br(U3)) & y;
    y = (br(DR) | br(UL)) & y;
    y = (br(UR) | br(DL)) & y;
    return make_uint2(~x & 0x80808080u, y & 0x80808080u);
}

// Per-cell scratch (LDS on the GPU).
struct CellScratch {
    uint8_t* T;        // [P * P], 4-byte aligned
    uint8_t* M;        // [P * P], 4-byte aligned
    uint16_t* list;    // [cell_list_cap<P>() + fast_list_slack(waves)] wave-private candidate
                       // lists (offsets into T/M) and the sink entries
    int32_t* wcnt;     // [waves]
    // device only (fast_cell_tables): per 4-bit pre-test mask, the positions of its set bits as
    // u16 pairs (p0 | p1 << 16, p2 | p3 << 16), and the detection-pixel mask of each dword group
    const uint2* lut = nullptr;  // [16]
    const uint32_t* emask = nullptr;  // [ng <= 20]: 0x80 in the bytes of detection pixels
    int32_t* wovf = nullptr;          // [waves]: capped lists, a wave's overflow flag
};

// List entries past cell_list_cap on the device: each wave's list is followed by 4 spare
// entries (the compaction writes 4 slots per lane, the ones past the lane's candidates are
// overwritten by later lanes or land in the spare entries), then 4 sink entries.
__host__ __device__ constexpr int fast_list_slack(int waves) { return 4 * waves + 4; }

// The positions of the set bits of every 4-bit pre-test mask as u16 pairs (p0 | p1 << 16,
// p2 | p3 << 16): a constant table, copied to LDS per workgroup (one load per lane, not the ~45
// VALU per wave of building it).
struct FastLutTable {
    uint32_t v[32];
};
constexpr FastLutTable make_fast_lut() {
    FastLutTable t{};
    for (int m = 0; m < 16; ++m) {
        uint32_t pos[4] = {0, 0, 0, 0};
        int n = 0;
        for (int k = 0; k < 4; ++k)
            if ((m >> k) & 1) pos[n++] = (uint32_t)k;
        t.v[2 * m] = pos[0] | (pos[1] << 16);
        t.v[2 * m + 1] = pos[2] | (pos[3] << 16);
    }
    return t;
}
__constant__ FastLutTable c_fast_lut = make_fast_lut();

// Builds CellScratch's lut / emask tables (threads < 16 and < ng); the caller syncs before
// fast_cell_detect.
template <int CP>
__device__ inline void fast_cell_tables(const CellGeom& g, int sh, uint2* lut, uint32_t* emask) {
    const int tid = threadIdx.x;
    if (tid < 16) lut[tid] = make_uint2(c_fast_lut.v[2 * tid], c_fast_lut.v[2 * tid + 1]);
    const int dc = g.cols - 6 > 0 ? g.cols - 6 : 0;
    const int xs = 3 + sh, xe = 3 + sh + dc;
    const int g0 = xs >> 2;
    const int ng = dc > 0 ? ((xe - 1) >> 2) - g0 + 1 : 0;
    if (tid < ng) {  // the first and last groups' masks are workgroup-uniform (scalar)
        auto bytes = [](uint32_t m4) {
            return (m4 & 1u ? 0x80u : 0u) | (m4 & 2u ? 0x8000u : 0u) | (m4 & 4u ? 0x800000u : 0u) |
                   (m4 & 8u ? 0x80000000u : 0u);
        };
        const uint32_t first = bytes(0xFu & ~((1u << (xs - 4 * g0)) - 1u));
        const uint32_t last = bytes((1u << (xe - 4 * (g0 + ng - 1))) - 1u);
        emask[tid] = (tid == 0 ? first : 0x80808080u) & (tid == ng - 1 ? last : 0x80808080u);
    }
}

// Stages the cell ROI in LDS (T) and clears the strength plane (M); the caller syncs.
template <int CP, class Pol, class Ld16>
__host__ __device__ void fast_cell_stage(Pol& p, const uint8_t* src, long long pitch, int sh,
                                         bool dword_ok, const CellGeom& g, const CellScratch& cs,
                                         Ld16 ld16) {
    const int tid = p.tid(), NT = p.nthreads();
    const int rows = g.rows, cols = g.cols;
    uint8_t* T = cs.T;
    uint8_t* M = cs.M;
    constexpr int RW = CP / 4;  // dwords per LDS row (constant divisors only)
    if (CP % 16 == 0 && dword_ok) {
        // 16-byte row chunks (ld16: bounds-checked load of 16 bytes at src + offset; bytes past
        // the ROI row are loaded but never read)
        constexpr int RQ = CP / 16;
        const int nq = (sh + cols + 15) >> 4;
        uint4* T128 = reinterpret_cast<uint4*>(T);
        uint4* M128 = reinterpret_cast<uint4*>(M);
        // the first kIt chunks per thread are all loaded before any is stored, so their round
        // trips overlap (a rolled load -> wait -> store loop pays one round trip per chunk);
        // kIt covers every chunk at fast_threads<CP>() threads (the device's workgroup), the loop after it the rest
        constexpr int kIt = (CP * RQ + fast_threads<CP>() - 1) / fast_threads<CP>();
        uint4 v[kIt];
#pragma unroll
        for (int k = 0; k < kIt; ++k) {
            const int i = tid + k * NT, r = i / RQ, q = i % RQ;
#if defined(__HIP_DEVICE_COMPILE__)  // rows < 2^8, pitch < 2^24: one full-rate 24-bit multiply
            if (i < rows * RQ && q < nq) v[k] = ld16((int)__umul24((uint32_t)r, (uint32_t)pitch) + 16 * q);
#else
            if (i < rows * RQ && q < nq) v[k] = ld16((long long)r * pitch + 16 * q);
#endif
        }
#pragma unroll
        for (int k = 0; k < kIt; ++k) {
            const int i = tid + k * NT, q = i % RQ;
            if (i < rows * RQ && q < nq) {
                T128[i] = v[k];
                M128[i] = make_uint4(0, 0, 0, 0);
            }
        }
        for (int i = tid + kIt * NT; i < rows * RQ; i += NT) {
            const int r = i / RQ, q = i % RQ;
            if (q < nq) {
                T128[i] = ld16((long long)r * pitch + 16 * q);
                M128[i] = make_uint4(0, 0, 0, 0);
            }
        }
    } else if (dword_ok) {
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
        for (int i = tid; i < rows * CP; i += NT) {
            const int r = i / CP, c = i % CP;
            if (c < cols) {
                T[r * CP + c + sh] = src[(long long)r * pitch + c];
                M[r * CP + c + sh] = 0;
            }
        }
    }
}

// The detection pixels are split into one contiguous row-major range per wave, so the wave
// lists concatenated in wave order are row-major: ordered output needs only a prefix over waves.
// Runs on a staged ROI (fast_cell_stage + sync); returns the cell's kept count.
// kCap: the candidate list's capacity.  Below cell_list_cap<CP>() (one wave per cell only: the
// small-list k_fast_cells<48>, whose 1 KB list lets 27 instead of 19 workgroups share a CU) a
// pre-test pass whose candidates would not fit returns kFastOverflow before writing past the
// list, and the cell is redone by the full-list kernel.
constexpr int kFastOverflow = -1;
template <int CP, int kCap = cell_list_cap<CP>(), class Pol>
__host__ __device__ int fast_cell_detect(Pol& p, int sh, const CellGeom& g, int ini_th, int min_th,
                                         const CellScratch& cs, uint32_t* keys_out) {
    static_assert(kCap <= cell_list_cap<CP>(), "list capacity");
    constexpr bool kCapped = kCap < cell_list_cap<CP>();
    const int rows = g.rows, cols = g.cols;
    uint8_t* T = cs.T;
    uint8_t* M = cs.M;
    const int dr = rows - 6 > 0 ? rows - 6 : 0;
    const int dc = cols - 6 > 0 ? cols - 6 : 0;
    const int nd = dr * dc;
    (void)nd;
    const int tini = ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th);
    const int tmin = min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th);
    const int W = p.nwaves(), w = p.wave(), L = p.wave_width(), lane = p.lane();
    (void)lane;
#if defined(__HIP_DEVICE_COMPILE__)
    // device: the pre-test takes 4 pixels per lane (fw_pretest4); a wave owns a contiguous
    // row-major range of (row, dword group) items, and its list starts after the detection
    // pixels of the items before it
    const int xs = 3 + sh, xe = 3 + sh + dc;
    const int g0 = xs >> 2;
    const int ng = dc > 0 ? ((xe - 1) >> 2) - g0 + 1 : 0;
    const int items = dr * ng;
    const int j0 = w * items / W, j1 = (w + 1) * items / W;
    // v_rcp_f32 (1 ulp): every quotient below is (k + 0.5) / ng with k < 1500, at least 0.5 / ng
    // (>= 0.025) from an integer, far beyond the error -- the floors are exact
    const float inv_ng = ng > 0 ? __builtin_amdgcn_rcpf((float)ng) : 0.f;
    auto pix_before = [&](int j) {  // detection pixels of the items before item j
        if (ng == 0) return 0;
        const int r = (int)(((float)j + 0.5f) * inv_ng), q = j - __mul24(r, ng);
        const int c = 4 * (g0 + q) - xs;
        return __mul24(r, dc) + (c < 0 ? 0 : (c > dc ? dc : c));
    };
    const int i0 = pix_before(j0);
    (void)lane;
#else
    const int i0 = w * nd / W, i1 = (w + 1) * nd / W;  // nd <= 4900, W <= 16: no overflow
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    // 4 spare entries after each wave's list; a capped list gives each wave kCap / W entries
    const int capw = kCap / W;
    uint16_t* list = cs.list + (kCapped ? w * capw : i0) + 4 * w;
    uint16_t* sink = cs.list + kCap + 4 * W;  // 4 entries (fast_list_slack)
#else
    uint16_t* list = cs.list + i0;
#endif
#if !defined(__HIP_DEVICE_COMPILE__)
    const float inv_dc = dc > 0 ? 1.f / (float)dc : 0.f;
    auto off_of = [&](int i) {
        const int r = (int)(((float)i + 0.5f) * inv_dc);  // exact: i < 4900, dc < 70
        return (3 + r) * CP + 3 + sh + (i - r * dc);
    };
#endif
    // candidates -> corners at t -> exact strength; returns this wave's corner count
    auto build = [&](int t) {
        int na = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        {
            constexpr int RW = CP / 4;
            const uint8_t* const Tb = T;
            const uint8_t* const Eb = reinterpret_cast<const uint8_t*>(cs.emask);
            auto T32 = [&](int byte_off) { return *reinterpret_cast<const uint32_t*>(Tb + byte_off); };
            const uint32_t tt = (uint32_t)t * 0x00010001u, kt = (uint32_t)(255 - t) * 0x00010001u;
            // this lane's item (row r, dword group q) as byte offsets (qb = 4 q into the edge-mask
            // table, db = 4 dw into T: the LDS addresses themselves, no per-item shift), advanced by
            // L items per iteration without a division: L = dr rows + dq groups (plus one row on wrap)
            int qb = 0, db = 0, dqb = 0, ddb = 0;
            if (ng > 0) {
                const int i = j0 + lane;
                const int r = (int)(((float)i + 0.5f) * inv_ng);  // exact: i < 69 * 19 + 64
                const int q = i - __mul24(r, ng);                 // (24-bit products: full rate)
                qb = 4 * q;
                db = 4 * (__mul24(r + 3, RW) + g0 + q);
                const int dr = (int)(((float)L + 0.5f) * inv_ng);
                const int dq = L - __mul24(dr, ng);
                dqb = 4 * dq;
                ddb = 4 * (__mul24(dr, RW) + dq);
            }
            const int ngb = 4 * ng, wrapb = 4 * (RW - ng);
            for (int base = j0; base < j1; base += L) {
                uint32_t m8 = 0;  // 0x80 per passing pixel
                if (lane < j1 - base) {
                    const uint2 sd = fw_pretest4(T32(db), T32(db - 4), T32(db + 4), T32(db - 12 * RW), T32(db + 12 * RW),
                                                 T32(db - 8 * RW - 4), T32(db - 8 * RW), T32(db - 8 * RW + 4),
                                                 T32(db + 8 * RW - 4), T32(db + 8 * RW), T32(db + 8 * RW + 4), tt, kt);
                    // detection pixels of the row's first / last group
                    m8 = (sd.x | sd.y) & *reinterpret_cast<const uint32_t*>(Eb + qb);
                }
                // the 4-bit pass mask (bit k = byte k) by one v_dot4_u32_u8 of the 0x80 bytes:
                // 128 m4, so m4's 8-byte LUT entry sits at byte offset 128 m4 >> 4 (one shift)
                const uint32_t m4x128 = __builtin_amdgcn_udot4(m8, 0x08040201u, 0u, false);
                const int c = __builtin_popcount(m8);
                // this lane's list position: an inclusive scan of c over the wave by DPP (rows of
                // 16 by row_shr 1 / 2 / 4 / 8, then row_bcast 15 / 31 across rows; 6 v_add_u32_dpp),
                // instead of bit-sliced ballots + 6 v_mbcnt (16 VALU)
                int incl = c;
                incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, true);  // row_shr:1
                incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, true);  // row_shr:2
                incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, true);  // row_shr:4
                incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, true);  // row_shr:8
                incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1, 3
                incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2, 3
                const int wave_total = __builtin_amdgcn_readlane(incl, 63);
                if (kCapped && na + wave_total > capw) {  // wave-uniform
                    na = kFastOverflow;
                    break;
                }
                // the lane's c entries 4 dw + (set bit positions), as u16 pairs from the table,
                // written to 4 consecutive slots from na + incl - c; slots past c hold garbage that
                // a later lane's entry overwrites (its slot index k is smaller, and the slots are
                // written in the order k = 3, 2, 1, 0) or that lands in the wave's spare entries;
                // lanes without candidates write the sink
                const uint2 lv = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(cs.lut) + (m4x128 >> 4));
                const uint32_t e01 = __umul24((uint32_t)db, 0x10001u) + lv.x;  // v_mad_u32_u24
                const uint32_t e23 = __umul24((uint32_t)db, 0x10001u) + lv.y;
                uint16_t* const lw = list + na;  // wave-uniform
                uint16_t* d = c ? lw + (incl - c) : sink;
                d[3] = (uint16_t)(e23 >> 16);
                asm volatile("" ::: "memory");  // keep the slot order (k = 3 .. 0)
                d[2] = (uint16_t)e23;
                asm volatile("" ::: "memory");
                d[1] = (uint16_t)(e01 >> 16);
                asm volatile("" ::: "memory");
                d[0] = (uint16_t)e01;
                na += wave_total;
                qb += dqb;
                db += ddb;
                if (qb >= ngb) {
                    qb -= ngb;
                    db += wrapb;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the list is read by other lanes
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (kCapped && na == kFastOverflow) return kFastOverflow;
        }
#else
        for (int base = i0; base < i1; base += L) {
            const bool in = base + lane < i1;
            const int i = in ? base + lane : i1 - 1;  // tail lanes recompute i1-1
            const int o = off_of(i);
            const uint8_t* c = &T[o];
            const int v = c[0], lo = v - t, hi = v + t;
            const int p0 = c[3 * CP], p4 = c[3], p8 = c[-3 * CP], p12 = c[-3];
            const int p2 = c[2 + 2 * CP], p6 = c[2 - 2 * CP], p10 = c[-2 - 2 * CP], p14 = c[-2 + 2 * CP];
            // the device's pre-test (fw_pretest4): for each antipodal pair {0,8}, {2,10}, {4,12},
            // {6,14} one point beyond t on the same side <=> a min/max over the pairs
            const int dk = imax(imax(imin(p0, p8), imin(p4, p12)), imax(imin(p2, p10), imin(p6, p14)));
            const int bk = imin(imin(imax(p0, p8), imax(p4, p12)), imin(imax(p2, p10), imax(p6, p14)));
            const bool cand = in & ((dk < lo) | (bk > hi));
            const uint64_t m = p.ballot(cand);
            if (cand) list[na + p.rank(m)] = (uint16_t)o;
            na += p.popc64(m);
        }
#endif
        // exact strength of every candidate (m > t <=> corner at t), corners kept in order; the
        // next batch's list entries are read one batch ahead (the in-place writes of a batch
        // land below its own start, never on entries not yet read)
        int nb = 0;
        int o_next = na > 0 ? list[lane < na ? lane : na - 1] : 0;
        for (int base = 0; base < na; base += L) {
            const int j = base + lane;
            const int o = o_next;
            if (base + L < na) o_next = list[base + L + lane < na ? base + L + lane : na - 1];
            const int sm = fast_strength_packed<CP>(&T[o]);
            const bool f = j < na && sm > t;
            const uint64_t m = p.ballot(j < na) & p.ballot(sm > t);  // two compares' masks, ANDed on the SALU
            if (f) {
                list[nb + p.rank(m)] = (uint16_t)o;  // in place: never passes the reads
                M[o] = (uint8_t)sm;
            }
            nb += p.popc64(m);
        }
        return nb;
    };
    // nonmax at t for every corner of the list; the verdict is kept in bit 15 of the entry
    // (LDS offsets < 6400 use 13 bits) for the ordered write
    auto count_kept = [&](int nb, int t) {
        int c = 0;
        for (int base = 0; base < nb; base += L) {
            const int j = base + lane;
            const bool in = j < nb;
            const int o = list[in ? j : nb - 1] & 0x1FFF;  // tail lanes re-test the last entry
            const bool k = in & fast_kept<CP>(M, o, t);
            if (in) list[j] = (uint16_t)(o | (k ? 0x8000 : 0));
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
    // a capped list: the workgroup agrees on an overflow of any wave before its next barrier
    auto overflowed = [&](int nbw) {
        if (W == 1) return nbw == kFastOverflow;
        if (lane == 0) cs.wovf[w] = nbw == kFastOverflow ? 1 : 0;
        p.sync();
        int any = 0;
        for (int v = 0; v < W; ++v) any |= cs.wovf[v];
        return any != 0;
    };
    int nb = build(tini);
    if (kCapped && overflowed(nb)) return kFastOverflow;
    p.sync();  // M complete: nonmax reads neighbours owned by other waves
    int2 cb = count_kept(nb, tini);
    int t = tini;
    if (cb.x == 0) {  // the cell kept nothing at iniThFAST: rerun at minThFAST (:845-861)
        t = tmin;
        p.sync();
        if (tmin < tini) {
            nb = build(tmin);
            if (kCapped && overflowed(nb)) return kFastOverflow;
            p.sync();
        }
        cb = count_kept(nb, t);
    }
    int run = 0;
    for (int base = 0; base < nb; base += L) {
        const int j = base + lane;
        const int e = j < nb ? list[j] : 0;
        const bool k = (e & 0x8000) != 0;
        const uint64_t m = p.ballot(k);
        if (k) {
            const int o = e & 0x1FFF;
            const int r = o / CP, c = o % CP - sh;
            const int resp = M[o] - 1;  // cornerScore<16> = m - 1
            keys_out[cb.y + run + p.rank(m)] =
                make_key(g.iniX + c - g.minBorder, g.iniY + r - g.minBorder, resp);
        }
        run += p.popc64(m);
    }
    return cb.x;
}

template <int CP, int kCap = cell_list_cap<CP>(), class Pol, class Ld16>
__host__ __device__ int fast_cell_run(Pol& p, const uint8_t* src, long long pitch, int sh,
                                      bool dword_ok, const CellGeom& g, int ini_th, int min_th,
                                      const CellScratch& cs, uint32_t* keys_out, Ld16 ld16) {
    fast_cell_stage<CP>(p, src, pitch, sh, dword_ok, g, cs, ld16);
    p.sync();
    return fast_cell_detect<CP, kCap>(p, sh, g, ini_th, min_th, cs, keys_out);
}

}  // namespace orbgpu
