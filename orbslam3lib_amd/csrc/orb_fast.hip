// orb_fast.hip -- cell FAST of ComputeKeyPointsOctTree (cpp/src/ORBextractor_old.cc:807-871) as
// a dense, threshold-independent pass over bands of cells.
//
// For every detection pixel the FAST strength m (orb_math.h) is computed in registers:
//   m = max(v - A, B - v, 0),  A = min over the 16 cyclic 9-arcs of the arc's maximum,
//                              B = max over the arcs of the arc's minimum,
// so that for ANY threshold t, "FAST corner at t" is m > t and cornerScore<16> = m - 1.  The
// 3x3 nonmax of cv::FAST(cell ROI, ..., nonmax=true) is threshold-independent too: p is kept at
// t iff m > t, m >= 2 and m > m(q) for every 8-neighbour q inside the same cell's detection
// rectangle (a neighbour q with m(q) >= m > t is itself a corner at t; one with m(q) < m never
// suppresses p).  So one pass yields R = (m if m beats its in-cell neighbours else 0) per
// pixel, and the cell loop's iniThFAST / minThFAST fallback (:845-861) becomes a choice of
// comparison at emission: keys are the pixels with R > max(t, 1), t = iniThFAST if the cell has
// any at iniThFAST, else minThFAST.  No pixel is evaluated twice and there is no candidate list.
//
// Work split: one workgroup per (image, band segment) -- a band is one row of cells of a level,
// a segment a run of whole cells of it (up to kFastBandMaxWaves waves wide).  Each lane owns a
// column quad (4 pixels, one dword per row) of the segment and walks the band's rows top to
// bottom; lanes 0 and 63 of a wave are halos that compute the quads beside the wave's 62 owned
// ones (the ring and the nonmax need a neighbour quad on each side).  Row data comes straight
// from HBM / L2 (one dword load per lane and row, issued 7 rows ahead); the neighbour dwords
// arrive by DPP wave shifts, and the 16 ring values of the 4 pixels are 16-bit pairs
// (pixels 0/2 and 1/3) built by v_perm / v_alignbyte from a 7-row window kept in registers.
// The two arc trees of each pair run on biased halves (0x04xx: normal f16 of one exponent, so
// v_pk_maximum3_f16 / v_pk_minimum3_f16 order them as integers).  R goes to an LDS plane of
// the segment; after a barrier, one wave per cell emits its keys in row-major order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "orb_fast_cell.h"
#include "orb_kernels.h"
#include "orb_math.h"
#include "orb_octree.h"

namespace orbgpu {

namespace {

typedef unsigned short fd_u16x2 __attribute__((ext_vector_type(2)));
__device__ inline fd_u16x2 h2(uint32_t x) { return __builtin_bit_cast(fd_u16x2, x); }
__device__ inline uint32_t w32(fd_u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ inline uint32_t pmin(uint32_t a, uint32_t b) { return w32(__builtin_elementwise_min(h2(a), h2(b))); }
__device__ inline uint32_t pmax(uint32_t a, uint32_t b) { return w32(__builtin_elementwise_max(h2(a), h2(b))); }
__device__ inline uint32_t pmin3(uint32_t a, uint32_t b, uint32_t c) { return w32(pk_min3(h2(a), h2(b), h2(c))); }
__device__ inline uint32_t pmax3(uint32_t a, uint32_t b, uint32_t c) { return w32(pk_max3(h2(a), h2(b), h2(c))); }
__device__ inline uint32_t psubs(uint32_t a, uint32_t b) { return w32(__builtin_elementwise_sub_sat(h2(a), h2(b))); }

// wave shifts (DPP wave_shr:1 / wave_shl:1): lane i gets lane i-1's / i+1's value; lane 0 / 63
// keeps `edge`
__device__ inline uint32_t from_left(uint32_t v, uint32_t edge) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ inline uint32_t from_right(uint32_t v, uint32_t edge) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)v, 0x130, 0xF, 0xF, false);
}

// The 8 pair values of one row for the lane's quad x0..x0+3 (biased halves 0x04pp):
// F[d + 3] = (p[x0 + d], p[x0 + d + 2]) for d = -3 .. 4; pixels 0/2 read F[dx + 3], pixels 1/3
// F[dx + 4] for a ring offset dx.
struct Row8 {
    uint32_t f[8];
};
__device__ inline Row8 row_pairs(uint32_t D, uint32_t Dp, uint32_t Dn) {
    constexpr uint32_t K = 0x04040404u;
    Row8 r;
    const uint32_t E = __builtin_amdgcn_perm(K, D, 0x04020400u);    // p0, p2
    const uint32_t O = __builtin_amdgcn_perm(K, D, 0x04030401u);    // p1, p3
    const uint32_t Ep = __builtin_amdgcn_perm(K, Dp, 0x04020400u);  // p-4, p-2
    const uint32_t Op = __builtin_amdgcn_perm(K, Dp, 0x04030401u);  // p-3, p-1
    const uint32_t En = __builtin_amdgcn_perm(K, Dn, 0x04020400u);  // p4, p6
    const uint32_t On = __builtin_amdgcn_perm(K, Dn, 0x04030401u);  // p5, p7
    r.f[0] = Op;                                      // d = -3
    r.f[1] = __builtin_amdgcn_alignbyte(E, Ep, 2);    // d = -2: p-2, p0
    r.f[2] = __builtin_amdgcn_alignbyte(O, Op, 2);    // d = -1: p-1, p1
    r.f[3] = E;                                       // d = 0
    r.f[4] = O;                                       // d = 1
    r.f[5] = __builtin_amdgcn_alignbyte(En, E, 2);    // d = 2: p2, p4
    r.f[6] = __builtin_amdgcn_alignbyte(On, O, 2);    // d = 3: p3, p5
    r.f[7] = En;                                      // d = 4: p4, p6
    return r;
}

// Both arc trees over 16 ring pairs x[k] (fast_strength_packed's pairing of the 16 arcs: arcs
// [2j, 2j+8] and [2j+1, 2j+9] share the 8 points [2j+1, 2j+8]): bmax = max over arcs of the
// arc minimum, amin = min over arcs of the arc maximum.
__device__ inline void arc_trees(const uint32_t (&x)[16], uint32_t& bmax, uint32_t& amin) {
    uint32_t a2[8], b2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a2[j] = pmin(x[2 * j + 1], x[(2 * j + 2) & 15]);
        b2[j] = pmax(x[2 * j + 1], x[(2 * j + 2) & 15]);
    }
    uint32_t a4[8], b4[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a4[j] = pmin(a2[j], a2[(j + 1) & 7]);  // min over [2j+1, 2j+4]
        b4[j] = pmax(b2[j], b2[(j + 1) & 7]);
    }
    uint32_t pr[8], qr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t e0 = x[2 * j], e1 = x[(2 * j + 9) & 15];
        pr[j] = pmin3(a4[j], a4[(j + 2) & 7], pmax(e0, e1));  // max(min arc 2j, min arc 2j+1)
        qr[j] = pmax3(b4[j], b4[(j + 2) & 7], pmin(e0, e1));  // min(max arc 2j, max arc 2j+1)
    }
    bmax = pmax(pmax3(pr[0], pr[1], pr[2]), pmax3(pr[3], pr[4], pmax3(pr[5], pr[6], pr[7])));
    amin = pmin(pmin3(qr[0], qr[1], qr[2]), pmin3(qr[3], qr[4], pmin3(qr[5], qr[6], qr[7])));
}

}  // namespace

// Segment geometry shared by the host record and the device: cells [j0, j1) of cell row i.
// rtab record {level, i, j0, j1}.  FB_WPE (measurement builds): minimum waves per SIMD the
// register allocation must allow.
#ifndef FB_WPE
#define FB_WPE 0
#endif
#if FB_WPE > 0
#define FB_ATTR __attribute__((amdgpu_waves_per_eu(FB_WPE)))
#else
#define FB_ATTR
#endif
template <int NW, bool kDw>
__global__ __launch_bounds__(NW * 64) FB_ATTR void k_fast_bands(BatchArgs a, int rec0, uint32_t nseg_magic) {
    extern __shared__ uint32_t fb_lds[];
    const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    const int irel = gridDim.x == 1 ? wg : (int)__umulhi((uint32_t)wg, nseg_magic);
    const int img = a.img0 + irel;
    const int4 rec = a.rtab[a.fast_band_off + rec0 + (wg - irel * (int)gridDim.x)];
    const int l = rec.x, ci = rec.y, j0 = rec.z, j1 = rec.w;
    const LevelGeom G = a.lv[l];
    int32_t* cnt_out = a.cellcnt + (long long)img * a.cellcnt_img_stride + G.cellcnt_off + ci * G.nCols;
    uint32_t* key_base = a.cellkeys + (long long)img * a.cellkeys_img_stride + G.cellkey_off;
    // the band's rows (:809-815) and the segment's detection columns (:819-825)
    const int iniY = kMinBorder + ci * G.hCell;
    const int maxY = min(iniY + G.hCell + 6, G.maxBY);
    const bool row_skip = iniY >= G.maxBY - 3;
    const int ry0 = iniY + 3, ry1 = maxY - 3;
    auto cell_x0 = [&](int j) { return kMinBorder + j * G.wCell + 3; };  // first detection column
    auto cell_x1 = [&](int j) {                                           // past the last one
        const int iniX = kMinBorder + j * G.wCell;
        return iniX >= G.maxBX - 6 ? cell_x0(j) : min(iniX + G.wCell + 6, G.maxBX) - 3;
    };
    const int xs = cell_x0(j0);
    int xe = xs;
    for (int j = j0; j < j1; ++j) xe = max(xe, cell_x1(j));
    const int qlo = xs >> 2, nq = xe > xs ? ((xe - 1) >> 2) - qlo + 1 : 0;
    const int nrows = row_skip ? 0 : max(ry1 - ry0, 0);
    int* cnt_ini = reinterpret_cast<int*>(fb_lds);              // [j1 - j0]: kept at iniThFAST
    uint32_t* Rp = fb_lds + 16 * ((j1 - j0 + 15) / 16);         // [nrows][nq]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if ((int)threadIdx.x < j1 - j0) cnt_ini[threadIdx.x] = 0;
    if (nrows == 0 || nq == 0) {
        if ((int)threadIdx.x < j1 - j0) cnt_out[j0 + threadIdx.x] = 0;
        return;
    }
    __syncthreads();
    const int tini = min(max(a.ini_th, 0), 255), tmin = min(max(a.min_th, 0), 255);
    // ---- pass 1: R for every pixel of the segment -------------------------------------------
    const int qown = 62 * wave + lane - 1;  // segment quad of this lane (-1 / 62: halos)
    const bool owner = lane >= 1 && lane <= 62 && qown < nq;
    if (62 * wave < nq) {  // waves past the segment's quads only join the emission
        const int x0 = 4 * (qlo + qown);
        // per pixel: its cell (or -1 outside every detection range) and whether its left /
        // right neighbour lies in the same cell
        int cid[6];
#pragma unroll
        for (int k = -1; k < 5; ++k) {
            const int x = x0 + k;
            int c = -1;
            if (x >= xs && x < xe) {
                const int j = (x - kMinBorder - 3) / G.wCell;  // absolute cell column
                if (j >= j0 && j < j1 && x >= cell_x0(j) && x < cell_x1(j)) c = j;
            }
            cid[k + 1] = c;
        }
        auto msk = [](bool b0, bool b1) { return (b0 ? 0xFFFFu : 0u) | (b1 ? 0xFFFF0000u : 0u); };
        auto same = [&](int k, int n) { return cid[k + 1] >= 0 && cid[n + 1] == cid[k + 1]; };
        const bool own_ok = owner;
        const uint32_t mLE = msk(same(0, -1), same(2, 1)), mRE = msk(same(0, 1), same(2, 3));
        const uint32_t mLO = msk(same(1, 0), same(3, 2)), mRO = msk(same(1, 2), same(3, 4));
        const uint32_t mSE = own_ok ? msk(cid[1] >= 0, cid[3] >= 0) : 0u;
        const uint32_t mSO = own_ok ? msk(cid[2] >= 0, cid[4] >= 0) : 0u;
        // the (at most two) cells of this quad, and byte masks of their pixels for the counts
        const int cA = cid[1] >= 0 ? cid[1] : cid[2] >= 0 ? cid[2] : cid[3] >= 0 ? cid[3] : cid[4];
        uint32_t bA = 0, bB = 0;
        int cB = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (cid[k + 1] < 0) continue;
            if (cid[k + 1] == cA) bA |= 0x80u << (8 * k);
            else {
                cB = cid[k + 1];
                bB |= 0x80u << (8 * k);
            }
        }
        if (!own_ok) bA = bB = 0;
        // row loads: own dword and the halo lanes' outer neighbour (lane 0: left, 63: right).
        // Planes with dword-aligned rows load one dword; otherwise (level 0 of an odd-width
        // input) the two aligned dwords around it are funnel-shifted (no unaligned access)
        const uint8_t* plane = a.lvl_base[l] + (long long)img * G.img_stride;
        const int xmax = G.pitch - 4;
        const int xo = min(max(x0, 0), xmax);
        const int xe_ld = min(max(lane == 0 ? x0 - 4 : lane == 63 ? x0 + 4 : x0, 0), xmax);
        auto ld = [&](int y, int x) -> uint32_t {
            const uint8_t* p = plane + (size_t)__mul24(y, G.pitch) + x;
            if constexpr (kDw) {
                return *reinterpret_cast<const uint32_t*>(p);
            } else {
                const uintptr_t u = reinterpret_cast<uintptr_t>(p);
                const uint32_t* q = reinterpret_cast<const uint32_t*>(u & ~(uintptr_t)3);
                return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(u & 3));
            }
        };
        // window of 7 rows (slot (y - ry0 + 3) % 7) and raw loads 7 rows ahead
        Row8 W[7];
        uint32_t rawD[7], rawE[7];
        const int ylast = ry1 + 2;  // last row the ring reads
#pragma unroll
        for (int k = 0; k < 7; ++k) {  // rows ry0-3 .. ry0+3 into the raw buffer (slot k)
            const int y = min(ry0 - 3 + k, ylast);
            rawD[k] = ld(y, xo);
            rawE[k] = ld(y, xe_ld);
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {  // rows ry0-3 .. ry0+2 into the window
            W[k] = row_pairs(rawD[k], from_left(rawD[k], rawE[k]), from_right(rawD[k], rawE[k]));
            const int y = min(ry0 + 4 + k, ylast);  // refill: row ry0-3+k+7
            rawD[k] = ld(y, xo);
            rawE[k] = ld(y, xe_ld);
        }
        // nonmax state (biased m, 0 = outside): m(y-1); H2(y-1); H3(y-2), H3(y-1)
        uint32_t mEp = 0, mOp = 0, h2Ep = 0, h2Op = 0, h3Epp = 0, h3Opp = 0, h3Ep = 0, h3Op = 0;
        uint32_t cntA = 0, cntB = 0;
        const uint32_t tA = (uint32_t)(255 - max(tini, 1)) * 0x01010101u;  // ~T for v_lerp_u8
        auto emit_row = [&](int y, uint32_t h3En, uint32_t h3On) {
            // nonmax of row y (= the previous row): neighbours H3(y-1), H2(y), H3(y+1)
            const uint32_t nE = pmax3(h3Epp, h2Ep, h3En), nO = pmax3(h3Opp, h2Op, h3On);
            const uint32_t one = 0x00010001u;
            const uint32_t kE = pmin(psubs(mEp, nE), one), kO = pmin(psubs(mOp, nO), one);
            // R = m if kept else 0 (unbiased), masked to this lane's detection pixels
            const uint32_t bias = 0x04000400u;
            const uint32_t RE = w32(h2(psubs(mEp, bias)) * h2(kE)) & mSE;
            const uint32_t RO = w32(h2(psubs(mOp, bias)) * h2(kO)) & mSO;
            const uint32_t R = __builtin_amdgcn_perm(RO, RE, 0x06020400u);
            if (owner) Rp[__mul24(y - ry0, nq) + qown] = R;
            // pixels kept at iniThFAST, per cell (bit 7 of each byte: R > max(tini, 1))
            const uint32_t gt = __builtin_amdgcn_lerp(R, tA, 0u);
            cntA += __builtin_popcount(gt & bA);
            cntB += __builtin_popcount(gt & bB);
        };
        // whole blocks of 7 rows (no exit inside the unrolled body); rows past the band are computed
        // from clamped rows and dropped: the first of them closes the last row's nonmax
        const int nblk = nrows / 7 + 1;
        for (int b = 0; b < nblk; ++b) {
#pragma unroll
            for (int u = 0; u < 7; ++u) {
                const int y = ry0 + 7 * b + u;
                // row y + 3 enters the window (slot (u + 6) % 7); its raw slot refills 7 rows ahead
                {
                    const int s = (u + 6) % 7;
                    W[s] = row_pairs(rawD[s], from_left(rawD[s], rawE[s]), from_right(rawD[s], rawE[s]));
                    const int yn = min(y + 10, ylast);
                    rawD[s] = ld(yn, xo);
                    rawE[s] = ld(yn, xe_ld);
                }
                // the 16 ring pairs of pixels 0/2 (E) and 1/3 (O)
                uint32_t xE[16], xO[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const Row8& R8 = W[(u + 3 + ring_dy(k) + 7) % 7];
                    xE[k] = R8.f[ring_dx(k) + 3];
                    xO[k] = R8.f[ring_dx(k) + 4];
                }
                const Row8& C8 = W[(u + 3) % 7];
                uint32_t bE, aE, bO, aO;
                arc_trees(xE, bE, aE);
                arc_trees(xO, bO, aO);
                // m = max(v - A, B - v) on the biased halves (the bias cancels), re-biased
                const uint32_t bias = 0x04000400u;
                const uint32_t vE = C8.f[3], vO = C8.f[4];
                const uint32_t mE = pmax(psubs(vE, aE), psubs(bE, vE)) + bias;
                const uint32_t mO = pmax(psubs(vO, aO), psubs(bO, vO)) + bias;
                // horizontal neighbours inside the pixel's cell (0 = none): pixels 0/2 have
                // (p-1, p1) on the left and (p1, p3) on the right; pixels 1/3 (p0, p2) and (p2, p4)
                const uint32_t mOl = from_left(mO, 0u), mEr = from_right(mE, 0u);
                const uint32_t LE = __builtin_amdgcn_alignbyte(mO, mOl, 2) & mLE, RE = mO & mRE;
                const uint32_t LO = mE & mLO, RO = __builtin_amdgcn_alignbyte(mEr, mE, 2) & mRO;
                const uint32_t h2E = pmax(LE, RE), h2O = pmax(LO, RO);
                const bool inside = y < ry1;
                const uint32_t h3E = inside ? pmax3(LE, mE, RE) : 0u, h3O = inside ? pmax3(LO, mO, RO) : 0u;
                if (y > ry0 && y <= ry1) emit_row(y - 1, h3E, h3O);
                h3Epp = h3Ep;
                h3Opp = h3Op;
                h3Ep = h3E;
                h3Op = h3O;
                h2Ep = h2E;
                h2Op = h2O;
                mEp = mE;
                mOp = mO;
            }
        }
        if (own_ok) {
            if (bA && cntA) atomicAdd(&cnt_ini[cA - j0], (int)cntA);
            if (bB && cntB) atomicAdd(&cnt_ini[cB - j0], (int)cntB);
        }
    }
    __syncthreads();
    // ---- pass 2: each cell's keys in row-major order (one wave per cell) --------------------
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int j = j0 + wave; j < j1; j += NW) {
        const int cx0 = cell_x0(j), cx1 = cell_x1(j);
        const int t = cnt_ini[j - j0] > 0 ? tini : tmin;
        const uint32_t tn = (uint32_t)(255 - max(t, 1)) * 0x01010101u;
        uint32_t* kout = key_base + (long long)(ci * G.nCols + j) * G.cell_cap;
        const int qa = (cx0 >> 2) - qlo, qb = cx1 > cx0 ? ((cx1 - 1) >> 2) - qlo : qa - 1;
        const int cq = qb - qa + 1;
        int run = 0;
        if (cq > 0) {
            const float inv = 1.f / (float)cq;
            for (int base = 0; base < nrows * cq; base += 64) {
                const int it = base + lane;
                const int r = (int)(((float)it + 0.5f) * inv);  // exact: it < 2^16, cq < 1024
                const int q = it - r * cq;
                uint32_t sel = 0;
                int x0 = 0;
                if (it < nrows * cq) {
                    const uint32_t R = Rp[__mul24(r, nq) + qa + q];
                    x0 = 4 * (qlo + qa + q);
                    uint32_t cm = 0;  // bytes of this cell
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (x0 + k >= cx0 && x0 + k < cx1) cm |= 0x80u << (8 * k);
                    sel = __builtin_amdgcn_lerp(R, tn, 0u) & cm;  // bytes with R > max(t, 1)
                }
                const int c = __builtin_popcount(sel);
                const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
                const int pos = run + __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
                if (sel) {
                    const uint32_t R = Rp[__mul24(r, nq) + qa + q];
                    int o = pos;
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (sel & (0x80u << (8 * k))) {
                            const int resp = (int)((R >> (8 * k)) & 0xFFu) - 1;  // cornerScore = m - 1
                            kout[o++] = make_key(x0 + k - kMinBorder, ry0 + r - kMinBorder, resp);
                        }
                }
                run += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
            }
        }
        if (lane == 0) cnt_out[j] = run;
    }
}

// ---------------------------------------------------------------------------------------------
// k_fast_sb: the sparse cell FAST of k_fast_cells (pre-test, strength of the candidates only) with
// k_fast_bands' row walk.  One wave per run of whole cells of one cell row (<= 62 column quads
// plus a halo quad each side).  Lane L owns quad qa - 1 + L and walks the band's rows:
//  * rows arrive as one dword per lane from HBM / L2, 7 rows ahead, into a 7-row register window
//    (the SWAR pre-test reads its 11 dwords from there; neighbours by DPP) and into a 16-row LDS
//    ring (the candidates' ring reads);
//  * pre-test candidates go to a wave FIFO (u16: row slot, byte column) and are evaluated 64 at a
//    time (fast strength on the 16 LDS ring bytes); corners at t put m into an 8-row LDS ring M;
//  * three rows behind, each lane reads its M dword of rows y-1, y, y+1 and keeps the pixels that
//    beat their in-cell neighbours, appending their keys to their cell in row-major order (the
//    wave owns its cells: a per-row prefix over lanes, the cell's start fetched by ds_bpermute,
//    running counts in LDS).
// Cells that keep nothing at iniThFAST are redone at minThFAST by a second walk that emits only
// for them (ORBextractor_old.cc:845-861).
constexpr int kSbRing = 16, kSbMRing = 8, kSbFifo = 512, kSbMaxCells = 8;

__device__ inline int sb_strength(const uint8_t* T, int rs, int col) {
    // ring byte k of the pixel at (row slot rs, byte column col) of the LDS ring
    const int v = T[(rs & (kSbRing - 1)) * 256 + col];
    const uint32_t cv = (uint32_t)(v + kFastBias) + ((uint32_t)(kFastBias - v) << 16);
    orb_u16x2 x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t p = T[((rs + ring_dy(k)) & (kSbRing - 1)) * 256 + col + ring_dx(k)];
        x[k] = __builtin_bit_cast(orb_u16x2, p * 65535u + cv);
    }
    orb_u16x2 a2[8], a4[8], pr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a2[j] = __builtin_elementwise_min(x[2 * j + 1], x[(2 * j + 2) & 15]);
#pragma unroll
    for (int j = 0; j < 8; ++j) a4[j] = __builtin_elementwise_min(a2[j], a2[(j + 1) & 7]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
        pr[j] = pk_min3(a4[j], a4[(j + 2) & 7], __builtin_elementwise_max(x[2 * j], x[(2 * j + 9) & 15]));
    const orb_u16x2 best = __builtin_elementwise_max(pk_max3(pr[0], pr[1], pr[2]),
                                                     pk_max3(pr[3], pr[4], pk_max3(pr[5], pr[6], pr[7])));
    int sc = (int)(best.x > best.y ? best.x : best.y) - kFastBias;
    sc = sc < 0 ? 0 : sc;
    return sc > 255 ? 255 : sc;
}

template <bool kDw>
__global__ __launch_bounds__(64) void k_fast_sb(BatchArgs a, uint32_t nseg_magic) {
    __shared__ uint32_t T32[kSbRing * 64];
    __shared__ uint32_t M32[kSbMRing * 64];
    __shared__ uint16_t fifo[kSbFifo];
    __shared__ uint2 lut[16];
    __shared__ int cnt[kSbMaxCells];
    __shared__ int tail_at[8];
    const uint8_t* Tb = reinterpret_cast<const uint8_t*>(T32);
    uint8_t* Mb = reinterpret_cast<uint8_t*>(M32);
    const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    const int irel = gridDim.x == 1 ? wg : (int)__umulhi((uint32_t)wg, nseg_magic);
    const int img = a.img0 + irel;
    const int4 rec = a.rtab[a.fast_sb_off + (wg - irel * (int)gridDim.x)];
    const int l = rec.x, ci = rec.y, ja = rec.z, jb = rec.w;
    const LevelGeom G = a.lv[l];
    const int lane = threadIdx.x;
    int32_t* cnt_out = a.cellcnt + (long long)img * a.cellcnt_img_stride + G.cellcnt_off + ci * G.nCols;
    uint32_t* key_base = a.cellkeys + (long long)img * a.cellkeys_img_stride + G.cellkey_off +
                         (long long)ci * G.nCols * G.cell_cap;
    const int iniY = kMinBorder + ci * G.hCell;
    const int maxY = min(iniY + G.hCell + 6, G.maxBY);
    const bool row_skip = iniY >= G.maxBY - 3;
    const int ry0 = iniY + 3, ry1 = maxY - 3;
    auto cell_x0 = [&](int j) { return kMinBorder + j * G.wCell + 3; };
    auto cell_x1 = [&](int j) {
        const int iniX = kMinBorder + j * G.wCell;
        return iniX >= G.maxBX - 6 ? cell_x0(j) : min(iniX + G.wCell + 6, G.maxBX) - 3;
    };
    const int xs = cell_x0(ja);
    int xe = xs;
    for (int j = ja; j < jb; ++j) xe = max(xe, cell_x1(j));
    const int qa = xs >> 2, nq = xe > xs ? ((xe - 1) >> 2) - qa + 1 : 0;
    const int nrows = row_skip ? 0 : max(ry1 - ry0, 0);
    if (nrows == 0 || nq == 0) {
        if (lane < jb - ja) cnt_out[ja + lane] = 0;
        return;
    }
    // ---- per-lane static geometry -----------------------------------------------------------
    const int x0 = 4 * (qa - 1 + lane);
    const bool owner = lane >= 1 && lane <= nq;
    int cid[6];
#pragma unroll
    for (int k = -1; k < 5; ++k) {
        const int x = x0 + k;
        int c = -1;
        if (owner || k < 0 || k > 3) {
            if (x >= xs && x < xe) {
                const int j = (x - kMinBorder - 3) / G.wCell;
                if (j >= ja && j < jb && x >= cell_x0(j) && x < cell_x1(j)) c = j;
            }
        }
        cid[k + 1] = c;
    }
    if (!owner) {
#pragma unroll
        for (int k = 0; k < 4; ++k) cid[k + 1] = -1;
    }
    auto msk = [](bool b0, bool b1) { return (b0 ? 0xFFFFu : 0u) | (b1 ? 0xFFFF0000u : 0u); };
    auto same = [&](int k, int n) { return cid[k + 1] >= 0 && cid[n + 1] == cid[k + 1]; };
    const uint32_t mLE = msk(same(0, -1), same(2, 1)), mRE = msk(same(0, 1), same(2, 3));
    const uint32_t mLO = msk(same(1, 0), same(3, 2)), mRO = msk(same(1, 2), same(3, 4));
    const uint32_t mSE = msk(cid[1] >= 0, cid[3] >= 0), mSO = msk(cid[2] >= 0, cid[4] >= 0);
    // the quad's (at most two) cells: part A = the first valid pixels, part B = the rest
    int cA = -1, cB = -1;
    uint32_t bA = 0, bB = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = cid[k + 1];
        if (c < 0) continue;
        if (cA < 0 || c == cA) {
            cA = c;
            bA |= 0x80u << (8 * k);
        } else {
            cB = c;
            bB |= 0x80u << (8 * k);
        }
    }
    // first lane of cell cA, and whether that lane's part A is the previous cell (a straddler)
    int F = lane, strF = 0;
    if (cA >= 0) {
        const int x = cell_x0(cA);
        F = (x >> 2) - (qa - 1);
        // pixels of quad F left of x belong to cell cA - 1 when that cell is this wave's
        strF = ((x & 3) != 0 && cA - 1 >= ja && (x - 1) >= cell_x0(cA - 1) && (x - 1) < cell_x1(cA - 1)) ? 1 : 0;
    }
    // part A / B ends its cell here (the next pixel is in no or another cell): this lane writes
    // the cell's running count after each row
    const bool lastA = cA >= 0 && (cB >= 0 || cid[5] != cA);
    const bool lastB = cB >= 0 && cid[5] != cB;
    // ---- tables --------------------------------------------------------------------------
    if (lane < 16) {
        int pos[4] = {0, 0, 0, 0}, n = 0;
        for (int k = 0; k < 4; ++k)
            if ((lane >> k) & 1) pos[n++] = k;
        lut[lane] = make_uint2((uint32_t)pos[0] | ((uint32_t)pos[1] << 16), (uint32_t)pos[2] | ((uint32_t)pos[3] << 16));
    }
    if (lane < kSbMaxCells) cnt[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint8_t* plane = a.lvl_base[l] + (long long)img * G.img_stride;
    const int xo = min(max(x0, 0), G.pitch - 4);
    auto ld = [&](int y) -> uint32_t {
        const uint8_t* p = plane + (size_t)__mul24(y, G.pitch) + xo;
        if constexpr (kDw) {
            return *reinterpret_cast<const uint32_t*>(p);
        } else {
            const uintptr_t u = reinterpret_cast<uintptr_t>(p);
            const uint32_t* q = reinterpret_cast<const uint32_t*>(u & ~(uintptr_t)3);
            return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(u & 3));
        }
    };
    const int tini = min(max(a.ini_th, 0), 255), tmin = min(max(a.min_th, 0), 255);
    auto rank = [](uint64_t b) {
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    };
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    const int ylast = ry1 + 2;
    constexpr int D = 3;  // rows between the pre-test of a row and its nonmax
    // one walk over the band at threshold t, emitting keys for the cells in `emit` (bit j - ja)
    auto walk = [&](int t, uint32_t emit) {
        const bool eA = cA >= 0 && ((emit >> (cA - ja)) & 1u), eB = cB >= 0 && ((emit >> (cB - ja)) & 1u);
        const uint32_t pre_mask = (eA ? bA : 0u) | (eB ? bB : 0u);  // pixels this walk evaluates
        const uint32_t tt = (uint32_t)t * 0x00010001u, kt = (uint32_t)(255 - t) * 0x00010001u;
        const uint32_t tn = (uint32_t)(255 - max(t, 1)) * 0x01010101u;  // ~T for v_lerp_u8
        uint32_t Wr[7], raw[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) raw[k] = ld(min(ry0 - 3 + k, ylast));
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            Wr[k] = raw[k];
            T32[((ry0 - 3 + k) & (kSbRing - 1)) * 64 + lane] = raw[k];
            raw[k] = ld(min(ry0 + 4 + k, ylast));
        }
        Wr[6] = 0;
        int head = 0, tail = 0;
        uint32_t mEp = 0, mOp = 0;  // nonmax state: M of row yn, H2 / H3 of rows yn - 1, yn
        uint32_t h3Epp = 0, h3Opp = 0, h3Ep = 0, h3Op = 0, h2Ep = 0, h2Op = 0;
        const int nsteps = nrows + D + 1;
        const int nblk = (nsteps + 6) / 7;
        for (int b = 0; b < nblk; ++b) {
#pragma unroll
            for (int u = 0; u < 7; ++u) {
                const int s = ry0 + 7 * b + u;
                if (s < ry1) {
                    // row s + 3 enters the window and the LDS ring; its raw slot refills 7 rows ahead
                    const int sl = (u + 6) % 7;
                    Wr[sl] = raw[sl];
                    T32[((s + 3) & (kSbRing - 1)) * 64 + lane] = raw[sl];
                    raw[sl] = ld(min(s + 10, ylast));
                    M32[(s & (kSbMRing - 1)) * 64 + lane] = 0u;  // row s of the strength ring
                    wsync();
                    // SWAR pre-test of row s (orb_fast_cell.h fw_pretest4) for this walk's pixels
                    const uint32_t C = Wr[(u + 3) % 7];
                    const uint32_t U2 = Wr[(u + 1) % 7], D2 = Wr[(u + 5) % 7];
                    uint32_t m8 = fw_pretest4(C, from_left(C, 0u), from_right(C, 0u), Wr[u % 7], Wr[(u + 6) % 7],
                                              from_left(U2, 0u), U2, from_right(U2, 0u), from_left(D2, 0u), D2,
                                              from_right(D2, 0u), tt, kt) & pre_mask;
                    // compaction into the FIFO: entries (row & 15) << 8 | byte column
                    const int c = __builtin_popcount(m8);
                    const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
                    const int pos = tail + rank(b0) + 2 * rank(b1) + 4 * rank(b2);
                    if (c) {
                        const uint2 lv = lut[__builtin_amdgcn_udot4(m8, 0x08040201u, 0u, false) >> 7];
                        const uint32_t base = (((uint32_t)s & 15u) << 8) | (uint32_t)(4 * lane);
                        const uint32_t e01 = base * 0x10001u + lv.x, e23 = base * 0x10001u + lv.y;
                        fifo[(pos + 3) & (kSbFifo - 1)] = (uint16_t)(e23 >> 16);
                        asm volatile("" ::: "memory");
                        fifo[(pos + 2) & (kSbFifo - 1)] = (uint16_t)e23;
                        asm volatile("" ::: "memory");
                        fifo[(pos + 1) & (kSbFifo - 1)] = (uint16_t)(e01 >> 16);
                        asm volatile("" ::: "memory");
                        fifo[pos & (kSbFifo - 1)] = (uint16_t)e01;
                    }
                    tail += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
                    if (lane == 0) tail_at[s & 7] = tail;
                    wsync();
                }
                // strengths: full batches, then whatever rows <= s - 2 still hold (the nonmax of
                // row s - 3 reads M of rows s - 4 .. s - 2)
                {
                    const int need = s - 2 >= ry0 ? (s - 2 < ry1 ? __builtin_amdgcn_readfirstlane(tail_at[(s - 2) & 7]) : tail)
                                                  : head;
                    while (tail - head >= 64 || head < need) {
                        const int nb = min(tail - head, 64);
                        if (lane < nb) {
                            const uint32_t e = fifo[(head + lane) & (kSbFifo - 1)];
                            const int rs = (int)(e >> 8), col = (int)(e & 255u);
                            const int m = sb_strength(Tb, rs, col);
                            if (m > t) Mb[(rs & (kSbMRing - 1)) * 256 + col] = (uint8_t)m;
                        }
                        head += nb;
                    }
                    wsync();
                }
                // nonmax + keys of row yn = s - 3
                const int yn = s - D;
                if (yn >= ry0 && yn < ry1) {
                    const uint32_t bias = 0x04000400u;
                    // M of rows yn (current) and yn + 1 (next) as E / O pairs biased by 0x0400 (so
                    // v_pk_maximum3_f16 orders them; masked-out neighbours are 0, below all)
                    auto pairs = [&](int y, uint32_t& E, uint32_t& O) {
                        const uint32_t Mw = (y >= ry0 && y < ry1) ? M32[(y & (kSbMRing - 1)) * 64 + lane] : 0u;
                        E = __builtin_amdgcn_perm(0x04040404u, Mw, 0x04020400u);
                        O = __builtin_amdgcn_perm(0x04040404u, Mw, 0x04030401u);
                    };
                    uint32_t mE, mO;
                    if (yn == ry0) {
                        pairs(yn, mE, mO);
                    } else {
                        mE = mEp;
                        mO = mOp;
                    }
                    uint32_t nE, nO;
                    pairs(yn + 1, nE, nO);
                    // masked horizontal neighbours (0 = none) of a row's biased pairs
                    auto hsums = [&](uint32_t E, uint32_t O, uint32_t& h2E, uint32_t& h2O, uint32_t& h3E,
                                     uint32_t& h3O) {
                        const uint32_t Ol = from_left(O, 0u), Er = from_right(E, 0u);
                        const uint32_t LE = __builtin_amdgcn_alignbyte(O, Ol, 2) & mLE, RE = O & mRE;
                        const uint32_t LO = E & mLO, RO = __builtin_amdgcn_alignbyte(Er, E, 2) & mRO;
                        h2E = pmax(LE, RE);
                        h2O = pmax(LO, RO);
                        h3E = pmax3(LE, E, RE);
                        h3O = pmax3(LO, O, RO);
                    };
                    uint32_t h2E, h2O, h3E, h3O, h2nE, h2nO, h3nE, h3nO;
                    if (yn == ry0) {
                        hsums(mE, mO, h2E, h2O, h3E, h3O);
                        h3Epp = 0;  // row ry0 - 1 is outside the cells
                        h3Opp = 0;
                    } else {
                        h2E = h2Ep;
                        h2O = h2Op;
                        h3E = h3Ep;
                        h3O = h3Op;
                    }
                    hsums(nE, nO, h2nE, h2nO, h3nE, h3nO);
                    if (yn + 1 >= ry1) {
                        h3nE = 0;
                        h3nO = 0;
                    }
                    const uint32_t bE = pmax3(h3Epp, h2E, h3nE), bO = pmax3(h3Opp, h2O, h3nO);
                    // kept: m beats its in-cell neighbours (pairs are biased: 0x0400 = strength 0)
                    const uint32_t one = 0x00010001u;
                    const uint32_t kE = pmin(psubs(mE, bE), one), kO = pmin(psubs(mO, bO), one);
                    const uint32_t RE = w32(h2(psubs(mE, bias)) * h2(kE)) & mSE;
                    const uint32_t RO = w32(h2(psubs(mO, bias)) * h2(kO)) & mSO;
                    const uint32_t R = __builtin_amdgcn_perm(RO, RE, 0x06020400u);
                    const uint32_t sel = __builtin_amdgcn_lerp(R, tn, 0u) & pre_mask;  // R > max(t, 1)
                    const int ea = __builtin_popcount(sel & bA), eb = __builtin_popcount(sel & bB);
                    const int e = ea + eb;
                    const uint64_t c0 = __ballot(e & 1), c1 = __ballot(e & 2), c2 = __ballot(e & 4);
                    const int P = rank(c0) + 2 * rank(c1) + 4 * rank(c2);
                    // start of cell cA in this row's sequence: lane F's prefix (+ its part A when
                    // that part is the previous cell)
                    const int pf = __builtin_amdgcn_ds_bpermute(4 * F, P | (ea << 16));
                    const int SA = (pf & 0xFFFF) + (strF ? (pf >> 16) : 0);
                    const int baseA = cA >= 0 ? cnt[cA - ja] : 0, baseB = cB >= 0 ? cnt[cB - ja] : 0;
                    int pa = baseA + P - SA, pb = baseB;
                    if (sel) {
                        const int ry = yn - kMinBorder;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t bit = 0x80u << (8 * k);
                            if (sel & bit) {
                                const int resp = (int)((R >> (8 * k)) & 0xFFu) - 1;  // cornerScore = m - 1
                                const uint32_t key = make_key(x0 + k - kMinBorder, ry, resp);
                                if (bA & bit) key_base[(long long)(cA)*G.cell_cap + pa++] = key;
                                else key_base[(long long)(cB)*G.cell_cap + pb++] = key;
                            }
                        }
                    }
                    wsync();  // every lane has read the counts before they move on
                    if (lastA && eA) cnt[cA - ja] = baseA + (P - SA) + ea;
                    if (lastB && eB) cnt[cB - ja] = baseB + eb;
                    wsync();
                    h3Epp = h3E;
                    h3Opp = h3O;
                    h3Ep = h3nE;
                    h3Op = h3nO;
                    h2Ep = h2nE;
                    h2Op = h2nO;
                    mEp = nE;
                    mOp = nO;
                }
            }
        }
    };
    const uint32_t all = (jb - ja) >= 32 ? 0xFFFFFFFFu : ((1u << (jb - ja)) - 1u);
    walk(tini, all);
    wsync();
    uint32_t redo = 0;
    for (int j = ja; j < jb; ++j)
        if (cnt[j - ja] == 0) redo |= 1u << (j - ja);
    redo = __builtin_amdgcn_readfirstlane(redo);
    if (redo) {
        wsync();
        walk(tmin, redo);
    }
    wsync();
    if (lane < jb - ja) cnt_out[ja + lane] = cnt[lane];
}

hipError_t launch_fast_sb(const BatchArgs& a, hipStream_t s) {
    const int n = a.fast_sb_n;
    if (n <= 0) return hipSuccess;
    const uint32_t d = (uint32_t)n;
    const uint32_t magic = d > 1 ? 0xFFFFFFFFu / d + 1u : 0u;
    const bool dw = ((a.lv[0].pitch | (int)a.lv[0].img_stride) & 3) == 0 &&
                    (reinterpret_cast<uintptr_t>(a.lvl_base[0]) & 3) == 0;
    if (dw) hipLaunchKernelGGL((k_fast_sb<true>), dim3(n, a.nimages), dim3(64), 0, s, a, magic);
    else hipLaunchKernelGGL((k_fast_sb<false>), dim3(n, a.nimages), dim3(64), 0, s, a, magic);
    return hipGetLastError();
}

// One launch per segment width (1 .. kFastBandMaxWaves waves): records [grp[w-1], grp[w]).
hipError_t launch_fast_bands(const BatchArgs& a, hipStream_t s) {
    constexpr int kMaxDevices = 64;
    static std::atomic<int> lds_set[kMaxDevices][2 * kFastBandMaxWaves];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = kMaxDevices - 1;
    for (int nw = 1; nw <= kFastBandMaxWaves; ++nw) {
        const int r0 = a.fast_band_grp[nw - 1], r1 = a.fast_band_grp[nw];
        if (r1 <= r0) continue;
        const int lds = a.fast_band_lds[nw - 1];
        // level 0 is the caller's input (row stride = width): dword rows only for widths % 4 == 0
        const bool dw = ((a.lv[0].pitch | (int)a.lv[0].img_stride) & 3) == 0 &&
                        (reinterpret_cast<uintptr_t>(a.lvl_base[0]) & 3) == 0;
        const void* fn = nw == 1 ? (dw ? reinterpret_cast<const void*>(k_fast_bands<1, true>) : reinterpret_cast<const void*>(k_fast_bands<1, false>))
                         : nw == 2 ? (dw ? reinterpret_cast<const void*>(k_fast_bands<2, true>) : reinterpret_cast<const void*>(k_fast_bands<2, false>))
                         : nw == 3 ? (dw ? reinterpret_cast<const void*>(k_fast_bands<3, true>) : reinterpret_cast<const void*>(k_fast_bands<3, false>))
                                   : (dw ? reinterpret_cast<const void*>(k_fast_bands<4, true>) : reinterpret_cast<const void*>(k_fast_bands<4, false>));
        std::atomic<int>& set = lds_set[dev][2 * (nw - 1) + (dw ? 0 : 1)];
        if (lds > 65536 && lds > set.load()) {
            hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e != hipSuccess) return e;
            int cur = set.load();
            while (lds > cur && !set.compare_exchange_weak(cur, lds)) {}
        }
        const uint32_t d = (uint32_t)(r1 - r0);
        const uint32_t magic = d > 1 ? 0xFFFFFFFFu / d + 1u : 0u;
        const dim3 grid(r1 - r0, a.nimages), block(64 * nw);
#define FB_LAUNCH(W)                                                                              \
    do {                                                                                          \
        if (dw) hipLaunchKernelGGL((k_fast_bands<W, true>), grid, block, lds, s, a, r0, magic);   \
        else hipLaunchKernelGGL((k_fast_bands<W, false>), grid, block, lds, s, a, r0, magic);     \
    } while (0)
        if (nw == 1) FB_LAUNCH(1);
        else if (nw == 2) FB_LAUNCH(2);
        else if (nw == 3) FB_LAUNCH(3);
        else FB_LAUNCH(4);
#undef FB_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace orbgpu
