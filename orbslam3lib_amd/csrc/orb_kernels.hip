// orb_kernels.hip -- gfx950 kernels of the ORB front-end.  Integer/byte work: no MFMA.
//
// Pipeline for a batch of B images (one launch per stage, or per sub-batch stream and stage):
//   k_blur_resize x (L-1)  level l-1's 7x7 Gaussian (sigma 2, fixed point, REFLECT_101) and the
//                          cascaded INTER_LINEAR resize to level l from one read of level l-1
//   k_blur        x 1      the last level's blur
//   k_fast_cells  x 1-3    one workgroup per (image, level, 35-px cell): FAST-9 strength,
//                          3x3 nonmax at iniTh / minTh fallback, ordered compaction (one launch
//                          per LDS tile size)
//   k_octree      x 1      one workgroup per (image, level): DistributeOctTree
//   k_orient_desc x 1      32 lanes per keypoint: IC_Angle + rBRIEF 256 bit
//   k_finalize    x 1      one workgroup per image: scale + mono/stereo partition
//   k_knn2_mfma   x 1      Hamming k=2 brute force on the i8 matrix cores
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "orb_kernels.h"
#include "orb_math.h"
#include "orb_fast_cell.h"
#include "orb_octree.h"
#include "orb_pattern_data.h"
#include "orb_policy.h"

namespace orbgpu {

static_assert(sizeof(BatchArgs) <= 4096, "kernel argument block too large");

// rBRIEF pattern decoded at compile time from the hex data: 256 pairs (x0,y0,x1,y1) int8.
struct PatternTable {
    int8_t v[1024];
};
constexpr int hexval(char c) { return c <= '9' ? c - '0' : c - 'a' + 10; }
constexpr PatternTable make_pattern() {
    PatternTable t{};
    const char* h = ORBGPU_PATTERN_HEX;
    for (int i = 0; i < 1024; ++i) t.v[i] = (int8_t)(hexval(h[2 * i]) * 16 + hexval(h[2 * i + 1]));
    return t;
}

// umax[] of the ORBextractor ctor (ORBextractor_old.cc:455-470) for HALF_PATCH_SIZE = 15.
__constant__ int c_umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};


// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ inline u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ inline uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// cv::resize INTER_LINEAR (canonical ComputePyramid, ORBextractor_old.cc:1342-1344), fixed point.
// Four output pixels dx0 .. dx0+3 of one output row from source rows r0 / r1 (LDS window rows,
// indexed by source column).  The quad's taps lie in the 8 source bytes from its first left tap
// `base` (scale <= 2: the last right tap is at most base + 7), read as three aligned dwords per
// row and byte-aligned with v_alignbyte; sel[k] picks output k's two taps as a u16 pair (v_perm)
// and cw[k] holds its two x coefficients times 16 as a u16 pair (16 c <= 32768), so each
// horizontal sum is one v_dot2_u32_u16 yielding 16 D (exact: < 2^23).  Vertical rounding:
// OpenCV's SIMD body (VResizeLinearVec_32s8u) below simd_end,
//   out = (((D0 >> 4) b0 >> 16) + ((D1 >> 4) b1 >> 16) + 2) >> 2,
// where (D >> 4) << 8 = 16 D & ~0xFF and the row weights come as b << 8 (B0 / B1 <= 2^19), so
// each ((D >> 4) b) >> 16 is one v_mul_hi_u32_u24 of two 24-bit operands (the 48-bit product
// >> 32); the sum is <= 1022 (c0 + c1 = b0 + b1 = 2048), so no clamp is needed.  FixedPtCast
// after simd_end (only the last quads of a row take that branch).
// (a * b) >> 32 for 24-bit a, b: one v_mul_hi_u32_u24 (the masks tell the compiler the operand
// widths; both are no-ops on rs_quad's operands)
__device__ inline uint32_t mulhi_u24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (uint64_t)(b & 0xFFFFFFu)) >> 32);
}

__device__ inline uint32_t rs_quad(const uint8_t* r0, const uint8_t* r1, int base, int4 sel, int4 cw, int B0,
                                   int B1, int dx0, int simd_end) {
    const uint32_t* p0 = reinterpret_cast<const uint32_t*>(r0 + (base & ~3));
    const uint32_t* p1 = reinterpret_cast<const uint32_t*>(r1 + (base & ~3));
    const uint32_t sh = (uint32_t)(base & 3);
    const uint32_t a0 = p0[0], a1 = p0[1], a2 = p0[2];
    const uint32_t c0 = p1[0], c1 = p1[1], c2 = p1[2];
    const uint32_t lo0 = __builtin_amdgcn_alignbyte(a1, a0, sh), hi0 = __builtin_amdgcn_alignbyte(a2, a1, sh);
    const uint32_t lo1 = __builtin_amdgcn_alignbyte(c1, c0, sh), hi1 = __builtin_amdgcn_alignbyte(c2, c1, sh);
    const int sl[4] = {sel.x, sel.y, sel.z, sel.w};
    const int cl[4] = {cw.x, cw.y, cw.z, cw.w};
    uint32_t D0[4], D1[4];  // 16 D
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t0 = __builtin_amdgcn_perm(hi0, lo0, (uint32_t)sl[k]);
        const uint32_t t1 = __builtin_amdgcn_perm(hi1, lo1, (uint32_t)sl[k]);
        D0[k] = __builtin_amdgcn_udot2(as_u16x2(t0), as_u16x2((uint32_t)cl[k]), 0u, false);
        D1[k] = __builtin_amdgcn_udot2(as_u16x2(t1), as_u16x2((uint32_t)cl[k]), 0u, false);
    }
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o[k] = (mulhi_u24(D0[k] & 0x7FFF00u, (uint32_t)B0) + mulhi_u24(D1[k] & 0x7FFF00u, (uint32_t)B1) + 2u) >> 2;
    if (dx0 + 3 >= simd_end) {
        const unsigned b0 = (unsigned)B0 >> 8, b1 = (unsigned)B1 >> 8;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (dx0 + k >= simd_end) {
                // D < 2^19, b <= 2048: both 24-bit, products < 2^30 (full-rate multiplies)
                const uint32_t v = (__umul24(D0[k] >> 4, b0) + __umul24(D1[k] >> 4, b1) + (1u << 21)) >> 22;
                o[k] = v < 255u ? v : 255u;
            }
        }
    }
    return o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24);
}

// ---------------------------------------------------------------------------------------------
// k_blur: cv::GaussianBlur(Size(7,7), 2, 2, BORDER_REFLECT_101) on each level
// (ORBextractor_old.cc:1146-1147), bit-exact fixed point: kernel {18,34,48,56,48,34,18}/256,
// out = (sum_v w_v sum_h w_h p + 2^15) >> 16 with the horizontal sums exact (<= 65280, u16).
// Byte offset of (row y, column x) inside one plane: planes are < 16 M rows of < 16 MB pitch
// and < 2^32 bytes, so the row product is one full-rate 24-bit multiply (no 64-bit multiply
// per access).
__device__ inline size_t plane_off(int y, int pitch, int x) {
    uint32_t o;  // v_mad_u32_u24 kept as such (not re-associated into a 64-bit multiply-add)
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(o) : "v"(y), "v"(pitch), "v"(x));
    return (size_t)o;
}

__device__ inline int refl101(int p, int n) {
    p = p < 0 ? -p : p;
    return p >= n ? 2 * n - p - 2 : p;
}

// Horizontal 7-tap sums of 4 columns of two rows as u16 pairs (row a low, row b high), from the
// 12 window bytes of each row that start 1 byte before the first output's first tap (A[0] byte 1 =
// column x-3 of output 0): per row and output, the taps x-3 .. x as one byte window (v_alignbyte)
// times {18, 34, 48, 56} and x+1 .. x+3 times {48, 34, 18, 0}, two v_dot4_u32_u8 (sums <= 65280).
// 32 VALU per two rows of 4 columns (the u16-pair form with v_perm / v_pk_mad_u16 took 38).
__device__ inline void hsum_pair(const uint32_t A[3], const uint32_t B[3], uint32_t out[4]) {
    constexpr uint32_t W03 = 18u | (34u << 8) | (48u << 16) | (56u << 24);
    constexpr uint32_t W46 = 48u | (34u << 8) | (18u << 16);
    auto row = [&](const uint32_t* X, uint32_t h[4]) {
        const uint32_t lo[4] = {__builtin_amdgcn_alignbyte(X[1], X[0], 1), __builtin_amdgcn_alignbyte(X[1], X[0], 2),
                                __builtin_amdgcn_alignbyte(X[1], X[0], 3), X[1]};
        const uint32_t hi[4] = {__builtin_amdgcn_alignbyte(X[2], X[1], 1), __builtin_amdgcn_alignbyte(X[2], X[1], 2),
                                __builtin_amdgcn_alignbyte(X[2], X[1], 3), X[2]};
#pragma unroll
        for (int o = 0; o < 4; ++o)
            h[o] = __builtin_amdgcn_udot4(hi[o], W46, __builtin_amdgcn_udot4(lo[o], W03, 0u, false), false);
    };
    uint32_t ha[4], hb[4];
    row(A, ha);
    row(B, hb);
#pragma unroll
    for (int o = 0; o < 4; ++o) out[o] = ha[o] | (hb[o] << 16);
}

// Tile 128 x 32 outputs; the input window is rows ty0-4 .. ty0+35 (one spare row each side so
// rows pair up) x cols tx0-16 .. tx0+143, staged in LDS with 16-byte loads.
// Horizontal pass in "row-pair" u16x2 lanes: lane lo = row 2rp, lane hi = row 2rp+1 of the
// same column, 7 taps as two v_dot4_u32_u8 per row and column (hsum_pair).
// Vertical pass: each output row is 4 v_dot2_u32_u16 over row pairs with weight pairs
// {0,18}{34,48}{56,48}{34,18} (even rows) or {18,34}{48,56}{48,34}{18,0} (odd rows), the
// accumulator seeded with the 2^15 rounding term.

struct BlurTile {
    int l, ty0, tx0;
    const uint8_t* src;
    uint8_t* dst;
};

__device__ inline BlurTile blur_tile(const BatchArgs& a, int t) {
    BlurTile bt;
    const int img = a.img0 + t / a.total_tiles;
    int k = t % a.total_tiles;
    int l = 0;
    while (l + 1 < a.nlevels && k >= a.lv[l + 1].tile_first) ++l;
    const LevelGeom G = a.lv[l];
    k -= G.tile_first;
    bt.l = l;
    bt.ty0 = (k / G.tiles_x) * kBlurTH;
    bt.tx0 = (k % G.tiles_x) * kBlurTW;
    bt.src = a.lvl_base[l] + (long long)img * G.img_stride;
    bt.dst = a.blur_base[l] + (long long)img * G.bimg_stride;
    return bt;
}

// Window chunk i (16 bytes) of tile bt: rows reflected here (REFLECT_101), columns loaded as
// they are (bounds-checked buffer load; chunks left of the plane are zero) -- the few column
// bytes outside the plane that the taps reach are reflected in LDS afterwards (blur_fix_cols).
template <int kAux = 0>
__device__ inline uint4 blur_chunk(const BatchArgs& a, const BlurTile& bt, int i, int IWQ) {
    const LevelGeom G = a.lv[bt.l];
    const int r = i / IWQ, cq = i - r * IWQ;
    // rows beyond the reflected range feed only zero weights or unwritten outputs: clamp
    const int y = min(max(refl101(bt.ty0 + r - 4, G.h), 0), G.h - 1);
    const int x = bt.tx0 - 16 + 16 * cq;
    if (x < 0) return make_uint4(0, 0, 0, 0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)bt.src, (short)0, (int)min(G.img_stride, 0x7fffffffLL), 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, y * G.pitch + x, 0, kAux);
    return make_uint4(v[0], v[1], v[2], v[3]);
}


// The same 128 x 32 blur tile as two int8 GEMMs on the matrix cores (v_mfma_i32_32x32x32_i8; the
// 7-tap kernel is banded, the zeros cost MFMA cycles that are otherwise idle, and the VALU keeps
// only the operand and result packing).  Wave w owns output columns 32w .. 32w+31 of the tile.
//   pass 1 (horizontal): D1[y][x] = sum_j (p[y][j] - 128) g[j - x - 13] over window columns
//     32w .. 32w+63 (two K-steps), rows 0..31 and 32..63 of the window (two M-blocks; rows past
//     the window's 40 read row 39 and only meet zero weights).  A = pixel rows straight from LDS
//     (16 bytes per lane, ^0x80 makes them int8), B = the constant band.
//   the pass-1 results (lane: column x, rows (g&3) + 8(g>>2) + 4h of the M-block) are split into
//     two int8 planes, hi = byte 1 and lo = byte 0 ^ 0x80 of D1, so D1 + 128 = 256 hi + lo + 256;
//     they are pass 2's A operand as they stand (lane = column x, its 16 rows = the K slots; the
//     constant B is laid out for exactly that row order).
//   pass 2 (vertical, transposed): D2[x][y'] = sum_y A2[x][y] g[y - y' - 1] -- lane = output
//     row y', its 16 registers = columns (g&3) + 8(g>>2) + 4h, i.e. four runs of 4 consecutive
//     bytes.  With S = the integer blur sum (sum of g = 256): 256 D2hi + D2lo = S - 2^23 - 2^15, so
//     the rounded output byte (S + 2^15) >> 16 is byte 2 of 256 D2hi + D2lo + 2^16 (which stays
//     in [-2^23, 2^23)) with bit 7 flipped.  The + 2^16 rides in K slot 4 of M-block 1 (a row >= 40
//     that no output reads) in both lane halves: A2hi = -1 there, B = -128, 2 x 128 into D2hi.
// Exact integer arithmetic throughout (no intermediate rounding), so bit-exact with the fixed-point
// filter the oracle restates (tests/test_blur_mfma_model.py replays the lane layouts on the CPU).
typedef int blur_v4i __attribute__((ext_vector_type(4)));
typedef int blur_v16i __attribute__((ext_vector_type(16)));
struct BlurMfmaTab {
    uint32_t b1[2][64][4];  // pass-1 B: [K-step s][lane (x = l & 31, h)], byte j: window column 32s + 16h + j
    uint32_t b2[2][64][4];  // pass-2 B: [M-block mb][lane (y' = l & 31, h)], byte g: window row of slot g
};
constexpr BlurMfmaTab make_blur_mfma_tab() {
    BlurMfmaTab t{};
    const int g7[7] = {18, 34, 48, 56, 48, 34, 18};
    for (int k = 0; k < 2; ++k)
        for (int l = 0; l < 64; ++l) {
            const int n = l & 31, h = l >> 5;
            for (int j = 0; j < 16; ++j) {
                const int d1 = 32 * k + 16 * h + j - (n + 13);                            // column tap
                const int rho = 32 * k + (j & 3) + 8 * (j >> 2) + 4 * h, d2 = rho - (n + 1);  // row tap
                const uint32_t w1 = d1 >= 0 && d1 < 7 ? (uint32_t)g7[d1] : 0u;
                uint32_t w2 = d2 >= 0 && d2 < 7 ? (uint32_t)g7[d2] : 0u;
                if (k == 1 && j == 4) w2 = 0x80u;  // -128: the + 2^16 slot (both halves h: 2 x 128)
                t.b1[k][l][j >> 2] |= w1 << (8 * (j & 3));
                t.b2[k][l][j >> 2] |= w2 << (8 * (j & 3));
            }
        }
    return t;
}
__constant__ BlurMfmaTab c_blur_mfma = make_blur_mfma_tab();

__device__ inline void blur_tile_compute_mfma(const LevelGeom& G, int tx0, int ty0, uint8_t* dst,
                                              uint4 (*tin4)[(kBlurTW + 32) / 16],
                                              uint4 (*hp)[kBlurTW / 4], int rlo, int rhi) {
    constexpr int IW = kBlurTW + 32, IH = kBlurTH + 8;
    static_assert(kBlurTW == 128 && kBlurTH == 32, "one 32-column strip per wave, one output block");
    constexpr int OP = kBlurTW + 4;  // output staging pitch: 33 dwords, conflict-free column writes
    if (tx0 == 0 || tx0 + kBlurTW + 3 > G.w) {  // REFLECT_101 of the 3 columns past each edge
        uint8_t* wb = reinterpret_cast<uint8_t*>(&tin4[0][0]);
        for (int i = threadIdx.x; i < IH * 6; i += 256) {
            const int r = i / 6, k = i - 6 * r;
            const int xx = k < 3 ? -1 - k : G.w + (k - 3);
            const int wx = xx - (tx0 - 16);
            if (wx >= 0 && wx < IW && (k < 3 ? tx0 == 0 : true)) {
                const int sx = refl101(xx, G.w) - (tx0 - 16);
                wb[r * IW + wx] = wb[r * IW + sx];
            }
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n = lane & 31, h = lane >> 5;
    const uint8_t* wb = reinterpret_cast<const uint8_t*>(&tin4[0][0]);
    auto ldc = [&](const uint32_t* p) {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        return blur_v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
    };
    const blur_v4i B1[2] = {ldc(c_blur_mfma.b1[0][lane]), ldc(c_blur_mfma.b1[1][lane])};
    const blur_v4i B2[2] = {ldc(c_blur_mfma.b2[0][lane]), ldc(c_blur_mfma.b2[1][lane])};
    blur_v4i hi[2], lo[2];
    const blur_v16i zero = {};
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int row = min(32 * mb + n, IH - 1);
        const uint8_t* src = wb + row * IW + 32 * w + 16 * h;
        blur_v16i acc = zero;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint4 v = *reinterpret_cast<const uint4*>(src + 32 * k);
            const blur_v4i a = {(int)(v.x ^ 0x80808080u), (int)(v.y ^ 0x80808080u), (int)(v.z ^ 0x80808080u),
                                (int)(v.w ^ 0x80808080u)};
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, B1[k], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (mb == 1 && q > 0) {  // rows >= 40: no output row reads them; slot 4 carries the + 2^16
                hi[mb][q] = q == 1 ? 0x000000FF : 0;
                lo[mb][q] = 0;
                continue;
            }
            const uint32_t u0 = acc[4 * q], u1 = acc[4 * q + 1], u2 = acc[4 * q + 2], u3 = acc[4 * q + 3];
            hi[mb][q] = (int)(__builtin_amdgcn_perm(u1, u0, 0x0c0c0501u) | (__builtin_amdgcn_perm(u3, u2, 0x0c0c0501u) << 16));
            lo[mb][q] = (int)((__builtin_amdgcn_perm(u1, u0, 0x0c0c0400u) | (__builtin_amdgcn_perm(u3, u2, 0x0c0c0400u) << 16)) ^ 0x80808080u);
        }
    }
    blur_v16i ah = zero, al = zero;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(hi[mb], B2[mb], ah, 0, 0, 0);
        al = __builtin_amdgcn_mfma_i32_32x32x32_i8(lo[mb], B2[mb], al, 0, 0, 0);
    }
    // output row n: columns 32w + 8q + 4h .. +3 from registers 4q .. 4q+3, staged row-major in LDS
    uint32_t* ob = reinterpret_cast<uint32_t*>(&hp[0][0]);  // hp is free: callers sync before reusing it
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t t4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t4[k] = ((uint32_t)ah[4 * q + k] << 8) + (uint32_t)al[4 * q + k];
        const uint32_t packed = (__builtin_amdgcn_perm(t4[1], t4[0], 0x0c0c0602u) |
                                 (__builtin_amdgcn_perm(t4[3], t4[2], 0x0c0c0602u) << 16)) ^ 0x80808080u;
        ob[n * (OP / 4) + 8 * w + 2 * q + h] = packed;
    }
    __syncthreads();
    // stores as the VALU path: thread -> column quad cq, rows R rg .. R rg + R - 1
    constexpr int R = kBlurTH / 8;
    const int cq = threadIdx.x & 31, rg = threadIdx.x >> 5;
    const int x = tx0 + 4 * cq;
    const int ybase = ty0 + R * rg;
    const int ylo = max(rlo, ybase), yhi = x < G.w ? min(min(rhi, G.h), ybase + R) : ybase;
    const int olo = ylo - ybase, ohi = yhi - ybase;
    uint8_t* dbase = dst + plane_off(ybase, G.bpitch, x);
#pragma unroll
    for (int o = 0; o < R; ++o)
        if (o >= olo && o < ohi) *reinterpret_cast<uint32_t*>(dbase + o * G.bpitch) = ob[(R * rg + o) * (OP / 4) + cq];
}

// Persistent over the tiles of the launch (images x levels x tiles): the next tile's window
// is loaded into registers while the current one is filtered, so the global-memory round
// trip is hidden behind the arithmetic of the previous tile.
__global__ __launch_bounds__(256) void k_blur(BatchArgs a, int tile0, int ntile) {
    constexpr int IW = kBlurTW + 32, IH = kBlurTH + 8, IWQ = IW / 16, NRP = IH / 2;
    constexpr int NCH = (IH * IWQ + 255) / 256;  // window chunks per thread
    __shared__ uint4 tin4[IH][IWQ];
    __shared__ uint4 hp[NRP][kBlurTW / 4];  // [row pair][column quad]: 4 columns x (row0,row1)
    // tiles [tile0, tile0 + ntile) of every image (all levels: 0, total_tiles)
    auto tile_of = [&](int t) { return (t / ntile) * a.total_tiles + tile0 + t % ntile; };
    const int total = ntile * a.nimages;
    // a contiguous run of tiles per workgroup, runs placed XCD-contiguously (xcd_remap)
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int t_end = (int)((long long)(lb + 1) * total / gridDim.x);
    int t = (int)((long long)lb * total / gridDim.x);
    if (t >= t_end) return;
    BlurTile bt = blur_tile(a, tile_of(t));
    uint4 pre[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int i = threadIdx.x + 256 * c;
        if (i < IH * IWQ) pre[c] = blur_chunk(a, bt, i, IWQ);
    }
    for (; t < t_end; ++t) {
        const BlurTile cur = bt;
        const LevelGeom G = a.lv[cur.l];
        const int ty0 = cur.ty0, tx0 = cur.tx0;
        uint8_t* dst = cur.dst;
        __syncthreads();  // the previous tile's passes are done with tin4 / hp
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int i = threadIdx.x + 256 * c;
            if (i < IH * IWQ) (&tin4[0][0])[i] = pre[c];
        }
        const int tn = t + 1;
        if (tn < t_end) {  // prefetch the next window
            bt = blur_tile(a, tile_of(tn));
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const int i = threadIdx.x + 256 * c;
                if (i < IH * IWQ) pre[c] = blur_chunk(a, bt, i, IWQ);
            }
        }
        __syncthreads();
        blur_tile_compute_mfma(G, tx0, ty0, dst, tin4, hp, 0, G.h);
    }
}

// ---------------------------------------------------------------------------------------------
// k_blur_resize: one read of level l - 1 serves two stages.  A workgroup stages the 128 x 32
// blur tile's window of level l - 1 (rows ty0-4 .. ty0+35, columns tx0-16 .. tx0+143, 16-byte
// buffer loads, REFLECT_101 rows) once, filters it (GaussianBlur of level l - 1, :1146-1147) and
// makes the level-l outputs whose first source row / column fall inside the tile (cv::resize of
// ComputePyramid, :1342-1344; exact-2x levels by INTER_AREA): their taps (source rows <= ty0+32,
// columns <= tx0+134 for scales <= 2) all lie in the window's real pixels, so level l needs no
// second read of level l - 1 and the blur of level l - 1 none of its own.  Ownership tables
// (band_row / tile_quad) come from the host with the resize coefficients.
static_assert(kBrMaxQuads >= kBlurTW / 4 + 1 && kBrMaxRows >= kBlurTH + 1, "ownership caps");

struct BrSmem {
    uint4 tin4[kBlurTH + 8][(kBlurTW + 32) / 16];
    uint4 hp[(kBlurTH + 8) / 2][kBlurTW / 4];
    // per owned output quad (rs_quad): tap selectors, coefficient pairs, first left tap; one
    // array per field so a wave's consecutive quads read consecutive entries
    int4 xsel[kBrMaxQuads];
    int4 xcw[kBrMaxQuads];
    int xbase[kBrMaxQuads];
    int4 yts[kBrMaxRows];
};

// Blur tile k of level s = l - 1 of image img, and (resize) the level-l outputs it owns.  kAux:
// cache policy of the window loads (sc1 where level s was written by this launch).
template <int kAux>
__device__ inline void br_tile(const BatchArgs& a, int l, bool resize, int img, int by, int bx, BrSmem& sm) {
    constexpr int IW = kBlurTW + 32, IH = kBlurTH + 8, IWQ = IW / 16;
    constexpr int NCH = (IH * IWQ + 255) / 256;
    const LevelGeom S = a.lv[l - 1];
    const LevelGeom G = a.lv[resize ? l : l - 1];
    BlurTile bt;
    bt.l = l - 1;
    bt.ty0 = by * kBlurTH;
    bt.tx0 = bx * kBlurTW;
    bt.src = a.lvl_base[l - 1] + (long long)img * S.img_stride;
    bt.dst = a.blur_base[l - 1] + (long long)img * S.bimg_stride;
    uint4 pre[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int i = threadIdx.x + 256 * c;
        if (i < IH * IWQ) pre[c] = blur_chunk<kAux>(a, bt, i, IWQ);
    }
    // the level-l outputs this tile owns, and their coefficients
    int r0 = 0, nr = 0, q0 = 0, nq = 0;
    if (resize) {
        const int* band_row = reinterpret_cast<const int*>(a.rtab) + G.band_row_off;
        const int* tile_quad = reinterpret_cast<const int*>(a.rtab) + G.tile_quad_off;
        r0 = band_row[by];
        q0 = tile_quad[bx];
        nr = min(band_row[by + 1] - r0, kBrMaxRows);
        nq = min(tile_quad[bx + 1] - q0, kBrMaxQuads);
        if (!G.area2) {
            if (threadIdx.x < nq) {
                const int q = threadIdx.x;
                int4 x[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) x[k] = a.rtab[G.xtab_off + min(4 * (q0 + q) + k, G.w - 1)];
                const int base = x[0].x;
                int sl[4], cl[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // taps relative to base: 0 .. 7 (scale <= 2)
                    sl[k] = (x[k].x - base) | 0x0c00 | ((x[k].y - base) << 16) | 0x0c000000;
                    cl[k] = (x[k].z << 4) | (x[k].w << 20);  // 16 c (rs_quad)
                }
                sm.xsel[q] = make_int4(sl[0], sl[1], sl[2], sl[3]);
                sm.xcw[q] = make_int4(cl[0], cl[1], cl[2], cl[3]);
                sm.xbase[q] = base;
            }
            if (threadIdx.x < nr) {  // (y0, y1, b0 << 8, b1 << 8): rs_quad's v_mul_hi_u32_u24 operands
                const int4 y = a.rtab[G.ytab_off + r0 + threadIdx.x];
                sm.yts[threadIdx.x] = make_int4(y.x, y.y, y.z << 8, y.w << 8);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int i = threadIdx.x + 256 * c;
        if (i < IH * IWQ) (&sm.tin4[0][0])[i] = pre[c];
    }
    __syncthreads();
    blur_tile_compute_mfma(S, bt.tx0, bt.ty0, bt.dst, sm.tin4, sm.hp, 0, S.h);  // fixes only off-plane columns
    if (!resize) return;
    // resize from the window: window row r = source row ty0 - 4 + r, column c = tx0 - 16 + c
    const uint8_t* wb = reinterpret_cast<const uint8_t*>(&sm.tin4[0][0]);
    const int wy0 = bt.ty0 - 4, wx0 = bt.tx0 - 16;
    uint8_t* dst = a.lvl_base[l] + (long long)img * G.img_stride;
    // thread -> (quad q, rows rr0, rr0 + step, ...): the quad's selectors and coefficients are
    // read once per tile, one division per tile instead of one per output quad
    if (nq <= 0) return;
    // t / nq and 256 / nq by v_rcp_f32 (1 ulp): (t + 0.5) / nq for t <= 256, nq <= kBrMaxQuads
    // lies >= 0.5 / nq from an integer, far beyond the error, so the floors are exact (a full
    // integer division here cost ~20 VALU per thread and tile)
    const float rnq = __builtin_amdgcn_rcpf((float)nq);
    const int step = max((int)(256.5f * rnq), 1);
    const int rr0 = (int)(((float)threadIdx.x + 0.5f) * rnq), q = (int)threadIdx.x - rr0 * nq;
    if (rr0 >= step) return;
    const int dx0 = 4 * (q0 + q);
    if (G.area2) {
        for (int rr = rr0; rr < nr; rr += step) {
            const int dy = r0 + rr;
            const uint8_t* s0 = wb + __mul24(2 * dy - wy0, IW) - wx0;
            const uint8_t* s1 = s0 + IW;
            uint32_t packed = 0;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int dx = min(dx0 + kk, G.w - 1);
                const int o = (s0[2 * dx] + s0[2 * dx + 1] + s1[2 * dx] + s1[2 * dx + 1] + 2) >> 2;
                packed |= (uint32_t)o << (8 * kk);
            }
            *reinterpret_cast<uint32_t*>(dst + plane_off(dy, G.pitch, dx0)) = packed;
        }
    } else {
        const int4 xsel = sm.xsel[q], xcw = sm.xcw[q];
        const int xbase = sm.xbase[q];
        for (int rr = rr0; rr < nr; rr += step) {
            const int dy = r0 + rr;
            const int4 yt = sm.yts[rr];
            const uint8_t* row0 = wb + __mul24(yt.x - wy0, IW) - wx0;
            const uint8_t* row1 = wb + __mul24(yt.y - wy0, IW) - wx0;
            const uint32_t packed = rs_quad(row0, row1, xbase, xsel, xcw, yt.z, yt.w, dx0, G.simd_end);
            *reinterpret_cast<uint32_t*>(dst + plane_off(dy, G.pitch, dx0)) = packed;
        }
    }
}

// n / d for a launch constant d by a mul-high with the host's magic ceil(2^32 / d) (d >= 2;
// magic 0 stands for d == 1); exact for 0 <= n < 2^32 / d
__device__ inline int div_magic(int n, uint32_t magic) {
    return magic ? (int)__umulhi((uint32_t)n, magic) : n;
}

__global__ __launch_bounds__(256) void k_blur_resize(BatchArgs a, int l, uint32_t per_magic, uint32_t tx_magic) {
    __shared__ BrSmem sm;
    const LevelGeom S = a.lv[l - 1];
    const int per = S.tiles_x * S.tiles_y;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);  // an image's tiles on one XCD
    const int irel = div_magic(wg, per_magic);
    const int k = wg - irel * per;
    const int by = div_magic(k, tx_magic), bx = k - by * S.tiles_x;
    br_tile<0>(a, l, true, a.img0 + irel, by, bx, sm);
}


// k_level_linear: level l from level l - 1 in HBM for any scale step (ComputePyramid's cv::resize
// INTER_LINEAR, ORBextractor_old.cc:1342-1344; the generic 2-tap path of OpenCV 4.2's resize, as
// oracle/orb_oracle.cpp resize_linear restates it).  k_blur_resize stages one blur tile of level
// l - 1 and makes the outputs whose taps it holds, which needs scale steps <= 2 (rs_quad reads the
// 8 source bytes from a quad's first tap); scale factors above 2 (accepted by ORBextractor, not
// used by ORB-SLAM3's configurations) take this kernel and then k_blur per level.  Thread = one
// output quad of one row; every tap is a byte load from the previous level.
__global__ __launch_bounds__(256) void k_level_linear(BatchArgs a, int l) {
    const LevelGeom G = a.lv[l], S = a.lv[l - 1];
    const int nq = (G.w + 3) >> 2;
    const int item = blockIdx.x * 256 + threadIdx.x;
    if (item >= nq * G.h) return;
    const int img = a.img0 + blockIdx.y;
    const int dy = item / nq, q = item - dy * nq;
    const uint8_t* src = a.lvl_base[l - 1] + (long long)img * S.img_stride;
    uint8_t* dst = a.lvl_base[l] + (long long)img * G.img_stride;
    const int4 yt = a.rtab[G.ytab_off + dy];  // (sy0, sy1, b0, b1), rows clamped
    const uint8_t* r0 = src + plane_off(yt.x, S.pitch, 0);
    const uint8_t* r1 = src + plane_off(yt.y, S.pitch, 0);
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int dx = min(4 * q + k, G.w - 1);
        const int4 xt = a.rtab[G.xtab_off + dx];  // (sx0, sx1, a0, a1), a1 = 0 past the last pair
        const int d0 = r0[xt.x] * xt.z + r0[xt.y] * xt.w;
        const int d1 = r1[xt.x] * xt.z + r1[xt.y] * xt.w;
        int o;
        if (dx < G.simd_end) {  // VResizeLinearVec_32s8u: v_mul_hi of the packed (D >> 4), v_rshr_pack_u<2>
            const int t0 = min(d0 >> 4, 32767), t1 = min(d1 >> 4, 32767);
            const int sum = min(max(((t0 * yt.z) >> 16) + ((t1 * yt.w) >> 16), -32768), 32767);
            o = (sum + 2) >> 2;
        } else {  // FixedPtCast<int, uchar, 22>
            o = (d0 * yt.z + d1 * yt.w + (1 << 21)) >> 22;
        }
        packed |= (uint32_t)min(max(o, 0), 255) << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(dst + plane_off(dy, G.pitch, 4 * q)) = packed;
}

hipError_t launch_level_linear(const BatchArgs& a, int l, hipStream_t s) {
    const LevelGeom G = a.lv[l];
    const int items = ((G.w + 3) >> 2) * G.h;
    hipLaunchKernelGGL(k_level_linear, dim3((items + 255) / 256, a.nimages), dim3(256), 0, s, a, l);
    return hipGetLastError();
}

hipError_t launch_blur_resize(const BatchArgs& a, int l, hipStream_t s) {
    const LevelGeom S = a.lv[l - 1];
    auto magic = [](uint32_t d) { return d > 1 ? 0xFFFFFFFFu / d + 1u : 0u; };  // exact for n < 2^32 / d
    hipLaunchKernelGGL(k_blur_resize, dim3(S.tiles_x * S.tiles_y * a.nimages), dim3(256), 0, s, a, l,
                       magic((uint32_t)(S.tiles_x * S.tiles_y)), magic((uint32_t)S.tiles_x));
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// k_pyr_tail: the small levels of the pyramid in ONE launch, one 1024-thread workgroup per image.
// Level s0 = tail0 - 1 (made by the last k_blur_resize) is loaded into LDS once; then for
// s = s0 .. L-1 the workgroup writes level s's blur (GaussianBlur 7x7, :1146-1147) and makes level
// s + 1 (cv::resize INTER_LINEAR / exact-2x INTER_AREA, :1342-1344) from the LDS copy into the
// other LDS buffer and to HBM.  Each of these levels took its own launch of a few thousand
// 128 x 32 tiles before, and every such launch was latency-bound (level 7: 32 us per 512 images
// for 24 K pixels per image).  Two buffers alternate (level s0 + 2k in buffer 0, s0 + 2k + 1 in
// buffer 1; each level is smaller than the one two steps before).  Row pitch Pitch(l) holds kTailPad
// bytes on the left (REFLECT_101 columns -3 .. -1) and >= 12 on the right (resize reads 12
// bytes from a quad's first tap), so the blur and rs_quad read the same window layout as k_blur.
constexpr int kTailThreads = 1024;

__device__ inline void tail_fill_pads(uint8_t* buf, int P, int w, int h) {
    for (int i = threadIdx.x; i < h * 6; i += kTailThreads) {
        const int y = i / 6, k = i - 6 * y;
        uint8_t* row = buf + __mul24(y, P) + kTailPad;
        if (k < 3) row[-1 - k] = row[1 + k];          // columns -1, -2, -3 <- 1, 2, 3
        else row[w + k - 3] = row[w - 2 - (k - 3)];    // columns w, w+1, w+2 <- w-2, w-3, w-4
    }
}

// Horizontal 7-tap sums of the 4 columns 4cq .. 4cq+3 of two LDS rows as u16 pairs (row a, row b):
// hsum_pair, as blur_tile_compute (window bytes 4cq+12 .. 4cq+23).
__device__ inline void tail_hpair(const uint8_t* ra, const uint8_t* rb, int cq, uint32_t out[4]) {
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(ra) + cq + 3;
    const uint32_t* pb = reinterpret_cast<const uint32_t*>(rb) + cq + 3;
    uint32_t A[3], B[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        A[d] = pa[d];
        B[d] = pb[d];
    }
    hsum_pair(A, B, out);
}

// Blur of one LDS-resident level.  Task = (column quad, segment of R rows), with the segment
// count chosen so the workgroup's 1024 threads get one task each where the level allows; a task
// slides down its rows with the last five row pairs in registers, so every row's horizontal sums
// are formed once (plus four pairs of prologue).  Row pair j of a task covers rows
// y0-4+2j, y0-3+2j (REFLECT_101 by index); output rows y0+2m / y0+2m+1 take pairs m .. m+3 with the
// even weights / m+1 .. m+4 with the odd ones (blur_tile_compute's vertical pass).
__device__ inline void tail_blur(const uint8_t* buf, int P, const LevelGeom& G, uint8_t* dst) {
    const int nq = (G.w + 3) >> 2;
    const int per = kTailThreads / nq > 0 ? kTailThreads / nq : 1;  // segments per column
    int R = (G.h + per - 1) / per;
    R = (R + 1) & ~1;
    const int nseg = (G.h + R - 1) / R;
    const u16x2 WE[4] = {as_u16x2(0u | (18u << 16)), as_u16x2(34u | (48u << 16)),
                         as_u16x2(56u | (48u << 16)), as_u16x2(34u | (18u << 16))};
    const u16x2 WO[4] = {as_u16x2(18u | (34u << 16)), as_u16x2(48u | (56u << 16)),
                         as_u16x2(48u | (34u << 16)), as_u16x2(18u | (0u << 16))};
    // REFLECT_101 of rows -4 .. h + 4 as min(|y|, 2h - 2 - |y|): one reflection suffices, every
    // level has >= 2 kEdge + 4 rows (the host's level check); rows >= 0 skip the |y|
    const int h2 = 2 * G.h - 2;
    auto row = [&](int y) {
        const int ay = max(y, -y);
        return buf + __mul24(min(ay, h2 - ay), P);
    };
    auto row_lo = [&](int y) { return buf + __mul24(min(y, h2 - y), P); };
    for (int t0 = 0; t0 < nq * nseg; t0 += kTailThreads) {
        const int t = t0 + (int)threadIdx.x;
        const int sg = t / nq, cq = t - sg * nq;  // one division per task
        if (sg >= nseg) break;
        const int y0 = sg * R, y1 = min(y0 + R, G.h);
        // the last five row pairs' sums in five register sets, the loop unrolled by five so that
        // each step names them in rotated order (no register moves between rows)
        uint32_t V0[4], V1[4], V2[4], V3[4], V4[4];
        tail_hpair(row(y0 - 4), row(y0 - 3), cq, V0);
        tail_hpair(row(y0 - 2), row(y0 - 1), cq, V1);
        tail_hpair(row(y0), row(y0 + 1), cq, V2);
        tail_hpair(row(y0 + 2), row(y0 + 3), cq, V3);
        uint8_t* d = dst + plane_off(y0, G.bpitch, 4 * cq);
        using Pair4 = uint32_t[4];
        // output row from pairs p0 .. p3 (weights W): 4 columns, bytes 2 of the sums
        auto vsum = [&](const Pair4& p0, const Pair4& p1, const Pair4& p2, const Pair4& p3, const u16x2* W) {
            uint32_t sv[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                uint32_t acc = 1u << 15;
                acc = __builtin_amdgcn_udot2(as_u16x2(p0[c]), W[0], acc, false);
                acc = __builtin_amdgcn_udot2(as_u16x2(p1[c]), W[1], acc, false);
                acc = __builtin_amdgcn_udot2(as_u16x2(p2[c]), W[2], acc, false);
                acc = __builtin_amdgcn_udot2(as_u16x2(p3[c]), W[3], acc, false);
                sv[c] = acc;
            }
            return __builtin_amdgcn_perm(sv[1], sv[0], 0x0c0c0602u) | __builtin_amdgcn_perm(sv[3], sv[2], 0x06020c0cu);
        };
        // rows y, y + 1 from pairs m .. m + 3 (even weights) and m + 1 .. m + 4 (odd), pair m + 4
        // (rows y + 4, y + 5) loaded into n
        auto step = [&](const Pair4& a, const Pair4& b, const Pair4& c, const Pair4& e, Pair4& n, int y) {
            tail_hpair(row_lo(y + 4), row_lo(y + 5), cq, n);
            *reinterpret_cast<uint32_t*>(d) = vsum(a, b, c, e, WE);
            if (y + 1 < y1) *reinterpret_cast<uint32_t*>(d + G.bpitch) = vsum(b, c, e, n, WO);
            d += 2 * G.bpitch;
        };
        for (int y = y0;;) {  // y0 < y1: at least one step
            step(V0, V1, V2, V3, V4, y);
            if ((y += 2) >= y1) break;
            step(V1, V2, V3, V4, V0, y);
            if ((y += 2) >= y1) break;
            step(V2, V3, V4, V0, V1, y);
            if ((y += 2) >= y1) break;
            step(V3, V4, V0, V1, V2, y);
            if ((y += 2) >= y1) break;
            step(V4, V0, V1, V2, V3, y);
            if ((y += 2) >= y1) break;
        }
    }
}

__global__ __launch_bounds__(kTailThreads) void k_pyr_tail(BatchArgs a) {
    extern __shared__ uint4 tail_lds[];
    uint8_t* lds = reinterpret_cast<uint8_t*>(tail_lds);
    const int img = a.img0 + blockIdx.x;
    const int s0 = a.tail0 - 1, L = a.nlevels;
    // buffers as offsets from the LDS base (an array of pointers would decay to generic
    // pointers: flat accesses, which fault on the 4-byte-aligned 12-byte row reads)
    auto buf = [&](int k) { return lds + (k ? a.tail_buf1 : 0); };
    int4* xsel = reinterpret_cast<int4*>(lds + a.tail_tab);
    int4* xcw = xsel + a.tail_maxq;
    int4* yts = xcw + a.tail_maxq;
    int* xbase = reinterpret_cast<int*>(yts + a.tail_maxrows);
    {   // level s0 from HBM (16-byte loads, 16-byte aligned LDS rows)
        const LevelGeom S = a.lv[s0];
        const uint8_t* src = a.lvl_base[s0] + (long long)img * S.img_stride;
        const int nch = (S.w + 15) >> 4, P = S.tpitch;
        for (int i = threadIdx.x; i < nch * S.h; i += kTailThreads) {
            const int y = i / nch, c = i - y * nch;
            *reinterpret_cast<uint4*>(buf(0) + __mul24(y, P) + kTailPad + 16 * c) =
                *reinterpret_cast<const uint4*>(src + plane_off(y, S.pitch, 16 * c));
        }
        __syncthreads();
        tail_fill_pads(buf(0), P, S.w, S.h);
        __syncthreads();
    }
    for (int s = s0; s < L; ++s) {
        const LevelGeom S = a.lv[s];
        const uint8_t* cur = buf((s - s0) & 1);
        const bool resize = s + 1 < L;
        const LevelGeom G = a.lv[resize ? s + 1 : s];
        const int nq = (G.w + 3) >> 2;
        if (resize && !G.area2) {  // level s + 1's quad and row coefficients (as br_tile)
            for (int q = threadIdx.x; q < nq; q += kTailThreads) {
                int4 xx[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) xx[k] = a.rtab[G.xtab_off + min(4 * q + k, G.w - 1)];
                const int base = xx[0].x;
                int sl[4], cl[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    sl[k] = (xx[k].x - base) | 0x0c00 | ((xx[k].y - base) << 16) | 0x0c000000;
                    cl[k] = (xx[k].z << 4) | (xx[k].w << 20);
                }
                xsel[q] = make_int4(sl[0], sl[1], sl[2], sl[3]);
                xcw[q] = make_int4(cl[0], cl[1], cl[2], cl[3]);
                xbase[q] = base;
            }
            for (int r = threadIdx.x; r < G.h; r += kTailThreads) {
                const int4 y = a.rtab[G.ytab_off + r];
                yts[r] = make_int4(y.x, y.y, y.z << 8, y.w << 8);
            }
        }
        tail_blur(cur, S.tpitch, S, a.blur_base[s] + (long long)img * S.bimg_stride);
        if (!resize) break;
        __syncthreads();  // coefficient tables
        uint8_t* nxt = buf((s + 1 - s0) & 1);
        uint8_t* dst = a.lvl_base[s + 1] + (long long)img * G.img_stride;
        const uint8_t* rowp = cur + kTailPad;
        // thread -> (quad q, rows dy0, dy0 + step, ...): one division per level
        const int step = max(kTailThreads / nq, 1);
        const int q = (int)threadIdx.x % nq, dyt = (int)threadIdx.x / nq;
        for (int dy = dyt; dy < G.h && dyt < step; dy += step) {
            const int dx0 = 4 * q;
            uint32_t packed = 0;
            if (G.area2) {
                const uint8_t* s0r = rowp + __mul24(2 * dy, S.tpitch);
                const uint8_t* s1r = s0r + S.tpitch;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int dx = min(dx0 + kk, G.w - 1);
                    const int o = (s0r[2 * dx] + s0r[2 * dx + 1] + s1r[2 * dx] + s1r[2 * dx + 1] + 2) >> 2;
                    packed |= (uint32_t)o << (8 * kk);
                }
            } else {
                const int4 yt = yts[dy];
                packed = rs_quad(rowp + __mul24(yt.x, S.tpitch), rowp + __mul24(yt.y, S.tpitch), xbase[q], xsel[q],
                                 xcw[q], yt.z, yt.w, dx0, G.simd_end);
            }
            *reinterpret_cast<uint32_t*>(nxt + __mul24(dy, G.tpitch) + kTailPad + dx0) = packed;
            *reinterpret_cast<uint32_t*>(dst + plane_off(dy, G.pitch, dx0)) = packed;
        }
        __syncthreads();  // level s + 1 complete in LDS; level s's buffer and the tables are free
        tail_fill_pads(nxt, G.tpitch, G.w, G.h);
        __syncthreads();
    }
}

hipError_t launch_pyr_tail(const BatchArgs& a, hipStream_t s) {
    // the dynamic-LDS limit is raised once per size and device (see launch_octree)
    constexpr int kMaxDevices = 64;
    static std::atomic<int> lds_set[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = kMaxDevices - 1;
    if (a.tail_lds > 65536 && a.tail_lds > lds_set[dev].load()) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_pyr_tail),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, a.tail_lds);
        if (e != hipSuccess) return e;
        int cur = lds_set[dev].load();
        while (a.tail_lds > cur && !lds_set[dev].compare_exchange_weak(cur, a.tail_lds)) {}
    }
    hipLaunchKernelGGL(k_pyr_tail, dim3(a.nimages), dim3(kTailThreads), a.tail_lds, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// k_fast_cells: one workgroup per (level, cell), image = blockIdx.y.  Restates the cell loop of
// ComputeKeyPointsOctTree (ORBextractor_old.cc:807-871) with cv::FAST(cell, kps, th, true):
// detection on [3,rows-3)x[3,cols-3) of the cell ROI, 3x3 nonmax inside the cell only, iniTh
// then minTh if the cell yields nothing, keys emitted in row-major order.

// One cell of image img (flattened cell index gcell) with a candidate list of kCap entries;
// returns the kept count (written to the cell's count) or kFastOverflow (nothing written).
template <int CP, int kCap>
__device__ __attribute__((always_inline)) inline int fast_cell_one(const BatchArgs& a, int img, int gcell, uint8_t* T,
                                                                   uint8_t* M, uint16_t* list, uint2* lut,
                                                                   uint32_t* emask, int32_t* wcnt, int32_t* wovf,
                                                                   int* scratch) {
    constexpr int kFastThreads = fast_threads<CP>();
    // the cell's record (host: the cell loop's geometry, :807-821)
    const int4 e0 = a.rtab[a.fast_tab_off + 2 * gcell];
    const int4 e1 = a.rtab[a.fast_tab_off + 2 * gcell + 1];
    const int l = e0.x;
    const LevelGeom G = a.lv[l];
    int32_t* cnt_out = a.cellcnt + (long long)img * a.cellcnt_img_stride + e1.x;
    uint32_t* key_out = a.cellkeys + (long long)img * a.cellkeys_img_stride + e1.y;
    CellGeom g;
    g.iniX = e0.y;
    g.iniY = e0.z;
    g.minBorder = kMinBorder;
    if (e1.z) {  // :812, :821
        if (threadIdx.x == 0) *cnt_out = 0;
        return 0;
    }
    g.rows = e0.w & 0xFFFF;
    g.cols = e0.w >> 16;
    const bool dword_ok = ((G.pitch | G.img_stride) & 3) == 0;
    const int sh = dword_ok ? (g.iniX & 3) : 0;
    const uint8_t* base = a.lvl_base[l] + (long long)img * G.img_stride;
    const long long roi = (long long)g.iniY * G.pitch + (g.iniX - sh);
    const uint8_t* src = base + roi;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)base, (short)0, (int)min(G.img_stride, 0x7fffffffLL), 0x00020000);
    const int roi32 = (int)roi;  // planes are < 2 GB (buffer offsets are 32-bit)
    auto ld16 = [&](long long off) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, roi32 + (int)off, 0, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
    };
    FixedDevPolicy<kFastThreads> p{{scratch}};
    fast_cell_tables<CP>(g, sh, lut, emask);  // synced with the ROI staging (fast_cell_run)
    CellScratch cs{T, M, list, wcnt, lut, emask, wovf};
    const int n = fast_cell_run<CP, kCap>(p, src, G.pitch, sh, dword_ok, g, a.ini_th, a.min_th, cs, key_out, ld16);
    if (n != kFastOverflow && threadIdx.x == 0) *cnt_out = n;
    return n;
}

// k_fast_cells<CP, kSmall>: one workgroup per (image, cell) of the tile's cells.  kSmall (the
// 48- and 64-byte tiles of launches of more than kFastMergeMaxImages images): a capped candidate
// list, kFastSmallList<CP> entries split over the waves (48: LDS 5.9 instead of 8.4 KB per
// workgroup, 26 instead of 19 resident per CU; 64: 11 instead of 15.2 KB; round 6: residency
// moves this kernel by up to ~20%).  A cell whose pre-test passes more pixels than fit (none of
// the bench frames' cells at iniThFAST, where the most is 441 of 1225 in a 48-byte cell) is
// queued (a.fast_ovf, per-launch slice by img0) and redone by k_fast_cells_ovf.
template <int CP, bool kSmall>
__global__ __launch_bounds__(fast_threads<CP>()) void k_fast_cells(BatchArgs a, int cell0, uint32_t ncell_magic) {
    constexpr int kList = kSmall ? kFastSmallList<CP>() : cell_list_cap<CP>(), kFastThreads = fast_threads<CP>();
    __shared__ __attribute__((aligned(16))) uint8_t T[CP * CP];
    __shared__ __attribute__((aligned(16))) uint8_t M[CP * CP];  // 16-byte rows when CP % 16 == 0
    __shared__ __attribute__((aligned(8))) uint16_t list[kList + fast_list_slack(kFastThreads / 64)];
    __shared__ uint2 lut[16];
    __shared__ uint32_t emask[32];
    __shared__ int32_t wcnt[kFastThreads / 64], wovf[kFastThreads / 64];
    __shared__ int scratch[16];
    const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    // wg / gridDim.x by the host's magic multiplier (exact for wg < 2^32 / gridDim.x)
    const int irel = gridDim.x == 1 ? wg : (int)__umulhi((uint32_t)wg, ncell_magic);
    const int img = a.img0 + irel;
    const int gcell = cell0 + (wg - irel * (int)gridDim.x);  // flattened over the levels
    const int n = (kSmall && a.fast_ovf_all) ? kFastOverflow  // diagnostics: every cell to the full-list pass
                                             : fast_cell_one<CP, kList>(a, img, gcell, T, M, list, lut, emask, wcnt, wovf, scratch);
    if (kSmall && n == kFastOverflow && threadIdx.x == 0) {
        const int q = __hip_atomic_fetch_add(a.fast_ovf_cnt + 2 * a.img0, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.fast_ovf[(long long)a.img0 * a.fast_qcap + q] = make_int2(img, gcell);
    }
}

// The cells k_fast_cells<CP, true> queued, with the full candidate list: a small grid walks the
// launch's queue (the count is read after the queueing launch finished: same stream); the last
// workgroup to finish resets the count and its own arrival counter for the next launch.
template <int CP>
__global__ __launch_bounds__(fast_threads<CP>()) void k_fast_cells_ovf(BatchArgs a) {
    constexpr int kList = cell_list_cap<CP>(), kFastThreads = fast_threads<CP>();
    __shared__ __attribute__((aligned(16))) uint8_t T[CP * CP];
    __shared__ __attribute__((aligned(16))) uint8_t M[CP * CP];
    __shared__ __attribute__((aligned(8))) uint16_t list[kList + fast_list_slack(kFastThreads / 64)];
    __shared__ uint2 lut[16];
    __shared__ uint32_t emask[32];
    __shared__ int32_t wcnt[kFastThreads / 64], wovf[kFastThreads / 64];
    __shared__ int scratch[16];
    int* const cnt = a.fast_ovf_cnt + 2 * a.img0;  // [0] queued cells, [1] finished workgroups
    // written by the previous launch on this stream (complete before this one starts): a plain
    // load; with nothing queued (the usual case) the launch ends here, no counter to reset
    const int nq = *cnt;
    if (nq == 0) return;
    for (int q = blockIdx.x; q < nq; q += gridDim.x) {
        const int2 e = a.fast_ovf[(long long)a.img0 * a.fast_qcap + q];
        fast_cell_one<CP, kList>(a, e.x, e.y, T, M, list, lut, emask, wcnt, wovf, scratch);
        __syncthreads();  // the LDS scratch is reused by the next cell
    }
    if (threadIdx.x == 0) {
        // every workgroup has read the count once it arrives here (the loop above depends on the
        // value), so the last one may clear both; the counters order nothing else (relaxed)
        const int done = __hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (int)gridDim.x - 1) {
            __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_octree: one workgroup per (level, image).  Gathers the level's cell lists in cell order
// (vToDistributeKeys, :807-871) then runs DistributeOctTree (orb_octree.h) with the node
// state in LDS (80 KB: two workgroups per CU).
// kOctRetry: the level did not fit the LDS instantiation (node capacity, cell offsets or more
// than kOctLdsKeys candidates); k_octree_retry then redoes it with generic pointers.
constexpr int kOctRetry = -7;

template <bool kLdsPath>
__device__ __attribute__((always_inline)) inline void octree_level(const BatchArgs& a, int img, int l,
                                                                   uint8_t* nodemem_lds, int* scratch,
                                                                   OctShared& sh, const OctCfg q) {
    const LevelGeom G = a.lv[l];
    DevPolicy p{scratch};
    const int32_t* cnt = a.cellcnt + (long long)img * a.cellcnt_img_stride + G.cellcnt_off;
    const uint32_t* ck = a.cellkeys + (long long)img * a.cellkeys_img_stride + G.cellkey_off;
    uint8_t* ws = a.octws + (long long)img * a.octws_img_stride + G.oct_off;
    const OctLayout L = oct_layout(G.cand_cap, G.oct_cap);
    uint32_t* keys = reinterpret_cast<uint32_t*>(ws + L.keys);
    void* nm = G.oct_cap <= q.lds_nodes ? (void*)nodemem_lds : (void*)(ws + L.nodemem);
    // exclusive scan of the cell counts into LDS (the node area is free until the octree's
    // gather has read it)
    int32_t* cell_off = reinterpret_cast<int32_t*>(nodemem_lds);
    const bool off_in_lds = G.ncells <= q.nq_off / 4;
    if (!off_in_lds) cell_off = reinterpret_cast<int32_t*>(ws + L.nq);  // huge levels only
    auto scan_cells = [&]() {
        int carry = 0;
        for (int base = 0; base < G.ncells; base += blockDim.x) {
            const int i = base + threadIdx.x;
            const int v = i < G.ncells ? cnt[i] : 0;
            int tot;
            const int ex = p.scan_excl(v, &tot);
            if (i < G.ncells) cell_off[i] = carry + ex;
            carry += tot;
        }
        __syncthreads();
        return carry;
    };
    const int n = scan_cells();
    uint32_t* out_keys = a.lvlkey + (long long)img * a.lvlkp_img_stride + G.kp_off;
    unsigned long long* dbg = a.octdbg ? a.octdbg + ((long long)img * kMaxLevels + l) * 8 : nullptr;
    int r = n > G.cand_cap ? -3 : 0;
    // node state and cell offsets in LDS; the per-key labels too up to q.lds_keys keys, in the
    // global workspace above that (dense levels of large frames: the label passes are parallel
    // and streaming, the serial node phases stay in LDS)
    const bool nodes_fit = off_in_lds && G.oct_cap <= q.lds_nodes && !a.oct_force_retry;
    // the count pyramid takes the LDS the level's node state and cell offsets leave (orb_octree.h)
    const int pyr_off = (int)((max(oct_nodemem_bytes(G.oct_cap), (size_t)(4 * G.ncells)) + 15) & ~(size_t)15);
    // (the pyramid names keys by cell * cell_cap + slot in 24 bits)
    const int pyrD = kLdsPath && q.lds_bytes > pyr_off && (long long)G.ncells * G.cell_cap < (1 << 24)
                         ? oct_pyr_depth((size_t)(q.lds_bytes - pyr_off), G.W, G.H, a.oct_pyr_max)
                         : 0;
    uint16_t* xtbl = reinterpret_cast<uint16_t*>(nodemem_lds + pyr_off + oct_pyr_bytes(pyrD, oct_nini(G.W, G.H)));
    if (kLdsPath && r == 0 && !nodes_fit) r = kOctRetry;
    if (kLdsPath && r == 0 && n > q.lds_keys) {
        OctWST<kLdsAS, kGlobalAS, kGlobalAS> w;
        w.keys = (asp<kGlobalAS, uint32_t>)keys;
        w.n = n;
        w.nq = (asp<kGlobalAS, uint16_t>)(ws + L.nq);
        w.m = oct_nodemem_carve<kLdsAS>(nodemem_lds, G.oct_cap);
        w.cap = G.oct_cap;
        w.out_keys = (asp<kGlobalAS, uint32_t>)out_keys;
        w.out_cap = G.kp_cap;
        w.dbg = dbg;
        w.cell_off = (asp<kLdsAS, const int32_t>)cell_off;
        w.cellkeys = (asp<kGlobalAS, const uint32_t>)ck;
        w.ncells = G.ncells;
        w.cell_cap = G.cell_cap;
        w.pyr = (asp<kLdsAS, uint32_t>)(nodemem_lds + pyr_off);
        w.pyrD = pyrD;
        w.xcode = (asp<kLdsAS, uint16_t>)xtbl;
        w.ycode = (asp<kLdsAS, uint16_t>)(xtbl + G.W + 1);
        r = octree_distribute(p, w, (asp<kLdsAS, OctShared>)&sh, G.W, G.H, G.N);
        if (r == kOctDeep) {  // deeper than the pyramid: the label passes from the start
            __syncthreads();
            scan_cells();  // the node state overwrote the cell offsets
            w.pyrD = 0;
            r = octree_distribute(p, w, (asp<kLdsAS, OctShared>)&sh, G.W, G.H, G.N);
        }
    } else if (kLdsPath && r == 0) {
        // everything node- and label-sized in LDS: ds_* accesses throughout
        OctWST<kLdsAS, kGlobalAS> w;
        w.keys = (asp<kGlobalAS, uint32_t>)keys;
        w.n = n;
        w.nq = (asp<kLdsAS, uint16_t>)(nodemem_lds + q.nq_off);
        w.m = oct_nodemem_carve<kLdsAS>(nodemem_lds, G.oct_cap);
        w.cap = G.oct_cap;
        w.out_keys = (asp<kGlobalAS, uint32_t>)out_keys;
        w.out_cap = G.kp_cap;
        w.dbg = dbg;
        w.cell_off = (asp<kLdsAS, const int32_t>)cell_off;
        w.cellkeys = (asp<kGlobalAS, const uint32_t>)ck;
        w.ncells = G.ncells;
        w.cell_cap = G.cell_cap;
        w.pyr = (asp<kLdsAS, uint32_t>)(nodemem_lds + pyr_off);
        w.pyrD = pyrD;
        w.xcode = (asp<kLdsAS, uint16_t>)xtbl;
        w.ycode = (asp<kLdsAS, uint16_t>)(xtbl + G.W + 1);
        r = octree_distribute(p, w, (asp<kLdsAS, OctShared>)&sh, G.W, G.H, G.N);
        if (r == kOctDeep) {  // deeper than the pyramid: the label passes from the start
            __syncthreads();
            scan_cells();  // the node state overwrote the cell offsets
            w.pyrD = 0;
            r = octree_distribute(p, w, (asp<kLdsAS, OctShared>)&sh, G.W, G.H, G.N);
        }
    } else if (!kLdsPath && r == 0) {
        // huge levels: node state / labels / cell offsets in the global workspace where needed
        OctWST<kGeneric, kGeneric> w;
        w.keys = keys;
        w.n = n;
        w.nq = n <= q.lds_keys && off_in_lds ? reinterpret_cast<uint16_t*>(nodemem_lds + q.nq_off)
                                             : reinterpret_cast<uint16_t*>(ws + L.nq);
        w.m = oct_nodemem_carve<kGeneric>(nm, G.oct_cap);
        w.cap = G.oct_cap;
        w.out_keys = out_keys;
        w.out_cap = G.kp_cap;
        w.dbg = dbg;
        w.cell_off = cell_off;
        w.cellkeys = ck;
        w.ncells = G.ncells;
        w.cell_cap = G.cell_cap;
        w.pyr = nullptr;
        w.pyrD = 0;
        w.xcode = w.ycode = nullptr;
        if (!off_in_lds && n > q.lds_keys) r = -3;  // cell offsets occupy L.nq
        else r = octree_distribute(p, w, &sh, G.W, G.H, G.N);
    }
    if (threadIdx.x == 0) {
        a.lvlcnt[img * kMaxLevels + l] = r < 0 ? 0 : r;
        a.status[img * kMaxLevels + l] = r < 0 ? r : 0;
    }
}

// One workgroup per (image, level l0 + blockIdx.y), level-major dispatch: the long level-0
// groups go first.  NT = 512 for the leading levels, kOctSmallThreads for the short ones.
template <int NT>
__global__ __launch_bounds__(NT) void k_octree(BatchArgs a, int l0, OctCfg q) {
    extern __shared__ __attribute__((aligned(16))) uint8_t nodemem_lds[];  // per-launch size
    __shared__ int scratch[16];
    __shared__ OctShared sh;
    octree_level<true>(a, a.img0 + blockIdx.x, l0 + blockIdx.y, nodemem_lds, scratch, sh, q);
}

// The levels k_octree left with kOctRetry, redone with generic pointers: a small persistent
// grid walks all (image, level) slots, so the usual no-retry case costs one status read each.
__global__ __launch_bounds__(512, 1) void k_octree_retry(BatchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t nodemem_lds[];  // a.oct_lds_bytes
    __shared__ int scratch[16];
    __shared__ OctShared sh;
    for (int s = blockIdx.x; s < a.nimages * a.nlevels; s += gridDim.x) {
        const int img = a.img0 + s / a.nlevels, l = s % a.nlevels;
        if (a.status[img * kMaxLevels + l] != kOctRetry) continue;  // uniform per workgroup
        octree_level<false>(a, img, l, nodemem_lds, scratch, sh, OctCfg{a.oct_nq_off, a.oct_lds_nodes, kOctLdsKeys, a.oct_lds_bytes});
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
constexpr int kOdLanes = 32;                   // lanes per keypoint
constexpr int kOdPairs = 256 / kOdLanes;       // test pairs per lane
static_assert(kOdLanes == 32, "k_orient_desc: one disc row and 8 test pairs per lane");
static_assert(kOdKpBlock == 256 / kOdLanes, "orb_kernels.h kOdKpBlock");

constexpr int kOdPatchR = 18;                    // |rotated pattern offset| <= 13*sqrt(2) < 19
constexpr int kOdPatchRows = 2 * kOdPatchR + 1;  // 37
constexpr int kOdPatchPitch = 48;                // 3 x 16 B: covers x-18..x+18 from the dword below
constexpr int kOdPatchChunks = kOdPatchRows * 3; // 16-byte chunks per patch
constexpr int kOdPatchIt = (kOdPatchChunks + kOdLanes - 1) / kOdLanes;

// Sum of v over each 32-lane group of the wave, in every lane: DPP quad_perm xor 1 / xor 2, row
// half-mirror (pairs the two quads of 8 lanes) and row mirror (the two halves of a 16-lane row),
// then the other row of the 32 through ds_swizzle (xor mask 16).
__device__ inline int od_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror
    return v + __builtin_amdgcn_ds_swizzle(v, 0x401F);               // lane ^ 16 within 32
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// k_orient_desc's two LDS tables, built at compile time and copied once per workgroup (building
// them in the kernel took ~200 VALU per wave, comparable to a whole keypoint pass):
//   rng[m * 17 + n]: 0xFF in bytes [m, n) of a 16-byte chunk (none if n <= m);
//   pat[b * kOdLanes + lane]: float bit patterns {x0, x1, y0, y1} of test pair 8 lane + b.
struct OdTables {
    uint32_t rng[17 * 17][4];
    uint32_t pat[kOdPairs * kOdLanes][4];
};
constexpr OdTables make_od_tables() {
    OdTables t{};
    for (int m = 0; m < 17; ++m)
        for (int n = 0; n < 17; ++n)
            for (int j = 0; j < 16; ++j)
                if (j >= m && j < n) t.rng[m * 17 + n][j >> 2] |= 0xFFu << (8 * (j & 3));
    const PatternTable pt = make_pattern();
    for (int b = 0; b < kOdPairs; ++b)
        for (int lane = 0; lane < kOdLanes; ++lane) {
            const int8_t* pv = pt.v + 4 * (kOdPairs * lane + b);  // x0, y0, x1, y1
            t.pat[b * kOdLanes + lane][0] = __builtin_bit_cast(uint32_t, (float)pv[0]);
            t.pat[b * kOdLanes + lane][1] = __builtin_bit_cast(uint32_t, (float)pv[2]);
            t.pat[b * kOdLanes + lane][2] = __builtin_bit_cast(uint32_t, (float)pv[1]);
            t.pat[b * kOdLanes + lane][3] = __builtin_bit_cast(uint32_t, (float)pv[3]);
        }
    return t;
}
__constant__ OdTables c_od_tab = make_od_tables();

// cv::KeyPoint as written to the outputs (orbgpu_keypoint): pt.x, pt.y, size, angle, response,
// octave, class_id
struct KP28 {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

// k_orient_desc: IC_Angle on the raw level (ORBextractor_old.cc:78-105) then
// computeOrbDescriptor on the blurred level (:108-148): a = (float)cos, b = (float)sin of
// angle*pi/180 (float), sample center[cvRound(x*b + y*a)*step + cvRound(x*a - y*b)].
// 32 lanes per keypoint (two independent groups per wave): lane `sub` owns disc row v = sub - 15
// for the moments and test pairs [8 sub, 8 sub + 8), sampled from the keypoint's blurred patch
// staged in LDS.  The kernel waits on dependent memory round trips per keypoint (key, moment
// rows + patch); few vector-memory instructions and registers per lane keep many of them in
// flight.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_orient_desc(
    BatchArgs a, uint32_t nblk_magic) {
    // per keypoint group: the blurred patch around the keypoint, staged with 16-byte loads
    __shared__ __attribute__((aligned(16))) uint8_t patch[kOdKpBlock][kOdPatchRows * kOdPatchPitch];
    const int wg = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
    // wg / gridDim.x by the host's magic multiplier; the block's level from a host record (no
    // level search with dependent kernarg loads)
    const int irel = gridDim.x == 1 ? wg : (int)__umulhi((uint32_t)wg, nblk_magic);
    const int img = a.img0 + irel, bx = wg - irel * (int)gridDim.x;
    const int l = a.rtab[a.od_tab_off + bx].x;
    const LevelGeom G = a.lv[l];
    const int sub = threadIdx.x % kOdLanes, grp = threadIdx.x / kOdLanes;
    const int count = a.lvlcnt[img * kMaxLevels + l];
    const long long kbase = (long long)img * a.lvlkp_img_stride + G.kp_off;
    const uint8_t* lvl = a.lvl_base[l] + (long long)img * G.img_stride;
    const uint8_t* blr = a.blur_base[l] + (long long)img * G.bimg_stride;
    const bool raw_dw = ((G.pitch | G.img_stride) & 3) == 0;
    // raw buffer over this image's blurred level (dword 3 = gfx9 raw-buffer format word)
    const __amdgpu_buffer_rsrc_t brs =
        __builtin_amdgcn_make_buffer_rsrc((void*)blr, (short)0, G.bpitch * G.h, 0x00020000);
    const int stride_k = G.od_blocks * kOdKpBlock;
    // a.fuse_out (every image of the batch has no lapping area, so every keypoint is mono): the
    // assembly of k_finalize (ORBextractor_old.cc:1130-1190) is done here -- keypoint j of level l
    // goes to output row off[l] + j, with pt *= mvScaleFactor[l], size, octave, class_id -1 --
    // and k_finalize does not run.  off[l] and the image's total come from the level counts (16
    // scalar loads); a level the octree could not finish or a total past out_cap writes the status
    // word instead, as k_finalize does.
    int out_row0 = 0;
    bool out_ok = false;
    if (a.fuse_out) {
        int total = 0;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < kMaxLevels; ++k)
            if (k < a.nlevels) {
                if (k < l) out_row0 += a.lvlcnt[img * kMaxLevels + k];
                total += a.lvlcnt[img * kMaxLevels + k];
                bad |= a.status[img * kMaxLevels + k] != 0;
            }
        out_ok = !bad && total <= a.out_cap;
        if (bx == 0 && threadIdx.x == 0) {  // one workgroup per image writes the counts
            a.out_n[img] = bad ? -5 : total > a.out_cap ? -2 : total;
            a.out_mono[img] = out_ok ? total : 0;
        }
    }
    KP28* const out_kp = reinterpret_cast<KP28*>(a.out_kps) + (long long)img * a.out_cap + out_row0;
    uint8_t* const out_d = a.out_desc + ((long long)img * a.out_cap + out_row0) * 32;
    // Moments from coalesced row chunks: the 31 disc rows of a keypoint are read as 16-byte
    // aligned chunks of the 48-byte window that starts at xa16 = (x - 15) & ~15 (it holds
    // x - 15 .. x + 15 for every x).  Chunk slot i = sub + 32 it (it < 3) is disc row r = i / 3
    // (v = r - 15; r = 31 lies past the disc) and part i % 3, so the three lanes of a row read 48
    // contiguous bytes -- one or two cache lines per row instead of three 16-byte / dword loads
    // per row lane (round 4: ~105 of the ~160 L1 accesses per keypoint were those).  Each chunk
    // adds its masked byte sums: s = sum of p, c = sum of (column - xa16) p over the disc span
    // |u| <= umax[|v|], i.e. chunk bytes [m, n) with m, n from the alignment a = (x - 15) & 15 and
    // two per-lane constants; the byte masks of every [m, n) are an LDS table, so a chunk is one
    // b128 LDS read, 4 ANDs and 8 v_dot4_u32_u8.  Then m_10 = sum c - (15 + a) sum s and
    // m_01 = sum v s.
    __shared__ __attribute__((aligned(16))) uint4 s_rng[17][17];  // bytes [m, n) of 16 (none if n <= m)
    __shared__ __attribute__((aligned(16))) uint4 s_pat[kOdPairs][kOdLanes];
    static_assert(kOdPairs * kOdLanes == 256 && 17 * 17 <= 2 * 256, "table copy: one / two entries per thread");
    const uint4* rng_src = reinterpret_cast<const uint4*>(c_od_tab.rng);
    const uint4 rng0 = rng_src[threadIdx.x];
    const uint4 pat0 = reinterpret_cast<const uint4*>(c_od_tab.pat)[threadIdx.x];
    if (threadIdx.x < 17 * 17 - 256) (&s_rng[0][0])[threadIdx.x + 256] = rng_src[threadIdx.x + 256];
    (&s_rng[0][0])[threadIdx.x] = rng0;
    (&s_pat[0][0])[threadIdx.x] = pat0;
    __syncthreads();
    // this lane's three chunk slots: row v, chunk bytes [lo + a, hi + a) clamped to [0, 16) are
    // the disc span (lo = 15 - d - 16 part, hi = 16 + d - 16 part, d = umax[|v|], -1 past the
    // disc), the part's column offset and the byte offset from the window
    int mv[3], mlo[3], mhi[3], mofs[3], mp16[3];
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const int i = sub + 32 * it, r = i / 3, part = i - 3 * r;
        mv[it] = r - 15;
        const int d = r < 31 ? c_umax[mv[it] < 0 ? -mv[it] : mv[it]] : -1;
        mlo[it] = 15 - d - 16 * part;
        mhi[it] = 16 + d - 16 * part;
        mofs[it] = (r < 31 ? mv[it] : 15) * G.pitch + 16 * part;
        mp16[it] = 16 * part;
    }
    const __amdgpu_buffer_rsrc_t lrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)lvl, (short)0, (int)min((long long)G.pitch * G.h, 0x7fffffffLL), 0x00020000);
    uint8_t* pt = patch[grp];
    // uniform trip count per wave so the group shuffles see all lanes
    const int wave_first = (bx - G.od_first) * kOdKpBlock + (threadIdx.x >> 6) * 2;
    // each iteration's key is loaded one iteration ahead, so its round trip overlaps the
    // previous keypoint's work
    auto key_at = [&](int kb) {
        const int kp = kb + (grp & 1);
        return kp < count ? a.lvlkey[kbase + kp] : a.lvlkey[kbase + kb];
    };
    uint32_t key_next = wave_first < count ? key_at(wave_first) : 0u;
    for (int kb = wave_first; kb < count; kb += stride_k) {
        const int kp = kb + (grp & 1);
        const bool valid = kp < count;
        const uint32_t key = key_next;
        if (kb + stride_k < count) key_next = key_at(kb + stride_k);
        const int x = key_x(key) + kMinBorder, y = key_y(key) + kMinBorder;
        const int al = (x - 15) & 15;
        const int wofs = y * G.pitch + (x - 15 - al);  // the 48-byte window of disc row 0
        // the three moment chunks (round trip 1) and the 37 x 37 blurred patch (rows y-18..y+18
        // from the dword at or below x-18, 16-byte buffer loads, out-of-range bytes read as 0
        // and never sampled) are both requested before either is used, so the two round trips
        // overlap; window bytes past x + 15 (or past the plane: 0) only meet zero masks
        uint4 mc[3];
#pragma unroll
        for (int it = 0; it < 3; ++it) {
            if (raw_dw) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(lrs, wofs + mofs[it], 0, 0);
                mc[it] = make_uint4(q[0], q[1], q[2], q[3]);
            } else {  // level-0 rows not 4-byte aligned: bytes
                const uint8_t* q = lvl + wofs + mofs[it];
                uint32_t d4[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    d4[k] = (uint32_t)q[4 * k] | ((uint32_t)q[4 * k + 1] << 8) | ((uint32_t)q[4 * k + 2] << 16) |
                            ((uint32_t)q[4 * k + 3] << 24);
                mc[it] = make_uint4(d4[0], d4[1], d4[2], d4[3]);
            }
        }
        const int xb = (x - kOdPatchR) & ~3;
        const int pofs = (y - kOdPatchR) * G.bpitch + xb;
        uint4 pv[kOdPatchIt];
#pragma unroll
        for (int it = 0; it < kOdPatchIt; ++it) {
            const int c = sub + it * kOdLanes;
            const int r = c / 3, part = c - 3 * r;
            if (c < kOdPatchChunks) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(brs, pofs + r * G.bpitch + 16 * part, 0, 0);
                pv[it] = make_uint4(q[0], q[1], q[2], q[3]);
            }
        }
        // IC_Angle (:78-105) over this lane's three chunks
        int s_all = 0, c_all = 0, m01p = 0;
#pragma unroll
        for (int it = 0; it < 3; ++it) {
            const int m = min(max(mlo[it] + al, 0), 16), n = min(max(mhi[it] + al, 0), 16);
            const uint4 mk = s_rng[m][n];
            const uint32_t p0 = mc[it].x & mk.x, p1 = mc[it].y & mk.y, p2 = mc[it].z & mk.z, p3 = mc[it].w & mk.w;
            uint32_t sc = __builtin_amdgcn_udot4(p0, 0x01010101u, 0u, false);
            sc = __builtin_amdgcn_udot4(p1, 0x01010101u, sc, false);
            sc = __builtin_amdgcn_udot4(p2, 0x01010101u, sc, false);
            sc = __builtin_amdgcn_udot4(p3, 0x01010101u, sc, false);
            uint32_t cc = __builtin_amdgcn_udot4(p0, 0x03020100u, 0u, false);  // column within the chunk
            cc = __builtin_amdgcn_udot4(p1, 0x07060504u, cc, false);
            cc = __builtin_amdgcn_udot4(p2, 0x0B0A0908u, cc, false);
            cc = __builtin_amdgcn_udot4(p3, 0x0F0E0D0Cu, cc, false);
            s_all += (int)sc;
            c_all += (int)cc + mp16[it] * (int)sc;
            m01p += mv[it] * (int)sc;
        }
        // sums over the keypoint's lanes (DPP, no LDS round trip but the last step)
        const int m10 = od_sum(c_all - (15 + al) * s_all), m01 = od_sum(m01p);
        const float angle = fast_atan2_deg((float)m01, (float)m10);
        // computeOrbDescriptor (:108-148): lane `sub` makes bits [8 sub, 8 sub + 8)
        const float factorPI = (float)(3.14159265358979323846 / 180.0);
        float sn, ca;  // std::sin(float) / std::cos(float) (:114-115): libm sinf / cosf
        libm_sincosf(angle * factorPI, &sn, &ca);
        // the patch to LDS: every sample is then an LDS byte read (4 vector-memory instructions
        // per lane instead of one scattered byte load per sample)
#pragma unroll
        for (int it = 0; it < kOdPatchIt; ++it) {
            const int c = sub + it * kOdLanes;
            const int r = c / 3, part = c - 3 * r;
            if (c < kOdPatchChunks) *reinterpret_cast<uint4*>(pt + r * kOdPatchPitch + 16 * part) = pv[it];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the group's own lanes read it
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int pc = kOdPatchR * kOdPatchPitch + (x - xb);  // patch offset of the keypoint
        // both samples of a test pair as packed f32 (each element an IEEE single operation, no
        // contraction): row = x*b + y*a, col = x*a - y*b as the reference's float expressions
        // (:116-121), then cvRound by adding 1.5 * 2^23 (round to nearest even, |value| < 19),
        // whose low 24 bits are 2^22 + the rounded value: the LDS offset is one v_mad_u32_u24 of
        // the two bit patterns and a per-keypoint constant (no v_rndne / v_cvt per sample)
        const float magic = 12582912.0f;
        const uint32_t kofs = (uint32_t)pc - 0x4B400000u - 0x400000u * (uint32_t)kOdPatchPitch;
        const f32x2 snv = {sn, sn}, cav = {ca, ca}, mg = {magic, magic};
        // the LDS address of a sample is v_mad_u32_u24(R, pitch, C) + kpb, the patch base folded
        // into the per-keypoint constant: one full-rate v_add_u32 per sample where the compiler's
        // own association gave a v_add3_u32 (slow class, profiles/r06/valu_rates.json)
        typedef const __attribute__((address_space(3))) uint8_t lds_u8;
        const uint32_t kpb = kofs + (uint32_t)(uintptr_t)(lds_u8*)pt;
        uint32_t bits = 0;
#pragma unroll
        for (int b = kOdPairs - 1; b >= 0; --b) {  // bit b of the byte is pair b's test
            uint4 pw = s_pat[b][sub];  // float bit patterns {x0, x1, y0, y1}
            asm volatile("" : "+v"(pw.x), "+v"(pw.y), "+v"(pw.z), "+v"(pw.w));  // not hoisted
            const f32x2 X = {__uint_as_float(pw.x), __uint_as_float(pw.y)};
            const f32x2 Y = {__uint_as_float(pw.z), __uint_as_float(pw.w)};
            const f32x2 R = (X * snv + Y * cav) + mg;
            const f32x2 C = (X * cav - Y * snv) + mg;
            // the unsigned sums wrap to the small patch offsets
            uint32_t m0 = __umul24(__float_as_uint(R.x), (uint32_t)kOdPatchPitch) + __float_as_uint(C.x);
            uint32_t m1 = __umul24(__float_as_uint(R.y), (uint32_t)kOdPatchPitch) + __float_as_uint(C.y);
            asm volatile("" : "+v"(m0), "+v"(m1));  // keep the mad's addend C (not re-associated)
            const uint32_t p0 = *(lds_u8*)(uintptr_t)(m0 + kpb), p1 = *(lds_u8*)(uintptr_t)(m1 + kpb);
            // p0 < p1 <=> the sign of p0 - p1: shifted to bit b and merged by one v_bitop3
            // (A | (B & C)) -- full-rate ops instead of v_cmp + v_cndmask + a shift-or
            bits = __builtin_amdgcn_bitop3_b32(bits, (p0 - p1) >> (31 - b), 1u << b, 0xf8);
        }
        if (valid && !out_ok) {  // the level arrays, for k_finalize (or a status image)
            if (sub == 0) a.lvlangle[kbase + kp] = angle;
            a.lvldesc[(kbase + kp) * 32 + sub] = (uint8_t)bits;
        }
        if (valid) {
            if (out_ok) {  // the assembled output row (k_finalize's arithmetic): lanes 0-6 its 7 dwords
                out_d[kp * 32 + sub] = (uint8_t)bits;
                if (sub < 7) {
                    float px = (float)(x), py = (float)(y);
                    if (l != 0) {
                        px = px * G.scale;
                        py = py * G.scale;
                    }
                    const uint32_t w7[7] = {__float_as_uint(px), __float_as_uint(py), __float_as_uint((float)G.patch),
                                            __float_as_uint(angle), __float_as_uint((float)key_resp(key)),
                                            (uint32_t)l, 0xFFFFFFFFu};
                    uint32_t v = w7[0];
#pragma unroll
                    for (int k = 1; k < 7; ++k) v = sub == k ? w7[k] : v;
                    reinterpret_cast<uint32_t*>(out_kp + kp)[sub] = v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_finalize: ORBextractor::operator() assembly (ORBextractor_old.cc:1130-1190): levels in
// order, pt *= mvScaleFactor[level] for level > 0, keypoints inside [lap0, lap1] written from
// the back, the others from the front; returns monoIndex.

// The image's keypoints are walked as one sequence (level l's keypoint j at off[l] + j), in
// batches of kFinU chunks of kFinThreads whose loads are all issued before the first chunk's partition,
// so a batch costs one memory round trip instead of one per level and chunk.  The mono / stereo
// ranks come from per-wave ballots and one barrier per chunk.
constexpr int kFinU = 2;
#ifndef FIN_WIDE_MAX
#define FIN_WIDE_MAX 8
#endif
constexpr int kFinWideMaxImages = FIN_WIDE_MAX;

template <int kFinThreads>  // a chunk is one keypoint per thread
__global__ __launch_bounds__(kFinThreads) void k_finalize(BatchArgs a) {
    __shared__ int4 s_lv[kMaxLevels];  // {level key base (image-relative), off[l], scale bits, patch}
    __shared__ int s_wave[2][kFinThreads / 64];  // per-wave stereo counts, double-buffered over chunks
    const int img = a.img0 + blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int L = a.nlevels;
    int off[kMaxLevels];  // uniform: first sequence index of each level
    int total = 0;
    bool bad = false;
#pragma unroll
    for (int l = 0; l < kMaxLevels; ++l) {
        off[l] = total;
        if (l < L) {
            total += a.lvlcnt[img * kMaxLevels + l];
            bad |= a.status[img * kMaxLevels + l] != 0;
        }
    }
    if (bad || total > a.out_cap) {
        if (tid == 0) {
            a.out_n[img] = bad ? -5 : -2;
            a.out_mono[img] = 0;
        }
        return;
    }
    if (tid == 0) {  // uniform level loop: the level records are read with scalar loads
#pragma unroll
        for (int l = 0; l < kMaxLevels; ++l)
            if (l < L) s_lv[l] = make_int4(a.lv[l].kp_off, off[l], __float_as_int(l == 0 ? 1.f : a.lv[l].scale), a.lv[l].patch);
    }
    __syncthreads();
    const float lap0 = (float)a.laps[2 * img], lap1 = (float)a.laps[2 * img + 1];
    KP28* out = reinterpret_cast<KP28*>(a.out_kps) + (long long)img * a.out_cap;
    uint8_t* od = a.out_desc + (long long)img * a.out_cap * 32;
    const long long ibase = (long long)img * a.lvlkp_img_stride;
    const uint64_t lt = (1ull << lane) - 1ull;
    int mono = 0, stereo = 0, chunk_no = 0;
    for (int base = 0; base < total; base += kFinThreads * kFinU) {
        uint32_t key[kFinU];
        float ang[kFinU];
        uint4 d0[kFinU], d1[kFinU];
        int lev[kFinU];
#pragma unroll
        for (int u = 0; u < kFinU; ++u) {
            const int i = base + u * kFinThreads + tid;
            int l = 0;
#pragma unroll
            for (int k = 1; k < kMaxLevels; ++k) l += (k < L && i >= off[k]) ? 1 : 0;
            lev[u] = l;
            if (i < total) {
                const int4 info = s_lv[l];
                const long long kb = ibase + info.x + (i - info.y);
                key[u] = a.lvlkey[kb];
                ang[u] = a.lvlangle[kb];
                const uint4* s4 = reinterpret_cast<const uint4*>(a.lvldesc + kb * 32);
                d0[u] = s4[0];
                d1[u] = s4[1];
            }
        }
#pragma unroll
        for (int u = 0; u < kFinU; ++u) {
            const int cb = base + u * kFinThreads;
            if (cb >= total) continue;  // uniform (the batch's last chunks)
            const int i = cb + tid;
            const bool valid = i < total;
            KP28 k;
            bool st = false;
            if (valid) {
                const int l = lev[u];
                const int4 info = s_lv[l];
                k.x = (float)(key_x(key[u]) + kMinBorder);
                k.y = (float)(key_y(key[u]) + kMinBorder);
                if (l != 0) {
                    k.x = k.x * __int_as_float(info.z);
                    k.y = k.y * __int_as_float(info.z);
                }
                k.size = (float)info.w;
                k.angle = ang[u];
                k.response = (float)key_resp(key[u]);
                k.octave = l;
                k.class_id = -1;
                st = (k.x >= lap0 && k.x <= lap1);
            }
            const uint64_t bal = __ballot(st);
            const int buf = chunk_no & 1;
            if (lane == 0) s_wave[buf][w] = __popcll(bal);
            __syncthreads();
            int before = 0, tst = 0;
#pragma unroll
            for (int v = 0; v < kFinThreads / 64; ++v) {
                const int c = s_wave[buf][v];
                tst += c;
                before += v < w ? c : 0;
            }
            const int exs = before + __popcll(bal & lt);
            const int exm = tid - exs;  // earlier lanes of this chunk are all valid
            if (valid) {
                const int dst = st ? (total - 1 - (stereo + exs)) : (mono + exm);
                out[dst] = k;
                uint4* d4 = reinterpret_cast<uint4*>(od + (long long)dst * 32);
                d4[0] = d0[u];
                d4[1] = d1[u];
            }
            const int chunk = min(kFinThreads, total - cb);
            stereo += tst;
            mono += chunk - tst;
            ++chunk_no;
        }
    }
    if (threadIdx.x == 0) {
        a.out_n[img] = total;
        a.out_mono[img] = mono;
    }
}

// ---------------------------------------------------------------------------------------------
__device__ inline uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    return max(min(a, b), min(max(a, b), c));  // lowers to v_med3_u32
}

__device__ inline void knn2_store(uint32_t k1, uint32_t k2, int qi, int32_t* i1, int32_t* d1,
                                  int32_t* i2, int32_t* d2) {
    i1[qi] = k1 == 0xFFFFFFFFu ? -1 : (int32_t)(k1 & 0xFFFF);
    d1[qi] = k1 == 0xFFFFFFFFu ? 0x7fffffff : (int32_t)(k1 >> 16);
    i2[qi] = k2 == 0xFFFFFFFFu ? -1 : (int32_t)(k2 & 0xFFFF);
    d2[qi] = k2 == 0xFFFFFFFFu ? 0x7fffffff : (int32_t)(k2 >> 16);
}

// ---------------------------------------------------------------------------------------------
// k_knn2_mfma: BFMatcher(NORM_HAMMING).knnMatch(k=2) on the block-scaled FP4 matrix cores.
// Every descriptor bit becomes one e2m1 element, +1 (0x2) for a clear bit and -1 (0xA) for a set
// one, on both operands; with an E8M0 scale of 2^6 per 32-element block on each side,
// v_mfma_scale_f32_32x32x64_f8f6f4 gives 4096 * (64 - 2 H) over its K = 64 bits, so a train tile
// of 32 rows against 32 queries is 4 MFMAs over the 256 bits, at twice the MACs per cycle of the
// i8 form (MI355X_MICROARCH.md: FP4 32x32x64 takes the cycles of BF16 32x32x16).  The f32
// accumulator is preloaded with 4095 - (t mod 4096), so acc = 4096 (256 - 2H) + 4095 - t_local
// (every value an integer below 2^24, exact) orders like (H, t) ascending and the best two train
// rows are the two largest accumulators: no popcount, no per-pair VALU beyond the top-2 update.
// Train rows are walked in 4096-row segments (12-bit local index); each segment's winners are
// folded into (H << 16 | t) keys.
//   workgroup = 8 waves x 32 queries; per 32-row train tile each wave issues 4 MFMAs: A = the
//   train tile (expanded once per workgroup into LDS, double-buffered), B = the wave's queries
//   (expanded once into registers).
// C/D layout (cdna_hip_programming.md §3): lane l holds column l & 31 (its query) and rows
// (reg & 3) + 8 (reg >> 2) + 4 (l >> 5) of the tile (train rows); the K order inside a fragment is
// the same map for A and B, so any consistent bit -> element assignment is exact.
// Measured and replaced (round 6, single stream, 512 images): the i8 form
// (v_mfma_i32_32x32x32_i8, bits as +-64 bytes, 8 MFMAs per tile) 230-238 us against 159-167 us;
// two query sets per wave on the i8 form (each LDS-read train fragment feeding two MFMAs; 186
// VGPRs, 2 waves per SIMD) 256 us, and with one accumulator set selected after its own tile 237 us.
// Round 2's FP4 attempt lost to its nibble expansion; here a dword expands to its 32 nibbles with
// one shift and one v_and_or_b32 per 8 nibbles.
typedef int knn_v8i __attribute__((ext_vector_type(8)));
typedef float knn_v16f __attribute__((ext_vector_type(16)));
constexpr int kKnnWaves = 8;
constexpr int kKnnThreads = 64 * kKnnWaves;
constexpr int kKnnQ = 32 * kKnnWaves;    // queries per workgroup
static_assert(kKnnQ == kKnnQueries, "orb_kernels.h kKnnQueries (grid and arrival counters)");
constexpr int kKnnSeg = 4096;            // train rows per key segment
constexpr int kKnnPitch4 = 144;          // bytes per expanded train row (128 + 16: conflict-free b128 reads)
// bit 3 of each nibble from ws, nibble = 0x2 (+1) or 0xA (-1): one v_and_or_b32
__device__ inline uint32_t knn_nib_of(uint32_t ws) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(ws), "v"(0x88888888u), "v"(0x22222222u));
    return r;
}
// 8 nibbles of output dword m (m = 0..3) = bits m, m + 4, .., m + 28 of w, each +1 (0x2) or -1 (0xA)
__device__ inline knn_v8i knn4_expand(uint32_t w) {
    knn_v8i v;
    v[0] = (int)knn_nib_of(w << 3);
    v[1] = (int)knn_nib_of(w << 2);
    v[2] = (int)knn_nib_of(w << 1);
    v[3] = (int)knn_nib_of(w);
    v[4] = v[5] = v[6] = v[7] = 0;  // the e2m1 form reads four registers
    return v;
}
__device__ inline float knn_med3_f32(float a, float b, float c) {
    float r;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ inline float knn_max3_f32(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __attribute__((always_inline)) inline void knn2_fp4_block(
    const uint8_t* q, int nq, const uint8_t* t, int nt, int qb, int ts, int te, int32_t* i1, int32_t* d1,
    int32_t* i2, int32_t* d2, uint2* part, uint8_t* lds) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int qi = qb * kKnnQ + wave * 32 + r;
    // B fragments: lane (r, h) of MFMA s holds bits 64 s + 32 h + [0, 32) = dword 2 s + h of query qi
    knn_v8i qf[4];
    {
        const uint4* qp = reinterpret_cast<const uint4*>(q + (long long)min(qi, max(nq - 1, 0)) * 32);
        const uint4 qa = qp[0], qc = qp[1];
        qf[0] = knn4_expand(h ? qa.y : qa.x);
        qf[1] = knn4_expand(h ? qa.w : qa.z);
        qf[2] = knn4_expand(h ? qc.y : qc.x);
        qf[3] = knn4_expand(h ? qc.w : qc.z);
    }
    uint32_t g1 = 0xFFFFFFFFu, g2 = 0xFFFFFFFFu;
    // expansion: threads < 256 take (row tid >> 3, dword tid & 7) of a tile, one 16-byte store
    // (8 lanes write 128 contiguous bytes)
    const int er = tid >> 3, ed = tid & 7;
    const bool expander = tid < 256;
    auto load_packed = [&](int tile) __attribute__((always_inline)) {
        const int row = min(tile * 32 + er, nt - 1);
        return expander ? *reinterpret_cast<const uint32_t*>(t + (long long)row * 32 + 4 * ed) : 0u;
    };
    auto tile_lds = [&](int u) __attribute__((always_inline)) { return lds + ((u - ts) & 1) * (32 * kKnnPitch4); };
    auto store_expanded = [&](int u, uint32_t w) __attribute__((always_inline)) {
        if (expander) {
            const knn_v8i v = knn4_expand(w);
            *reinterpret_cast<uint4*>(tile_lds(u) + er * kKnnPitch4 + 16 * ed) = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };
    uint32_t pk0 = 0, pk1 = 0;
    if (te > ts) {
        store_expanded(ts, load_packed(ts));
        pk1 = load_packed(ts + 1);  // ts is even
    }
    auto rowc = [](int g) { return (g & 3) + 8 * (g >> 2); };
    knn_v16f C0;
#pragma unroll
    for (int g = 0; g < 16; ++g) C0[g] = (float)(4095 - 4 * h - rowc(g));
    const float kNone = -1073741824.0f;  // -2^30: below every key, and stays below after +32 per tile
    for (int seg0 = (ts * 32 / kKnnSeg) * kKnnSeg; seg0 < te * 32; seg0 += kKnnSeg) {
        const int tile0 = max(seg0 >> 5, ts), tile1 = min(te, (seg0 + kKnnSeg) >> 5);
        float ka1 = kNone, ka2 = kNone, kb1 = kNone, kb2 = kNone;
        auto select = [&](const knn_v16f& v, bool shift) __attribute__((always_inline)) {
            if (shift) {
                ka1 += 32.f;
                ka2 += 32.f;
                kb1 += 32.f;
                kb2 += 32.f;
            }
#pragma unroll
            for (int g = 0; g < 16; g += 4) {
                const float x0 = v[g], y0 = v[g + 1], x1 = v[g + 2], y1 = v[g + 3];
                ka2 = fmaxf(ka2, knn_med3_f32(ka1, x0, y0));
                ka1 = knn_max3_f32(ka1, x0, y0);
                kb2 = fmaxf(kb2, knn_med3_f32(kb1, x1, y1));
                kb1 = knn_max3_f32(kb1, x1, y1);
            }
        };
        auto body = [&](int ti, auto par, knn_v16f& acc, const knn_v16f& prev) __attribute__((always_inline)) {
            constexpr int PAR = decltype(par)::value;
            uint32_t& pk_use = PAR ? pk0 : pk1;
            uint32_t& pk_load = PAR ? pk1 : pk0;
            __syncthreads();  // tile ti expanded; the other buffer is free
            pk_load = load_packed(ti + 2);
            const uint8_t* ab = tile_lds(ti) + r * kKnnPitch4 + 16 * h;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const uint4 a4 = *reinterpret_cast<const uint4*>(ab + 32 * s);
                const knn_v8i a = {(int)a4.x, (int)a4.y, (int)a4.z, (int)a4.w, 0, 0, 0, 0};
                acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, qf[s], s ? acc : C0, 4, 4, 0, 133, 0, 133);
            }
            if (ti > tile0) select(prev, ti - 1 > tile0);
            if (ti + 1 < te) store_expanded(ti + 1, pk_use);
            if (ti * 32 + 32 > nt) {  // partial last tile: padding rows never win
#pragma unroll
                for (int g = 0; g < 16; ++g)
                    if (ti * 32 + rowc(g) + 4 * h >= nt) acc[g] = kNone;
            }
        };
        using P0 = std::integral_constant<int, 0>;
        using P1 = std::integral_constant<int, 1>;
        knn_v16f acc0, acc1;
        int ti = tile0;
        for (; ti + 1 < tile1; ti += 2) {
            body(ti, P0{}, acc0, acc1);
            body(ti + 1, P1{}, acc1, acc0);
        }
        if (ti < tile1) {
            body(ti, P0{}, acc0, acc1);
            select(acc0, ti > tile0);
        } else if (tile1 > tile0) {
            select(acc1, tile1 - 1 > tile0);
        }
        const int unbias = 32 * (tile1 - 1 - tile0);
        const int k1 = (int)fmaxf(ka1, kb1) - unbias;
        const int k2 = (int)fmaxf(fminf(ka1, kb1), fmaxf(ka2, kb2)) - unbias;
        auto fold = [&](int k) __attribute__((always_inline)) {
            if (k < -(1 << 24)) return;  // padding rows only
            const int tl = 4095 - (k & 4095), dotp = k >> 12;
            const uint32_t key = ((uint32_t)((256 - dotp) >> 1) << 16) | (uint32_t)(32 * tile0 + tl);
            g2 = med3_u32(g1, g2, key);
            g1 = min(g1, key);
        };
        fold(k1);
        fold(k2);
    }
    const uint32_t o1 = __shfl_xor(g1, 32), o2 = __shfl_xor(g2, 32);
    g2 = med3_u32(g1, g2, o1);
    g1 = min(g1, o1);
    g2 = med3_u32(g1, g2, o2);
    g1 = min(g1, o2);
    if (h == 0 && qi < nq) {
        if (part) part[qi] = make_uint2(g1, g2);
        else knn2_store(g1, g2, qi, i1, d1, i2, d2);
    }
}
constexpr int kKnnLdsBytes = 2 * 32 * kKnnPitch4;  // two expanded train tiles

__global__ __launch_bounds__(kKnnThreads) void k_knn2_mfma_pairs(MatchArgs m) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kKnnLdsBytes];
    const int pair = m.pair0 + blockIdx.y;
    const int qimg = 2 * pair, timg = 2 * pair + 1;
    const int qn = m.out_n[qimg], tn = m.out_n[timg];
    const int q0 = m.stereo_only ? m.out_mono[qimg] : 0;
    const int tq0 = m.stereo_only ? m.out_mono[timg] : 0;
    const int nq = qn > q0 ? qn - q0 : 0, nt = tn > tq0 ? tn - tq0 : 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) m.nq[pair] = nq;
    if ((int)blockIdx.x * kKnnQ >= nq) return;
    const uint8_t* q = m.desc + ((long long)qimg * m.out_cap + q0) * 32;
    const uint8_t* t = m.desc + ((long long)timg * m.out_cap + tq0) * 32;
    const long long o = (long long)pair * m.out_cap;
    // train split blockIdx.z of gridDim.z: tile ranges on 2-tile boundaries
    const int npt = (((nt + 31) >> 5) + 1) >> 1, S = gridDim.z, sp = blockIdx.z;  // tile pairs
    const int ts = 2 * (npt * sp / S), te = min((nt + 31) >> 5, 2 * (npt * (sp + 1) / S));
    uint2* part = m.part ? m.part + ((long long)(blockIdx.y * S + sp)) * m.out_cap : nullptr;
    knn2_fp4_block(q, nq, t, nt, blockIdx.x, ts, te, m.idx1 + o, m.dist1 + o, m.idx2 + o, m.dist2 + o, part, lds);
    if (!part || !m.cnt || S == 1) return;
    // fused merge: the last of the S split workgroups of this query block merges their partial
    // top-2 lists (k_knn2_merge's work, without its launch).  The hand-off follows
    // cdna_hip_programming.md Guideline 16 (counter form): every wave drains its partial stores,
    // one lane releases at agent scope (other XCDs' L2s), waits, and takes a ticket; the last
    // arriver resets the counter (zeroed when allocated) and acquires before any wave reads the
    // other splits' partials.  The "last" verdict goes through the kernel's one LDS array (a second
    // __shared__ object can add vmcnt waits to the tile loop).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* s_last = reinterpret_cast<int*>(lds);  // every wave is past its last tile read
    if (threadIdx.x == 0) {
        uint32_t* c = m.cnt + blockIdx.y * gridDim.x + blockIdx.x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const bool last = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(S - 1);
        if (last) {
            __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *s_last = last ? 1 : 0;
    }
    __syncthreads();
    if (!*s_last) return;
    const long long pb = (long long)blockIdx.y * S * m.out_cap;
    for (int i = threadIdx.x; i < kKnnQ; i += kKnnThreads) {
        const int qi = blockIdx.x * kKnnQ + i;
        if (qi >= nq) break;
        uint32_t g1 = 0xFFFFFFFFu, g2 = 0xFFFFFFFFu;
        for (int k = 0; k < S; ++k) {
            const uint2 kk = m.part[pb + (long long)k * m.out_cap + qi];
            g2 = med3_u32(g1, g2, kk.x);
            g1 = min(g1, kk.x);
            g2 = med3_u32(g1, g2, kk.y);
            g1 = min(g1, kk.y);
        }
        knn2_store(g1, g2, qi, m.idx1 + o, m.dist1 + o, m.idx2 + o, m.dist2 + o);
    }
}

// The split launch's partial top-2 lists of one query, merged (keys are distinct train rows).
__global__ __launch_bounds__(256) void k_knn2_merge(MatchArgs m, int nsplit) {
    const int pair = m.pair0 + blockIdx.y;
    const int qimg = 2 * pair, timg = 2 * pair + 1;
    const int qn = m.out_n[qimg], tn = m.out_n[timg];
    const int q0 = m.stereo_only ? m.out_mono[qimg] : 0;
    const int nq = qn > q0 ? qn - q0 : 0;
    (void)tn;
    const int qi = blockIdx.x * 256 + threadIdx.x;
    if (qi >= nq) return;
    uint32_t g1 = 0xFFFFFFFFu, g2 = 0xFFFFFFFFu;
    for (int sp = 0; sp < nsplit; ++sp) {
        const uint2 k = m.part[((long long)(blockIdx.y * nsplit + sp)) * m.out_cap + qi];
        g2 = med3_u32(g1, g2, k.x);
        g1 = min(g1, k.x);
        g2 = med3_u32(g1, g2, k.y);
        g1 = min(g1, k.y);
    }
    const long long o = (long long)pair * m.out_cap;
    knn2_store(g1, g2, qi, m.idx1 + o, m.dist1 + o, m.idx2 + o, m.dist2 + o);
}

__global__ __launch_bounds__(kKnnThreads) void k_knn2_mfma_plain(const uint8_t* q, int nq, const uint8_t* t, int nt,
                                                         int32_t* i1, int32_t* d1, int32_t* i2, int32_t* d2) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kKnnLdsBytes];
    knn2_fp4_block(q, nq, t, nt, blockIdx.x, 0, (nt + 31) >> 5, i1, d1, i2, d2, nullptr, lds);
}

// ---------------------------------------------------------------------------------------------
hipError_t launch_blur_level(const BatchArgs& a, int l, hipStream_t s) {
    const LevelGeom G = a.lv[l];
    const int n = G.tiles_x * G.tiles_y;
    hipLaunchKernelGGL(k_blur, dim3(std::min(n * a.nimages, 8192)), dim3(256), 0, s, a, G.tile_first, n);
    return hipGetLastError();
}
void fast_cell_range(const BatchArgs& a, int tile, int* c0, int* c1) {
    const int s48 = a.fast_n48, s64 = a.fast_n64;
    *c0 = tile == kCellPitchTiny ? 0 : tile == kCellPitchSmall ? s48 : s64;
    *c1 = tile == kCellPitchTiny ? s48 : tile == kCellPitchSmall ? s64 : a.total_cells;
}
hipError_t launch_fast_cells(const BatchArgs& a, int tile, hipStream_t s) {
    // smaller tiles = less LDS per workgroup = more cells resident per CU
    int c0, c1;
    fast_cell_range(a, tile, &c0, &c1);
    // a launch of a few images (the latency shape) leaves the GPU mostly idle: the 48- and 64-byte
    // cells go in ONE 64-byte launch instead of two back to back (every 48 cell fits 64)
    const bool merge = a.nimages <= kFastMergeMaxImages && a.fast_small <= 0 && a.fast_n48 > 0 && a.fast_n64 > a.fast_n48;
    if (merge && tile == kCellPitchSmall) return hipSuccess;  // done by the 48 launch
    if (merge && tile == kCellPitchTiny) {
        tile = kCellPitchSmall;
        c1 = a.fast_n64;
    }
    if (c1 <= c0) return hipSuccess;
    const dim3 grid(c1 - c0, a.nimages);
    const dim3 block(tile == kCellPitchTiny ? fast_threads<kCellPitchTiny>() : tile == kCellPitchSmall ? fast_threads<kCellPitchSmall>()
                                                                                                      : fast_threads<kCellMax>());
    const uint32_t d = (uint32_t)(c1 - c0);
    const uint32_t magic = d > 1 ? 0xFFFFFFFFu / d + 1u : 0u;  // ceil(2^32 / d) for d >= 2
    // the small-list 48- and 64-byte kernels and their overflow passes for the batch shape
    // (a.fast_small); the two tiles' launches share the queue slot (one after the other on the
    // stream, each overflow pass resets it)
    const bool small = (tile == kCellPitchTiny || tile == kCellPitchSmall) && a.fast_ovf &&
                       (a.fast_small > 0 || (a.fast_small < 0 && a.nimages > kFastMergeMaxImages));
    // one overflow pass after both tiles: the 64-byte full-list kernel redoes the cells either
    // queued (every 48-byte cell fits the 64-byte tile, as in the merged launch of small batches)
    const dim3 oblock(fast_threads<kCellPitchSmall>());
    if (small && tile == kCellPitchTiny) {
        hipLaunchKernelGGL((k_fast_cells<kCellPitchTiny, true>), grid, block, 0, s, a, c0, magic);
        int d0, d1;
        fast_cell_range(a, kCellPitchSmall, &d0, &d1);
        if (d1 <= d0) hipLaunchKernelGGL(k_fast_cells_ovf<kCellPitchSmall>, dim3(kFastOvfBlocks), oblock, 0, s, a);
    } else if (small) {
        hipLaunchKernelGGL((k_fast_cells<kCellPitchSmall, true>), grid, block, 0, s, a, c0, magic);
        hipLaunchKernelGGL(k_fast_cells_ovf<kCellPitchSmall>, dim3(kFastOvfBlocks), oblock, 0, s, a);
    } else if (tile == kCellPitchTiny) hipLaunchKernelGGL((k_fast_cells<kCellPitchTiny, false>), grid, block, 0, s, a, c0, magic);
    else if (tile == kCellPitchSmall) hipLaunchKernelGGL((k_fast_cells<kCellPitchSmall, false>), grid, block, 0, s, a, c0, magic);
    else hipLaunchKernelGGL((k_fast_cells<kCellMax, false>), grid, block, 0, s, a, c0, magic);
    return hipGetLastError();
}
hipError_t launch_octree(const BatchArgs& a, hipStream_t s) {
    // the dynamic-LDS limit is raised once per size and device (the attribute is per device; not
    // on every launch: the launch sequence may be captured into a hipGraph, orb_runtime.cpp)
    constexpr int kMaxDevices = 64;
    static std::atomic<int> lds_set[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = kMaxDevices - 1;
    std::atomic<int>& set = lds_set[dev];
    if (a.oct_lds_bytes > 65536 && a.oct_lds_bytes > set.load()) {
        for (const void* f : {reinterpret_cast<const void*>(k_octree<512>),
                              reinterpret_cast<const void*>(k_octree_retry)}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, a.oct_lds_bytes);
            if (e != hipSuccess) return e;
        }
        int cur = set.load();
        while (a.oct_lds_bytes > cur && !set.compare_exchange_weak(cur, a.oct_lds_bytes)) {}
    }
    const int split = a.nimages < a.oct_split_min_images ? a.nlevels : std::min(a.oct_split, a.nlevels);
    if (split > 0)
        hipLaunchKernelGGL(k_octree<512>, dim3(a.nimages, split), dim3(512), a.oct_lds_bytes, s, a, 0,
                           OctCfg{a.oct_nq_off, a.oct_lds_nodes, kOctLdsKeys, a.oct_lds_bytes});
    if (split < a.nlevels) {
        const OctCfg q{a.oct2_nq_off, a.oct2_lds_nodes, a.oct2_lds_keys, a.oct2_lds_bytes};
        if (a.oct2_threads == 128)
            hipLaunchKernelGGL(k_octree<128>, dim3(a.nimages, a.nlevels - split), dim3(128), a.oct2_lds_bytes, s, a,
                               split, q);
        else
            hipLaunchKernelGGL(k_octree<256>, dim3(a.nimages, a.nlevels - split), dim3(256), a.oct2_lds_bytes, s, a,
                               split, q);
    }
    // levels that did not fit the LDS instantiation (rare: node state or cell offsets too large)
    if (a.oct_may_retry)
        hipLaunchKernelGGL(k_octree_retry, dim3(std::min(a.nimages * a.nlevels, 64)), dim3(512),
                           a.oct_lds_bytes, s, a);
    return hipGetLastError();
}
hipError_t launch_orient_desc(const BatchArgs& a, hipStream_t s) {
    const uint32_t d = (uint32_t)a.total_od_blocks;
    const uint32_t magic = d > 1 ? 0xFFFFFFFFu / d + 1u : 0u;  // ceil(2^32 / d) for d >= 2
    hipLaunchKernelGGL(k_orient_desc, dim3(a.total_od_blocks, a.nimages), dim3(256), 0, s, a, magic);
    return hipGetLastError();
}
hipError_t launch_finalize(const BatchArgs& a, hipStream_t s) {
    // few images (the latency shape): 1024 / 512 threads per image (one load round trip covers
    // 2048 / 1024 keypoints); full batches: 256
    if (a.nimages <= 2) hipLaunchKernelGGL(k_finalize<1024>, dim3(a.nimages), dim3(1024), 0, s, a);
    else if (a.nimages <= kFinWideMaxImages) hipLaunchKernelGGL(k_finalize<512>, dim3(a.nimages), dim3(512), 0, s, a);
    else hipLaunchKernelGGL(k_finalize<256>, dim3(a.nimages), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_knn2_pairs(const MatchArgs& m, int npairs, hipStream_t s) {
    // few pairs (the latency shape): the train rows split over S workgroups per query block, so
    // the launch has ~256 workgroups instead of 8 per pair, and k_knn2_merge combines the splits
    const int S = m.part ? std::max(1, std::min(kKnnMaxSplit, kKnnSplitSlots / std::max(npairs, 1))) : 1;
    const int qblocks = (m.out_cap + kKnnQ - 1) / kKnnQ;
    if (S > 1) {
        // the partial lists take npairs * S slots of out_cap rows, the fused merge one arrival
        // counter per (pair, query block): refuse a launch that would index past either
        if (npairs * S > kKnnSplitSlots || (m.cnt && (long long)npairs * qblocks > m.cnt_slots))
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_knn2_mfma_pairs, dim3(qblocks, npairs, S), dim3(kKnnThreads), 0, s, m);
        if (!m.cnt) hipLaunchKernelGGL(k_knn2_merge, dim3((m.out_cap + 255) / 256, npairs), dim3(256), 0, s, m, S);
        return hipGetLastError();
    }
    MatchArgs m1 = m;
    m1.part = nullptr;
    hipLaunchKernelGGL(k_knn2_mfma_pairs, dim3(qblocks, npairs), dim3(kKnnThreads), 0, s, m1);
    return hipGetLastError();
}
hipError_t launch_knn2_plain(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* i1,
                             int32_t* d1, int32_t* i2, int32_t* d2, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(k_knn2_mfma_plain, dim3((nq + kKnnQ - 1) / kKnnQ), dim3(kKnnThreads), 0, s, q, nq, t, nt, i1,
                       d1, i2, d2);
    return hipGetLastError();
}

}  // namespace orbgpu
