// host_harness.hip -- TEST INFRASTRUCTURE: runs the device algorithm headers of the product
// (orb_octree.h, orb_fast_cell.h, orb_introsort.h, orb_math.h) on the host with SerialPolicy so
// they can be checked against the CPU oracle without a GPU.  Not part of liborbgpu.so.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../orbslam3lib_amd/csrc/orb_fast_cell.h"
#include "../../orbslam3lib_amd/csrc/orb_introsort.h"
#include "../../orbslam3lib_amd/csrc/orb_math.h"
#include "../../orbslam3lib_amd/csrc/orb_octree.h"
#include "../../orbslam3lib_amd/csrc/orb_policy.h"

using namespace orbgpu;

// node state is read and written as 16-byte records (orb_octree.h on_ld / on_st)
static uint8_t* align16(uint8_t* p) { return (uint8_t*)(((uintptr_t)p + 15) & ~(uintptr_t)15); }

extern "C" {

// libm_sincosf (orb_math.h) against the host's own sinf / cosf on every `stride`-th float of
// [lo, hi): returns the number of mismatching values (sin or cos), *checked = floats visited.
long long harness_libm_sincosf_mismatches(float lo, float hi, int stride, long long* checked) {
    uint32_t u = __builtin_bit_cast(uint32_t, lo);
    const uint32_t end = __builtin_bit_cast(uint32_t, hi);
    long long bad = 0, n = 0;
    for (; u < end; u += (uint32_t)stride) {
        volatile float y = __builtin_bit_cast(float, u);
        const float c = cosf(y), s = sinf(y);
        float ms, mc;
        libm_sincosf(y, &ms, &mc);
        bad += (__builtin_bit_cast(uint32_t, c) != __builtin_bit_cast(uint32_t, mc)) ||
               (__builtin_bit_cast(uint32_t, s) != __builtin_bit_cast(uint32_t, ms));
        ++n;
    }
    if (checked) *checked = n;
    return bad;
}

// libm_atanf / libm_tanf (orb_math.h) against the host's atanf / tanf on every `stride`-th float
// of [lo, hi) (lo >= 0, or both negative: floats are walked by bit pattern).
long long harness_libm_atanf_tanf_mismatches(float lo, float hi, int stride, int which, long long* checked) {
    uint32_t u = __builtin_bit_cast(uint32_t, lo);
    const uint32_t end = __builtin_bit_cast(uint32_t, hi);
    long long bad = 0, n = 0;
    for (; u < end; u += (uint32_t)stride) {
        volatile float y = __builtin_bit_cast(float, u);
        const float ref = which ? tanf(y) : atanf(y);
        const float got = which ? libm_tanf(y) : libm_atanf(y);
        bad += __builtin_bit_cast(uint32_t, ref) != __builtin_bit_cast(uint32_t, got);
        ++n;
    }
    if (checked) *checked = n;
    return bad;
}

// libm_atan2f against the host's atan2f on n pseudo-random pairs (xorshift from seed): raw bit
// patterns, [-3, 3]^2 and the |y| ~ |x| band, one quarter each.
long long harness_libm_atan2f_random(long long n, unsigned long long seed) {
    unsigned long long s = seed | 1;
    auto rnd = [&]() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return (uint32_t)s;
    };
    long long bad = 0;
    for (long long i = 0; i < n; ++i) {
        const uint32_t a = rnd(), b = rnd();
        float y, x;
        switch (i & 3) {
            case 0: y = __builtin_bit_cast(float, a); x = __builtin_bit_cast(float, b); break;
            case 1: y = (float)(int32_t)a / 2147483648.0f * 3.0f; x = (float)(int32_t)b / 2147483648.0f * 3.0f; break;
            case 2: y = __builtin_bit_cast(float, a & 0x3fffffffu); x = __builtin_bit_cast(float, b & 0x3fffffffu) * ((b >> 31) ? -1.f : 1.f); break;
            default:
                y = __builtin_bit_cast(float, 0x3f000000u + (a & 0x00ffffffu));
                x = y * (0.5f + (float)(b & 0xffff) / 65536.0f) * ((a >> 31) ? -1.f : 1.f);
        }
        volatile float vy = y, vx = x;
        const float ref = atan2f(vy, vx), got = libm_atan2f(vy, vx);
        bad += __builtin_bit_cast(uint32_t, ref) != __builtin_bit_cast(uint32_t, got) && !(ref != ref && got != got);
    }
    return bad;
}

int harness_octree(const uint32_t* keys, int n, int W, int H, int N, uint32_t* out, int out_cap) {
    const int nIni = std::max(1, (int)std::round((float)W / (float)H));
    const int cap = std::max(N + 3, 4 * nIni) + 8;
    std::vector<uint16_t> nq(n + 1);
    std::vector<uint8_t> mem(oct_nodemem_bytes(cap) + 64);
    OctWST<kGeneric, kGeneric> w;
    w.keys = const_cast<uint32_t*>(keys);  // read-only without a cell gather
    w.n = n;
    w.nq = nq.data();
    w.cell_off = nullptr;
    w.cellkeys = nullptr;
    w.ncells = 0;
    w.cell_cap = 0;
    w.m = oct_nodemem_carve<kGeneric>(align16(mem.data()), cap);
    w.cap = cap;
    w.out_keys = out;
    w.out_cap = out_cap;
    w.dbg = nullptr;
    w.pyr = nullptr;
    w.pyrD = 0;
    w.xcode = w.ycode = nullptr;
    OctShared sh;
    SerialPolicy p;
    return octree_distribute(p, w, &sh, W, H, N);
}

// The count-pyramid formulation with a pyramid of depth D (orb_octree.h), rerun with the label
// passes when a node below depth D must be divided, as the kernel does.  *deep = 1 when it was.
// ncells > 0: the keys arrive as per-cell lists (cell c holds counts[c] keys at cells[c * cap]),
// the kernel's layout, so the cell search and the pyramid's cell-slot key names are exercised.
int harness_octree_cells(const uint32_t* cells, const int32_t* counts, int ncells, int cap, int W, int H, int N,
                         uint32_t* out, int out_cap, int D, int* deep) {
    const int nIni = oct_nini(W, H);
    const int ocap = std::max(N + 3, 4 * nIni) + 8;
    std::vector<int32_t> off(ncells + 1, 0);
    for (int c = 0; c < ncells; ++c) off[c + 1] = off[c] + counts[c];
    const int n = off[ncells];
    std::vector<uint32_t> keys(n + 1);
    std::vector<uint16_t> nq(n + 1);
    std::vector<uint8_t> mem(oct_nodemem_bytes(ocap) + 64);
    std::vector<uint32_t> pyr(oct_pyr_bytes(D, nIni) / 4 + 1);
    std::vector<uint16_t> tbl(W + H + 2);
    OctWST<kGeneric, kGeneric> w;
    w.keys = keys.data();
    w.n = n;
    w.nq = nq.data();
    w.cell_off = off.data();
    w.cellkeys = cells;
    w.ncells = ncells;
    w.cell_cap = cap;
    w.m = oct_nodemem_carve<kGeneric>(align16(mem.data()), ocap);
    w.cap = ocap;
    w.out_keys = out;
    w.out_cap = out_cap;
    w.dbg = nullptr;
    w.pyr = pyr.data();
    w.pyrD = D;
    w.xcode = tbl.data();
    w.ycode = tbl.data() + W + 1;
    OctShared sh;
    SerialPolicy p;
    int r = octree_distribute(p, w, &sh, W, H, N);
    *deep = r == kOctDeep;
    if (r == kOctDeep) {
        w.pyrD = 0;
        r = octree_distribute(p, w, &sh, W, H, N);
    }
    return r;
}

int harness_octree_pyr(const uint32_t* keys, int n, int W, int H, int N, uint32_t* out, int out_cap, int D,
                       int* deep) {
    const int nIni = oct_nini(W, H);
    const int cap = std::max(N + 3, 4 * nIni) + 8;
    std::vector<uint16_t> nq(n + 1);
    std::vector<uint8_t> mem(oct_nodemem_bytes(cap) + 64);
    std::vector<uint32_t> pyr(oct_pyr_bytes(D, nIni) / 4 + 1);
    std::vector<uint16_t> tbl(W + H + 2);
    OctWST<kGeneric, kGeneric> w;
    w.keys = const_cast<uint32_t*>(keys);
    w.n = n;
    w.nq = nq.data();
    w.cell_off = nullptr;
    w.cellkeys = nullptr;
    w.ncells = 0;
    w.cell_cap = 0;
    w.m = oct_nodemem_carve<kGeneric>(align16(mem.data()), cap);
    w.cap = cap;
    w.out_keys = out;
    w.out_cap = out_cap;
    w.dbg = nullptr;
    w.pyr = pyr.data();
    w.pyrD = D;
    w.xcode = tbl.data();
    w.ycode = tbl.data() + W + 1;
    OctShared sh;
    SerialPolicy p;
    int r = octree_distribute(p, w, &sh, W, H, N);
    *deep = r == kOctDeep;
    if (r == kOctDeep) {
        w.pyrD = 0;
        r = octree_distribute(p, w, &sh, W, H, N);
    }
    return r;
}

void harness_introsort(const int32_t* size, const int32_t* ulx, int n, int32_t* perm) {
    std::vector<SortElem> a(n);
    for (int i = 0; i < n; ++i) a[i] = SortElem{size[i], ulx[i], i};
    introsort_like_libstdcxx(a.data(), n);
    for (int i = 0; i < n; ++i) perm[i] = a[i].node;
}

void harness_introsort_parallel(const int32_t* size, const int32_t* ulx, int n, int32_t* perm) {
    std::vector<SortElem> a(n + 1), tmp(n + 1);
    for (int i = 0; i < n; ++i) a[i] = SortElem{size[i], ulx[i], i};
    std::vector<uint16_t> lex(n + 2), rex(n + 2), segof(n + 1), lpos(n + 1), rpos(n + 1), rank(n + 1);
    const int S = n / 16 + 4;
    std::vector<uint16_t> seg(6 * S);
    std::vector<int32_t> segK(S);
    SortScratch ss;
    ss.tmp = tmp.data();
    ss.lex = lex.data();
    ss.rex = rex.data();
    ss.segof = segof.data();
    ss.lpos = lpos.data();
    ss.rpos = rpos.data();
    ss.rank = rank.data();
    for (int b = 0; b < 2; ++b) {
        ss.segF[b] = seg.data() + (3 * b + 0) * S;
        ss.segL[b] = seg.data() + (3 * b + 1) * S;
        ss.segD[b] = seg.data() + (3 * b + 2) * S;
    }
    ss.segK = segK.data();
    int nseg = 0;
    SerialPolicy p;
    introsort_parallel<kGeneric>(p, a.data(), n, ss, &nseg);
    for (int i = 0; i < n; ++i) perm[i] = a[i].node;
}

int harness_fast_strength(const uint8_t* img, int stride, int x, int y, int tlow) {
    return fast_strength(img + (long long)y * stride + x, stride, tlow);
}

float harness_fast_atan2(float y, float x) { return fast_atan2_deg(y, x); }

// Packed (both polarities per word) strength vs the scalar corner strength on the same pixel.
int harness_fast_strength_packed64(const uint8_t* img, int x, int y) {
    return fast_strength_packed<64>(img + (long long)y * 64 + x);
}
int harness_fast_strength_corner(const uint8_t* img, int stride, int x, int y) {
    return fast_strength_corner(img + (long long)y * stride + x, stride);
}

// ComputeKeyPointsOctTree cell loop geometry (same formulas as orb_runtime.cpp) + fast_cell_run.
int harness_level_candidates(const uint8_t* lvl, int w, int h, int ini, int mn, uint32_t* out,
                             int cap) {
    const int minB = 16, maxBX = w - 16, maxBY = h - 16;
    const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
    const int nCols = (int)(width / 35.f), nRows = (int)(height / 35.f);
    const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
    std::vector<uint32_t> T32(kCellMax * kCellMax / 4), M32(kCellMax * kCellMax / 4);
    uint8_t* T = reinterpret_cast<uint8_t*>(T32.data());
    uint8_t* M = reinterpret_cast<uint8_t*>(M32.data());
    std::vector<uint16_t> list(cell_list_cap<kCellMax>() + 1);
    std::vector<int32_t> wcnt(4);
    std::vector<uint32_t> tmp(kCellMax * kCellMax);
    int total = 0, cnt = 0;
    SerialPolicy p;
    for (int i = 0; i < nRows; ++i)
        for (int j = 0; j < nCols; ++j) {
            CellGeom g;
            g.iniY = minB + i * hCell;
            g.iniX = minB + j * wCell;
            g.minBorder = minB;
            if (g.iniY >= maxBY - 3 || g.iniX >= maxBX - 6) continue;
            g.rows = std::min(g.iniY + hCell + 6, maxBY) - g.iniY;
            g.cols = std::min(g.iniX + wCell + 6, maxBX) - g.iniX;
            // alternate the two load paths (dword-aligned window / plain bytes) across cells
            const bool dw = ((i + j) & 1) == 0 && (w & 3) == 0;
            const int sh = dw ? (g.iniX & 3) : 0;
            CellScratch cs{T, M, list.data(), wcnt.data()};
            // the small tile whenever the cells fit it (as the runtime picks it), else the general one
            const bool small = wCell + 9 <= kCellPitchSmall && hCell + 6 <= kCellPitchSmall;
            const long long roi = (long long)g.iniY * w + g.iniX - sh;
            const uint8_t* src = lvl + roi;
            const long long size = (long long)w * h;
            auto ld16 = [&](long long off) {  // bounds-checked like the device buffer load
                uint8_t b[16];
                for (int k = 0; k < 16; ++k) b[k] = roi + off + k < size ? src[off + k] : 0;
                uint4 v;
                std::memcpy(&v, b, 16);
                return v;
            };
            const int m = small ? fast_cell_run<kCellPitchSmall>(p, src, w, sh, dw, g, ini, mn, cs, tmp.data(), ld16)
                                : fast_cell_run<kCellMax>(p, src, w, sh, dw, g, ini, mn, cs, tmp.data(), ld16);
            for (int k = 0; k < m; ++k) {
                if (total < cap) out[total] = tmp[k];
                ++total;
            }
        }
    return total;
}

}  // extern "C"
