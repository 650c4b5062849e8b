// orb_octree.h -- quadtree keypoint culling (DistributeOctTree) as a data-parallel program.
//
// Restates cpp/src/ORBextractor_old.cc:557-781 (+ DivideNode :482-538, compareNodes :540-555)
// without std::list.  The reference list semantics reduce to a deterministic rebuild rule that
// is applied once per round:
//   * a round divides a set of nodes in a "division order" (phase 1: every non-frozen node in
//     list order, :624-683; final phase: the compareNodes-sorted candidates from the back,
//     stopping as soon as the list reaches N, :694-755);
//   * each division push_front()s its non-empty children n1..n4 and erases the parent, so the
//     next list is  [children of the LAST division (n4,n3,n2,n1)] ... [children of the FIRST
//     division] ++ [undivided nodes in their old order];
//   * vSizeAndPointerToNode = children with >1 keys, in (division order, n1..n4) order, and
//     those are exactly the next round's division candidates (phase 1: every node with >1 key
//     is a fresh child; phase 2: vPrev).
// Keys never move: a key's node is tracked by index (nq = node << 2 | quadrant), and a node's
// key list is always the input order filtered, so "first key with max response" (:762-778)
// is an atomic max over (response, -input index).
//
// Live nodes never exceed max(N + 3, 4 * nIni): a phase-1 round that would pass N triggers
// the final phase instead (:691), which stops at N.  The node state therefore fits in LDS for
// N <= ~1000; larger levels pass global scratch through the same flat pointers.
//
// Written once against a policy P (tid/nthreads/sync/atomics/block scan): the GPU kernel
// instantiates it with one workgroup per (image, level), the host test harness with a serial
// policy, so the exact same code is checked against the CPU oracle on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_addrspace.h"
#include "orb_kernels.h"
#include "orb_introsort.h"

namespace orbgpu {

struct alignas(16) OctNode {
    uint16_t x0, y0, x1, y1;  // UL = (x0,y0), BR = (x1,y1), relative to minBorder
    int32_t cnt;              // number of keys (bNoMore <=> cnt == 1)
    uint32_t path;            // depth << 27 | quadrant-path index (count pyramid, see below)
};
static_assert(sizeof(OctNode) == 16, "OctNode: 16 bytes");

// ---- count pyramid ------------------------------------------------------------------------
// Every node's bounds follow from its initial node and its quadrant path alone (oct_child), so a
// key's node at depth d is fixed by its coordinates: path index = initial node * 4^d + the
// quadrants of depths 1..d in base 4.  A histogram of the keys at depth D, summed up the levels,
// gives the key count of EVERY node of depth <= D -- and therefore the child counts that the
// label passes of the original formulation recount in every round -- plus, as a max over
// (response, -input index), every node's retained key (:759-778).  Level d holds nIni * 4^d
// entries from pyr_base(d): counts first, then the best values (same indexing).
constexpr int kOctPyrMaxD = 7;
constexpr int kOctDeep = -8;  // a node below depth D would be divided: rerun with label passes
__host__ __device__ inline int pyr_base(int d, int nIni) { return nIni * (((1 << (2 * d)) - 1) / 3); }
__host__ __device__ inline size_t oct_pyr_bytes(int D, int nIni) { return 8 * (size_t)pyr_base(D + 1, nIni); }
__host__ __device__ inline uint32_t oct_path_code(int d, uint32_t idx) { return ((uint32_t)d << 27) | idx; }
__host__ __device__ inline int oct_path_depth(uint32_t code) { return (int)(code >> 27); }
__host__ __device__ inline uint32_t oct_path_idx(uint32_t code) { return code & 0x7FFFFFFu; }
__host__ __device__ inline int oct_nini(int W, int H) {
    const int nIni = (int)roundf((float)W / (float)H);
    return nIni < 1 ? 1 : nIni;  // reference divides by zero here; never reached at sane sizes
}
// the per-axis path tables (u16 x codes for columns 0..W, y codes for rows 0..H)
__host__ __device__ inline size_t oct_tbl_bytes(int W, int H) { return ((size_t)2 * (W + H + 2) + 15) & ~(size_t)15; }
// deepest pyramid that fits `bytes` with the tables (0: none), at most Dmax
__host__ __device__ inline int oct_pyr_depth(size_t bytes, int W, int H, int Dmax) {
    const int nIni = oct_nini(W, H);
    const size_t t = oct_tbl_bytes(W, H);
    int D = 0;
    while (D < Dmax && D < kOctPyrMaxD && oct_pyr_bytes(D + 1, nIni) + t <= bytes &&
           ((size_t)nIni << (2 * (D + 1))) <= 65536)
        ++D;
    return D;
}

// Packed candidate key: x | y << 12 | response << 24 (relative coords < 4096, response < 256).
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__host__ __device__ inline int key_resp(uint32_t k) { return (int)(k >> 24); }
__host__ __device__ inline uint32_t make_key(int x, int y, int resp) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)resp << 24);
}

// Node-state scratch for capacity C nodes (LDS on the GPU when it fits), in address space AS.
template <int AS>
struct OctNodeMemT {
    asp<AS, OctNode> nodesA;     // [C]
    asp<AS, OctNode> nodesB;     // [C]  (also the sort buffer between the sort and the rebuild)
    asp<AS, int32_t> cntA;       // [4C] child key counts of the current candidates (double-buffered)
    asp<AS, int32_t> cntB;       // [4C]
    asp<AS, uint16_t> childpos;  // [4C]
    asp<AS, int32_t> divrank;    // [C]  -1 undivided, >=0 division rank
    asp<AS, uint16_t> undivpos;  // [C]
    asp<AS, uint16_t> blockoff;  // [C]
    asp<AS, uint16_t> expoff;    // [C]
    asp<AS, uint16_t> vsizeA;    // [C]
    asp<AS, uint16_t> vsizeB;    // [C]
};

// oct_nodemem_bytes (orb_kernels.h) = C * kOctNodeMemPerNode + 64, the carve below per node:
static_assert(2 * sizeof(OctNode) + 2 * 16 + 8 + 4 + 5 * 2 == kOctNodeMemPerNode, "node state bytes per node");

// Carves an OctNodeMemT out of `base` (16-byte aligned, in address space AS).
template <int AS>
__host__ __device__ inline OctNodeMemT<AS> oct_nodemem_carve(void* base, int C) {
    uint8_t* p = (uint8_t*)base;
    OctNodeMemT<AS> m;
    m.cntA = (asp<AS, int32_t>)p; p += 16 * (size_t)C;
    m.cntB = (asp<AS, int32_t>)p; p += 16 * (size_t)C;
    m.nodesA = (asp<AS, OctNode>)p; p += sizeof(OctNode) * (size_t)C;
    m.nodesB = (asp<AS, OctNode>)p; p += sizeof(OctNode) * (size_t)C;
    m.divrank = (asp<AS, int32_t>)p; p += 4 * (size_t)C;
    m.childpos = (asp<AS, uint16_t>)p; p += 8 * (size_t)C;
    m.undivpos = (asp<AS, uint16_t>)p; p += 2 * (size_t)C;
    m.blockoff = (asp<AS, uint16_t>)p; p += 2 * (size_t)C;
    m.expoff = (asp<AS, uint16_t>)p; p += 2 * (size_t)C;
    m.vsizeA = (asp<AS, uint16_t>)p; p += 2 * (size_t)C;
    m.vsizeB = (asp<AS, uint16_t>)p; p += 2 * (size_t)C;
    return m;
}

// LAS: address space of the node state and the cell offsets (LDS on the GPU); GAS: address
// space of the key arrays (global on the GPU); NAS: address space of the per-key labels (LDS
// while they fit, global for levels with more than kOctLdsKeys candidate keys).
template <int LAS, int GAS, int NAS = LAS>
struct OctWST {
    asp<GAS, uint32_t> keys;    // [n] in vToDistributeKeys order (written by the gather if any)
    int n;
    asp<NAS, uint16_t> nq;      // [n] node index << 2 | quadrant of each key
    OctNodeMemT<LAS> m;
    int cap;                    // node capacity C (>= max(N+3, 4*nIni) + 4)
    asp<GAS, uint32_t> out_keys;  // [out_cap]
    int out_cap;
    unsigned long long* dbg;    // diagnostic phase clocks (8 slots) or nullptr
    // optional gather of keys[] from per-cell lists (ComputeKeyPointsOctTree cell order):
    // key k lives in the last cell c with cell_off[c] <= k, at cellkeys[c * cell_cap + k - off]
    asp<LAS, const int32_t> cell_off;  // [ncells] exclusive scan of the cell counts, or null
    asp<GAS, const uint32_t> cellkeys;
    int ncells, cell_cap;
    // count pyramid (LDS): depth pyrD > 0 runs the label-free formulation, 0 the label passes
    asp<LAS, uint32_t> pyr;  // [oct_pyr_bytes(pyrD, nIni) / 4]
    int pyrD;
    asp<LAS, uint16_t> xcode;  // [W + 1] oct_xcode of every column (pyrD > 0)
    asp<LAS, uint16_t> ycode;  // [H + 1] oct_ycode of every row
};

constexpr int kOctUnroll = 8;         // keys per thread per batch in the key passes
#ifndef OCT_HIST_VEC
#define OCT_HIST_VEC 1  // pyramid histogram: 16-byte key loads when the cell capacity is a multiple of 4
#endif

struct OctShared {
    int size, prev_size, nexp, ndiv, phase, done, nchild, nundiv, status, jstop, deep;
};

__host__ __device__ inline int oct_half(int a, int b) { return (b - a + 1) >> 1; }  // ceil((b-a)/2.f)

__host__ __device__ inline int oct_quadrant(uint32_t key, OctNode nd) {
    const int hx = nd.x0 + oct_half(nd.x0, nd.x1);
    const int hy = nd.y0 + oct_half(nd.y0, nd.y1);
    const int x = key_x(key), y = key_y(key);
    if (x < hx) return (y < hy) ? 0 : 2;
    return (y < hy) ? 1 : 3;
}

// One axis of a key's path at depth D: bit d of the quadrant (x >= hx, or y >= hy) in base-4
// digit D - d, with the bounds updated exactly as oct_child / oct_quadrant do.  A key's path
// index is init * 4^D + code_x + 2 * code_y (init: its initial node, :585 kp.pt.x / hX).
__host__ __device__ inline uint32_t oct_axis_code(int v, int lo, int hi, int D) {
    uint32_t c = 0;
    for (int d = 0; d < D; ++d) {
        const int h = lo + oct_half(lo, hi);
        const int b = v >= h;
        c = 4 * c + (uint32_t)b;
        lo = b ? h : lo;
        hi = b ? hi : h;
    }
    return c;
}
__host__ __device__ inline int oct_init_node(int x, float hX, int nIni) {
    const int i = (int)((float)x / hX);
    return i >= nIni ? nIni - 1 : i;
}
// x part of the path index: init * 4^D + code_x
__host__ __device__ inline uint32_t oct_xcode(int x, int D, float hX, int nIni) {
    const int i = oct_init_node(x, hX, nIni);
    const int x0 = (uint16_t)(int)(hX * (float)i), x1 = (uint16_t)(int)(hX * (float)(i + 1));
    return ((uint32_t)i << (2 * D)) + oct_axis_code(x, x0, x1, D);
}
__host__ __device__ inline uint32_t oct_ycode(int y, int D, int H) { return 2 * oct_axis_code(y, 0, (uint16_t)H, D); }

__host__ __device__ inline OctNode oct_child(OctNode nd, int q, int cnt) {
    const int hx = nd.x0 + oct_half(nd.x0, nd.x1);
    const int hy = nd.y0 + oct_half(nd.y0, nd.y1);
    OctNode c;
    c.x0 = (uint16_t)((q & 1) ? hx : nd.x0);
    c.x1 = (uint16_t)((q & 1) ? nd.x1 : hx);
    c.y0 = (uint16_t)((q & 2) ? hy : nd.y0);
    c.y1 = (uint16_t)((q & 2) ? nd.y1 : hy);
    c.cnt = cnt;
    c.path = oct_path_code(oct_path_depth(nd.path) + 1, 4 * oct_path_idx(nd.path) + (uint32_t)q);
    return c;
}

// Runs DistributeOctTree for one level.  Coordinates are relative to (minBorderX, minBorderY);
// W = maxBorderX-minBorderX, H = maxBorderY-minBorderY, N = mnFeaturesPerLevel[level].
// Returns the number of output nodes (keys written to ws.out_keys in list order), or <0.
//
// Work split: node-level phases (division order, sort, rebuild: a few hundred nodes) run on
// p.node() -- wave 0 alone on the GPU, so their many scans need no workgroup barrier -- and
// the key passes (relabel + child counts) run on every thread with the global key loads
// software-pipelined; a phase-1 round costs two workgroup barriers.
// whole nodes as one 16-byte access (the node phases run on one wave: fewer LDS instructions)
template <class NP>
__host__ __device__ inline OctNode on_ld(NP a, int i) {
    const orb_u32x4 v = as_vec4(a)[i];
    OctNode n;
    n.x0 = (uint16_t)(v.x & 0xFFFFu);
    n.y0 = (uint16_t)(v.x >> 16);
    n.x1 = (uint16_t)(v.y & 0xFFFFu);
    n.y1 = (uint16_t)(v.y >> 16);
    n.cnt = (int32_t)v.z;
    n.path = v.w;
    return n;
}
template <class NP>
__host__ __device__ inline void on_st(NP a, int i, OctNode n) {
    orb_u32x4 v;
    v.x = (uint32_t)n.x0 | ((uint32_t)n.y0 << 16);
    v.y = (uint32_t)n.x1 | ((uint32_t)n.y1 << 16);
    v.z = (uint32_t)n.cnt;
    v.w = n.path;
    as_vec4(a)[i] = v;
}

template <int LAS, int GAS, int NAS, class P>
__host__ __device__ __attribute__((always_inline)) inline int octree_distribute(P& p, const OctWST<LAS, GAS, NAS> ws,
                                          asp<LAS, OctShared> sh, int W, int H, int N) {
    const int tid = p.tid(), NT = p.nthreads();
    const int n = ws.n;
    const OctNodeMemT<LAS> M = ws.m;
    auto cur = M.nodesA;
    auto nxt = M.nodesB;
    auto ccur = M.cntA;   // child counts of the current round's candidates
    auto cnxt = M.cntB;
    auto vsz = M.vsizeA;
    auto vsz2 = M.vsizeB;
    auto nq = ws.nq;
    const bool nw = p.node_worker();
    unsigned long long t_prev = p.now();
    auto mark = [&](int slot) __attribute__((always_inline)) {
        if (ws.dbg && tid == 0) {
            const unsigned long long t = p.now();
            ws.dbg[slot] += t - t_prev;
            t_prev = t;
        }
    };
    if (ws.cap > 16383) return -3;  // node index must fit 14 bits of nq
    const int nIni = oct_nini(W, H);
    const float hX = (float)W / (float)nIni;
    if (nIni + 4 > ws.cap) return -3;
    // count-pyramid formulation (ws.pyrD > 0): one histogram of the keys replaces every label pass
    const int D = ws.pyrD;
    const bool fast = D > 0;
    auto pcnt = ws.pyr;
    auto pbest = fast ? ws.pyr + pyr_base(D + 1, nIni) : ws.pyr;  // (no offset on a null pyr)
    const int bD = pyr_base(D, nIni);
    if (fast) {
        for (int e = tid; e < (nIni << (2 * D)); e += NT) {
            pcnt[bD + e] = 0;
            pbest[bD + e] = 0;
        }
        p.sync();
#ifdef OCT_DIAG
        mark(1);
#endif
    }
    // every key pass: f(base, key[kOctUnroll]) handles keys k = base + u * NT + tid (u <
    // kOctUnroll; k >= n are padding) in stages across the batch so the LDS round trips of
    // different keys overlap; the global key loads run one batch ahead
    auto for_keys = [&](auto f) __attribute__((always_inline)) {
        if (n <= 0) return;
        uint32_t key[kOctUnroll], nkey[kOctUnroll];
#pragma unroll
        for (int u = 0; u < kOctUnroll; ++u) {
            const int k = u * NT + tid;
            key[u] = ws.keys[k < n ? k : n - 1];
        }
        for (int base = 0; base < n; base += kOctUnroll * NT) {
            // the next batch's loads are in flight while this batch runs its LDS chains
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + (kOctUnroll + u) * NT + tid;
                nkey[u] = ws.keys[k < n ? k : n - 1];
            }
            f(base, key);
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) key[u] = nkey[u];
        }
    };

    // ---- keys: the histogram (pyramid) or the gather into vToDistributeKeys order -------
    // The pyramid reads the cell lists as they are and names a key by kid = cell * cell_cap +
    // slot (monotone in the input index k, and the key's own address): no gathered copy.  The
    // gather locates each k's cell by a fixed-length binary search over the cell offsets, many
    // keys per thread in lockstep so their LDS reads and global loads overlap.
    int steps = 0;
    if (ws.cell_off)
        while ((1 << steps) < ws.ncells) ++steps;
    if (fast) {
        // the path index is init * 4^D + code_x + 2 * code_y: one table per axis
        for (int x = tid; x <= W; x += NT) ws.xcode[x] = (uint16_t)oct_xcode(x, D, hX, nIni);
        for (int y = tid; y <= H; y += NT) ws.ycode[y] = (uint16_t)oct_ycode(y, D, H);
        p.sync();
#ifdef OCT_DIAG
        mark(1);
#endif
    }
    auto pyr_add = [&](uint32_t key, int kid) __attribute__((always_inline)) {
        const int x = key_x(key), y = key_y(key);
        const int e = bD + (x <= W && y <= H ? (int)ws.xcode[x] + (int)ws.ycode[y]
                                             : (int)(oct_xcode(x, D, hX, nIni) + oct_ycode(y, D, H)));
#ifndef OCT_NOATOM
        p.atomic_add(&pcnt[e], 1);
        p.atomic_max(&pbest[e], ((uint32_t)key_resp(key) << 24) | (0xFFFFFFu - (uint32_t)kid));
#else
        if (kid == -5) pcnt[e] = 1;
#endif
    };
    if (fast && n > 0 && ws.cell_off) {
        // cell lists as they are (no search for a key's cell; kid = cell * cell_cap + slot):
        // consecutive threads take consecutive cells, K threads per cell interleaving its slots,
        // so the lanes of one atomic instruction hit different pyramid entries (a cell's own
        // keys share a few entries: lanes on one cell would serialize on them)
        const int nc = ws.ncells;
        int K = 1;
        while (2 * K * nc <= NT) K *= 2;
        const int slots = K * nc;
        constexpr int U = 16;  // keys in flight per thread
        for (int t = tid; t < slots; t += NT) {
            const int c = t % nc, ph = t / nc;
            const int cnt_c = (c + 1 < nc ? ws.cell_off[c + 1] : n) - ws.cell_off[c];
            const int cb = c * ws.cell_cap;
#if OCT_HIST_VEC
            if ((ws.cell_cap & 3) == 0 && K <= 4) {
                // 16-byte loads, 4 keys each (chunk q = keys 4q .. 4q+3 of the cell; a chunk's
                // bytes past cnt_c lie inside the cell's capacity, a multiple of 4): a full cell
                // takes 4x fewer load round trips than one key per load.  Levels with few cells
                // (K > 4 threads per cell) keep one key per thread and load: their cells hold a
                // few keys each, and whole chunks would put them on fewer threads.
                // One pair (tools/octree_stamps.py 1): level-0 histogram 11.6 -> 9.9 us.
                constexpr int U4 = 8;  // chunks in flight per thread
                for (int q0 = ph; 4 * q0 < cnt_c; q0 += U4 * K) {
                    orb_u32x4 kv[U4];
#pragma unroll
                    for (int u = 0; u < U4; ++u) {
                        const int q = q0 + u * K;
                        kv[u] = as_vec4(ws.cellkeys + cb)[4 * q < cnt_c ? q : q0];
                    }
#pragma unroll
                    for (int u = 0; u < U4; ++u) {
                        const int j = 4 * (q0 + u * K);
                        if (j < cnt_c) pyr_add(kv[u].x, cb + j);
                        if (j + 1 < cnt_c) pyr_add(kv[u].y, cb + j + 1);
                        if (j + 2 < cnt_c) pyr_add(kv[u].z, cb + j + 2);
                        if (j + 3 < cnt_c) pyr_add(kv[u].w, cb + j + 3);
                    }
                }
                continue;
            }
#endif
            for (int j0 = ph; j0 < cnt_c; j0 += U * K) {
                uint32_t key[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {  // clamped, unpredicated: all U loads in flight
                    const int j = j0 + u * K;
                    key[u] = ws.cellkeys[cb + (j < cnt_c ? j : cnt_c - 1)];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = j0 + u * K;
                    if (j < cnt_c) pyr_add(key[u], cb + j);
                }
            }
        }
        p.sync();
        mark(5);
    } else if (fast && n > 0) {
        for (int k = tid; k < n; k += NT) pyr_add(ws.keys[k], k);
        p.sync();
        mark(5);
    } else if (ws.cell_off && n > 0) {
        for (int base = 0; base < n; base += kOctUnroll * NT) {
            int kk[kOctUnroll], lo[kOctUnroll];
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT + tid;
                kk[u] = k < n ? k : n - 1;
                lo[u] = 0;
            }
            for (int it = 0; it < steps; ++it) {
                const int half = 1 << (steps - 1 - it);
#pragma unroll
                for (int u = 0; u < kOctUnroll; ++u) {
                    const int mid = lo[u] + half;
                    const int midc = mid < ws.ncells ? mid : ws.ncells - 1;
                    if (mid < ws.ncells && ws.cell_off[midc] <= kk[u]) lo[u] = mid;
                }
            }
            uint32_t key[kOctUnroll];
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u)
                key[u] = ws.cellkeys[lo[u] * ws.cell_cap + (kk[u] - ws.cell_off[lo[u]])];
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u)
                if (base + u * NT + tid < n) ws.keys[kk[u]] = key[u];
        }
        p.sync();  // the cell offsets share memory with the node state written below
    }
    if (fast) {  // the levels above D: sums and maxima of the four children
        for (int d = D - 1; d >= 0; --d) {
            const int b = pyr_base(d, nIni), b1 = pyr_base(d + 1, nIni);
            for (int e = tid; e < (nIni << (2 * d)); e += NT) {
                const int c = b1 + 4 * e;
                pcnt[b + e] = pcnt[c] + pcnt[c + 1] + pcnt[c + 2] + pcnt[c + 3];
                const uint32_t m0 = pbest[c] > pbest[c + 1] ? pbest[c] : pbest[c + 1];
                const uint32_t m1 = pbest[c + 2] > pbest[c + 3] ? pbest[c + 2] : pbest[c + 3];
                pbest[b + e] = m0 > m1 ? m0 : m1;
            }
            p.sync();
        }
        mark(6);
    }
    // ---- initial nodes (:561-603) ------------------------------------------------------
    for (int i = tid; i < nIni; i += NT) {
        OctNode nd;
        nd.x0 = (uint16_t)(int)(hX * (float)i);
        nd.x1 = (uint16_t)(int)(hX * (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = (uint16_t)H;
        nd.cnt = fast ? (int)pcnt[i] : 0;
        nd.path = oct_path_code(0, (uint32_t)i);
        on_st(cur, i, nd);
    }
    p.sync();
    if (!fast) {
        for_keys([&](int base, const uint32_t* key) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT + tid;
                int idx = (int)((float)key_x(key[u]) / hX);
                if (idx >= nIni) idx = nIni - 1;  // unreachable for in-range keys; keeps memory safe
                if (k < n) nq[k] = (uint16_t)(idx << 2);
                p.run_add(&cur[idx].cnt, idx, k < n);
            }
        });
        p.sync();
    }
    if (nw) {  // drop the empty initial nodes (:594-603)
        auto np = p.node();
        const int ntid = np.tid(), NNT = np.nthreads();
        int carry = 0;
        for (int base = 0; base < nIni; base += NNT) {
            const int i = base + ntid;
            const int v = (i < nIni && cur[i].cnt > 0) ? 1 : 0;
            int tot;
            const int ex = np.scan_small(v, &tot);
            if (v) {
                const OctNode nd = on_ld(cur, i);
                on_st(nxt, carry + ex, nd);
                M.undivpos[i] = (uint16_t)(carry + ex);
                // round 1's candidates (>1 key): their child counts from the pyramid
                const int b1 = pyr_base(1, nIni) + 4 * i;
                for (int q = 0; q < 4; ++q)
                    ccur[4 * (carry + ex) + q] = (fast && nd.cnt > 1) ? (int)pcnt[b1 + q] : 0;
            }
            carry += tot;
        }
        if (ntid == 0) {
            sh->size = carry;
            sh->nexp = 0;
            sh->phase = 1;
            sh->done = 0;
            sh->status = 0;
            sh->deep = 0;
        }
    }
    {
        auto t = cur;
        cur = nxt;
        nxt = t;
    }
    p.sync();
    // relabel to the compacted list + count round 1 (every node with >1 key is a candidate)
    if (!fast) {
        for_keys([&](int base, const uint32_t* key) __attribute__((always_inline)) {
            int v[kOctUnroll];
            OctNode nd[kOctUnroll];
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT + tid;
                v[u] = M.undivpos[nq[k < n ? k : n - 1] >> 2];
            }
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) nd[u] = on_ld(cur, v[u]);
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT + tid;
                const bool split = k < n && nd[u].cnt > 1;
                const int q = split ? oct_quadrant(key[u], nd[u]) : 0;
                p.run_add(&ccur[4 * v[u] + q], 4 * v[u] + q, split);
                if (k < n) nq[k] = (uint16_t)((v[u] << 2) | q);
            }
        });
        p.sync();
    }
    mark(0);

    // ---- rounds (:612-757) -----------------------------------------------------------
    int guard = 0;
    // sort scratch of the final phase (every array is free until step 3 / the rebuild)
    auto sort_scratch = [&](asp<LAS, int32_t> cn) __attribute__((always_inline)) {
        const int C = ws.cap;
        SortScratchT<LAS> ss;
        ss.tmp = reinterpret_cast<asp<LAS, SortElem>>(cn);
        ss.lex = M.childpos;
        ss.rex = M.childpos + (C + 1);
        ss.segof = M.childpos + 2 * (C + 1);
        ss.lpos = M.undivpos;
        ss.rpos = M.blockoff;
        ss.rank = M.expoff;
        auto seg = reinterpret_cast<asp<LAS, uint16_t>>(M.divrank);
        const int S = C / 16 + 4;
        for (int b = 0; b < 2; ++b) {
            ss.segF[b] = seg + (3 * b + 0) * S;
            ss.segL[b] = seg + (3 * b + 1) * S;
            ss.segD[b] = seg + (3 * b + 2) * S;
        }
        ss.segK = reinterpret_cast<asp<LAS, int32_t>>(seg + 6 * S + 2);
        return ss;
    };
    while (!sh->done) {
        if (++guard > 4096) return -4;
        if (sh->phase != 1) {  // final phase: libstdc++-ordered sort of vPrev
            // partition rounds: one wave per segment, one workgroup barrier per round
            const int m = sh->nexp;
            auto sb = reinterpret_cast<asp<LAS, SortElem>>(nxt);  // nxt is free until the rebuild
            for (int j = tid; j < m; j += NT) {
                const int v = vsz[j];
                SortElem e;
                e.size = cur[v].cnt;
                e.ulx = cur[v].x0;
                e.node = v;
                e.pad = 0;
                se_st(sb, j, e);
            }
            p.sync();
            introsort_partition<LAS>(p, sb, m, sort_scratch(cnxt), &sh->jstop);
        }
        if (sh->phase != 1) {  // the O(m^2) stable rank pass spreads over the whole block
            p.sync();
            introsort_final<LAS>(p, reinterpret_cast<asp<LAS, SortElem>>(nxt), sh->nexp,
                                 sort_scratch(cnxt));
            p.sync();
            mark(3);
        }
        if (nw) {
            auto np = p.node();
            const int ntid = np.tid(), NNT = np.nthreads();
            const int size = sh->size;
            const int phase = sh->phase;
            if (ntid == 0) sh->prev_size = size;
            // 1. division order
            if (phase == 1) {  // every non-frozen node, in list order
                int carry = 0;
                for (int base = 0; base < size; base += NNT) {
                    const int i = base + ntid;
                    const int v = (i < size && cur[i].cnt > 1) ? 1 : 0;
                    int tot;
                    const int ex = np.scan_small(v, &tot);
                    if (i < size) M.divrank[i] = v ? carry + ex : -1;
                    carry += tot;
                }
                if (ntid == 0) sh->ndiv = carry;
                // children block offsets: rank r lands after all ranks > r
                int c1 = 0, c2 = 0;
                for (int base = 0; base < size; base += NNT) {
                    const int i = base + ntid;
                    int nc = 0, ne = 0;
                    if (i < size && cur[i].cnt > 1) {
                        for (int q = 0; q < 4; ++q) {
                            const int c = ccur[4 * i + q];
                            nc += c > 0;
                            ne += c > 1;
                        }
                    }
                    int t1, t2;
                    const int e1 = np.scan_small(nc, &t1);
                    const int e2 = np.scan_small(ne, &t2);
                    if (i < size && cur[i].cnt > 1) {
                        M.blockoff[i] = (uint16_t)(c1 + e1 + nc);  // inclusive; finalised below
                        M.expoff[i] = (uint16_t)(c2 + e2);
                    }
                    c1 += t1;
                    c2 += t2;
                }
                if (ntid == 0) {
                    sh->nchild = c1;
                    sh->nexp = c2;
                }
                np.sync();
                for (int i = ntid; i < size; i += NNT)
                    if (M.divrank[i] >= 0) M.blockoff[i] = (uint16_t)(c1 - M.blockoff[i]);
                mark(1);
            } else {  // final phase: divide the sorted vPrev from the back until N
                const int m = sh->nexp;
                const auto sb = reinterpret_cast<asp<LAS, const SortElem>>(nxt);
                for (int i = ntid; i < size; i += NNT) M.divrank[i] = -1;
                np.sync();
                // S_j = size + sum_{j'>=j} (nc_j' - 1) is non-increasing in j; divide [jstop, m)
                if (ntid == 0) sh->jstop = 0;
                np.sync();
                int carry = 0;
                for (int base = 0; base < m; base += NNT) {  // scan in reversed sorted order
                    const int t = base + ntid;
                    const int j = m - 1 - t;
                    int d = 0;
                    if (t < m) {
                        const int v = sb[j].node;
                        for (int q = 0; q < 4; ++q) d += ccur[4 * v + q] > 0;
                        d -= 1;
                    }
                    // d in [-1, 3]: scan d + 1 over the valid lanes (a prefix of the wave)
                    const int nvalid = m - base < NNT ? m - base : NNT;
                    int tot;
                    const int ex = np.scan_small(t < m ? d + 1 : 0, &tot) - (ntid < nvalid ? ntid : nvalid);
                    tot -= nvalid;
                    if (t < m && size + carry + ex + d >= N) np.atomic_max_int(&sh->jstop, j);
                    carry += tot;
                }
                np.sync();
                const int jstop = sh->jstop;
                // ranks, block offsets (division order = j descending) and vsize offsets
                int c1 = 0, c2 = 0;
                for (int base = jstop; base < m; base += NNT) {
                    const int j = base + ntid;
                    int nc = 0, ne = 0, v = -1;
                    if (j < m) {
                        v = sb[j].node;
                        for (int q = 0; q < 4; ++q) {
                            const int c = ccur[4 * v + q];
                            nc += c > 0;
                            ne += c > 1;
                        }
                    }
                    int t1, t2;
                    const int e1 = np.scan_small(nc, &t1);  // children of ranks > r (j' < j)
                    const int e2 = np.scan_small(ne, &t2);
                    if (j < m) {
                        M.divrank[v] = m - 1 - j;
                        M.blockoff[v] = (uint16_t)(c1 + e1);
                        M.expoff[v] = (uint16_t)(c2 + e2);
                    }
                    c1 += t1;
                    c2 += t2;
                }
                if (ntid == 0) {
                    sh->ndiv = m - jstop;
                    sh->nchild = c1;
                }
                np.sync();
                // vsize order is division order (j descending): reverse the expoff offsets
                for (int j = jstop + ntid; j < m; j += NNT) {
                    const int v = sb[j].node;
                    int ne = 0;
                    for (int q = 0; q < 4; ++q) ne += ccur[4 * v + q] > 1;
                    M.expoff[v] = (uint16_t)(c2 - M.expoff[v] - ne);
                }
                if (ntid == 0) sh->nexp = c2;
            }
            np.sync();
            // 2. rebuild: undivided nodes keep their order after all children; one pass over the
            // nodes (each node's record and division rank read once) places both kinds
            {
                const int nchild = sh->nchild;
                int carry = 0;
                for (int base = 0; base < size; base += NNT) {
                    const int i = base + ntid;
                    const bool in = i < size;
                    const int dr = in ? M.divrank[i] : 0;
                    const OctNode nd = on_ld(cur, in ? i : 0);
                    const int v = (in && dr < 0) ? 1 : 0;
                    int tot;
                    const int ex = np.scan_small(v, &tot);
                    if (v) {
                        const int pos = nchild + carry + ex;
                        M.undivpos[i] = (uint16_t)pos;
                        on_st(nxt, pos, nd);
                        if (!fast)
                            for (int q = 0; q < 4; ++q) cnxt[4 * pos + q] = 0;
                    } else if (in) {
                        int pos = M.blockoff[i];
                        int e = M.expoff[i];
                        for (int q = 3; q >= 0; --q) {  // push_front n1..n4 => front reads n4,n3,n2,n1
                            const int c = ccur[4 * i + q];
                            if (c > 0) {
                                const OctNode ch = oct_child(nd, q, c);
                                on_st(nxt, pos, ch);
                                // a fresh child with >1 key is a candidate of the next round: with
                                // the pyramid, its child counts are looked up after this phase (all
                                // threads), which needs it above depth D
                                if (fast) {
                                    if (c > 1 && oct_path_depth(ch.path) >= D) sh->deep = 1;
                                } else {
                                    for (int qq = 0; qq < 4; ++qq) cnxt[4 * pos + qq] = 0;
                                }
                                M.childpos[4 * i + q] = (uint16_t)pos;
                                ++pos;
                            }
                        }
                        for (int q = 0; q < 4; ++q)  // vSizeAndPointerToNode push_back order n1..n4
                            if (ccur[4 * i + q] > 1) vsz2[e++] = M.childpos[4 * i + q];
                    }
                    carry += tot;
                }
                if (ntid == 0) sh->nundiv = carry;
            }
            np.sync();
            // 4. next round's state (read by every thread after the barrier)
            if (ntid == 0) {
                const int nsize = sh->nchild + sh->nundiv;
                sh->size = nsize;
                if (nsize > ws.cap - 4) {
                    sh->status = -3;
                    sh->done = 1;
                } else if (nsize >= N || nsize == sh->prev_size) {
                    sh->done = 1;
                } else if (sh->phase == 1 && nsize + sh->nexp * 3 > N) {
                    sh->phase = 2;
                }
                // the next round would divide a node whose children lie below the pyramid
                if (!sh->done && sh->deep) {
                    sh->status = kOctDeep;
                    sh->done = 1;
                }
                if (ws.dbg) ws.dbg[7] += 1;
            }
            mark(4);
        }
        p.sync();
        mark(2);
        // 3. the next round's candidates (fresh children with >1 key): their child counts from
        // the pyramid, or relabel the keys and count them
        if (fast && !sh->done) {
            const int ne = sh->nexp;
            for (int j = tid; j < ne; j += NT) {
                const int pos = vsz2[j];
                const uint32_t path = nxt[pos].path;
                const int b = pyr_base(oct_path_depth(path) + 1, nIni) + 4 * (int)oct_path_idx(path);
                for (int qq = 0; qq < 4; ++qq) cnxt[4 * pos + qq] = (int)pcnt[b + qq];
            }
        }
        if (!fast) for_keys([&](int base, const uint32_t* key) __attribute__((always_inline)) {
            int e[kOctUnroll], nv[kOctUnroll];
            bool dv[kOctUnroll];
            OctNode nd[kOctUnroll];
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT + tid;
                e[u] = nq[k < n ? k : n - 1];
            }
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int v = e[u] >> 2;
                dv[u] = M.divrank[v] >= 0;
                const int cpos = M.childpos[4 * v + (e[u] & 3)];
                const int upos = M.undivpos[v];
                nv[u] = dv[u] ? cpos : upos;
            }
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) nd[u] = on_ld(nxt, nv[u]);
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT + tid;
                const bool split = k < n && dv[u] && nd[u].cnt > 1;
                const int q = split ? oct_quadrant(key[u], nd[u]) : 0;
                p.run_add(&cnxt[4 * nv[u] + q], 4 * nv[u] + q, split);
                if (k < n) nq[k] = (uint16_t)((nv[u] << 2) | q);
            }
        });
        {
            auto t = cur;
            cur = nxt;
            nxt = t;
            auto c = ccur;
            ccur = cnxt;
            cnxt = c;
            auto u = vsz;
            vsz = vsz2;
            vsz2 = u;
        }
        p.sync();
        mark(fast ? 2 : 5);  // diagnostics: with the pyramid, slot 5 = gather + histogram
    }
    if (sh->status) return sh->status;

    // ---- retain the best key per node (:759-778) ----------------------------------------
    const int size = sh->size;
    if (size > ws.out_cap) return -5;
    if (fast) {  // every node lies at depth <= D: its retained key is its pyramid maximum
        for (int i = tid; i < size; i += NT) {
            const uint32_t path = cur[i].path;
            const uint32_t v = pbest[pyr_base(oct_path_depth(path), nIni) + (int)oct_path_idx(path)];
            const int kid = (int)(0xFFFFFFu - (v & 0xFFFFFFu));
            ws.out_keys[i] = ws.cell_off ? ws.cellkeys[kid] : ws.keys[kid];
        }
        p.sync();
        mark(2);  // diagnostics: with the pyramid, slot 6 = the pyramid's reduction
        return size;
    }
    auto best = reinterpret_cast<asp<LAS, uint32_t>>(cnxt);
    for (int i = tid; i < size; i += NT) best[i] = 0;
    p.sync();
    for_keys([&](int base, const uint32_t* key) __attribute__((always_inline)) {
        int v[kOctUnroll];
#pragma unroll
        for (int u = 0; u < kOctUnroll; ++u) {
            const int k = base + u * NT + tid;
            v[u] = nq[k < n ? k : n - 1] >> 2;
        }
#pragma unroll
        for (int u = 0; u < kOctUnroll; ++u) {
            const int k = base + u * NT + tid;
            const uint32_t val = ((uint32_t)key_resp(key[u]) << 24) | (0xFFFFFFu - (uint32_t)k);
            if (k < n) p.atomic_max(&best[v[u]], val);
        }
    });
    p.sync();
    for (int i = tid; i < size; i += NT) {
        const int k = (int)(0xFFFFFFu - (best[i] & 0xFFFFFFu));
        ws.out_keys[i] = ws.keys[k];
    }
    p.sync();
    mark(6);
    return size;
}

}  // namespace orbgpu
