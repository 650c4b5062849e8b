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
// Keys never move: a key's node is tracked by index, and a node's key list is always the input
// order filtered, so "first key with max response" (:762-778) is an atomic max over
// (response, -input index).
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

#include "orb_introsort.h"

namespace orbgpu {

struct OctNode {
    uint16_t x0, y0, x1, y1;  // UL = (x0,y0), BR = (x1,y1), relative to minBorder
    int32_t cnt;              // number of keys (bNoMore <=> cnt == 1)
};

// Packed candidate key: x | y << 12 | response << 24 (relative coords < 4096, response < 256).
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__host__ __device__ inline int key_resp(uint32_t k) { return (int)(k >> 24); }
__host__ __device__ inline uint32_t make_key(int x, int y, int resp) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)resp << 24);
}

// Node-state scratch for capacity C nodes (LDS on the GPU when it fits).
struct OctNodeMem {
    OctNode* nodesA;     // [C]
    OctNode* nodesB;     // [C]  (also the sort buffer between the sort and the rebuild)
    int32_t* cntA;       // [4C] child key counts of the current candidates (double-buffered)
    int32_t* cntB;       // [4C]
    uint16_t* childpos;  // [4C]
    int32_t* divrank;    // [C]  -1 undivided, >=0 division rank
    uint16_t* undivpos;  // [C]
    uint16_t* blockoff;  // [C]
    uint16_t* expoff;    // [C]
    uint16_t* vsizeA;    // [C]
    uint16_t* vsizeB;    // [C]
};

__host__ __device__ inline size_t oct_nodemem_bytes(int C) {
    return (size_t)C * (2 * sizeof(OctNode) + 2 * 16 + 8 + 4 + 5 * 2) + 64;
}

// Carves an OctNodeMem out of `base` (16-byte aligned).
__host__ __device__ inline OctNodeMem oct_nodemem_carve(void* base, int C) {
    uint8_t* p = (uint8_t*)base;
    OctNodeMem m;
    m.cntA = (int32_t*)p; p += 16 * (size_t)C;
    m.cntB = (int32_t*)p; p += 16 * (size_t)C;
    m.nodesA = (OctNode*)p; p += sizeof(OctNode) * (size_t)C;
    m.nodesB = (OctNode*)p; p += sizeof(OctNode) * (size_t)C;
    m.divrank = (int32_t*)p; p += 4 * (size_t)C;
    m.childpos = (uint16_t*)p; p += 8 * (size_t)C;
    m.undivpos = (uint16_t*)p; p += 2 * (size_t)C;
    m.blockoff = (uint16_t*)p; p += 2 * (size_t)C;
    m.expoff = (uint16_t*)p; p += 2 * (size_t)C;
    m.vsizeA = (uint16_t*)p; p += 2 * (size_t)C;
    m.vsizeB = (uint16_t*)p; p += 2 * (size_t)C;
    return m;
}

struct OctWS {
    const uint32_t* keys;   // [n] in vToDistributeKeys order
    int n;
    uint16_t* knode;        // [n] current node index of each key
    uint8_t* kq;            // [n] quadrant of each key inside its (candidate) node
    OctNodeMem m;
    int cap;                // node capacity C (>= max(N+3, 4*nIni) + 4)
    uint32_t* out_keys;     // [out_cap]
    int out_cap;
    unsigned long long* dbg;  // diagnostic phase clocks (8 slots) or nullptr
};

constexpr int kOctUnroll = 4;  // keys per thread per batch in the key passes

struct OctShared {
    int size, prev_size, nexp, ndiv, phase, done, nchild, nundiv, status, jstop;
};

__host__ __device__ inline int oct_half(int a, int b) { return (b - a + 1) >> 1; }  // ceil((b-a)/2.f)

__host__ __device__ inline int oct_quadrant(uint32_t key, const OctNode& nd) {
    const int hx = nd.x0 + oct_half(nd.x0, nd.x1);
    const int hy = nd.y0 + oct_half(nd.y0, nd.y1);
    const int x = key_x(key), y = key_y(key);
    if (x < hx) return (y < hy) ? 0 : 2;
    return (y < hy) ? 1 : 3;
}

__host__ __device__ inline OctNode oct_child(const OctNode& nd, int q, int cnt) {
    const int hx = nd.x0 + oct_half(nd.x0, nd.x1);
    const int hy = nd.y0 + oct_half(nd.y0, nd.y1);
    OctNode c;
    c.x0 = (uint16_t)((q & 1) ? hx : nd.x0);
    c.x1 = (uint16_t)((q & 1) ? nd.x1 : hx);
    c.y0 = (uint16_t)((q & 2) ? hy : nd.y0);
    c.y1 = (uint16_t)((q & 2) ? nd.y1 : hy);
    c.cnt = cnt;
    return c;
}

// Runs DistributeOctTree for one level.  Coordinates are relative to (minBorderX, minBorderY);
// W = maxBorderX-minBorderX, H = maxBorderY-minBorderY, N = mnFeaturesPerLevel[level].
// Returns the number of output nodes (keys written to ws.out_keys in list order), or <0.
template <class P>
__host__ __device__ int octree_distribute(P& p, const OctWS& ws, OctShared* sh, int W, int H,
                                          int N) {
    const int tid = p.tid(), NT = p.nthreads();
    const int n = ws.n;
    const OctNodeMem& M = ws.m;
    OctNode* cur = M.nodesA;
    OctNode* nxt = M.nodesB;
    int32_t* ccur = M.cntA;   // child counts of the current round's candidates
    int32_t* cnxt = M.cntB;
    uint16_t* vsz = M.vsizeA;
    uint16_t* vsz2 = M.vsizeB;
    unsigned long long t_prev = p.now();
    auto mark = [&](int slot) {
        if (ws.dbg && tid == 0) {
            const unsigned long long t = p.now();
            ws.dbg[slot] += t - t_prev;
            t_prev = t;
        }
    };

    // ---- initial nodes (:561-603) ------------------------------------------------------
    int nIni = (int)roundf((float)W / (float)H);
    if (nIni < 1) nIni = 1;  // reference divides by zero here; never reached at sane sizes
    const float hX = (float)W / (float)nIni;
    if (nIni + 4 > ws.cap) return -3;
    for (int i = tid; i < nIni; i += NT) {
        OctNode nd;
        nd.x0 = (uint16_t)(int)(hX * (float)i);
        nd.x1 = (uint16_t)(int)(hX * (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = (uint16_t)H;
        nd.cnt = 0;
        cur[i] = nd;
    }
    p.sync();
    for (int k = tid; k < n; k += NT) {
        int idx = (int)((float)key_x(ws.keys[k]) / hX);
        if (idx >= nIni) idx = nIni - 1;  // unreachable for in-range keys; keeps memory safe
        ws.knode[k] = (uint16_t)idx;
        p.atomic_add(&cur[idx].cnt, 1);
    }
    p.sync();
    {
        int carry = 0;
        for (int base = 0; base < nIni; base += NT) {
            const int i = base + tid;
            const int v = (i < nIni && cur[i].cnt > 0) ? 1 : 0;
            int tot;
            const int ex = p.scan_excl(v, &tot);
            if (v) {
                nxt[carry + ex] = cur[i];
                M.undivpos[i] = (uint16_t)(carry + ex);
                for (int q = 0; q < 4; ++q) ccur[4 * (carry + ex) + q] = 0;
            }
            carry += tot;
        }
        if (tid == 0) {
            sh->size = carry;
            sh->nexp = 0;
            sh->phase = 1;
            sh->done = 0;
            sh->status = 0;
        }
    }
    {
        OctNode* t = cur;
        cur = nxt;
        nxt = t;
    }
    p.sync();
    // relabel to the compacted list + count round 1 (every node with >1 key is a candidate)
    for (int k = tid; k < n; k += NT) {
        const int v = M.undivpos[ws.knode[k]];
        ws.knode[k] = (uint16_t)v;
        if (cur[v].cnt > 1) {
            const int q = oct_quadrant(ws.keys[k], cur[v]);
            ws.kq[k] = (uint8_t)q;
            p.atomic_add(&ccur[4 * v + q], 1);
        }
    }
    p.sync();
    mark(0);

    // ---- rounds (:612-757) -----------------------------------------------------------
    int guard = 0;
    while (!sh->done) {
        if (++guard > 4096) return -4;
        const int size = sh->size;
        const int phase = sh->phase;
        if (tid == 0) sh->prev_size = size;
        // 1. division order
        if (phase == 1) {  // every non-frozen node, in list order
            int carry = 0;
            for (int base = 0; base < size; base += NT) {
                const int i = base + tid;
                const int v = (i < size && cur[i].cnt > 1) ? 1 : 0;
                int tot;
                const int ex = p.scan_excl(v, &tot);
                if (i < size) M.divrank[i] = v ? carry + ex : -1;
                carry += tot;
            }
            if (tid == 0) sh->ndiv = carry;
            p.sync();
            mark(1);
            // children block offsets: rank r lands after all ranks > r
            const int nd_ = sh->ndiv;
            int c1 = 0, c2 = 0;
            for (int base = 0; base < size; base += NT) {
                const int i = base + tid;
                int nc = 0, ne = 0;
                if (i < size && M.divrank[i] >= 0) {
                    for (int q = 0; q < 4; ++q) {
                        const int c = ccur[4 * i + q];
                        nc += c > 0;
                        ne += c > 1;
                    }
                }
                int t1, t2;
                const int e1 = p.scan_excl(nc, &t1);
                const int e2 = p.scan_excl(ne, &t2);
                if (i < size && M.divrank[i] >= 0) {
                    M.blockoff[i] = (uint16_t)(c1 + e1 + nc);  // inclusive; finalised below
                    M.expoff[i] = (uint16_t)(c2 + e2);
                }
                c1 += t1;
                c2 += t2;
            }
            if (tid == 0) {
                sh->nchild = c1;
                sh->nexp = c2;
            }
            p.sync();
            for (int i = tid; i < size; i += NT)
                if (M.divrank[i] >= 0) M.blockoff[i] = (uint16_t)(c1 - M.blockoff[i]);
            (void)nd_;
        } else {  // final phase: libstdc++-ordered sort of vPrev, divide from the back until N
            const int m = sh->nexp;
            SortElem* sb = reinterpret_cast<SortElem*>(nxt);  // nxt is free until the rebuild
            for (int j = tid; j < m; j += NT) {
                const int v = vsz[j];
                SortElem e;
                e.size = cur[v].cnt;
                e.ulx = cur[v].x0;
                e.node = v;
                sb[j] = e;
            }
            p.sync();
            {
                // scratch: every array below is free until step 3 / the rebuild
                const int C = ws.cap;
                SortScratch ss;
                ss.tmp = reinterpret_cast<SortElem*>(cnxt);
                ss.lex = M.childpos;
                ss.rex = M.childpos + (C + 1);
                ss.segof = M.childpos + 2 * (C + 1);
                ss.lpos = M.undivpos;
                ss.rpos = M.blockoff;
                ss.rank = M.expoff;
                uint16_t* seg = reinterpret_cast<uint16_t*>(M.divrank);
                const int S = C / 16 + 4;
                for (int b = 0; b < 2; ++b) {
                    ss.segF[b] = seg + (3 * b + 0) * S;
                    ss.segL[b] = seg + (3 * b + 1) * S;
                    ss.segD[b] = seg + (3 * b + 2) * S;
                }
                ss.segK = reinterpret_cast<int32_t*>(seg + 6 * S + 2);
                introsort_parallel(p, sb, m, ss, &sh->jstop);
            }
            for (int i = tid; i < size; i += NT) M.divrank[i] = -1;
            p.sync();
            mark(3);
            // S_j = size + sum_{j'>=j} (nc_j' - 1) is non-increasing in j; divide [jstop, m)
            if (tid == 0) sh->jstop = 0;
            int carry = 0;
            for (int base = 0; base < m; base += NT) {  // scan in reversed sorted order
                const int t = base + tid;
                const int j = m - 1 - t;
                int d = 0;
                if (t < m) {
                    const int v = sb[j].node;
                    for (int q = 0; q < 4; ++q) d += ccur[4 * v + q] > 0;
                    d -= 1;
                }
                int tot;
                const int ex = p.scan_excl(d, &tot);
                if (t < m && size + carry + ex + d >= N) p.atomic_max_int(&sh->jstop, j);
                carry += tot;
            }
            p.sync();
            const int jstop = sh->jstop;
            // ranks, block offsets (division order = j descending) and vsize offsets
            int c1 = 0, c2 = 0;
            for (int base = jstop; base < m; base += NT) {
                const int j = base + tid;
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
                const int e1 = p.scan_excl(nc, &t1);  // children of ranks > r (j' < j)
                const int e2 = p.scan_excl(ne, &t2);
                if (j < m) {
                    M.divrank[v] = m - 1 - j;
                    M.blockoff[v] = (uint16_t)(c1 + e1);
                    M.expoff[v] = (uint16_t)(c2 + e2);
                }
                c1 += t1;
                c2 += t2;
            }
            if (tid == 0) {
                sh->ndiv = m - jstop;
                sh->nchild = c1;
            }
            p.sync();
            // vsize order is division order (j descending): reverse the expoff offsets
            for (int j = jstop + tid; j < m; j += NT) {
                const int v = sb[j].node;
                int ne = 0;
                for (int q = 0; q < 4; ++q) ne += ccur[4 * v + q] > 1;
                M.expoff[v] = (uint16_t)(c2 - M.expoff[v] - ne);
            }
            if (tid == 0) sh->nexp = c2;
        }
        p.sync();
        mark(1);
        // 2. rebuild: undivided nodes keep their order after all children
        {
            const int nchild = sh->nchild;
            int carry = 0;
            for (int base = 0; base < size; base += NT) {
                const int i = base + tid;
                const int v = (i < size && M.divrank[i] < 0) ? 1 : 0;
                int tot;
                const int ex = p.scan_excl(v, &tot);
                if (v) {
                    const int pos = nchild + carry + ex;
                    M.undivpos[i] = (uint16_t)pos;
                    nxt[pos] = cur[i];
                    for (int q = 0; q < 4; ++q) cnxt[4 * pos + q] = 0;
                }
                carry += tot;
            }
            if (tid == 0) sh->nundiv = carry;
        }
        for (int i = tid; i < size; i += NT) {
            if (M.divrank[i] < 0) continue;
            int pos = M.blockoff[i];
            int e = M.expoff[i];
            const OctNode nd = cur[i];
            for (int q = 3; q >= 0; --q) {  // push_front n1..n4 => front reads n4,n3,n2,n1
                const int c = ccur[4 * i + q];
                if (c > 0) {
                    nxt[pos] = oct_child(nd, q, c);
                    for (int qq = 0; qq < 4; ++qq) cnxt[4 * pos + qq] = 0;
                    M.childpos[4 * i + q] = (uint16_t)pos;
                    ++pos;
                }
            }
            for (int q = 0; q < 4; ++q)  // vSizeAndPointerToNode push_back order n1..n4
                if (ccur[4 * i + q] > 1) vsz2[e++] = M.childpos[4 * i + q];
        }
        p.sync();
        mark(4);
        // 3. relabel keys, and count the next round's candidates (fresh children with >1 key);
        //    global loads of 4 keys per thread are issued together (latency-bound pass)
        for (int base = tid; base < n; base += kOctUnroll * NT) {
            int v[kOctUnroll], q0[kOctUnroll];
            uint32_t key[kOctUnroll];
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT;
                const bool in = k < n;
                v[u] = in ? ws.knode[k] : 0;
                q0[u] = in ? ws.kq[k] : 0;
                key[u] = in ? ws.keys[k] : 0;
            }
#pragma unroll
            for (int u = 0; u < kOctUnroll; ++u) {
                const int k = base + u * NT;
                if (k >= n) continue;
                const bool dv = M.divrank[v[u]] >= 0;
                const int nv = dv ? M.childpos[4 * v[u] + q0[u]] : M.undivpos[v[u]];
                ws.knode[k] = (uint16_t)nv;
                if (dv && nxt[nv].cnt > 1) {
                    const int q = oct_quadrant(key[u], nxt[nv]);
                    ws.kq[k] = (uint8_t)q;
                    p.atomic_add(&cnxt[4 * nv + q], 1);
                }
            }
        }
        if (tid == 0) {
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
            if (ws.dbg) ws.dbg[7] += 1;
        }
        {
            OctNode* t = cur;
            cur = nxt;
            nxt = t;
            int32_t* c = ccur;
            ccur = cnxt;
            cnxt = c;
            uint16_t* u = vsz;
            vsz = vsz2;
            vsz2 = u;
        }
        p.sync();
        mark(5);
    }
    if (sh->status) return sh->status;

    // ---- retain the best key per node (:759-778) ----------------------------------------
    const int size = sh->size;
    if (size > ws.out_cap) return -5;
    uint32_t* best = reinterpret_cast<uint32_t*>(cnxt);
    for (int i = tid; i < size; i += NT) best[i] = 0;
    p.sync();
    for (int base = tid; base < n; base += kOctUnroll * NT) {
        uint32_t key[kOctUnroll];
        int v[kOctUnroll];
#pragma unroll
        for (int u = 0; u < kOctUnroll; ++u) {
            const int k = base + u * NT;
            key[u] = k < n ? ws.keys[k] : 0;
            v[u] = k < n ? ws.knode[k] : 0;
        }
#pragma unroll
        for (int u = 0; u < kOctUnroll; ++u) {
            const int k = base + u * NT;
            if (k >= n) continue;
            const uint32_t val = ((uint32_t)key_resp(key[u]) << 24) | (0xFFFFFFu - (uint32_t)k);
            p.atomic_max(&best[v[u]], val);
        }
    }
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
