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
//   * vSizeAndPointerToNode = children with >1 keys, in (division order, n1..n4) order.
// Keys never move: a key's node is tracked by index, and a node's key list is always the input
// order filtered, so "first key with max response" (:762-778) is an atomic max over
// (response, -input index).
//
// The algorithm is written once against a policy P (tid/nthreads/sync/atomics/block scan):
// the GPU kernel instantiates it with one workgroup per (image, level), the host test harness
// with a serial policy, so the exact same code is checked against the CPU oracle on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_introsort.h"

namespace orbgpu {

struct OctNode {
    int32_t x0, y0, x1, y1;  // UL = (x0,y0), BR = (x1,y1) (relative to minBorder)
    int32_t cnt;             // number of keys
    int32_t nomore;          // bNoMore
};

// Packed candidate key: x | y << 12 | response << 24 (relative coords < 4096, response < 256).
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__host__ __device__ inline int key_resp(uint32_t k) { return (int)(k >> 24); }
__host__ __device__ inline uint32_t make_key(int x, int y, int resp) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)resp << 24);
}

// Per-(image,level) scratch; every array has `cap` entries (x4 where noted), caller-owned.
struct OctWS {
    const uint32_t* keys;  // [n] in vToDistributeKeys order
    int n;
    int cap;               // >= max(n, nIni) + 4
    int32_t* knode;        // [n]
    uint8_t* kq;           // [n]
    OctNode* nodesA;       // [cap]
    OctNode* nodesB;       // [cap]
    int32_t* childcnt;     // [4*cap]
    int32_t* childpos;     // [4*cap]
    int32_t* divrank;      // [cap]
    int32_t* rank2node;    // [cap]
    int32_t* rankoff;      // [cap]
    int32_t* expoff;       // [cap]
    int32_t* undivpos;     // [cap]
    int32_t* vsizeA;       // [cap]
    int32_t* vsizeB;       // [cap]
    SortElem* sortbuf;     // [cap]
    uint32_t* best;        // [cap]
    uint32_t* out_keys;    // [out_cap]
    int out_cap;
};

struct OctShared {
    int size, prev_size, nexp, ndiv, phase, done, nchild, nundiv, status;
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
    c.x0 = (q & 1) ? hx : nd.x0;
    c.x1 = (q & 1) ? nd.x1 : hx;
    c.y0 = (q & 2) ? hy : nd.y0;
    c.y1 = (q & 2) ? nd.y1 : hy;
    c.cnt = cnt;
    c.nomore = (cnt == 1);
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
    OctNode* cur = ws.nodesA;
    OctNode* nxt = ws.nodesB;
    int32_t* vsz = ws.vsizeA;
    int32_t* vsz2 = ws.vsizeB;

    // ---- initial nodes (:561-603) ------------------------------------------------------
    int nIni = (int)roundf((float)W / (float)H);
    if (nIni < 1) nIni = 1;  // reference divides by zero here; never reached at sane sizes
    const float hX = (float)W / (float)nIni;
    if (tid == 0) {
        sh->status = (nIni + 4 > ws.cap) ? -3 : 0;
    }
    p.sync();
    if (sh->status) return sh->status;
    for (int i = tid; i < nIni; i += NT) {
        OctNode nd;
        nd.x0 = (int)(hX * (float)i);
        nd.x1 = (int)(hX * (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = H;
        nd.cnt = 0;
        nd.nomore = 0;
        cur[i] = nd;
    }
    p.sync();
    for (int k = tid; k < n; k += NT) {
        int idx = (int)((float)key_x(ws.keys[k]) / hX);
        if (idx >= nIni) idx = nIni - 1;  // unreachable for in-range keys; keeps memory safe
        ws.knode[k] = idx;
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
                OctNode nd = cur[i];
                nd.nomore = (nd.cnt == 1);
                nxt[carry + ex] = nd;
                ws.undivpos[i] = carry + ex;
            }
            carry += tot;
        }
        if (tid == 0) {
            sh->size = carry;
            sh->nexp = 0;
            sh->phase = 1;
            sh->done = 0;
        }
    }
    p.sync();
    for (int k = tid; k < n; k += NT) ws.knode[k] = ws.undivpos[ws.knode[k]];
    {
        OctNode* t = cur;
        cur = nxt;
        nxt = t;
    }
    p.sync();

    // ---- rounds (:612-757) -----------------------------------------------------------
    int guard = 0;
    while (!sh->done) {
        if (++guard > 4096) {
            if (tid == 0) sh->status = -4;
            p.sync();
            return -4;
        }
        const int size = sh->size;
        const int phase = sh->phase;
        if (tid == 0) sh->prev_size = size;
        // 1. choose division candidates
        if (phase == 1) {
            int carry = 0;
            for (int base = 0; base < size; base += NT) {
                const int i = base + tid;
                const int v = (i < size && !cur[i].nomore) ? 1 : 0;
                int tot;
                const int ex = p.scan_excl(v, &tot);
                if (i < size) ws.divrank[i] = v ? carry + ex : -1;
                carry += tot;
            }
            if (tid == 0) sh->ndiv = carry;
        } else {
            for (int i = tid; i < size; i += NT) ws.divrank[i] = -1;
            p.sync();
            for (int j = tid; j < sh->nexp; j += NT) ws.divrank[vsz[j]] = 0x40000000;  // candidate
        }
        for (int i = tid; i < 4 * size; i += NT) ws.childcnt[i] = 0;
        p.sync();
        // 2. count keys per child quadrant of every candidate node (DivideNode :512-527)
        for (int k = tid; k < n; k += NT) {
            const int v = ws.knode[k];
            if (ws.divrank[v] != -1) {
                const int q = oct_quadrant(ws.keys[k], cur[v]);
                ws.kq[k] = (uint8_t)q;
                p.atomic_add(&ws.childcnt[4 * v + q], 1);
            }
        }
        p.sync();
        // 3. final phase: libstdc++-ordered sort of vPrev, divide from the back until >= N
        if (phase == 2) {
            if (tid == 0) {
                const int m = sh->nexp;
                for (int j = 0; j < m; ++j) {
                    const int v = vsz[j];
                    SortElem e;
                    e.size = cur[v].cnt;
                    e.ulx = cur[v].x0;
                    e.node = v;
                    ws.sortbuf[j] = e;
                }
                introsort_like_libstdcxx(ws.sortbuf, m);
                int sz = size, r = 0, j = m - 1;
                for (; j >= 0; --j) {
                    const int v = ws.sortbuf[j].node;
                    int nc = 0;
                    for (int q = 0; q < 4; ++q) nc += ws.childcnt[4 * v + q] > 0;
                    sz += nc - 1;
                    ws.divrank[v] = r++;
                    if (sz >= N) break;
                }
                for (int jj = (j < 0 ? 0 : j) - 1; jj >= 0; --jj) ws.divrank[ws.sortbuf[jj].node] = -1;
                sh->ndiv = r;
            }
            p.sync();
        }
        const int ndiv = sh->ndiv;
        // 4. rebuild the list
        for (int i = tid; i < size; i += NT) {
            const int r = ws.divrank[i];
            if (r >= 0) {
                int nc = 0, ne = 0;
                for (int q = 0; q < 4; ++q) {
                    const int c = ws.childcnt[4 * i + q];
                    nc += c > 0;
                    ne += c > 1;
                }
                ws.rank2node[r] = i;
                ws.rankoff[r] = nc;   // temporarily the counts
                ws.expoff[r] = ne;
            }
        }
        p.sync();
        {
            // children blocks: rank r goes after all ranks r' > r -> scan in reversed rank order
            int carry = 0;
            for (int base = 0; base < ndiv; base += NT) {
                const int t = base + tid;
                const int r = ndiv - 1 - t;
                const int v = (t < ndiv) ? ws.rankoff[r] : 0;
                int tot;
                const int ex = p.scan_excl(v, &tot);
                p.sync();
                if (t < ndiv) ws.rankoff[r] = carry + ex;
                carry += tot;
            }
            if (tid == 0) sh->nchild = carry;
            int ecarry = 0;
            for (int base = 0; base < ndiv; base += NT) {
                const int r = base + tid;
                const int v = (r < ndiv) ? ws.expoff[r] : 0;
                int tot;
                const int ex = p.scan_excl(v, &tot);
                p.sync();
                if (r < ndiv) ws.expoff[r] = ecarry + ex;
                ecarry += tot;
            }
            if (tid == 0) sh->nexp = ecarry;
        }
        p.sync();
        {
            const int nchild = sh->nchild;
            int carry = 0;
            for (int base = 0; base < size; base += NT) {
                const int i = base + tid;
                const int v = (i < size && ws.divrank[i] < 0) ? 1 : 0;
                int tot;
                const int ex = p.scan_excl(v, &tot);
                if (v) {
                    ws.undivpos[i] = nchild + carry + ex;
                    nxt[nchild + carry + ex] = cur[i];
                }
                carry += tot;
            }
            if (tid == 0) sh->nundiv = carry;
        }
        for (int r = tid; r < ndiv; r += NT) {
            const int i = ws.rank2node[r];
            int pos = ws.rankoff[r];
            int e = ws.expoff[r];
            const OctNode nd = cur[i];
            for (int q = 3; q >= 0; --q) {  // push_front n1..n4 => front reads n4,n3,n2,n1
                const int c = ws.childcnt[4 * i + q];
                if (c > 0) {
                    nxt[pos] = oct_child(nd, q, c);
                    ws.childpos[4 * i + q] = pos;
                    ++pos;
                }
            }
            for (int q = 0; q < 4; ++q) {   // vSizeAndPointerToNode push_back order n1..n4
                if (ws.childcnt[4 * i + q] > 1) vsz2[e++] = ws.childpos[4 * i + q];
            }
        }
        p.sync();
        for (int k = tid; k < n; k += NT) {
            const int v = ws.knode[k];
            ws.knode[k] = (ws.divrank[v] >= 0) ? ws.childpos[4 * v + ws.kq[k]] : ws.undivpos[v];
        }
        p.sync();
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
        }
        {
            OctNode* t = cur;
            cur = nxt;
            nxt = t;
            int32_t* u = vsz;
            vsz = vsz2;
            vsz2 = u;
        }
        p.sync();
    }
    if (sh->status) return sh->status;

    // ---- retain the best key per node (:759-778) ----------------------------------------
    const int size = sh->size;
    if (size > ws.out_cap) return -5;
    for (int i = tid; i < size; i += NT) ws.best[i] = 0;
    p.sync();
    for (int k = tid; k < n; k += NT) {
        const uint32_t val = ((uint32_t)key_resp(ws.keys[k]) << 24) | (0xFFFFFFu - (uint32_t)k);
        p.atomic_max(&ws.best[ws.knode[k]], val);
    }
    p.sync();
    for (int i = tid; i < size; i += NT) {
        const int k = (int)(0xFFFFFFu - (ws.best[i] & 0xFFFFFFu));
        ws.out_keys[i] = ws.keys[k];
    }
    p.sync();
    return size;
}

}  // namespace orbgpu
