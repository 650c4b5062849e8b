// orb_introsort.h -- deterministic introsort whose permutation equals libstdc++'s std::sort.
//
// Why: DistributeOctTree sorts (size, node*) pairs with compareNodes (reference
// cpp/src/ORBextractor_old.cc:540-555, sort call :702).  compareNodes is not a strict total
// order on ties (equal size and equal UL.x), so which of two tied nodes is divided first --
// and therefore the keypoint order and the set kept at the N cut -- is whatever GNU libstdc++'s
// introsort does.  This header restates that algorithm (GCC bits/stl_algo.h / stl_heap.h:
// __introsort_loop with threshold 16 and depth 2*lg(n), median-of-three into *first,
// __unguarded_partition, heap-sort fallback, __final_insertion_sort) on plain arrays so one
// GPU thread can reproduce the exact permutation.  Host-testable (tests/test_host_harness.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_addrspace.h"

namespace orbgpu {

// Element sorted by the octree: key = (size << 16 | ulx) would NOT reproduce libstdc++ on
// ties, so the comparator is kept separate and the payload (node index) travels with it.
struct alignas(16) SortElem {
    int32_t size;
    int32_t ulx;
    int32_t node;
    int32_t pad;  // 16 bytes: one ds_read_b128 / ds_write_b128 per element
};

__host__ __device__ inline bool node_less(SortElem a, SortElem b) {
    if (a.size < b.size) return true;
    if (a.size > b.size) return false;
    return a.ulx < b.ulx;
}

// Whole-element access that works for any address space (the implicit copy operations of a
// struct take generic references, which an LDS-qualified lvalue cannot bind to).
template <class EP>
__host__ __device__ inline SortElem se_ld(EP a, int i) {
    const orb_u32x4 v = as_vec4(a)[i];
    SortElem e;
    e.size = (int32_t)v.x;
    e.ulx = (int32_t)v.y;
    e.node = (int32_t)v.z;
    e.pad = 0;
    return e;
}
template <class EP>
__host__ __device__ inline void se_st(EP a, int i, SortElem e) {
    orb_u32x4 v;
    v.x = (uint32_t)e.size;
    v.y = (uint32_t)e.ulx;
    v.z = (uint32_t)e.node;
    v.w = 0;
    as_vec4(a)[i] = v;
}

template <class EP>
__host__ __device__ inline void isort_swap(EP a, int i, int j) {
    // whole 16-byte elements (a struct temporary could be placed in scratch memory by hipcc)
    const orb_u32x4 x = as_vec4(a)[i], y = as_vec4(a)[j];
    as_vec4(a)[i] = y;
    as_vec4(a)[j] = x;
}

__host__ __device__ inline int isort_lg(int n) {
    int k = 0;
    while ((n >> (k + 1)) > 0) ++k;
    return k;
}

template <class EP>
__host__ __device__ inline void isort_push_heap(EP a, int hole, int top, SortElem v) {
    int parent = (hole - 1) / 2;
    while (hole > top && node_less(se_ld(a, parent), v)) {
        se_st(a, hole, se_ld(a, parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    se_st(a, hole, v);
}

template <class EP>
__host__ __device__ inline void isort_adjust_heap(EP a, int hole, int len, SortElem v) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (node_less(se_ld(a, second), se_ld(a, second - 1))) second--;
        se_st(a, hole, se_ld(a, second));
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        se_st(a, hole, se_ld(a, second - 1));
        hole = second - 1;
    }
    isort_push_heap(a, hole, top, v);
}

// std::__partial_sort(first, last, last) == __make_heap + __sort_heap on [first, last).
template <class EP>
__host__ __device__ inline void isort_heapsort(EP a, int n) {
    if (n >= 2) {
        int parent = (n - 2) / 2;
        while (true) {
            SortElem v = se_ld(a, parent);
            isort_adjust_heap(a, parent, n, v);
            if (parent == 0) break;
            parent--;
        }
    }
    while (n > 1) {
        --n;
        SortElem v = se_ld(a, n);
        se_st(a, n, se_ld(a, 0));
        isort_adjust_heap(a, 0, n, v);
    }
}

template <class EP>
__host__ __device__ inline void isort_median_to_first(EP a, int result, int i, int j, int k) {
    if (node_less(se_ld(a, i), se_ld(a, j))) {
        if (node_less(se_ld(a, j), se_ld(a, k))) isort_swap(a, result, j);
        else if (node_less(se_ld(a, i), se_ld(a, k))) isort_swap(a, result, k);
        else isort_swap(a, result, i);
    } else if (node_less(se_ld(a, i), se_ld(a, k))) {
        isort_swap(a, result, i);
    } else if (node_less(se_ld(a, j), se_ld(a, k))) {
        isort_swap(a, result, k);
    } else {
        isort_swap(a, result, j);
    }
}

template <class EP>
__host__ __device__ inline int isort_unguarded_partition(EP a, int first, int last,
                                                         int pivot) {
    while (true) {
        while (node_less(se_ld(a, first), se_ld(a, pivot))) ++first;
        --last;
        while (node_less(se_ld(a, pivot), se_ld(a, last))) --last;
        if (!(first < last)) return first;
        isort_swap(a, first, last);
        ++first;
    }
}

template <class EP>
__host__ __device__ inline void isort_unguarded_linear_insert(EP a, int last) {
    SortElem v = se_ld(a, last);
    int next = last - 1;
    while (node_less(v, se_ld(a, next))) {
        se_st(a, last, se_ld(a, next));
        last = next;
        --next;
    }
    se_st(a, last, v);
}

template <class EP>
__host__ __device__ inline void isort_insertion(EP a, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (node_less(se_ld(a, i), se_ld(a, first))) {
            SortElem v = se_ld(a, i);
            for (int k = i; k > first; --k) se_st(a, k, se_ld(a, k - 1));
            se_st(a, first, v);
        } else {
            isort_unguarded_linear_insert(a, i);
        }
    }
}

// Iterative form of __introsort_loop: libstdc++ recurses on the right part and loops on the
// left; an explicit stack of (first, last, depth) frames visited in the same order is
// equivalent because the two halves are disjoint.
template <class EP>
__host__ __device__ inline void introsort_like_libstdcxx(EP a, int n) {
    if (n <= 1) return;
    const int kThreshold = 16;
    struct Frame { int first, last, depth; };
    Frame stack[64];
    int sp = 0;
    stack[sp++] = {0, n, 2 * isort_lg(n)};
    while (sp > 0) {
        Frame f = stack[--sp];
        int first = f.first, last = f.last, depth = f.depth;
        while (last - first > kThreshold) {
            if (depth == 0) {
                isort_heapsort(a + first, last - first);
                break;
            }
            --depth;
            int mid = first + (last - first) / 2;
            isort_median_to_first(a, first, first + 1, mid, last - 1);
            int cut = isort_unguarded_partition(a, first + 1, last, first);
            // libstdc++: __introsort_loop(cut, last, depth) first, then continue with last=cut.
            // Push the left remainder so that the right part is fully processed first.
            stack[sp++] = {first, cut, depth};
            first = cut;
        }
    }
    if (n > kThreshold) {
        isort_insertion(a, 0, kThreshold);
        for (int i = kThreshold; i < n; ++i) isort_unguarded_linear_insert(a, i);
    } else {
        isort_insertion(a, 0, n);
    }
}

// ---------------------------------------------------------------------------------------------
// Data-parallel form of the same permutation (policy-templated, one workgroup).
//
// 1. __introsort_loop only partitions: segments > 16 elements are split with median-of-three +
//    __unguarded_partition until depth runs out (then that segment is heap-sorted).  Segments of
//    one recursion level are disjoint and are partitioned together.  The two-pointer Hoare scan
//    is reproduced exactly from the original values: with L'_k the k-th "left stopper"
//    (!(a[i] < pivot), i > f, ascending) and R'_k the k-th "right stopper" (!(pivot < a[i]),
//    descending), the scan swaps (L'_k, R'_k) for every k with L'_k < R'_k (a prefix, K pairs)
//    and returns cut = min(L'_K, R'_{K-1}) -- the positions it revisits after a swap never
//    change a stop decision before the pointers cross.
// 2. __final_insertion_sort over the whole partitioned array is a stable insertion sort (its
//    leftmost segment holds the minimum, so the unguarded inserts are exact): it equals a stable
//    sort of the partitioned array, done here as a parallel rank sort.
template <int AS>
struct SortScratchT {
    asp<AS, SortElem> tmp;       // [m]
    asp<AS, uint16_t> lex;       // [m+1]
    asp<AS, uint16_t> rex;       // [m+1]
    asp<AS, uint16_t> segof;     // [m]
    asp<AS, uint16_t> lpos;      // [m]
    asp<AS, uint16_t> rpos;      // [m]
    asp<AS, uint16_t> rank;      // [m]
    asp<AS, uint16_t> segF[2];   // [S]
    asp<AS, uint16_t> segL[2];   // [S]
    asp<AS, uint16_t> segD[2];   // [S]
    asp<AS, int32_t> segK;       // [S]
};
using SortScratch = SortScratchT<kGeneric>;

// Step 1 (partition phase) on policy p: segments are independent, so each is partitioned by
// ONE wave (wave w takes segments w, w + waves, ...) with ballot scans inside the wave, and a
// round of the recursion costs a single workgroup barrier.  The next round's segments are
// appended through a counter (their order does not matter: segments are disjoint).
template <int AS, class P>
__host__ __device__ __attribute__((always_inline)) inline void introsort_partition(
    P& p, asp<AS, SortElem> a, int m, const SortScratchT<AS>& s, asp<AS, int> /*unused*/) {
    const int tid = p.tid(), NT = p.nthreads();
    const int lane = p.lane(), wv = p.wave(), Wv = p.nwaves(), Lw = p.wave_width();
    const uint64_t lt = p.lanemask_lt();
    if (m <= 1) return;
    // s.rank[i] = first index of the final segment holding i (a segment of <= 16 elements is
    // never partitioned again), 0xFFFF inside a heap-sorted segment (step 2 reads it)
    if (m <= 16) {
        for (int i = tid; i < m; i += NT) s.rank[i] = 0;
        p.sync();
        return;
    }
    // s.segK[0..2]: segment counters of rounds r, r + 1, r + 2 (mod 3)
    if (tid == 0) {
        s.segF[0][0] = 0;
        s.segL[0][0] = (uint16_t)m;
        s.segD[0][0] = (uint16_t)(2 * isort_lg(m));
        s.segK[0] = 1;
        s.segK[1] = 0;
        s.segK[2] = 0;
    }
    p.sync();
    int cur = 0;
    for (int r = 0;; ++r) {
        const int nseg = s.segK[r % 3];
        if (nseg == 0) break;
        if (tid == 0) s.segK[(r + 2) % 3] = 0;  // last read in round r - 1, appended in r + 1
        const auto F = cur ? s.segF[1] : s.segF[0];
        const auto L = cur ? s.segL[1] : s.segL[0];
        const auto D = cur ? s.segD[1] : s.segD[0];
        const auto NF = cur ? s.segF[0] : s.segF[1];
        const auto NL = cur ? s.segL[0] : s.segL[1];
        const auto ND = cur ? s.segD[0] : s.segD[1];
        const auto nxt_cnt = s.segK + (r + 1) % 3;
        for (int g = wv; g < nseg; g += Wv) {  // wave-uniform
            const int f = F[g], l = L[g], d = D[g];
            if (d == 0) {  // depth exhausted: std::__partial_sort, in place
                if (lane == 0) isort_heapsort(a + f, l - f);
                for (int i = f + lane; i < l; i += Lw) s.rank[i] = 0xFFFF;
                p.wave_sync();
                continue;
            }
            if (lane == 0) isort_median_to_first(a, f, f + 1, f + (l - f) / 2, l - 1);
            p.wave_sync();
            const SortElem pv = se_ld(a, f);
            // left stoppers L'_k (i > f, !(a[i] < pivot)) ascending into lpos[f + k]; right
            // stoppers (!(pivot < a[i])) counted from the left into rex[i], then placed
            // descending into rpos[f + k]
            int nl = 0, nr = 0;
            for (int i0 = f; i0 < l; i0 += Lw) {
                const int i = i0 + lane;
                bool lf = false, rf = false;
                if (i < l) {
                    const SortElem x = se_ld(a, i);
                    lf = i > f && !node_less(x, pv);
                    rf = !node_less(pv, x);
                }
                const uint64_t bl = p.ballot(lf), br = p.ballot(rf);
                if (lf) s.lpos[f + nl + p.popc64(bl & lt)] = (uint16_t)i;
                if (i < l) s.rex[i] = rf ? (uint16_t)(nr + p.popc64(br & lt)) : (uint16_t)0xFFFF;
                nl += p.popc64(bl);
                nr += p.popc64(br);
            }
            p.wave_sync();
            for (int i = f + lane; i < l; i += Lw) {
                const int k = s.rex[i];
                if (k != 0xFFFF) s.rpos[f + nr - 1 - k] = (uint16_t)i;
            }
            p.wave_sync();
            // the scan swaps (L'_k, R'_k) while L'_k < R'_k: a prefix of k (L' ascends, R'
            // descends) of K pairs, no position in two of them, so every pair swaps in place
            const int np = nl < nr ? nl : nr;
            int K = 0;
            for (int k0 = 0; k0 < np; k0 += Lw) {
                const int k = k0 + lane;
                const bool sw = k < np && s.lpos[f + k] < s.rpos[f + k];
                if (sw) isort_swap(a, s.lpos[f + k], s.rpos[f + k]);
                K += p.popc64(p.ballot(sw));
            }
            p.wave_sync();
            int cut = K < nl ? s.lpos[f + K] : 0x7fffffff;
            if (K > 0) {
                const int rk = s.rpos[f + K - 1];
                cut = cut < rk ? cut : rk;
            }
            // children: > 16 elements go to the next round, the others are final segments
            if (lane == 0) {
                if (cut - f > 16) {
                    const int o = p.atomic_add(nxt_cnt, 1);
                    NF[o] = (uint16_t)f;
                    NL[o] = (uint16_t)cut;
                    ND[o] = (uint16_t)(d - 1);
                }
                if (l - cut > 16) {
                    const int o = p.atomic_add(nxt_cnt, 1);
                    NF[o] = (uint16_t)cut;
                    NL[o] = (uint16_t)l;
                    ND[o] = (uint16_t)(d - 1);
                }
            }
            if (cut - f <= 16)
                for (int i = f + lane; i < cut; i += Lw) s.rank[i] = (uint16_t)f;
            if (l - cut <= 16)
                for (int i = cut + lane; i < l; i += Lw) s.rank[i] = (uint16_t)cut;
            p.wave_sync();
        }
        p.sync();
        cur ^= 1;
    }
}

// Step 2: stable sort of the partitioned array on policy p.  Partitioning leaves every element
// of a segment <= every element of the segments to its right, so the stable sort of the whole
// array is the stable sort of each final segment (<= 16 elements: a rank among them; a
// heap-sorted segment is already in order and keeps its positions).
template <int AS, class P>
__host__ __device__ __attribute__((always_inline)) inline void introsort_final(
    P& p, asp<AS, SortElem> a, int m, const SortScratchT<AS>& s) {
    const int tid = p.tid(), NT = p.nthreads();
    if (m <= 1) return;
    for (int i = tid; i < m; i += NT) {
        const SortElem x = se_ld(a, i);
        const int s0 = s.rank[i];
        int r = i;
        if (s0 != 0xFFFF) {
            r = s0;
            for (int j = s0; j < m && s.rank[j] == s0; ++j) {
                const SortElem y = se_ld(a, j);
                r += node_less(y, x) || (j < i && !node_less(x, y));
            }
        }
        se_st(s.tmp, r, x);
    }
    p.sync();
    for (int i = tid; i < m; i += NT) se_st(a, i, se_ld(s.tmp, i));
    p.sync();
}

template <int AS, class P>
__host__ __device__ __attribute__((always_inline)) inline void introsort_parallel(
    P& p, asp<AS, SortElem> a, int m, const SortScratchT<AS>& s, asp<AS, int> sh_nseg) {
    introsort_partition<AS>(p, a, m, s, sh_nseg);
    introsort_final<AS>(p, a, m, s);
}

}  // namespace orbgpu
