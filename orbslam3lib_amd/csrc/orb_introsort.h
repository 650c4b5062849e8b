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

namespace orbgpu {

// Element sorted by the octree: key = (size << 16 | ulx) would NOT reproduce libstdc++ on
// ties, so the comparator is kept separate and the payload (node index) travels with it.
struct SortElem {
    int32_t size;
    int32_t ulx;
    int32_t node;
};

__host__ __device__ inline bool node_less(const SortElem& a, const SortElem& b) {
    if (a.size < b.size) return true;
    if (a.size > b.size) return false;
    return a.ulx < b.ulx;
}

__host__ __device__ inline void isort_swap(SortElem* a, int i, int j) {
    SortElem t = a[i];
    a[i] = a[j];
    a[j] = t;
}

__host__ __device__ inline int isort_lg(int n) {
    int k = 0;
    while ((n >> (k + 1)) > 0) ++k;
    return k;
}

__host__ __device__ inline void isort_push_heap(SortElem* a, int hole, int top, SortElem v) {
    int parent = (hole - 1) / 2;
    while (hole > top && node_less(a[parent], v)) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = v;
}

__host__ __device__ inline void isort_adjust_heap(SortElem* a, int hole, int len, SortElem v) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (node_less(a[second], a[second - 1])) second--;
        a[hole] = a[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[hole] = a[second - 1];
        hole = second - 1;
    }
    isort_push_heap(a, hole, top, v);
}

// std::__partial_sort(first, last, last) == __make_heap + __sort_heap on [first, last).
__host__ __device__ inline void isort_heapsort(SortElem* a, int n) {
    if (n >= 2) {
        int parent = (n - 2) / 2;
        while (true) {
            SortElem v = a[parent];
            isort_adjust_heap(a, parent, n, v);
            if (parent == 0) break;
            parent--;
        }
    }
    while (n > 1) {
        --n;
        SortElem v = a[n];
        a[n] = a[0];
        isort_adjust_heap(a, 0, n, v);
    }
}

__host__ __device__ inline void isort_median_to_first(SortElem* a, int result, int i, int j, int k) {
    if (node_less(a[i], a[j])) {
        if (node_less(a[j], a[k])) isort_swap(a, result, j);
        else if (node_less(a[i], a[k])) isort_swap(a, result, k);
        else isort_swap(a, result, i);
    } else if (node_less(a[i], a[k])) {
        isort_swap(a, result, i);
    } else if (node_less(a[j], a[k])) {
        isort_swap(a, result, k);
    } else {
        isort_swap(a, result, j);
    }
}

__host__ __device__ inline int isort_unguarded_partition(SortElem* a, int first, int last,
                                                         int pivot) {
    while (true) {
        while (node_less(a[first], a[pivot])) ++first;
        --last;
        while (node_less(a[pivot], a[last])) --last;
        if (!(first < last)) return first;
        isort_swap(a, first, last);
        ++first;
    }
}

__host__ __device__ inline void isort_unguarded_linear_insert(SortElem* a, int last) {
    SortElem v = a[last];
    int next = last - 1;
    while (node_less(v, a[next])) {
        a[last] = a[next];
        last = next;
        --next;
    }
    a[last] = v;
}

__host__ __device__ inline void isort_insertion(SortElem* a, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (node_less(a[i], a[first])) {
            SortElem v = a[i];
            for (int k = i; k > first; --k) a[k] = a[k - 1];
            a[first] = v;
        } else {
            isort_unguarded_linear_insert(a, i);
        }
    }
}

// Iterative form of __introsort_loop: libstdc++ recurses on the right part and loops on the
// left; an explicit stack of (first, last, depth) frames visited in the same order is
// equivalent because the two halves are disjoint.
__host__ __device__ inline void introsort_like_libstdcxx(SortElem* a, int n) {
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

}  // namespace orbgpu
