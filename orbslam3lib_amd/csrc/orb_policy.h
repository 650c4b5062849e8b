// orb_policy.h -- execution policies for the data-parallel algorithms in orb_octree.h.
//
// DevPolicy: one HIP workgroup (blockDim.x a multiple of 64), LDS scratch for the block scan.
// SerialPolicy: a single host thread; used only by the host test harness (tests/) so the same
// algorithm source that runs on the GPU is also checked against the oracle on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_addrspace.h"

namespace orbgpu {

// Wave 0 of a workgroup working alone (the octree's node-level phases): block-wide ops become
// wave-wide, so "sync" costs a counter wait instead of a workgroup barrier.
struct WaveScanPolicy {
    int* scratch;  // unused (interface parity with DevPolicy)
    __device__ int tid() const { return (int)(threadIdx.x & 63); }
    __device__ int nthreads() const { return 64; }
    __device__ void sync() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0);  // LDS and global (node state may live in global memory)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    template <class T>
    __device__ int atomic_add(T p, int v) {
        return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    template <class T>
    __device__ uint32_t atomic_max(T p, uint32_t v) {
        return __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    template <class T>
    __device__ int atomic_max_int(T p, int v) {
        return __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ unsigned long long now() const { return wall_clock64(); }
    __device__ int popc64(uint64_t x) const { return __popcll(x); }
    __device__ int scan_excl(int v, int* total) {
        const int lane = (int)(threadIdx.x & 63);
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        *total = __shfl(x, 63, 64);
        return x - v;
    }
    // exclusive scan of values in [0, 7] by bit-sliced ballots (no cross-lane data movement)
    __device__ int scan_small(int v, int* total) {
        const uint64_t lt = (1ull << (threadIdx.x & 63)) - 1ull;
        const uint64_t b0 = __ballot(v & 1), b1 = __ballot(v & 2), b2 = __ballot(v & 4);
        *total = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        return __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
    }
    // exclusive scans of two 0/1 flags at once
    __device__ int2 scan_pair(int a, int b, int* ta, int* tb) {
        const uint64_t lt = (1ull << (threadIdx.x & 63)) - 1ull;
        const uint64_t ba = __ballot(a), bb = __ballot(b);
        *ta = __popcll(ba);
        *tb = __popcll(bb);
        return make_int2(__popcll(ba & lt), __popcll(bb & lt));
    }
};

struct DevPolicy {
    int* scratch;  // >= 16 ints of LDS
    // node-level work of the octree runs on wave 0 alone
    __device__ bool node_worker() const { return threadIdx.x < 64; }
    __device__ WaveScanPolicy node() const { return WaveScanPolicy{scratch}; }
    __device__ int tid() const { return (int)threadIdx.x; }
    __device__ int nthreads() const { return (int)blockDim.x; }
    __device__ void sync() { __syncthreads(); }
    // memory ordering among the lanes of the calling wave (LDS written by one lane, read by another)
    __device__ void wave_sync() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    template <class T>
    __device__ int atomic_add(T p, int v) {
        return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    template <class T>
    __device__ uint32_t atomic_max(T p, uint32_t v) {
        return __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    template <class T>
    __device__ int atomic_max_int(T p, int v) {
        return __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ unsigned long long now() const { return wall_clock64(); }  // 100 MHz
    // +1 on the counter `ptr` of every valid lane, where lanes naming the same counter `key` in a
    // run of neighbouring lanes add once (the run's first lane adds the run length).  The key
    // passes of the octree visit keys in cell order, so a wave's lanes mostly hit a few counters:
    // per-lane LDS atomics on one address serialize lane by lane.  All lanes must call it.
    template <class T>
    __device__ void run_add(T ptr, int key, bool valid) {
        const int lane = (int)(threadIdx.x & 63);
        const int k = valid ? key : -1 - lane;  // invalid lanes end runs
        const int prev = __shfl_up(k, 1, 64);
        const bool head = valid && (lane == 0 || prev != k);
        const uint64_t bound = __ballot(head || !valid);
        const uint64_t above = lane == 63 ? 0ull : (bound & (~0ull << (lane + 1)));
        const int next = above ? (int)__builtin_ctzll(above) : 64;
        if (head) __hip_atomic_fetch_add(ptr, next - lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ int popc64(uint64_t x) const { return __popcll(x); }
    __device__ int lane() const { return (int)(threadIdx.x & 63); }
    // wave-uniform by construction; readfirstlane lets the compiler keep it (and every loop
    // bound derived from it) in SGPRs
    __device__ int wave() const { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
    __device__ int nwaves() const { return (int)(blockDim.x >> 6); }
    __device__ int wave_width() const { return 64; }
    __device__ uint64_t ballot(bool f) const { return __ballot(f); }
    __device__ uint64_t lanemask_lt() const { return (1ull << (threadIdx.x & 63)) - 1ull; }
    // set bits of m below this lane: v_mbcnt_lo + v_mbcnt_hi (popc(m & lanemask_lt) costs 2 ANDs
    // and 2 v_bcnt)
    __device__ int rank(uint64_t m) const {
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    // OR of x over the 64 lanes of the calling wave (all lanes must participate)
    __device__ uint64_t wave_or(uint64_t x) const {
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) x |= __shfl_xor(x, o, 64);
        return x;
    }
    // Block-wide exclusive scan: every thread passes v, gets its exclusive prefix and the total.
    __device__ int scan_excl(int v, int* total) {
        const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
        const int nw = (int)((blockDim.x + 63) >> 6);
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        __syncthreads();  // scratch may still be read by the previous call
        if (lane == 63) scratch[wid] = x;
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < nw; ++w) {
            const int s = scratch[w];
            before += (w < wid) ? s : 0;
            tot += s;
        }
        *total = tot;
        return before + x - v;
    }
    // block-wide exclusive scan of values in [0, 7]: ballots inside the wave, one LDS hop
    __device__ int scan_small(int v, int* total) {
        const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
        const int nw = (int)((blockDim.x + 63) >> 6);
        const uint64_t lt = (1ull << lane) - 1ull;
        const uint64_t b0 = __ballot(v & 1), b1 = __ballot(v & 2), b2 = __ballot(v & 4);
        const int wtot = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        const int ex = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
        __syncthreads();  // scratch may still be read by the previous call
        if (lane == 0) scratch[wid] = wtot;
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < nw; ++w) {
            const int s = scratch[w];
            before += (w < wid) ? s : 0;
            tot += s;
        }
        *total = tot;
        return before + ex;
    }
    // block-wide exclusive scans of two 0/1 flags with one pair of barriers (<= 8 waves)
    __device__ int2 scan_pair(int a, int b, int* ta, int* tb) {
        const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
        const int nw = (int)((blockDim.x + 63) >> 6);
        const uint64_t lt = (1ull << lane) - 1ull;
        const uint64_t ba = __ballot(a), bb = __ballot(b);
        __syncthreads();  // scratch may still be read by the previous call
        if (lane == 0) {
            scratch[wid] = __popcll(ba);
            scratch[8 + wid] = __popcll(bb);
        }
        __syncthreads();
        int pa = 0, pb = 0, sa = 0, sb = 0;
        for (int w = 0; w < nw; ++w) {
            const int x = scratch[w], y = scratch[8 + w];
            pa += (w < wid) ? x : 0;
            pb += (w < wid) ? y : 0;
            sa += x;
            sb += y;
        }
        *ta = sa;
        *tb = sb;
        return make_int2(pa + __popcll(ba & lt), pb + __popcll(bb & lt));
    }
};

// A DevPolicy whose workgroup size is a compile-time constant (k_fast_cells: FAST_THREADS), so the
// per-wave loops of the policy-templated code have constant trip counts; a one-wave workgroup
// orders its LDS accesses with a wave barrier instead of s_barrier.
template <int NT>
struct FixedDevPolicy : DevPolicy {
    __device__ int nthreads() const { return NT; }
    __device__ int nwaves() const { return NT / 64; }
    __device__ int wave() const { return NT == 64 ? 0 : DevPolicy::wave(); }
    __device__ void sync() {
        if constexpr (NT == 64) wave_sync();
        else __syncthreads();
    }
};

// One wave on its own (64 lanes), e.g. one FAST cell per wave: "sync" is a wave-level memory
// ordering point (LDS ops of one wave complete in order; the fences stop compiler reordering).
struct WavePolicy {
    __device__ int tid() const { return (int)(threadIdx.x & 63); }
    __device__ int nthreads() const { return 64; }
    __device__ void sync() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __device__ int popc64(uint64_t x) const { return __popcll(x); }
    __device__ int lane() const { return (int)(threadIdx.x & 63); }
    __device__ int wave() const { return 0; }
    __device__ int nwaves() const { return 1; }
    __device__ int wave_width() const { return 64; }
    __device__ uint64_t ballot(bool f) const { return __ballot(f); }
    __device__ uint64_t lanemask_lt() const { return (1ull << (threadIdx.x & 63)) - 1ull; }
};

struct SerialPolicy {
    __host__ __device__ bool node_worker() const { return true; }
    __host__ __device__ SerialPolicy node() const { return SerialPolicy{}; }
    __host__ __device__ int tid() const { return 0; }
    __host__ __device__ int nthreads() const { return 1; }
    __host__ __device__ void sync() {}
    __host__ __device__ void wave_sync() {}
    template <class T>
    __host__ __device__ int atomic_add(T p, int v) {
        const int o = *p;
        *p = o + v;
        return o;
    }
    template <class T>
    __host__ __device__ uint32_t atomic_max(T p, uint32_t v) {
        const uint32_t o = *p;
        if (v > o) *p = v;
        return o;
    }
    template <class T>
    __host__ __device__ int atomic_max_int(T p, int v) {
        const int o = *p;
        if (v > o) *p = v;
        return o;
    }
    __host__ __device__ int scan_excl(int v, int* total) {
        *total = v;
        return 0;
    }
    template <class T>
    __host__ __device__ void run_add(T ptr, int, bool valid) {
        if (valid) *ptr += 1;
    }
    __host__ __device__ int scan_small(int v, int* total) {
        *total = v;
        return 0;
    }
    __host__ __device__ int2 scan_pair(int a, int b, int* ta, int* tb) {
        *ta = a;
        *tb = b;
        return make_int2(0, 0);
    }
    __host__ __device__ unsigned long long now() const { return 0; }
    __host__ __device__ int popc64(uint64_t x) const {
        int c = 0;
        for (; x; x &= x - 1) ++c;
        return c;
    }
    __host__ __device__ uint64_t wave_or(uint64_t x) const { return x; }
    __host__ __device__ int lane() const { return 0; }
    __host__ __device__ int wave() const { return 0; }
    __host__ __device__ int nwaves() const { return 1; }
    __host__ __device__ int wave_width() const { return 1; }
    __host__ __device__ uint64_t ballot(bool f) const { return f ? 1ull : 0ull; }
    __host__ __device__ uint64_t lanemask_lt() const { return 0ull; }
    __host__ __device__ int rank(uint64_t) const { return 0; }
};

}  // namespace orbgpu
