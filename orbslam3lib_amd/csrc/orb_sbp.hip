// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
// (cpp/src/ORBmatcher.cc:44-214) for pinhole frames (Nleft == -1), over frames whose keypoints,
// descriptors, grid (Frame::GetFeaturesInArea, Frame.cc:673-735) and mvuRight already live in HBM.
//
// The reference loop is sequential: a keypoint taken by an earlier map point (Observations() > 0)
// is skipped by every later one.  Two kernels keep the result identical:
//   k_sbp_candidates  one thread per map point walks its window with the pre-call occupancy and
//                     keeps its 4 lowest (distance, window position) candidates + their count.
//                     The reference's (best, second) pair is exactly the two lowest of that order
//                     (strict `<` keeps the earlier of equal distances), so removing a candidate
//                     outside the two lowest changes nothing.
//   k_sbp_resolve     one wave per frame replays the map points in order, 64 lanes at a time,
//                     from LDS-staged top-4 lists: the first two candidates not taken so far are
//                     the reference's (best, second); only when fewer than two survive out of a
//                     window holding more than four does a lane re-walk its window with the live
//                     occupancy.  Lanes whose examined candidates an earlier lane of the group
//                     takes are recomputed after the prefix before them commits.
#include <hip/hip_runtime.h>

#include "orb_kernels.h"

namespace orbgpu {
namespace {

constexpr int kTop = 4;

struct Top4 {
    int idx[kTop];
    int dist[kTop];
    int lvl[kTop];
    int n;  // candidates that passed every filter (the window after the skips)
};

// Insert in (distance, window position) order: candidates arrive in window order, so a new one
// goes after every kept one of equal distance (strict <).  Fully unrolled so the four slots stay
// in registers.
__device__ inline void top_insert(Top4& t, int idx, int dist, int lvl) {
    ++t.n;
    bool shift = false;  // once placed, every later slot moves one down
#pragma unroll
    for (int j = 0; j < kTop; ++j) {
        shift = shift || dist < t.dist[j];
        if (shift) {
            const int ti = t.idx[j], td = t.dist[j], tl = t.lvl[j];
            t.idx[j] = idx, t.dist[j] = dist, t.lvl[j] = lvl;
            idx = ti, dist = td, lvl = tl;
        }
    }
}

struct FrameView {
    const float* xy;       // mvKeysUn positions [out_cap][2]
    const uint8_t* kp;     // out_kps rows (octave at +20)
    const int32_t* cs;     // cell_start [3073]
    const int32_t* ci;     // cell_idx
    const uint8_t* desc;   // [out_cap][32]
    const float* uright;   // mvuRight or nullptr
};

__device__ inline int octave_of(const FrameView& F, int k) {
    return *reinterpret_cast<const int32_t*>(F.kp + (long long)k * 28 + 20);
}

__device__ inline int hamming32(const uint32_t q[8], const uint8_t* d) {
    const uint4 a = *reinterpret_cast<const uint4*>(d);
    const uint4 b = *reinterpret_cast<const uint4*>(d + 16);
    return __popc(q[0] ^ a.x) + __popc(q[1] ^ a.y) + __popc(q[2] ^ a.z) + __popc(q[3] ^ a.w) +
           __popc(q[4] ^ b.x) + __popc(q[5] ^ b.y) + __popc(q[6] ^ b.z) + __popc(q[7] ^ b.w);
}

// Map-point prologue (:50-73): false when the point is skipped, else true with the window
// half-size r * mvScaleFactors[level] in *rs (also the mvuRight tolerance, :91-95).
__device__ inline bool mp_window(const SbpArgs& a, const MapPointIn& mp, float* rs) {
    if (!(mp.flags & kMpInView)) return false;
    if (a.far_points && mp.depth > a.th_far) return false;
    if (mp.flags & kMpBad) return false;
    if (mp.level < 0 || mp.level >= a.nlevels) return false;
    float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:216-222)
    if (a.factor) r *= a.th;
    *rs = r * a.scale[mp.level];
    return true;
}

// GetFeaturesInArea (Frame.cc:673-735) + the per-candidate filters and distances of
// :86-118, calling emit(idx, dist, octave) for each surviving candidate in window order.
template <class Blocked, class Emit>
__device__ inline void walk_window(const SbpArgs& a, const FrameView& F, const MapPointIn& mp, float rs,
                                   const uint32_t q[8], Blocked blocked, Emit emit) {
    const float x = mp.proj_x, y = mp.proj_y;
    const int minX = max(0, (int)floorf((x - a.bounds[0] - rs) * a.grid_inv[0]));
    if (minX >= kGridCols) return;
    const int maxX = min(kGridCols - 1, (int)ceilf((x - a.bounds[0] + rs) * a.grid_inv[0]));
    if (maxX < 0) return;
    const int minY = max(0, (int)floorf((y - a.bounds[2] - rs) * a.grid_inv[1]));
    if (minY >= kGridRows) return;
    const int maxY = min(kGridRows - 1, (int)ceilf((y - a.bounds[2] + rs) * a.grid_inv[1]));
    if (maxY < 0) return;
    const int minLevel = mp.level - 1, maxLevel = mp.level;
    const bool checkLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = minX; ix <= maxX; ++ix) {
        const int j1 = F.cs[ix * kGridRows + maxY + 1];
        for (int j = F.cs[ix * kGridRows + minY]; j < j1; ++j) {  // cells iy = minY..maxY are adjacent
            const int k = F.ci[j];
            const int oct = octave_of(F, k);
            if (checkLevels) {
                if (oct < minLevel) continue;
                if (maxLevel >= 0 && oct > maxLevel) continue;
            }
            const float2 p = *reinterpret_cast<const float2*>(F.xy + 2LL * k);
            if (!(fabsf(p.x - x) < rs && fabsf(p.y - y) < rs)) continue;
            if (blocked(k)) continue;
            if (F.uright) {
                const float ur = F.uright[k];
                if (ur > 0 && fabsf(mp.proj_xr - ur) > rs) continue;
            }
            emit(k, hamming32(q, F.desc + 32LL * k), oct);
        }
    }
}

__device__ inline FrameView frame_view(const SbpArgs& a, int f) {
    const int img = (a.img0 + f) * a.image_step;
    FrameView F;
    F.xy = a.xy_un + 2LL * img * a.out_cap;
    F.kp = static_cast<const uint8_t*>(a.kps) + 28LL * img * a.out_cap;
    F.cs = a.cell_start + (long long)img * (kGridCols * kGridRows + 1);
    F.ci = a.cell_idx + (long long)img * a.out_cap;
    F.desc = a.desc + 32LL * img * a.out_cap;
    F.uright = a.uright ? a.uright + (long long)(a.img0 + f) * a.out_cap : nullptr;
    return F;
}

__device__ inline void load_desc(const MapPointIn& mp, uint32_t q[8]) {
    for (int w = 0; w < 8; ++w)
        q[w] = (uint32_t)mp.desc[4 * w] | ((uint32_t)mp.desc[4 * w + 1] << 8) |
               ((uint32_t)mp.desc[4 * w + 2] << 16) | ((uint32_t)mp.desc[4 * w + 3] << 24);
}

__global__ __launch_bounds__(256) void k_sbp_candidates(SbpArgs a) {
    const int f = blockIdx.y;
    const int m0 = a.mp_off[a.img0 + f], m1 = a.mp_off[a.img0 + f + 1];
    const int i = m0 + blockIdx.x * 256 + threadIdx.x;
    if (i >= m1) return;
    const MapPointIn mp = a.mps[i];
    SbpCand& out = a.cand[i];
    out.flags = mp.flags;
    float rs;
    if (!mp_window(a, mp, &rs)) {
        out.n = -1;
        return;
    }
    const FrameView F = frame_view(a, f);
    const uint8_t* blk = a.kp_block ? a.kp_block + (long long)(a.img0 + f) * a.out_cap : nullptr;
    uint32_t q[8];
    load_desc(mp, q);
    Top4 t;
    t.n = 0;
    for (int j = 0; j < kTop; ++j) {
        t.idx[j] = -1;
        t.dist[j] = 256;
        t.lvl[j] = -1;
    }
    walk_window(a, F, mp, rs, q, [&](int k) { return blk && blk[k]; },
                [&](int k, int d, int o) { top_insert(t, k, d, o); });
    out.n = t.n;
    for (int j = 0; j < kTop; ++j) {
        out.idx[j] = t.idx[j];
        out.key[j] = t.dist[j] | ((t.lvl[j] & 0xFFFF) << 16);
    }
}

constexpr int kResolveChunk = 256;

// Dynamic LDS of k_sbp_resolve for out_cap keypoints: the occupancy bitmap, two per-keypoint
// lane tables and the staged candidate lists.
__host__ __device__ inline int sbp_lds_words(int out_cap) { return (out_cap + 31) / 32 + 2 * out_cap; }
__host__ __device__ inline size_t sbp_lds_bytes(int out_cap) {
    return 4 * (size_t)sbp_lds_words(out_cap) + sizeof(SbpCand) * kResolveChunk;
}

// One wave per frame.  The map points are replayed 64 at a time: every pending lane computes
// its result against the occupancy so far, then the longest prefix of lanes whose examined
// candidates no earlier lane of the group takes is committed at once (the reference order makes
// exactly those results final), and the rest retry against the updated occupancy.
__global__ __launch_bounds__(64) void k_sbp_resolve(SbpArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nbits = (a.out_cap + 31) / 32;
    uint32_t* taken = lds;                       // keypoint held by an occupant with observations
    uint32_t* owner = lds + nbits;               // lowest lane of the group taking the keypoint
    int32_t* writer = reinterpret_cast<int32_t*>(owner + a.out_cap);  // last lane assigning it
    SbpCand* chunk = reinterpret_cast<SbpCand*>(lds + sbp_lds_words(a.out_cap));
    const int f = blockIdx.x, lane = threadIdx.x;
    const int img = (a.img0 + f) * a.image_step;
    const int nkp = a.out_n[img];
    const int m0 = a.mp_off[a.img0 + f], m1 = a.mp_off[a.img0 + f + 1];
    int32_t* match = a.match + (long long)(a.img0 + f) * a.out_cap;
    const uint8_t* blk = a.kp_block ? a.kp_block + (long long)(a.img0 + f) * a.out_cap : nullptr;
    for (int w = lane; w < (nkp + 31) / 32; w += 64) {
        uint32_t bits = 0;
        if (blk)
            for (int b = 0; b < 32 && w * 32 + b < nkp; ++b) bits |= (blk[w * 32 + b] ? 1u : 0u) << b;
        taken[w] = bits;
    }
    for (int k = lane; k < nkp; k += 64) {
        match[k] = -1;
        owner[k] = 64;
        writer[k] = -1;
    }
    __syncthreads();
    const FrameView F = frame_view(a, f);
    auto is_taken = [&](int k) { return ((taken[k >> 5] >> (k & 31)) & 1u) != 0; };
    int nmatches = 0;
    for (int c0 = m0; c0 < m1; c0 += kResolveChunk) {
        const int cn = min(kResolveChunk, m1 - c0);
        for (int j = lane; j < cn; j += 64) chunk[j] = a.cand[c0 + j];
        __syncthreads();
        for (int g0 = 0; g0 < cn; g0 += 64) {
            const int j = g0 + lane;
            bool pending = j < cn;
            SbpCand c;
            if (pending) c = chunk[j];
            while (__ballot(pending)) {
                int asg = -1, nexam = 0;
                bool all = false, blocking = false;
                if (pending && c.n > 0) {
                    int bi = -1, bd = 256, bl = -1, sd = 256, sl = -1, found = 0;
#pragma unroll
                    for (int t = 0; t < kTop; ++t) {
                        const int k = c.idx[t];
                        if (found >= 2 || k < 0) break;
                        nexam = t + 1;
                        if (is_taken(k)) continue;
                        const int d = c.key[t] & 0xFFFF, l = (int16_t)(c.key[t] >> 16);
                        if (found == 0) {
                            bi = k, bd = d, bl = l;
                        } else {
                            sd = d, sl = l;
                        }
                        ++found;
                    }
                    if (found < 2 && c.n > kTop) {  // the top 4 ran dry: walk the window again
                        all = true;
                        const MapPointIn mp = a.mps[c0 + j];
                        float rs;
                        mp_window(a, mp, &rs);
                        uint32_t q[8];
                        load_desc(mp, q);
                        bi = -1, bd = 256, bl = -1, sd = 256, sl = -1;
                        walk_window(a, F, mp, rs, q, is_taken, [&](int k, int d, int o) {
                            if (d < bd) {
                                sd = bd, sl = bl;
                                bd = d, bl = o, bi = k;
                            } else if (d < sd) {
                                sd = d, sl = o;
                            }
                        });
                    }
                    // TH_HIGH and the ratio test (:124-140)
                    if (bd <= 100 && !(bl == sl && (float)bd > a.nnratio * (float)sd) &&
                        (bl != sl || (float)bd <= a.nnratio * (float)sd)) {
                        asg = bi;
                        blocking = (c.flags & kMpHasObs) != 0;
                    }
                }
                // a lane is stale if an earlier pending lane takes a candidate it examined (a
                // lane that walked its whole window: if any earlier lane takes anything)
                const bool takes = pending && asg >= 0 && blocking;
                const uint64_t tm = __ballot(takes);
                if (takes) atomicMin(&owner[asg], (uint32_t)lane);
                bool stale = false;
                if (pending) {
                    if (all) stale = (tm & ((1ull << lane) - 1)) != 0;
#pragma unroll
                    for (int t = 0; t < kTop; ++t)
                        if (t < nexam) stale |= owner[c.idx[t]] < (uint32_t)lane;
                }
                if (takes) owner[asg] = 64;
                const uint64_t st = __ballot(pending && stale);
                const int first = st ? __builtin_ctzll(st) : 64;
                const bool commit = pending && lane < first;
                // the reference keeps the last of several assignments to one keypoint
                const bool assigns = commit && asg >= 0;
                if (assigns) atomicMax(&writer[asg], lane);
                if (assigns && writer[asg] == lane) match[asg] = c0 + j - m0;
                if (assigns) writer[asg] = -1;
                if (assigns && blocking) atomicOr(&taken[asg >> 5], 1u << (asg & 31));
                nmatches += __popcll(__ballot(assigns));
                pending = pending && !commit;
            }
        }
        __syncthreads();
    }
    if (lane == 0) a.nmatches[a.img0 + f] = nmatches;
}

}  // namespace

hipError_t launch_sbp(const SbpArgs& a, int nframes, int max_mps, hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    if (max_mps > 0)
        hipLaunchKernelGGL(k_sbp_candidates, dim3((max_mps + 255) / 256, nframes), dim3(256), 0, st, a);
    const size_t lds = sbp_lds_bytes(a.out_cap);
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_sbp_resolve),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_sbp_resolve, dim3(nframes), dim3(64), lds, st, a);
    return hipGetLastError();
}

}  // namespace orbgpu
