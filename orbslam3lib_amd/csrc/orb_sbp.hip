// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
// (cpp/src/ORBmatcher.cc:44-214) over frames whose keypoints, descriptors, grids
// (Frame::GetFeaturesInArea, Frame.cc:673-735) and mvuRight already live in HBM:
//   pinhole frames (Nleft == -1)   one image per frame, mvKeysUn + mvuRight test (:91-95)
//   two-camera frames (Nleft != -1) the left image's window (:63-139, no mvuRight test) and the
//                                  right image's window (:141-207), each assignment copied to the
//                                  stereo partner (mvLeftToRightMatch / mvRightToLeftMatch)
//
// The reference loop is sequential: a keypoint taken by an earlier map point (Observations() > 0)
// is skipped by every later one.  Two kernels keep the result identical:
//   k_sbp_candidates  one thread per map point walks its window(s) with the pre-call occupancy
//                     and keeps the 4 lowest (distance, window position) candidates + their
//                     count.  The reference's (best, second) pair is exactly the two lowest of
//                     that order (strict `<` keeps the earlier of equal distances), so removing a
//                     candidate outside the two lowest changes nothing.
//   k_sbp_resolve     one wave per frame replays the map points in order, 64 lanes at a time:
//                     each lane takes the first two candidates not taken so far from its lists
//                     (re-walking a window with the live occupancy when fewer than two survive
//                     out of more than four), then the prefix of lanes that no earlier lane of
//                     the group disturbs commits at once (see k_sbp_resolve).
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

__device__ inline void top_init(Top4& t) {
    t.n = 0;
#pragma unroll
    for (int j = 0; j < kTop; ++j) {
        t.idx[j] = -1;
        t.dist[j] = 256;
        t.lvl[j] = -1;
    }
}

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
    const float* xy;       // keypoint positions [out_cap][2] (mvKeysUn, or mvKeys / mvKeysRight)
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

// Map-point prologue shared by both windows (:50-61).
__device__ inline bool mp_live(const SbpArgs& a, const MapPointIn& mp) {
    const int views = a.two_cam ? (kMpInView | kMpInViewR) : kMpInView;
    if (!(mp.flags & views)) return false;
    if (a.far_points && mp.depth > a.th_far) return false;
    return !(mp.flags & kMpBad);
}

// The left (or only) window (:63-73): false when not searched, else its half-size
// r * mvScaleFactors[level] in *rs (also the mvuRight tolerance, :91-95).
__device__ inline bool mp_window(const SbpArgs& a, const MapPointIn& mp, float* rs) {
    if (!(mp.flags & kMpInView)) return false;
    if (mp.level < 0 || mp.level >= a.nlevels) return false;
    float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:216-222)
    if (a.factor) r *= a.th;
    *rs = r * a.scale[mp.level];
    return true;
}

// The right-camera window (:141-152): no th factor.
__device__ inline bool mp_window_r(const SbpArgs& a, const MapPointIn& mp, float* rs) {
    if (!a.two_cam || !(mp.flags & kMpInViewR)) return false;
    if (mp.level_r < 0 || mp.level_r >= a.nlevels) return false;
    const float r = (double)mp.view_cos_r > 0.998 ? 2.5f : 4.0f;
    *rs = r * a.scale[mp.level_r];
    return true;
}

// GetFeaturesInArea (Frame.cc:673-735) + the per-candidate filters and distances of
// :86-118 / :164-187, calling emit(idx, dist, octave) for each surviving candidate in window order.
template <class Blocked, class Emit>
__device__ inline void walk_window(const SbpArgs& a, const FrameView& F, float x, float y, int level, float rs,
                                   float proj_xr, const uint32_t q[8], Blocked blocked, Emit emit) {
    const int minX = max(0, (int)floorf((x - a.bounds[0] - rs) * a.grid_inv[0]));
    if (minX >= kGridCols) return;
    const int maxX = min(kGridCols - 1, (int)ceilf((x - a.bounds[0] + rs) * a.grid_inv[0]));
    if (maxX < 0) return;
    const int minY = max(0, (int)floorf((y - a.bounds[2] - rs) * a.grid_inv[1]));
    if (minY >= kGridRows) return;
    const int maxY = min(kGridRows - 1, (int)ceilf((y - a.bounds[2] + rs) * a.grid_inv[1]));
    if (maxY < 0) return;
    const int minLevel = level - 1, maxLevel = level;
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
                if (ur > 0 && fabsf(proj_xr - ur) > rs) continue;
            }
            emit(k, hamming32(q, F.desc + 32LL * k), oct);
        }
    }
}

__device__ inline FrameView frame_view(const SbpArgs& a, int f, int eye) {
    const int img = (a.img0 + f) * a.image_step + eye;
    FrameView F;
    F.xy = a.xy_un + 2LL * img * a.out_cap;
    F.kp = static_cast<const uint8_t*>(a.kps) + 28LL * img * a.out_cap;
    F.cs = a.cell_start + (long long)img * (kGridCols * kGridRows + 1);
    F.ci = a.cell_idx + (long long)img * a.out_cap;
    F.desc = a.desc + 32LL * img * a.out_cap;
    F.uright = a.uright && !a.two_cam ? a.uright + (long long)(a.img0 + f) * a.out_cap : nullptr;
    return F;
}

__device__ inline void load_desc(const MapPointIn& mp, uint32_t q[8]) {
    for (int w = 0; w < 8; ++w)
        q[w] = (uint32_t)mp.desc[4 * w] | ((uint32_t)mp.desc[4 * w + 1] << 8) |
               ((uint32_t)mp.desc[4 * w + 2] << 16) | ((uint32_t)mp.desc[4 * w + 3] << 24);
}

__device__ inline void top_store(const Top4& t, int32_t idx[kTop], int32_t key[kTop]) {
#pragma unroll
    for (int j = 0; j < kTop; ++j) {
        idx[j] = t.idx[j];
        key[j] = t.dist[j] | ((t.lvl[j] & 0xFFFF) << 16);
    }
}

__global__ __launch_bounds__(256) void k_sbp_candidates(SbpArgs a) {
    const int f = blockIdx.y;
    const int m0 = a.mp_off[a.img0 + f], m1 = a.mp_off[a.img0 + f + 1];
    const int i = m0 + blockIdx.x * 256 + threadIdx.x;
    if (i >= m1) return;
    const MapPointIn mp = a.mps[i];
    SbpCand& out = a.cand[i];
    out.flags = mp.flags;
    out.n = -1;
    out.nR = -1;
    if (!mp_live(a, mp)) return;
    const int ncomb = a.two_cam ? 2 * a.out_cap : a.out_cap;
    const uint8_t* blk = a.kp_block ? a.kp_block + (long long)(a.img0 + f) * ncomb : nullptr;
    const int nl = a.out_n[(a.img0 + f) * a.image_step];
    uint32_t q[8];
    load_desc(mp, q);
    float rs;
    if (mp_window(a, mp, &rs)) {
        const FrameView F = frame_view(a, f, 0);
        Top4 t;
        top_init(t);
        walk_window(a, F, mp.proj_x, mp.proj_y, mp.level, rs, mp.proj_xr, q,
                    [&](int k) { return blk && blk[k]; }, [&](int k, int d, int o) { top_insert(t, k, d, o); });
        out.n = t.n;
        top_store(t, out.idx, out.key);
    }
    if (mp_window_r(a, mp, &rs)) {
        const FrameView F = frame_view(a, f, 1);
        Top4 t;
        top_init(t);
        walk_window(a, F, mp.proj_xr, mp.proj_yr, mp.level_r, rs, 0.f, q,
                    [&](int k) { return blk && blk[nl + k]; }, [&](int k, int d, int o) { top_insert(t, k, d, o); });
        out.nR = t.n;
        top_store(t, out.idxR, out.keyR);
    }
}

constexpr int kResolveChunk = 128;

// Dynamic LDS of k_sbp_resolve for n keypoints per frame: the occupancy bitmap, two
// per-keypoint lane tables and the staged candidate lists.
__host__ __device__ inline int sbp_lds_words(int n) { return (n + 31) / 32 + 2 * n; }
__host__ __device__ inline size_t sbp_lds_bytes(int n) {
    return 4 * (size_t)sbp_lds_words(n) + sizeof(SbpCand) * kResolveChunk;
}

// Best / second from a top-4 list, skipping taken keypoints; nexam = entries looked at.
template <class Taken>
__device__ inline int top_pick(const int32_t idx[kTop], const int32_t key[kTop], Taken taken, int& bi, int& bd,
                               int& bl, int& sd, int& sl, int& nexam) {
    int found = 0;
    bi = -1, bd = 256, bl = -1, sd = 256, sl = -1, nexam = 0;
#pragma unroll
    for (int t = 0; t < kTop; ++t) {
        const int k = idx[t];
        if (found >= 2 || k < 0) break;
        nexam = t + 1;
        if (taken(k)) continue;
        const int d = key[t] & 0xFFFF, l = (int16_t)(key[t] >> 16);
        if (found == 0) {
            bi = k, bd = d, bl = l;
        } else {
            sd = d, sl = l;
        }
        ++found;
    }
    return found;
}

// One wave per frame.  The map points are replayed 64 at a time.  Every pending lane computes
// its assignments (up to 4: best and stereo partner per window) against the occupancy so far;
// every assigned keypoint records its lowest assigning lane (owner table).  A lane is stale if an
// earlier pending lane assigns a candidate it examined, anything at all when it walked a whole
// window, or frees a keypoint that was occupied before the call (those are missing from every
// candidate list: the rest of the frame then walks whole windows).  The prefix before the first
// stale lane commits at once -- the last assignment of a keypoint decides its match and
// occupancy, as the reference overwrites -- and the other lanes recompute.
__global__ __launch_bounds__(64) void k_sbp_resolve(SbpArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int ncap = a.two_cam ? 2 * a.out_cap : a.out_cap;
    const int nbits = (ncap + 31) / 32;
    uint32_t* taken = lds;                       // keypoint held by an occupant with observations
    uint32_t* owner = lds + nbits;               // lowest lane of the group assigning the keypoint
    int32_t* writer = reinterpret_cast<int32_t*>(owner + ncap);  // last lane assigning it
    SbpCand* chunk = reinterpret_cast<SbpCand*>(lds + sbp_lds_words(ncap));
    const int f = blockIdx.x, lane = threadIdx.x;
    const int img = (a.img0 + f) * a.image_step;
    const int nl = a.out_n[img];
    const int nr = a.two_cam ? a.out_n[img + 1] : 0;
    const int ncomb = nl + nr;
    const int m0 = a.mp_off[a.img0 + f], m1 = a.mp_off[a.img0 + f + 1];
    int32_t* match = a.match + (long long)(a.img0 + f) * ncap;
    const uint8_t* blk = a.kp_block ? a.kp_block + (long long)(a.img0 + f) * ncap : nullptr;
    const int32_t* l2r = a.two_cam && a.l2r ? a.l2r + (long long)(a.img0 + f) * a.out_cap : nullptr;
    const int32_t* r2l = a.two_cam && a.r2l ? a.r2l + (long long)(a.img0 + f) * a.out_cap : nullptr;
    for (int w = lane; w < (ncomb + 31) / 32; w += 64) {
        uint32_t bits = 0;
        if (blk)
            for (int b = 0; b < 32 && w * 32 + b < ncomb; ++b) bits |= (blk[w * 32 + b] ? 1u : 0u) << b;
        taken[w] = bits;
    }
    for (int k = lane; k < ncomb; k += 64) {
        match[k] = -1;
        owner[k] = 64;
        writer[k] = -1;
    }
    __syncthreads();
    const FrameView FL = frame_view(a, f, 0);
    const FrameView FR = frame_view(a, f, a.two_cam ? 1 : 0);
    auto is_taken = [&](int k) { return ((taken[k >> 5] >> (k & 31)) & 1u) != 0; };
    auto init_blocked = [&](int k) { return blk && blk[k]; };
    bool walk_all = false;  // a keypoint occupied before the call was freed: lists are incomplete
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
                // this lane's assignments, in the reference's order
                int ak0 = -1, ak1 = -1, ak2 = -1, ak3 = -1, na = 0;
                auto add = [&](int k) {
                    if (na == 0) ak0 = k;
                    else if (na == 1) ak1 = k;
                    else if (na == 2) ak2 = k;
                    else ak3 = k;
                    ++na;
                };
                bool walked = false, frees = false;
                int nexL = 0, nexR = 0;
                const bool obs = pending && (c.flags & kMpHasObs) != 0;
                if (pending && (c.n >= 0 || c.nR >= 0)) {
                    const MapPointIn* mpp = a.mps + c0 + j;
                    bool stop = false;  // the left ratio test's `continue` skips the right window
                    if (c.n >= 0) {
                        int bi, bd, bl, sd, sl;
                        const int found = top_pick(c.idx, c.key, is_taken, bi, bd, bl, sd, sl, nexL);
                        if (walk_all || (found < 2 && c.n > kTop)) {
                            walked = true;
                            const MapPointIn mp = *mpp;
                            float rs;
                            mp_window(a, mp, &rs);
                            uint32_t q[8];
                            load_desc(mp, q);
                            bi = -1, bd = 256, bl = -1, sd = 256, sl = -1;
                            walk_window(a, FL, mp.proj_x, mp.proj_y, mp.level, rs, mp.proj_xr, q, is_taken,
                                        [&](int k, int d, int o) {
                                            if (d < bd) {
                                                sd = bd, sl = bl;
                                                bd = d, bl = o, bi = k;
                                            } else if (d < sd) {
                                                sd = d, sl = o;
                                            }
                                        });
                        }
                        if (bd <= 100) {  // TH_HIGH and the ratio test (:124-140)
                            if (bl == sl && (float)bd > a.nnratio * (float)sd) {
                                stop = true;
                            } else if (bl != sl || (float)bd <= a.nnratio * (float)sd) {
                                add(bi);
                                if (l2r && l2r[bi] != -1) {
                                    const int pk = nl + l2r[bi];
                                    if (!obs && init_blocked(pk)) frees = true;
                                    add(pk);
                                }
                            }
                        }
                    }
                    if (!stop && c.nR >= 0) {
                        // the right window sees this lane's own left assignments
                        auto takenR = [&](int k) {
                            const int kc = nl + k;
                            if (na > 1 && ak1 == kc) return obs;
                            return is_taken(kc);
                        };
                        int bi, bd, bl, sd, sl;
                        const int found = top_pick(c.idxR, c.keyR, takenR, bi, bd, bl, sd, sl, nexR);
                        if (walk_all || frees || (found < 2 && c.nR > kTop)) {
                            walked = true;
                            const MapPointIn mp = *mpp;
                            float rs;
                            mp_window_r(a, mp, &rs);
                            uint32_t q[8];
                            load_desc(mp, q);
                            bi = -1, bd = 256, bl = -1, sd = 256, sl = -1;
                            walk_window(a, FR, mp.proj_xr, mp.proj_yr, mp.level_r, rs, 0.f, q, takenR,
                                        [&](int k, int d, int o) {
                                            if (d < bd) {
                                                sd = bd, sl = bl;
                                                bd = d, bl = o, bi = k;
                                            } else if (d < sd) {
                                                sd = d, sl = o;
                                            }
                                        });
                        }
                        if (bd <= 100 && !(bl == sl && (float)bd > a.nnratio * (float)sd)) {  // :189-207
                            if (r2l && r2l[bi] != -1) {
                                const int pk = r2l[bi];
                                if (!obs && init_blocked(pk)) frees = true;
                                add(pk);
                            }
                            add(nl + bi);
                        }
                    }
                }
                // staleness against the earlier pending lanes of the group
                // (pinhole frames: an assignment by a point without observations leaves the
                // keypoint free, so only the blocking ones can disturb a later lane)
                const bool reg = pending && na > 0 && (a.two_cam || obs);
                const uint64_t below = (1ull << lane) - 1;
                const uint64_t am = __ballot(reg);
                const uint64_t fm = __ballot(pending && frees);
                if (reg) {
                    if (na > 0) atomicMin(&owner[ak0], (uint32_t)lane);
                    if (na > 1) atomicMin(&owner[ak1], (uint32_t)lane);
                    if (na > 2) atomicMin(&owner[ak2], (uint32_t)lane);
                    if (na > 3) atomicMin(&owner[ak3], (uint32_t)lane);
                }
                bool stale = false;
                if (pending) {
                    stale = (fm & below) != 0 || (walked && (am & below) != 0);
#pragma unroll
                    for (int t = 0; t < kTop; ++t) {
                        if (t < nexL) stale |= owner[c.idx[t]] < (uint32_t)lane;
                        if (t < nexR) stale |= owner[nl + c.idxR[t]] < (uint32_t)lane;
                    }
                }
                if (reg) {
                    if (na > 0) owner[ak0] = 64;
                    if (na > 1) owner[ak1] = 64;
                    if (na > 2) owner[ak2] = 64;
                    if (na > 3) owner[ak3] = 64;
                }
                const uint64_t st = __ballot(pending && stale);
                const int first = st ? __builtin_ctzll(st) : 64;
                const bool commit = pending && lane < first;
                // the reference keeps the last assignment of a keypoint (its match and occupancy)
                const int val = c0 + j - m0;
                auto last = [&](int k) { return writer[k] == lane; };
                auto apply = [&](int k) {
                    match[k] = val;
                    if (obs) atomicOr(&taken[k >> 5], 1u << (k & 31));
                    else atomicAnd(&taken[k >> 5], ~(1u << (k & 31)));
                };
                if (commit) {
                    if (na > 0) atomicMax(&writer[ak0], lane);
                    if (na > 1) atomicMax(&writer[ak1], lane);
                    if (na > 2) atomicMax(&writer[ak2], lane);
                    if (na > 3) atomicMax(&writer[ak3], lane);
                }
                const bool w0 = commit && na > 0 && last(ak0), w1 = commit && na > 1 && last(ak1);
                const bool w2 = commit && na > 2 && last(ak2), w3 = commit && na > 3 && last(ak3);
                if (commit) {
                    if (na > 0) writer[ak0] = -1;
                    if (na > 1) writer[ak1] = -1;
                    if (na > 2) writer[ak2] = -1;
                    if (na > 3) writer[ak3] = -1;
                }
                if (w0) apply(ak0);
                if (w1) apply(ak1);
                if (w2) apply(ak2);
                if (w3) apply(ak3);
                int cnt = commit ? na : 0;
                for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
                nmatches += cnt;
                walk_all = walk_all || (__ballot(commit && frees) != 0);
                pending = pending && !commit;
            }
        }
        __syncthreads();
    }
    if (lane == 0) a.nmatches[a.img0 + f] = nmatches;
}

}  // namespace

size_t sbp_resolve_lds_bytes(int out_cap, int two_cam) { return sbp_lds_bytes(two_cam ? 2 * out_cap : out_cap); }

hipError_t launch_sbp(const SbpArgs& a, int nframes, int max_mps, hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    if (max_mps > 0)
        hipLaunchKernelGGL(k_sbp_candidates, dim3((max_mps + 255) / 256, nframes), dim3(256), 0, st, a);
    const size_t lds = sbp_resolve_lds_bytes(a.out_cap, a.two_cam);
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_sbp_resolve),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_sbp_resolve, dim3(nframes), dim3(64), lds, st, a);
    return hipGetLastError();
}

}  // namespace orbgpu
