// orb_stereo.hip -- Frame::ComputeStereoMatches (cpp/src/Frame.cc:827-997) on gfx950, over the
// device-resident results of a batch: pair p = left image 2p, right image 2p+1 (rectified
// pinhole stereo).  Integer/byte work (Hamming + 8-bit SAD), no MFMA.
//
//   k_stereo_rows    one workgroup per pair: counting sort of the right keypoints by row
//                    (floor y) -> CSR table in HBM (vRowIndices, :842-855, without the 2r band:
//                    the band test is applied per candidate)
//   k_stereo_match   one lane per left keypoint: band rows of the table, octave / disparity
//                    gates, Hamming best (TH_HIGH), then the 11x11 SAD over +-5 px on the left
//                    keypoint's unblurred level, parabola fit, disparity -> depth (:861-981)
//   k_stereo_median  one workgroup per pair: median of the accepted SAD distances (radix
//                    select), rejection of distances >= 1.5 * 1.4 * median (:984-996)
//
// Every float expression follows the reference's operation order; the file is compiled with
// -ffp-contract=off like the rest of the library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_kernels.h"

namespace orbgpu {

namespace {

struct Kp {  // orbgpu_keypoint / cv::KeyPoint (28 B)
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

constexpr int kThHigh = 100, kThLow = 50;  // ORBmatcher.cc:36-37
constexpr int kThOrbDist = (kThHigh + kThLow) / 2;
constexpr int kW = 5, kL = 5;              // SAD half window, search half range (Frame.cc:901,905)

__device__ inline const Kp* pair_kps(const StereoArgs& s, int img) {
    return reinterpret_cast<const Kp*>(s.kps) + (long long)img * s.out_cap;
}

// Dword-aligned loads of `n` dwords from byte address p & ~3, realigned to p: out[i] holds bytes
// p + 4i .. p + 4i + 3.  The extra bytes past a row end are inside the plane padding / the +256
// slack of every plane allocation.
template <int N>
__device__ inline void load_bytes(const uint8_t* p, uint32_t (&out)[N]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t w[N + 1];
#pragma unroll
    for (int i = 0; i <= N; ++i) w[i] = q[i];
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stereo_rows(StereoArgs s) {
    extern __shared__ int32_t cnt[];  // [H0 + 1]
    const int p = s.pair0 + blockIdx.x;
    const int H = s.H0;
    const int nR = s.out_n[2 * p + 1];
    const Kp* kr = pair_kps(s, 2 * p + 1);
    int32_t* start = s.row_start + (long long)p * (H + 1);
    int32_t* idx = s.row_idx + (long long)p * s.out_cap;
    for (int r = threadIdx.x; r <= H; r += 256) cnt[r] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nR; i += 256) {
        const int row = min(max((int)floorf(kr[i].y), 0), H - 1);
        atomicAdd(&cnt[row], 1);
    }
    __syncthreads();
    // exclusive scan over H rows: each thread a contiguous chunk, then a scan of the chunk sums
    __shared__ int32_t part[256];
    const int per = (H + 255) / 256;
    const int r0 = threadIdx.x * per, r1 = min(r0 + per, H);
    int sum = 0;
    for (int r = r0; r < r1; ++r) sum += cnt[r];
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int t = 0; t < 256; ++t) {
            const int v = part[t];
            part[t] = run;
            run += v;
        }
    }
    __syncthreads();
    int run = part[threadIdx.x];
    for (int r = r0; r < r1; ++r) {
        const int v = cnt[r];
        cnt[r] = run;  // becomes the scatter cursor
        start[r] = run;
        run += v;
    }
    if (threadIdx.x == 0) start[H] = nR;
    __syncthreads();
    for (int i = threadIdx.x; i < nR; i += 256) {
        const int row = min(max((int)floorf(kr[i].y), 0), H - 1);
        idx[atomicAdd(&cnt[row], 1)] = i;  // order inside a row is free: ties break on the index
    }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_stereo_match(StereoArgs s) {
    const int p = s.pair0 + blockIdx.y;
    const int iL = blockIdx.x * 64 + threadIdx.x;
    const int nL = s.out_n[2 * p];
    if (iL >= nL) return;
    float* uR_out = s.u_right + (long long)p * s.out_cap;
    float* dp_out = s.depth + (long long)p * s.out_cap;
    int32_t* sad_out = s.sad + (long long)p * s.out_cap;
    uR_out[iL] = -1.0f;
    dp_out[iL] = -1.0f;
    sad_out[iL] = -1;
    const Kp* kl = pair_kps(s, 2 * p);
    const Kp* kr = pair_kps(s, 2 * p + 1);
    const Kp kpL = kl[iL];
    const int H = s.H0;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int rowL = (int)vL;  // vRowIndices[vL]: float -> size_t
    if (rowL < 0 || rowL >= H) return;
    const float minZ = s.mb;
    const float minD = 0;
    const float maxD = s.mbf / minZ;
    const float minU = uL - maxD;
    const float maxU = uL - minD;
    if (maxU < 0) return;
    // band rows: a right keypoint of octave o lists rows floor(y - r) .. ceil(y + r), r = 2 s_o,
    // and only octaves levelL-1 .. levelL+1 can match, so its row floor(y) is within
    // ceil(rmax) + 1 of rowL
    const int omax = min(levelL + 1, s.nlevels - 1);
    const int band = (int)ceilf(2.0f * s.scale[omax]) + 1;
    const int ra = max(rowL - band, 0), rb = min(rowL + band, H - 1);
    const int32_t* start = s.row_start + (long long)p * (H + 1);
    const int32_t* idx = s.row_idx + (long long)p * s.out_cap;
    const uint4* dl4 = reinterpret_cast<const uint4*>(s.desc + ((long long)(2 * p) * s.out_cap + iL) * 32);
    const uint4 da = dl4[0], db = dl4[1];
    int bestDist = kThHigh, bestIdxR = 0x7fffffff;
    for (int j = start[ra], je = start[rb + 1]; j < je; ++j) {
        const int iR = idx[j];
        const Kp& kpR = kr[iR];
        const int octR = kpR.octave;
        if (octR < levelL - 1 || octR > levelL + 1) continue;
        const float kpY = kpR.y;
        const float r = 2.0f * s.scale[octR];
        const int maxr = (int)ceilf(kpY + r);
        const int minr = (int)floorf(kpY - r);
        if (rowL < minr || rowL > maxr) continue;  // not in vRowIndices[rowL]
        const float uR = kpR.x;
        if (uR >= minU && uR <= maxU) {
            const uint4* dr4 = reinterpret_cast<const uint4*>(s.desc + ((long long)(2 * p + 1) * s.out_cap + iR) * 32);
            const uint4 ea = dr4[0], eb = dr4[1];
            const int dist = __popc(da.x ^ ea.x) + __popc(da.y ^ ea.y) + __popc(da.z ^ ea.z) + __popc(da.w ^ ea.w) +
                             __popc(db.x ^ eb.x) + __popc(db.y ^ eb.y) + __popc(db.z ^ eb.z) + __popc(db.w ^ eb.w);
            // the reference scans vRowIndices[rowL] in ascending iR with a strict '<': the
            // lowest index wins among equal distances
            if (dist < bestDist || (dist == bestDist && dist < kThHigh && iR < bestIdxR)) {
                bestDist = dist;
                bestIdxR = iR;
            }
        }
    }
    if (!(bestDist < kThOrbDist)) return;
    // Subpixel match by correlation (:895-981)
    const float uR0 = kr[bestIdxR].x;
    const float scaleFactor = s.inv_scale[levelL];
    const float scaleduL = roundf(kpL.x * scaleFactor);
    const float scaledvL = roundf(kpL.y * scaleFactor);
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const float iniu = scaleduR0 + kL - kW;
    const float endu = scaleduR0 + kL + kW + 1;
    const int W = s.lw[levelL], Hl = s.lh[levelL], pitch = s.lpitch[levelL];
    if (iniu < 0 || endu >= W) return;
    const int r0 = (int)scaledvL - kW, c0 = (int)scaleduL - kW, cr = (int)scaleduR0 - kL - kW;
    if (r0 < 0 || r0 + 2 * kW + 1 > Hl || c0 < 0 || c0 + 2 * kW + 1 > W || cr < 0) return;
    const uint8_t* IL = s.lvl_base[levelL] + (long long)(2 * p) * s.limg_stride[levelL] + (long long)r0 * pitch + c0;
    const uint8_t* IR = s.lvl_base[levelL] + (long long)(2 * p + 1) * s.limg_stride[levelL] + (long long)r0 * pitch + cr;
    // dist[k] for incR = k - 5: SAD of the 11x11 left patch and the right window shifted by k
    uint32_t acc[2 * kL + 1];
#pragma unroll
    for (int k = 0; k < 2 * kL + 1; ++k) acc[k] = 0;
    for (int y = 0; y < 2 * kW + 1; ++y) {
        uint32_t a[3], b[6];
        load_bytes<3>(IL + (long long)y * pitch, a);
        load_bytes<6>(IR + (long long)y * pitch, b);
        a[2] &= 0x00ffffffu;  // 11 bytes
#pragma unroll
        for (int k = 0; k < 2 * kL + 1; ++k) {
            const uint32_t b0 = __builtin_amdgcn_alignbyte(b[(k >> 2) + 1], b[k >> 2], k & 3);
            const uint32_t b1 = __builtin_amdgcn_alignbyte(b[(k >> 2) + 2], b[(k >> 2) + 1], k & 3);
            const uint32_t b2 = __builtin_amdgcn_alignbyte(b[(k >> 2) + 3], b[(k >> 2) + 2], k & 3) & 0x00ffffffu;
            acc[k] = __builtin_amdgcn_sad_u8(a[0], b0, acc[k]);
            acc[k] = __builtin_amdgcn_sad_u8(a[1], b1, acc[k]);
            acc[k] = __builtin_amdgcn_sad_u8(a[2], b2, acc[k]);
        }
    }
    int sadBest = 0x7fffffff;
    int bestincR = 0;
    float vDists[2 * kL + 1];
#pragma unroll
    for (int k = 0; k < 2 * kL + 1; ++k) {
        const float dist = (float)acc[k];  // cv::norm(IL, IR, NORM_L1): exact
        if (dist < (float)sadBest) {
            sadBest = (int)dist;
            bestincR = k - kL;
        }
        vDists[k] = dist;
    }
    if (bestincR == -kL || bestincR == kL) return;
    float dist1 = 0, dist2 = 0, dist3 = 0;
#pragma unroll
    for (int k = 1; k < 2 * kL; ++k)
        if (k == kL + bestincR) dist1 = vDists[k - 1], dist2 = vDists[k], dist3 = vDists[k + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) return;
    float bestuR = s.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = (uL - bestuR);
    if (disparity >= minD && disparity < maxD) {
        if (disparity <= 0) {
            disparity = 0.01;
            bestuR = uL - 0.01;  // double arithmetic, as in the reference
        }
        dp_out[iL] = s.mbf / disparity;
        uR_out[iL] = bestuR;
        sad_out[iL] = sadBest;
    }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stereo_median(StereoArgs s) {
    __shared__ int32_t hist[256];
    __shared__ int32_t sel[2];
    const int p = s.pair0 + blockIdx.x;
    const int nL = s.out_n[2 * p];
    float* uR_out = s.u_right + (long long)p * s.out_cap;
    float* dp_out = s.depth + (long long)p * s.out_cap;
    const int32_t* sad = s.sad + (long long)p * s.out_cap;
    // k-th smallest accepted distance, k = count / 2 (vDistIdx sorted, [size/2].first);
    // distances <= 121 * 255 < 2^15: two radix passes of 8 and 7 bits
    hist[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nL; i += 256)
        if (sad[i] >= 0) atomicAdd(&hist[sad[i] >> 7], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int count = 0;
        for (int b = 0; b < 256; ++b) count += hist[b];
        int k = count / 2, b = 0;
        while (b < 256 && k >= hist[b]) k -= hist[b++];
        sel[0] = count > 0 ? b : -1;
        sel[1] = k;
    }
    __syncthreads();
    const int hb = sel[0];
    if (hb < 0) return;  // no accepted match (the reference indexes an empty vector here)
    const int kk = sel[1];
    __syncthreads();
    if (threadIdx.x < 128) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nL; i += 256)
        if (sad[i] >= 0 && (sad[i] >> 7) == hb) atomicAdd(&hist[sad[i] & 127], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int k = kk, b = 0;
        while (b < 127 && k >= hist[b]) k -= hist[b++];
        sel[0] = (hb << 7) | b;
    }
    __syncthreads();
    const float median = (float)sel[0];
    const float thDist = 1.5f * 1.4f * median;
    for (int i = threadIdx.x; i < nL; i += 256) {
        if (sad[i] >= 0 && !((float)sad[i] < thDist)) {
            uR_out[i] = -1;
            dp_out[i] = -1;
        }
    }
}

hipError_t launch_stereo(const StereoArgs& s, int npairs, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    const size_t smem = sizeof(int32_t) * (size_t)(s.H0 + 1);
    if (smem > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_stereo_rows),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_stereo_rows, dim3(npairs), dim3(256), smem, st, s);
    hipLaunchKernelGGL(k_stereo_match, dim3((s.out_cap + 63) / 64, npairs), dim3(64), 0, st, s);
    hipLaunchKernelGGL(k_stereo_median, dim3(npairs), dim3(256), 0, st, s);
    return hipGetLastError();
}

}  // namespace orbgpu
