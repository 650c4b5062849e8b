// Wire formats either side of the hot path.
//
// Ingest: the side-by-side stereo Y8 frame the reference receives from the headset (an
// AHardwareBuffer of 2W x H, ORBextractor.cc:131-143; the DSP copies the left half with row pitch
// 2W from column 0 and the right half from column W, orbslam_dsp.cpp:643-648) becomes batch
// images 2p (left) and 2p+1 (right) in the [image][row][col] layout the pyramid reads.
//
// Egress: the FastRPC result layout (orbslam3.idl:15-19): per eye int32 X, Y, angle, level
// arrays + N x 32 B descriptors, and int16 indices / distances1 / distances2 of the stereo kNN.
//   X, Y   (int) of the level-0 float coordinates (truncation, as the DSP's `int x = pos * scale`,
//          orbslam_dsp.cpp:447-453; coordinates are >= 0 so this is floor)
//   angle  (cos8 & 0xFF) | ((sin8 & 0xFF) << 8), cos8/sin8 = rint(64 * cos/sin of the keypoint
//          angle) with the same single-precision cos/sin the descriptor rotation uses
//          (ORBextractor_old.cc:114-115, libm cosf / sinf): the encoding the host decodes with
//          atan2(sin8 / 64, cos8 / 64) (LynxHardwareAccelerator.cpp:174-178)
//   level  octave
//   indices/distances: idx1 (-1 if absent), dist1, dist2 clamped to 32767 (absent = 32767)
// Both are pure HBM streaming kernels.
#include <hip/hip_runtime.h>

#include "orb_kernels.h"
#include "orb_math.h"

namespace orbgpu {

// One thread per 16 B chunk of a source row (aligned case) or per byte (general case).
template <bool kVec>
__global__ __launch_bounds__(256) void k_sbs_split(SbsArgs a) {
    const long long per_row = kVec ? (2LL * a.w) / 16 : 2LL * a.w;
    const long long total = per_row * a.h * a.nframes;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const long long row = t / per_row;
        const int col = (int)(t - row * per_row) * (kVec ? 16 : 1);
        const int f = (int)(row / a.h), r = (int)(row - (long long)f * a.h);
        const uint8_t* src = a.src + (long long)f * a.frame_bytes + (long long)r * a.stride + col;
        const int eye = col >= a.w;
        uint8_t* dst = a.dst + ((long long)(2 * f + eye) * a.h + r) * a.w + (col - eye * a.w);
        if constexpr (kVec) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
            *reinterpret_cast<u32x4*>(dst) = v;
        } else {
            *dst = *src;
        }
    }
}

hipError_t launch_sbs_split(const SbsArgs& a, hipStream_t st) {
    const bool vec = (a.w % 16) == 0 && (a.stride % 16) == 0 && (a.frame_bytes % 16) == 0 &&
                     ((uintptr_t)a.src % 16) == 0 && ((uintptr_t)a.dst % 16) == 0;
    const long long work = (vec ? (2LL * a.w) / 16 : 2LL * a.w) * a.h * a.nframes;
    // enough waves to cover every CU several times; the loop strides the rest
    const long long blocks = std::min<long long>((work + 255) / 256, 256LL * 32);
    if (blocks <= 0) return hipSuccess;
    if (vec)
        hipLaunchKernelGGL(k_sbs_split<true>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(k_sbs_split<false>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}

__device__ inline int16_t clamp16(int32_t d) { return (int16_t)(d > 32767 ? 32767 : d); }

// blockIdx.y < nimages: keypoints of image img0 + y -> SoA; otherwise matches of pair
// y - nimages -> int16.
__global__ __launch_bounds__(256) void k_pack_soa(SoaArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if ((int)blockIdx.y < a.nimages) {
        const int img = a.img0 + blockIdx.y;
        if (i >= a.out_n[img]) return;
        const long long o = (long long)img * a.out_cap + i;
        const float* kp = reinterpret_cast<const float*>(static_cast<const uint8_t*>(a.kps) + o * 28);
        const float x = kp[0], y = kp[1], ang = kp[3];
        const int oct = reinterpret_cast<const int32_t*>(kp)[5];
        // the descriptor rotation's cos/sin (ORBextractor_old.cc:114-115): angle * factorPI in
        // float, then the float overloads std::cos / std::sin (libm cosf / sinf)
        const float rad = ang * (float)(3.14159265358979323846 / 180.0);
        float sd, cd;
        libm_sincosf(rad, &sd, &cd);
        const int c8 = (int)rintf(64.0f * cd), s8 = (int)rintf(64.0f * sd);
        a.x[o] = (int32_t)x;
        a.y[o] = (int32_t)y;
        a.angle[o] = (c8 & 0xFF) | ((s8 & 0xFF) << 8);
        a.level[o] = oct;
    } else {
        const int pair = blockIdx.y - a.nimages;
        if (i >= a.nq[pair]) return;
        const long long o = (long long)pair * a.out_cap + i;
        a.idx16[o] = (int16_t)a.idx1[o];
        a.d1_16[o] = clamp16(a.dist1[o]);
        a.d2_16[o] = clamp16(a.dist2[o]);
    }
}

hipError_t launch_pack_soa(const SoaArgs& a, int npairs, hipStream_t st) {
    const unsigned gy = (unsigned)(a.nimages + npairs);
    if (gy == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_soa, dim3((a.out_cap + 255) / 256, gy), dim3(256), 0, st, a);
    return hipGetLastError();
}

// orbgpu_export_batch's packed layout (include/orbgpu.h), produced rows only.  blockIdx.y < nimages:
// image y's keypoints then descriptors (15 dwords per row); otherwise pair y - nimages's four match
// arrays (4 dwords per query row).  Each workgroup finds its unit's offset from the device counts
// (the host checked them: no status codes); workgroup (0, 0) also writes the header.
__global__ __launch_bounds__(256) void k_pack_export(ExportArgs a) {
    __shared__ long long s_off;
    const int y = blockIdx.y;
    const bool img = y < a.nimages;
    const int u = img ? y : y - a.nimages;
    if (threadIdx.x == 0) s_off = 0;
    __syncthreads();
    {   // offset in dwords past the header: 15 per row of every earlier image (all images before a
        // pair), 4 per query row of every earlier pair
        long long part = 0;
        const int nimg = img ? u : a.nimages;
        for (int i = threadIdx.x; i < nimg; i += 256) part += 15LL * a.out_n[i];
        if (!img)
            for (int p = threadIdx.x; p < u; p += 256) part += 4LL * a.nq[p];
        if (part) atomicAdd(reinterpret_cast<unsigned long long*>(&s_off), (unsigned long long)part);
    }
    __syncthreads();
    uint32_t* dst = reinterpret_cast<uint32_t*>(a.dst);
    const int hdr = 2 * a.nimages + a.npairs;
    if (blockIdx.x == 0 && y == 0)
        for (int i = threadIdx.x; i < hdr; i += 256)
            dst[i] = (uint32_t)(i < a.nimages ? a.out_n[i] : i < 2 * a.nimages ? a.out_mono[i - a.nimages]
                                                                                 : a.nq[i - 2 * a.nimages]);
    uint32_t* out = dst + hdr + s_off;
    const long long stride = (long long)gridDim.x * 256;
    if (img) {
        const long long n = a.out_n[u];
        const uint32_t* kp = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(a.kps) + (long long)u * a.out_cap * 28);
        const uint32_t* de = reinterpret_cast<const uint32_t*>(a.desc + (long long)u * a.out_cap * 32);
        for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < 15 * n; t += stride)
            out[t] = t < 7 * n ? kp[t] : de[t - 7 * n];
    } else {
        const long long n = a.nq[u], o = (long long)u * a.out_cap;
        for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < 4 * n; t += stride) {
            const long long k = t / n, r = t - k * n;
            const int32_t* s = k == 0 ? a.idx1 : k == 1 ? a.dist1 : k == 2 ? a.idx2 : a.dist2;
            out[t] = (uint32_t)s[o + r];
        }
    }
}

hipError_t launch_pack_export(const ExportArgs& a, hipStream_t st) {
    const unsigned gy = (unsigned)(a.nimages + a.npairs);
    if (gy == 0) return hipSuccess;
    // enough workgroups per unit for the largest image's 15 dwords per row
    const unsigned gx = (unsigned)std::max(1, std::min(64, (15 * a.out_cap + 1023) / 1024));
    hipLaunchKernelGGL(k_pack_export, dim3(gx, gy), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace orbgpu
