// orb_fisheye.hip -- Frame::ComputeStereoFishEyeMatches (cpp/src/Frame.cc:1142-1201) on gfx950,
// over the device-resident results of a batch: pair p = left image 2p, right image 2p+1, each
// left stereo row with its best right stereo row from the kNN2 of the same batch (BFMatchORB,
// :1164, orbgpu_match_stereo_batch with stereo_only = 1).
//
//   k_fisheye_stereo   one lane per left keypoint (rows [0, monoLeft) only reset their outputs):
//                      dist1 == 0 skip (:1171-1175), dist1 < 70 (:1177), the index checks
//                      (:1183-1189), KannalaBrandt8::TriangulateMatches (KannalaBrandt8.cpp:
//                      300-366) and the acceptance depth > 0.0001f (:1193).  mvRightToLeftMatch
//                      keeps the last accepted left row per right row, as the reference's loop
//                      does: an atomic max over a -1 preset.
//
// Float work per candidate: two Newton unprojections, a 4x4 two-sided Jacobi SVD (Eigen's
// JacobiSVD, restated), two projections.  Every expression follows the reference's operation
// order without contraction (-ffp-contract=off); cos / sin of the projection use the libm
// sincosf restatement (orb_math.h), atan2f / tanf the device library.  Parity with the reference
// is unpinned (Eigen's order and FMA use on the NDK, the Android libm's atan2f / tanf):
// tests/test_fisheye.py compares with the oracle restatement within tolerances.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "orb_kernels.h"
#include "orb_math.h"

namespace orbgpu {

namespace {

struct Kp {  // orbgpu_keypoint / cv::KeyPoint (28 B)
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

// KannalaBrandt8::unproject (KannalaBrandt8.cpp:110-137)
__device__ inline void kb8_unproject(const float* P, float precision, float u, float v, float r[3]) {
    const float pwx = (u - P[2]) / P[0], pwy = (v - P[3]) / P[1];
    float scale = 1.f;
    float theta_d = sqrtf(pwx * pwx + pwy * pwy);
    const float half_pi = (float)(3.14159265358979323846 / 2.0);  // CV_PI / 2.f as fmaxf sees it
    theta_d = fminf(fmaxf(-half_pi, theta_d), half_pi);
    if ((double)theta_d > 1e-8) {
        float theta = theta_d;
        for (int j = 0; j < 10; j++) {
            const float theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2,
                        theta8 = theta4 * theta4;
            const float k0_theta2 = P[4] * theta2, k1_theta4 = P[5] * theta4;
            const float k2_theta6 = P[6] * theta6, k3_theta8 = P[7] * theta8;
            const float theta_fix = (theta * (1 + k0_theta2 + k1_theta4 + k2_theta6 + k3_theta8) - theta_d) /
                                    (1 + 3 * k0_theta2 + 5 * k1_theta4 + 7 * k2_theta6 + 9 * k3_theta8);
            theta = theta - theta_fix;
            if (fabsf(theta_fix) < precision) break;
        }
        scale = libm_tanf(theta) / theta_d;
    }
    r[0] = pwx * scale;
    r[1] = pwy * scale;
    r[2] = 1.f;
}

// KannalaBrandt8::project(const Eigen::Vector3f&) (KannalaBrandt8.cpp:61-78)
__device__ inline void kb8_project(const float* P, const float x[3], float uv[2]) {
    const float x2_plus_y2 = x[0] * x[0] + x[1] * x[1];
    const float theta = libm_atan2f(sqrtf(x2_plus_y2), x[2]);
    const float psi = libm_atan2f(x[1], x[0]);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = theta + P[4] * theta3 + P[5] * theta5 + P[6] * theta7 + P[7] * theta9;
    float sn, cs;
    libm_sincosf(psi, &sn, &cs);
    uv[0] = P[0] * r * cs + P[2];
    uv[1] = P[1] * r * sn + P[3];
}

__device__ inline float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// Plane rotation of the pair (x, y) by (c, s): x' = c x + s y, y' = -s x + c y
// (Eigen apply_rotation_in_the_plane, identity rotations skipped as there)
__device__ inline void rot(float& x, float& y, float c, float s) {
    const float xi = x, yi = y;
    x = c * xi + s * yi;
    y = -s * xi + c * yi;
}

// Eigen::JacobiSVD<Matrix4f>(A, ComputeFullV).matrixV().col(3): two-sided Jacobi sweeps over the
// pairs (p, q), p = 1..3, q < p, until every off-diagonal entry is <= max(FLT_MIN, 2 eps max|diag|),
// then the columns of V sorted by descending singular value.
__device__ inline void svd4_last_v(float W[4][4], float v3[4]) {
    float scale = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) scale = fmaxf(scale, fabsf(W[i][j]));
    if (scale == 0.f) scale = 1.f;
    float V[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            W[i][j] = W[i][j] / scale;
            V[i][j] = i == j ? 1.f : 0.f;
        }
    const float precision = 2.f * FLT_EPSILON;
    float maxDiag = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) maxDiag = fmaxf(maxDiag, fabsf(W[i][i]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 64; ++sweep) {
        finished = true;
#pragma unroll
        for (int p = 1; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < p; ++q) {
                const float threshold = fmaxf(FLT_MIN, precision * maxDiag);
                if (!(fabsf(W[p][q]) > threshold || fabsf(W[q][p]) > threshold)) continue;
                finished = false;
                // real_2x2_jacobi_svd: rot1 symmetrizes the 2x2 block, j_right diagonalizes it
                const float m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                const float t = m00 + m11, d = m10 - m01;
                float c1 = 1.f, s1 = 0.f;
                if (!(fabsf(d) < FLT_MIN)) {
                    const float u = t / d;
                    const float tmp = sqrtf(1.f + u * u);
                    s1 = 1.f / tmp;
                    c1 = u / tmp;
                }
                const float n00 = c1 * m00 + s1 * m10, n01 = c1 * m01 + s1 * m11;
                const float n11 = -s1 * m01 + c1 * m11;
                float cr = 1.f, sr = 0.f;  // makeJacobi(n00, n01, n11)
                const float deno = 2.f * fabsf(n01);
                if (!(deno < FLT_MIN)) {
                    const float tau = (n00 - n11) / deno;
                    const float w = sqrtf(tau * tau + 1.f);
                    const float tt = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
                    const float sign_t = tt > 0.f ? 1.f : -1.f;
                    const float n = 1.f / sqrtf(tt * tt + 1.f);
                    sr = -sign_t * (n01 / fabsf(n01)) * fabsf(tt) * n;
                    cr = n;
                }
                const float cl = c1 * cr - s1 * -sr;  // j_left = rot1 * j_right^T
                const float sl = c1 * -sr + s1 * cr;
                if (!(cl == 1.f && sl == 0.f))
#pragma unroll
                    for (int k = 0; k < 4; ++k) rot(W[p][k], W[q][k], cl, sl);
                if (!(cr == 1.f && sr == 0.f)) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) rot(W[k][p], W[k][q], cr, -sr);
#pragma unroll
                    for (int k = 0; k < 4; ++k) rot(V[k][p], V[k][q], cr, -sr);
                }
                maxDiag = fmaxf(maxDiag, fmaxf(fabsf(W[p][p]), fabsf(W[q][q])));
            }
    }
    float sv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sv[i] = fabsf(W[i][i]) * scale;
    // descending order, the first maximum of the tail moving up (Eigen's maxCoeff(&pos))
    int col[4] = {0, 1, 2, 3};
    for (int i = 0; i < 4; ++i) {
        int pos = i;
        for (int j = i + 1; j < 4; ++j)
            if (sv[j] > sv[pos]) pos = j;
        if (sv[pos] == 0.f) break;
        if (pos != i) {
            const float tv = sv[i];
            sv[i] = sv[pos];
            sv[pos] = tv;
            const int tc = col[i];
            col[i] = col[pos];
            col[pos] = tc;
        }
    }
    const int c3 = col[3];
#pragma unroll
    for (int k = 0; k < 4; ++k) v3[k] = c3 == 0 ? V[k][0] : c3 == 1 ? V[k][1] : c3 == 2 ? V[k][2] : V[k][3];
}

// KannalaBrandt8::TriangulateMatches: z1 (> 0) or a negative code
__device__ inline float kb8_triangulate(const FisheyeArgs& f, float u1, float v1, float u2, float v2,
                                        float sigmaLevel, float unc, float p3D[3]) {
    float r1[3], r2[3];
    kb8_unproject(f.cam_l, f.prec_l, u1, v1, r1);
    kb8_unproject(f.cam_r, f.prec_r, u2, v2, r2);
    const float* R = f.R12;
    float r21[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) r21[i] = R[3 * i] * r2[0] + R[3 * i + 1] * r2[1] + R[3 * i + 2] * r2[2];
    const float cosParallaxRays = dot3(r1, r21) / (sqrtf(dot3(r1, r1)) * sqrtf(dot3(r21, r21)));
    if ((double)cosParallaxRays > 0.99998) return -1.f;
    float T2[3][4];  // Tcw2 = [R21 | -R21 t12], R21 = R12^T
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) T2[i][j] = R[3 * j + i];
        T2[i][3] = -(T2[i][0] * f.t12[0] + T2[i][1] * f.t12[1] + T2[i][2] * f.t12[2]);
    }
    // Triangulate (KannalaBrandt8.cpp:385-397), Tcw1 = [I | 0]
    float A[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float t1r2 = j == 2 ? 1.f : 0.f, t1r0 = j == 0 ? 1.f : 0.f, t1r1 = j == 1 ? 1.f : 0.f;
        A[0][j] = r1[0] * t1r2 - t1r0;
        A[1][j] = r1[1] * t1r2 - t1r1;
        A[2][j] = r2[0] * T2[2][j] - T2[0][j];
        A[3][j] = r2[1] * T2[2][j] - T2[1][j];
    }
    float h[4];
    svd4_last_v(A, h);
    const float x3D[3] = {h[0] / h[3], h[1] / h[3], h[2] / h[3]};
    const float z1 = x3D[2];
    if (z1 <= 0) return -2.f;
    const float z2 = (T2[2][0] * x3D[0] + T2[2][1] * x3D[1] + T2[2][2] * x3D[2]) + T2[2][3];
    if (z2 <= 0) return -3.f;
    float uv1[2];
    kb8_project(f.cam_l, x3D, uv1);
    const float errX1 = uv1[0] - u1, errY1 = uv1[1] - v1;
    if ((double)(errX1 * errX1 + errY1 * errY1) > 5.991 * 8 * sigmaLevel) return -4.f;
    float x3D2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) x3D2[i] = (T2[i][0] * x3D[0] + T2[i][1] * x3D[1] + T2[i][2] * x3D[2]) + T2[i][3];
    float uv2[2];
    kb8_project(f.cam_r, x3D2, uv2);
    const float errX2 = uv2[0] - u2, errY2 = uv2[1] - v2;
    if ((double)(errX2 * errX2 + errY2 * errY2) > 5.991 * 8 * unc) return -5.f;
    p3D[0] = x3D[0];
    p3D[1] = x3D[1];
    p3D[2] = x3D[2];
    return z1;
}

}  // namespace

// grid (row blocks, pairs): lane = left keypoint row
__global__ __launch_bounds__(256) void k_fisheye_stereo(FisheyeArgs f) {
    const int pair = f.pair0 + blockIdx.y;
    const int li = 2 * pair, ri = 2 * pair + 1;
    const int nL = max(f.out_n[li], 0), nR = max(f.out_n[ri], 0);
    const int mL = min(max(f.out_mono[li], 0), nL), mR = min(max(f.out_mono[ri], 0), nR);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // left keypoint
    if (i >= nL) return;
    const long long o = (long long)pair * f.out_cap;
    int32_t l2r = -1;
    float depth = -1.f, p[3] = {0.f, 0.f, 0.f};
    if (i >= mL) {
        const int q = i - mL;  // stereo row (query of the kNN2)
        const int d1 = f.dist1[o + q];
        const uint32_t d16 = (uint32_t)d1 & 0xFFFFu;  // BFMatchORB's uint16 distances
        if (d16 != 0 && d16 < 70 && d1 >= 0) {
            atomicAdd(&f.counts[2 * pair + 1], 1);  // descMatches
            const int rightPos = f.idx1[o + q];
            if (!(rightPos + mR >= nR || rightPos < 0)) {
                const Kp* kl = reinterpret_cast<const Kp*>(f.kps) + (long long)li * f.out_cap + i;
                const Kp* kr = reinterpret_cast<const Kp*>(f.kps) + (long long)ri * f.out_cap + rightPos + mR;
                const Kp a = *kl, b = *kr;
                const float sigma1 = f.sigma2[min(max(a.octave, 0), kMaxLevels - 1)];
                const float sigma2 = f.sigma2[min(max(b.octave, 0), kMaxLevels - 1)];
                float x[3];
                const float z = kb8_triangulate(f, a.x, a.y, b.x, b.y, sigma1, sigma2, x);
                if (z > 0.0001f) {
                    l2r = rightPos + mR;
                    depth = z;
                    p[0] = x[0];
                    p[1] = x[1];
                    p[2] = x[2];
                    atomicMax(&f.r2l[o + l2r], i);
                    atomicAdd(&f.counts[2 * pair], 1);
                }
            }
        }
    }
    f.l2r[o + i] = l2r;
    f.depth[o + i] = depth;
    float* pp = f.p3d + 3 * (o + i);
    pp[0] = p[0];
    pp[1] = p[1];
    pp[2] = p[2];
}

hipError_t launch_fisheye(const FisheyeArgs& f, int npairs, hipStream_t s) {
    hipLaunchKernelGGL(k_fisheye_stereo, dim3((f.out_cap + 255) / 256, npairs), dim3(256), 0, s, f);
    return hipGetLastError();
}

}  // namespace orbgpu
