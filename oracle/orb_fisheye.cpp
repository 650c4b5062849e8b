// orb_fisheye.cpp -- TEST INFRASTRUCTURE ONLY (CPU oracle; never linked into the product).
//
// Frame::ComputeStereoFishEyeMatches (cpp/src/Frame.cc:1142-1201) for one stereo frame, restated
// on the kNN2 result of the stereo rows (BFMatchORB, Frame.cc:1164): per left stereo row i,
//   dist1 == 0 -> skipped ("bugged point", :1171-1175), dist1 < 70 -> candidate (:1177),
//   index checks (:1183-1189), KannalaBrandt8::TriangulateMatches (KannalaBrandt8.cpp:300-366)
//   with sigma1 = mvLevelSigma2[left octave], unc = mvLevelSigma2[right octave], accepted when
//   the returned depth > 0.0001f (:1193): mvLeftToRightMatch, mvRightToLeftMatch (the last
//   accepted left row wins), mvDepth, mvStereo3Dpoints.
// KannalaBrandt8::unproject (:110-137, float Newton, std::tan), project (:61-78, atan2f and the
// float cos / sin), Triangulate (:385-397: Eigen::JacobiSVD<Matrix4f>(A, ComputeFullV), last
// column of V).  Eigen is an external dependency of the reference (not vendored, not installed
// here): the SVD below restates Eigen 3.3/3.4's JacobiSVD for a square real matrix (no QR
// preconditioner for square input, two-sided 2x2 Jacobi sweeps until every off-diagonal entry
// is <= max(FLT_MIN, 2 eps * max|diag|), singular values sorted descending with V's columns).
// PARITY UNPINNED: Eigen's evaluation order and the NDK's FMA contraction, and the Android
// libm's atan2f / tanf, cannot be reproduced here; the GPU kernel and this restatement share
// the arithmetic order (no contraction), and tests compare them with a tolerance (see
// tests/test_fisheye.py).  Besides the outputs it reports each row's decision code and the
// quantities tested against the thresholds, so that tests can tell a near-threshold flip.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "orb_oracle.h"

namespace {

struct Cam {
    const float* p;  // fx fy cx cy k0 k1 k2 k3
    float precision;
};

void unproject(const Cam& c, float u, float v, float r[3]) {
    const float* P = c.p;
    const float pwx = (u - P[2]) / P[0], pwy = (v - P[3]) / P[1];
    float scale = 1.f;
    float theta_d = std::sqrt(pwx * pwx + pwy * pwy);
    const float half_pi = (float)(3.14159265358979323846 / 2.0);  // fmaxf(-CV_PI / 2.f, ...)
    theta_d = std::fmin(std::fmax(-half_pi, theta_d), half_pi);
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
            if (std::fabs(theta_fix) < c.precision) break;
        }
        scale = std::tan(theta) / theta_d;
    }
    r[0] = pwx * scale;
    r[1] = pwy * scale;
    r[2] = 1.f;
}

void project(const Cam& c, const float x[3], float uv[2]) {
    const float* P = c.p;
    const float x2_plus_y2 = x[0] * x[0] + x[1] * x[1];
    const float theta = atan2f(std::sqrt(x2_plus_y2), x[2]);
    const float psi = atan2f(x[1], x[0]);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = theta + P[4] * theta3 + P[5] * theta5 + P[6] * theta7 + P[7] * theta9;
    uv[0] = P[0] * r * std::cos(psi) + P[2];
    uv[1] = P[1] * r * std::sin(psi) + P[3];
}

float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// Eigen JacobiSVD (square, real, ComputeFullV): returns column 3 of V (sorted).
void jacobi_svd4_lastv(const float Ain[4][4], float v3[4]) {
    float scale = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) scale = std::fmax(scale, std::fabs(Ain[i][j]));
    if (scale == 0.f) scale = 1.f;
    float W[4][4], V[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            W[i][j] = Ain[i][j] / scale;
            V[i][j] = i == j ? 1.f : 0.f;
        }
    const float considerAsZero = FLT_MIN, precision = 2.f * FLT_EPSILON;
    float maxDiag = 0.f;
    for (int i = 0; i < 4; ++i) maxDiag = std::fmax(maxDiag, std::fabs(W[i][i]));
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 64) {
        finished = true;
        ++sweeps;
        for (int p = 1; p < 4; ++p)
            for (int q = 0; q < p; ++q) {
                const float threshold = std::fmax(considerAsZero, precision * maxDiag);
                if (!(std::fabs(W[p][q]) > threshold || std::fabs(W[q][p]) > threshold)) continue;
                finished = false;
                // real_2x2_jacobi_svd on [[W(p,p) W(p,q)] [W(q,p) W(q,q)]]
                const float m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                const float t = m00 + m11, d = m10 - m01;
                float c1, s1;
                if (std::fabs(d) < FLT_MIN) {
                    s1 = 0.f;
                    c1 = 1.f;
                } else {
                    const float u = t / d;
                    const float tmp = std::sqrt(1.f + u * u);
                    s1 = 1.f / tmp;
                    c1 = u / tmp;
                }
                // m.applyOnTheLeft(0, 1, rot1): rows x = (m00, m01), y = (m10, m11)
                const float n00 = c1 * m00 + s1 * m10, n01 = c1 * m01 + s1 * m11;
                const float n11 = -s1 * m01 + c1 * m11;
                // j_right.makeJacobi(n00, n01, n11)
                float cr, sr;
                const float deno = 2.f * std::fabs(n01);
                if (deno < FLT_MIN) {
                    cr = 1.f;
                    sr = 0.f;
                } else {
                    const float tau = (n00 - n11) / deno;
                    const float w = std::sqrt(tau * tau + 1.f);
                    const float tt = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
                    const float sign_t = tt > 0.f ? 1.f : -1.f;
                    const float n = 1.f / std::sqrt(tt * tt + 1.f);
                    sr = -sign_t * (n01 / std::fabs(n01)) * std::fabs(tt) * n;
                    cr = n;
                }
                // j_left = rot1 * j_right.transpose(), transpose = (cr, -sr)
                const float cl = c1 * cr - s1 * -sr;
                const float sl = c1 * -sr + s1 * cr;
                // W.applyOnTheLeft(p, q, j_left): rows p, q
                if (!(cl == 1.f && sl == 0.f))
                    for (int k = 0; k < 4; ++k) {
                        const float xi = W[p][k], yi = W[q][k];
                        W[p][k] = cl * xi + sl * yi;
                        W[q][k] = -sl * xi + cl * yi;
                    }
                // W.applyOnTheRight(p, q, j_right) and V.applyOnTheRight(p, q, j_right): columns
                // p, q rotated by j_right.transpose() = (cr, -sr)
                if (!(cr == 1.f && sr == 0.f)) {
                    const float c = cr, s = -sr;
                    for (int k = 0; k < 4; ++k) {
                        const float xi = W[k][p], yi = W[k][q];
                        W[k][p] = c * xi + s * yi;
                        W[k][q] = -s * xi + c * yi;
                    }
                    for (int k = 0; k < 4; ++k) {
                        const float xi = V[k][p], yi = V[k][q];
                        V[k][p] = c * xi + s * yi;
                        V[k][q] = -s * xi + c * yi;
                    }
                }
                maxDiag = std::fmax(maxDiag, std::fmax(std::fabs(W[p][p]), std::fabs(W[q][q])));
            }
    }
    float sv[4];
    for (int i = 0; i < 4; ++i) sv[i] = std::fabs(W[i][i]) * scale;
    for (int i = 0; i < 4; ++i) {
        int pos = i;
        for (int j = i + 1; j < 4; ++j)
            if (sv[j] > sv[pos]) pos = j;  // maxCoeff: the first maximum
        if (sv[pos] == 0.f) break;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int k = 0; k < 4; ++k) std::swap(V[k][i], V[k][pos]);
        }
    }
    for (int k = 0; k < 4; ++k) v3[k] = V[k][3];
}

// TriangulateMatches; returns z1 (> 0) or the negative code; m[5] = cos parallax, z1, z2,
// reprojection error 1 minus its bound, reprojection error 2 minus its bound
float triangulate(const Cam& c1, const Cam& c2, float u1, float v1, float u2, float v2, const float R12[9],
                  const float t12[3], float sigmaLevel, float unc, float p3D[3], double m[5]) {
    float r1[3], r2[3];
    unproject(c1, u1, v1, r1);
    unproject(c2, u2, v2, r2);
    float r21[3];
    for (int i = 0; i < 3; ++i) r21[i] = R12[3 * i] * r2[0] + R12[3 * i + 1] * r2[1] + R12[3 * i + 2] * r2[2];
    const float cosParallaxRays = dot3(r1, r21) / (std::sqrt(dot3(r1, r1)) * std::sqrt(dot3(r21, r21)));
    m[0] = cosParallaxRays;
    if ((double)cosParallaxRays > 0.99998) return -1;
    // Tcw1 = [I | 0], Tcw2 = [R21 | -R21 t12], R21 = R12^T
    float T2[3][4];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T2[i][j] = R12[3 * j + i];
        T2[i][3] = -(T2[i][0] * t12[0] + T2[i][1] * t12[1] + T2[i][2] * t12[2]);
    }
    const float T1[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
    float A[4][4];
    for (int j = 0; j < 4; ++j) {
        A[0][j] = r1[0] * T1[2][j] - T1[0][j];
        A[1][j] = r1[1] * T1[2][j] - T1[1][j];
        A[2][j] = r2[0] * T2[2][j] - T2[0][j];
        A[3][j] = r2[1] * T2[2][j] - T2[1][j];
    }
    float h[4];
    jacobi_svd4_lastv(A, h);
    const float x3D[3] = {h[0] / h[3], h[1] / h[3], h[2] / h[3]};
    const float z1 = x3D[2];
    m[1] = z1;
    if (z1 <= 0) return -2;
    const float z2 = (T2[2][0] * x3D[0] + T2[2][1] * x3D[1] + T2[2][2] * x3D[2]) + T2[2][3];
    m[2] = z2;
    if (z2 <= 0) return -3;
    float uv1[2];
    project(c1, x3D, uv1);
    const float errX1 = uv1[0] - u1, errY1 = uv1[1] - v1;
    const float e1 = errX1 * errX1 + errY1 * errY1;
    m[3] = (double)e1 - 5.991 * 8 * sigmaLevel;
    if ((double)e1 > 5.991 * 8 * sigmaLevel) return -4;
    float x3D2[3];
    for (int i = 0; i < 3; ++i) x3D2[i] = (T2[i][0] * x3D[0] + T2[i][1] * x3D[1] + T2[i][2] * x3D[2]) + T2[i][3];
    float uv2[2];
    project(c2, x3D2, uv2);
    const float errX2 = uv2[0] - u2, errY2 = uv2[1] - v2;
    const float e2 = errX2 * errX2 + errY2 * errY2;
    m[4] = (double)e2 - 5.991 * 8 * unc;
    if ((double)e2 > 5.991 * 8 * unc) return -5;
    for (int i = 0; i < 3; ++i) p3D[i] = x3D[i];
    return z1;
}

}  // namespace

extern "C" int oracle_fisheye_stereo(const oracle_kp* kpsL, int nL, int monoL, const oracle_kp* kpsR, int nR,
                                     int monoR, const int32_t* idx1, const int32_t* dist1, const float* camL,
                                     const float* camR, float precL, float precR, const float* R12,
                                     const float* t12, const float* sigma2, int32_t* l2r, int32_t* r2l,
                                     float* depth, float* p3d, int32_t* code, double* margins) {
    const Cam c1{camL, precL}, c2{camR, precR};
    for (int i = 0; i < nL; ++i) {
        l2r[i] = -1;
        depth[i] = -1.f;
        p3d[3 * i] = p3d[3 * i + 1] = p3d[3 * i + 2] = 0.f;
    }
    for (int i = 0; i < nR; ++i) r2l[i] = -1;
    int nMatches = 0;
    const int nq = nL - monoL;
    for (int i = 0; i < nq; ++i) {
        double* m = margins + 5 * (size_t)i;
        for (int k = 0; k < 5; ++k) m[k] = NAN;
        code[i] = 0;
        const uint16_t d1 = (uint16_t)dist1[i];  // BFMatchORB returns uint16 distances
        if (d1 == 0) {  // "Bugged point"
            code[i] = 1;
            continue;
        }
        if (d1 >= 70) {
            code[i] = 2;
            continue;
        }
        const int leftPos = i, rightPos = idx1[i];
        if (rightPos + monoR >= nR || rightPos < 0 || leftPos + monoL >= nL) {
            code[i] = 3;
            continue;
        }
        const oracle_kp& k1 = kpsL[leftPos + monoL];
        const oracle_kp& k2 = kpsR[rightPos + monoR];
        float p[3];
        const float z = triangulate(c1, c2, k1.x, k1.y, k2.x, k2.y, R12, t12, sigma2[k1.octave], sigma2[k2.octave],
                                    p, m);
        if (z > 0.0001f) {
            l2r[leftPos + monoL] = rightPos + monoR;
            r2l[rightPos + monoR] = leftPos + monoL;
            depth[leftPos + monoL] = z;
            for (int k = 0; k < 3; ++k) p3d[3 * (leftPos + monoL) + k] = p[k];
            code[i] = 10;
            ++nMatches;
        } else {
            code[i] = z == -1 ? 4 : z == -2 ? 5 : z == -3 ? 6 : z == -4 ? 7 : z == -5 ? 8 : 9;
        }
    }
    return nMatches;
}
