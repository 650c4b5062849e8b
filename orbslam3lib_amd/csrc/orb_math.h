// orb_math.h -- bit-exact scalar primitives shared by the kernels (host-callable for tests).
//
// Compiled with -ffp-contract=off: every float expression below is evaluated as separately
// rounded IEEE single operations in source order, which is what the CPU reference does.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbgpu {

__host__ __device__ inline int imin(int a, int b) { return a < b ? a : b; }
__host__ __device__ inline int imax(int a, int b) { return a > b ? a : b; }

// cvRound(float) = round-half-to-even (lrintf / v_rndne_f32).
__host__ __device__ inline int cv_round(float v) { return (int)__builtin_rintf(v); }

// std::cos(float) / std::sin(float) as computeOrbDescriptor calls them: `(float)cos(angle)` with a
// float `angle` under `using namespace std` (cpp/src/ORBextractor_old.cc:68,114-115) is the float
// overload, i.e. libm cosf / sinf.  glibc >= 2.28 and Android bionic (arm64) both ship the same
// single-precision algorithm (ARM optimized-routines sincosf: double-precision Cody-Waite
// reduction by pi/2 for |x| < 120, then degree-8 / degree-7 polynomials in x^2).  Restated here for
// the domain the descriptor produces, 0 <= x < 2 pi (angles from fastAtan2 in [0, 360) degrees
// times factorPI); checked bit-exact against the host libm on every float of [0, 6.2832), with
// and without FMA contraction of the polynomial (tests/test_host_harness.py).
// sin polynomial x + x^3 s1 + x^7 (s2 + x^2 s3) and cos polynomial
// (c0 + x^2 c1) + x^4 c2 + x^6 (c3 + x^2 c4), each rounded to float as glibc's sincosf does
__host__ __device__ inline float libm_sin_poly(double x, double x2) {
    const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
    const double x3 = x * x2;
    const double t1 = s2 + x2 * s3;
    const double x7 = x3 * x2;
    const double s = x + x3 * s1;
    return (float)(s + x7 * t1);
}
__host__ __device__ inline float libm_cos_poly(double x2) {
    const double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                 c4 = 0x1.99343027bf8c3p-16;
    const double x4 = x2 * x2;
    const double t2 = c3 + x2 * c4;
    const double t1 = c0 + x2 * c1;
    const double x6 = x4 * x2;
    const double c = t1 + x4 * c2;
    return (float)(c + x6 * t2);
}
// libm sinf(y) and cosf(y) for 0 <= y < 120.  glibc evaluates, after the reduction to
// x in [-pi/4, pi/4] with quadrant n, sinf = poly(x s, n) and cosf = poly(x s, n ^ 1), where an
// odd selector takes the cos polynomial with coefficients negated for n & 2 (table 1) and
// s = {1, -1, -1, 1}[n & 3].  Both results therefore come from ONE sin and ONE cos polynomial
// of x s, swapped for odd n; the negated coefficients negate the cos polynomial exactly
// (every operation is sign-symmetric under round-to-nearest), so the sign is applied to the
// float result.
__host__ __device__ inline void libm_sincosf(float y, float* sn, float* cs) {
    double x = y;
    const uint32_t u = __builtin_bit_cast(uint32_t, y);
    const uint32_t top = (u >> 20) & 0x7ff;
    if (top < 0x398u) {  // |y| < 2^-12
        *sn = y;
        *cs = 1.0f;
        return;
    }
    int n = 0;
    if (top >= 0x3f4u) {  // |y| >= pi/4 (abstop12(0x1.921FB6p-1f)): reduce_fast
        // n = round(x * 2/pi) in 8.24 fixed point, r = x - n * pi/2, times {1, -1, -1, 1}[n & 3]
        const double r = x * 0x1.45F306DC9C883p+23;
        n = ((int32_t)r + 0x800000) >> 24;
        x = x - n * 0x1.921FB54442D18p0;
        x = ((n + 1) & 2) ? -x : x;
    }
    const double x2 = x * x;
    const float ps = libm_sin_poly(x, x2);
    float pc = libm_cos_poly(x2);
    pc = (n & 2) ? -pc : pc;
    *sn = (n & 1) ? pc : ps;
    *cs = (n & 1) ? ps : pc;
}

// atanf / atan2f / tanf of the host libm the oracle links (glibc 2.35, this image and the GPU
// box), for Frame::ComputeStereoFishEyeMatches' KannalaBrandt8 camera model (project:
// atan2f(sqrt(x^2 + y^2), z) and atan2f(y, x), CameraModels/KannalaBrandt8.cpp:61-78; unproject:
// std::tan(float theta) = tanf, :110-137).  glibc's single-precision atanf / atan2f are the
// fdlibm float algorithm (11-term odd/even polynomial after the 7/16, 11/16, 19/16, 39/16
// argument split; atan2f's quadrant and pi_lo corrections); its tanf is the fdlibm float kernel
// (13-term polynomial, the |x| >= 0.6744 pi/4 - x transform and the -1/(x + r) refinement) after a
// double-precision reduction by pi/2.  Checked against the host libm: atanf on every positive
// float (2,139,095,040 values, odd function), tanf on every float of [-2.35, 2.35] (the domain of
// the restated reduction, |x| < 3 pi / 4), atan2f on 4e8 random pairs (bit patterns, [-3, 3]^2,
// the near-diagonal band) -- tools/libm_fisheye_exhaustive.py, tests/test_host_harness.py.  No
// FMA contraction (-ffp-contract=off): every expression is rounded as written.
__host__ __device__ inline float libm_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f,  -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f,  -3.6531571299e-02f, 1.6285819933e-02f};
    const int32_t hx = __builtin_bit_cast(int32_t, x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {  // |x| < 0.4375
        if (ix < 0x31000000) return x;  // |x| < 2^-29
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {      // |x| < 1.1875
            if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000) {  // |x| < 2.4375
            id = 2;
            x = (x - 1.5f) / (1.0f + 1.5f * x);
        } else {
            id = 3;
            x = -1.0f / x;
        }
    }
    float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -z : z;
}

__host__ __device__ inline float libm_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = __builtin_bit_cast(int32_t, x), ix = hx & 0x7fffffff;
    const int32_t hy = __builtin_bit_cast(int32_t, y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;  // NaN
    if (hx == 0x3f800000) return libm_atanf(y);             // x = 1
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);       // 2 sign(x) + sign(y)
    if (iy == 0) return m <= 1 ? y : m == 2 ? pi + tiny : -pi - tiny;
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            const float r[4] = {pi_o_4 + tiny, -pi_o_4 - tiny, 3.0f * pi_o_4 + tiny, -3.0f * pi_o_4 - tiny};
            return r[m];
        }
        const float r[4] = {0.0f, -0.0f, pi + tiny, -pi - tiny};
        return r[m];
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;  // |y / x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0f;   // |y| / x < -2^60
    else z = libm_atanf(__builtin_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// __kernel_tanf(x, y, iy): tan(x + y) for |x + y| <= pi/4 (iy = 1), -1 / tan(x + y) (iy = -1).
__host__ __device__ inline float libm_kernel_tanf(float x, float y, int iy) {
    const float T[13] = {3.3333334327e-01f, 1.3333334029e-01f, 5.3968254477e-02f, 2.1869488060e-02f,
                         8.8632395491e-03f, 3.5920790397e-03f, 1.4562094584e-03f, 5.8804126456e-04f,
                         2.4646313977e-04f, 7.8179444245e-05f, 7.1407252108e-05f, -1.8558637748e-05f,
                         2.5907305826e-05f};
    const float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
    const int32_t hx = __builtin_bit_cast(int32_t, x), ix = hx & 0x7fffffff;
    if (ix < 0x39000000 && (int)x == 0) {  // |x| < 2^-13
        if ((ix | (iy + 1)) == 0) return 1.0f / __builtin_fabsf(x);
        return iy == 1 ? x : -1.0f / x;
    }
    if (ix >= 0x3f2ca140) {  // |x| >= 0.6744
        if (hx < 0) {
            x = -x;
            y = -y;
        }
        const float zz = pio4 - x, ww = pio4lo - y;
        x = zz + ww;
        y = 0.0f;
        if (__builtin_fabsf(x) < 0x1p-13f) return (float)((1 - ((hx >> 30) & 2)) * iy) * (1.0f - (float)(2 * iy) * x);
    }
    const float z = x * x;
    float w = z * z;
    float r = T[1] + w * (T[3] + w * (T[5] + w * (T[7] + w * (T[9] + w * T[11]))));
    float v = z * (T[2] + w * (T[4] + w * (T[6] + w * (T[8] + w * (T[10] + w * T[12])))));
    float s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T[0] * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    // -1 / (x + r) refined: z + v = r + x with z the high 12 bits of w
    const float zh = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, w) & 0xfffff000u);
    v = r - (zh - x);
    const float a = -1.0f / w;
    const float t = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, a) & 0xfffff000u);
    s = 1.0f + t * zh;
    return t + a * (s + t * v);
}

// tanf(x) for |x| < 3 pi / 4 (the restated reduction's domain; the fisheye unprojection's theta
// lies in [0, pi / 2]): |x| <= pi/4 straight to the kernel, else x - n pi/2 (n = +-1) in double,
// split into a float head and tail, and the kernel's -1 / tan form.
__host__ __device__ inline float libm_tanf(float x) {
    const int32_t ix = __builtin_bit_cast(int32_t, x) & 0x7fffffff;
    if (ix <= 0x3f490fda) return libm_kernel_tanf(x, 0.0f, 1);
    if (ix >= 0x7f800000) return x - x;
    const double xd = (double)x;
    const int n = xd > 0.0 ? 1 : -1;
    const double yd = xd - (double)n * 1.57079632679489661923;
    const float y0 = (float)yd, y1 = (float)(yd - (double)y0);
    return libm_kernel_tanf(y0, y1, -1);
}

// cv::fastAtan2 (OpenCV 4.2 core mathfuncs atanImpl<float>), degrees in [0, 360).
// Called by IC_Angle, cpp/src/ORBextractor_old.cc:104.
__host__ __device__ inline float fast_atan2_deg(float y, float x) {
    const float k180pi = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k180pi;
    const float p3 = -0.3258083974640975f * k180pi;
    const float p5 = 0.1555786518463281f * k180pi;
    const float p7 = -0.04432655554792128f * k180pi;
    const float eps = (float)2.220446049250313080847e-16;  // (float)DBL_EPSILON
    const float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// FAST-9/16 Bresenham ring (OpenCV makeOffsets, patternSize 16), (dx, dy).
__host__ __device__ inline int ring_dx(int k) {
    const int t[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    return t[k];
}
__host__ __device__ inline int ring_dy(int k) {
    const int t[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    return t[k];
}

// Threshold-independent FAST strength m(p) = clamp(max over the 16 cyclic 9-arcs of
// min(v - ring) [dark] or min(ring - v) [bright], 0, 255).  With it, for any threshold t >= 0:
//   cv::FAST corner at t      <=>  m > t
//   cornerScore<16>(p, t)      =   m - 1                     (for corners)
// and the 3x3 nonmax rule of FAST_t<16> becomes
//   kept_t(p) <=> m(p) > t && m(p) >= 2 && for each 8-neighbour q in the same cell detection
//                 region: m(q) <= t || m(p) > m(q).
// When a necessary-condition pre-test at t_min fails (the 4-point compass in fast_strength below,
// the 8-point antipodal-pair test in k_fast_cells), S_max <= t_min and 0 is stored instead (exact
// for every t >= t_min).  Reference call sites: cv::FAST at ORBextractor_old.cc:828,847.
// Exact strength of a pixel already known to be a corner at some t >= 0 (no pre-test).
__host__ __device__ inline int fast_strength_corner(const uint8_t* c, int stride) {
    const int v = c[0];
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - (int)c[ring_dx(k) + ring_dy(k) * stride];
    int a2[16], b2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int x = d[k], y = d[(k + 1) & 15];
        a2[k] = x < y ? x : y;
        b2[k] = x > y ? x : y;
    }
    int a4[16], b4[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int x = a2[k], y = a2[(k + 2) & 15];
        a4[k] = x < y ? x : y;
        const int u = b2[k], w = b2[(k + 2) & 15];
        b4[k] = u > w ? u : w;
    }
    int sdark = -1024, bmin = 1024;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        int a = a4[k] < a4[(k + 4) & 15] ? a4[k] : a4[(k + 4) & 15];
        a = a < d[(k + 8) & 15] ? a : d[(k + 8) & 15];
        sdark = sdark > a ? sdark : a;
        int b = b4[k] > b4[(k + 4) & 15] ? b4[k] : b4[(k + 4) & 15];
        b = b > d[(k + 8) & 15] ? b : d[(k + 8) & 15];
        bmin = bmin < b ? bmin : b;
    }
    int s = sdark > -bmin ? sdark : -bmin;
    s = s < 0 ? 0 : s;
    return s > 255 ? 255 : s;
}

// The same strength with both polarities in one 32-bit word per ring point: low half
// d + kFastBias, high half -d + kFastBias (d = v - p; both halves in [0x401, 0x5FF], so one
// v_mad_u32_u24 builds the word), then 9-arc minima and the maximum over arcs with packed
// 16-bit min/max: low = sdark + kFastBias, high = -bmin + kFastBias.  Exact for any pixel;
// m > t <=> FAST corner at t.  The bias puts every half in the normal f16 range with one
// exponent (0x0400 <= h <= 0x7BFF), where the f16 order of the bit patterns is their integer
// order, so the 3-input gfx950 v_pk_minimum3_f16 / v_pk_maximum3_f16 are exact integer
// min3 / max3 on them.
typedef unsigned short orb_u16x2 __attribute__((ext_vector_type(2)));
constexpr int kFastBias = 1280;  // 0x500

__host__ __device__ inline orb_u16x2 pk_min3(orb_u16x2 a, orb_u16x2 b, orb_u16x2 c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3"
        : "=v"(r)
        : "v"(__builtin_bit_cast(uint32_t, a)), "v"(__builtin_bit_cast(uint32_t, b)),
          "v"(__builtin_bit_cast(uint32_t, c)));
    return __builtin_bit_cast(orb_u16x2, r);
#else
    return __builtin_elementwise_min(__builtin_elementwise_min(a, b), c);
#endif
}

__host__ __device__ inline orb_u16x2 pk_max3(orb_u16x2 a, orb_u16x2 b, orb_u16x2 c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3"
        : "=v"(r)
        : "v"(__builtin_bit_cast(uint32_t, a)), "v"(__builtin_bit_cast(uint32_t, b)),
          "v"(__builtin_bit_cast(uint32_t, c)));
    return __builtin_bit_cast(orb_u16x2, r);
#else
    return __builtin_elementwise_max(__builtin_elementwise_max(a, b), c);
#endif
}

// max over the 16 9-arcs of the arc minimum, per u16 half.  The 16 arcs pair up: arcs [2j, 2j+8]
// and [2j+1, 2j+9] share the 8 points [2j+1, 2j+8], so max(min(arc 2j), min(arc 2j+1)) =
// min(a8[2j+1], max(x[2j], x[2j+9])), and a8[2j+1] = min(a4[j], a4[j+2]) with a4[j] = min over
// [2j+1, 2j+4]: 8 + 8 two-input mins, 8 max + 8 min3 for the pairs, 4 max3/max over the pairs =
// 36 packed ops (47 with two-input ops only, 79 for the 16 arcs taken one by one).
__host__ __device__ inline orb_u16x2 fast_arc_maxmin(const orb_u16x2 x[16]) {
    orb_u16x2 a2[8], a4[8], pr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a2[j] = __builtin_elementwise_min(x[2 * j + 1], x[(2 * j + 2) & 15]);
#pragma unroll
    for (int j = 0; j < 8; ++j) a4[j] = __builtin_elementwise_min(a2[j], a2[(j + 1) & 7]);   // [2j+1, 2j+4]
#pragma unroll
    for (int j = 0; j < 8; ++j)
        pr[j] = pk_min3(a4[j], a4[(j + 2) & 7], __builtin_elementwise_max(x[2 * j], x[(2 * j + 9) & 15]));
    return __builtin_elementwise_max(pk_max3(pr[0], pr[1], pr[2]), pk_max3(pr[3], pr[4], pk_max3(pr[5], pr[6], pr[7])));
}

template <int STRIDE>
__host__ __device__ inline int fast_strength_packed(const uint8_t* c) {
    const int v = c[0];
    const uint32_t cv = (uint32_t)(v + kFastBias) + ((uint32_t)(kFastBias - v) << 16);
    orb_u16x2 x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t p = c[ring_dx(k) + ring_dy(k) * STRIDE];
        x[k] = __builtin_bit_cast(orb_u16x2, p * 65535u + cv);
    }
    const orb_u16x2 best = fast_arc_maxmin(x);
    int s = (int)(best.x > best.y ? best.x : best.y) - kFastBias;
    s = s < 0 ? 0 : s;
    return s > 255 ? 255 : s;
}

__host__ __device__ inline int fast_strength(const uint8_t* c, int stride, int t_min) {
    const int v = c[0];
    // compass pre-test: any 9-arc holds two cyclically adjacent points of {0,4,8,12}
    int dm = 0, bm = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int d = v - (int)c[ring_dx(4 * q) + ring_dy(4 * q) * stride];
        dm |= (d > t_min) << q;
        bm |= (-d > t_min) << q;
    }
    const int dr = ((dm << 1) | (dm >> 3)) & 15, br = ((bm << 1) | (bm >> 3)) & 15;
    if (!(dm & dr) && !(bm & br)) return 0;
    return fast_strength_corner(c, stride);
}

}  // namespace orbgpu
