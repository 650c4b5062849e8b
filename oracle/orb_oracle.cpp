// orb_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
//
// Scalar CPU restatement of the reference CPU ORBextractor path.  Every function cites the
// reference file:line it follows (paths relative to the reference root, `cpp/` =
// app/src/main/cpp/).  OpenCV 4.2.0 primitives (absent here) are restated from the published
// OpenCV algorithm; their configuration-dependent choices are pinned in orb_oracle.h.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fno-fast-math).  Never linked into the
// product library.
#include "orb_oracle.h"

#include <algorithm>
#include <atomic>
#include <thread>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <list>
#include <utility>
#include <vector>
#include <atomic>
#include <thread>

#include "orb_pattern_data.h"

namespace {

// ------------------------------------------------------------------------------------------
// OpenCV rounding helpers (core/fast_math.hpp): cvRound = round-half-even via lrint.
inline int cvRound(double v) { return (int)std::lrint(v); }
inline int cvRound(float v) { return (int)std::lrintf(v); }
inline int cvFloor(float v) { int i = cvRound(v); return i - (float(i) > v); }
inline int cvFloor(double v) { int i = (int)v; return i - (i > v); }
inline int cvCeil(double v) { int i = (int)v; return i + (i < v); }
inline short sat_short(float v) {
    int i = cvRound(v);
    return (short)std::min(std::max(i, (int)SHRT_MIN), (int)SHRT_MAX);
}
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }

struct KeyPoint {  // cv::KeyPoint
    float x = 0, y = 0, size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};

struct Plane {
    std::vector<uint8_t> px;
    int w = 0, h = 0;
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
    uint8_t* row(int y) { return px.data() + (size_t)y * w; }
};

const int PATCH_SIZE = 31;       // ORBextractor_old.cc:73
const int HALF_PATCH_SIZE = 15;  // :74
const int EDGE_THRESHOLD = 19;   // :75

std::vector<int> pattern_table() {
    static const char* hex = ORACLE_PATTERN_HEX;
    std::vector<int> v(1024);
    for (int i = 0; i < 1024; ++i) {
        auto nib = [](char c) { return c <= '9' ? c - '0' : c - 'a' + 10; };
        int b = nib(hex[2 * i]) * 16 + nib(hex[2 * i + 1]);
        v[i] = (int8_t)b;
    }
    return v;
}

// ------------------------------------------------------------------------------------------
// cv::resize INTER_LINEAR, CV_8UC1 (OpenCV 4.2 imgproc/src/resize.cpp: hal::resize ->
// resizeGeneric_<HResizeLinear<uchar,int,short,2048,...>, VResizeLinear<...,FixedPtCast<22>,
// VResizeLinearVec_32s8u>>).  Called by canonical ComputePyramid, ORBextractor_old.cc:1344.
const int INTER_RESIZE_COEF_BITS = 11;
const int INTER_RESIZE_COEF_SCALE = 1 << INTER_RESIZE_COEF_BITS;

int simd_end(int width) {
    // VResizeLinearVec_32s8u: 16-pixel body while x <= width-16, then 8-pixel body while
    // x <= width-8 (128-bit universal intrinsics); FixedPtCast scalar tail afterwards.
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x <= width - 8; x += 8) {}
    return x;
}

void resize_linear(const uint8_t* src, int sw, int sh, int sstep, uint8_t* dst, int dw, int dh,
                   int dstep) {
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int iscale_x = cvRound(scale_x), iscale_y = cvRound(scale_y);
    bool is_area_fast = std::abs(scale_x - iscale_x) < DBL_EPSILON &&
                        std::abs(scale_y - iscale_y) < DBL_EPSILON;
    if (is_area_fast && iscale_x == 2 && iscale_y == 2) {
        // INTER_LINEAR with exact 2x downscale is serviced by INTER_AREA fast: 2x2 mean.
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x) {
                const uint8_t* s0 = src + (size_t)(2 * y) * sstep + 2 * x;
                const uint8_t* s1 = s0 + sstep;
                dst[(size_t)y * dstep + x] = (uint8_t)((s0[0] + s0[1] + s1[0] + s1[1] + 2) >> 2);
            }
        return;
    }
    std::vector<int> xofs(dw), yofs(dh);
    std::vector<short> ialpha(2 * dw), ibeta(2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        float cbuf0 = 1.f - fx, cbuf1 = fx;
        ialpha[2 * dx] = sat_short(cbuf0 * INTER_RESIZE_COEF_SCALE);
        ialpha[2 * dx + 1] = sat_short(cbuf1 * INTER_RESIZE_COEF_SCALE);
    }
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        yofs[dy] = sy;
        float cbuf0 = 1.f - fy, cbuf1 = fy;
        ibeta[2 * dy] = sat_short(cbuf0 * INTER_RESIZE_COEF_SCALE);
        ibeta[2 * dy + 1] = sat_short(cbuf1 * INTER_RESIZE_COEF_SCALE);
    }
    auto hresize = [&](int sy, std::vector<int>& D) {
        const uint8_t* S = src + (size_t)sy * sstep;
        int dx = 0;
        for (; dx < xmax; ++dx) {
            int sx = xofs[dx];
            D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
        }
        for (; dx < dw; ++dx) D[dx] = S[xofs[dx]] * INTER_RESIZE_COEF_SCALE;
    };
    std::vector<int> D0(dw), D1(dw);
    const int xs = simd_end(dw);
    for (int dy = 0; dy < dh; ++dy) {
        int sy0 = std::min(std::max(yofs[dy], 0), sh - 1);
        int sy1 = std::min(std::max(yofs[dy] + 1, 0), sh - 1);
        hresize(sy0, D0);
        hresize(sy1, D1);
        int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* out = dst + (size_t)dy * dstep;
        for (int x = 0; x < dw; ++x) {
            if (x < xs) {
                // v_mul_hi(v_pack(S>>4), beta) summed, v_rshr_pack_u<2>.
                int t0 = (int16_t)std::min(D0[x] >> 4, 32767);
                int t1 = (int16_t)std::min(D1[x] >> 4, 32767);
                int s = ((t0 * b0) >> 16) + ((t1 * b1) >> 16);
                s = std::min(std::max(s, -32768), 32767);
                out[x] = sat_u8((s + 2) >> 2);
            } else {
                out[x] = sat_u8((D0[x] * b0 + D1[x] * b1 + (1 << 21)) >> 22);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// cv::GaussianBlur(Size(7,7), 2, 2, BORDER_REFLECT_101) on a non-submatrix CV_8U clone
// (ORBextractor_old.cc:1146-1147): OpenCV's bit-exact fixed-point path.  Kernel = ufixedpoint16
// (8 fractional bits) with error-diffusion rounding; horizontal sums in 8.8, vertical in 16.16,
// final (v + 2^15) >> 16.
void blur_kernel7(int k[7]) {
    const int n = 7;
    const double sigma = 2.0;
    double scale2X = -0.5 / (sigma * sigma);
    double vals[7], sum = 0;
    for (int i = 0; i < n; ++i) {
        double x = i - (n - 1) * 0.5;
        vals[i] = std::exp(scale2X * x * x);
        sum += vals[i];
    }
    for (int i = 0; i < n; ++i) vals[i] /= sum;
    // getGaussianKernelFixedPoint_ED: error diffusion from the tails inwards, centre takes rest.
    double err = 0;
    long s = 0;
    for (int i = 0; i < n / 2; ++i) {
        double adj = vals[i] * 256.0 + err;
        long v0 = std::lrint(adj);
        err = adj - (double)v0;
        k[i] = k[n - 1 - i] = (int)v0;
        s += v0;
    }
    k[n / 2] = (int)(256 - 2 * s);
}

inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

void gaussian_blur(const Plane& src, Plane& dst) {
    int k[7];
    blur_kernel7(k);
    const int w = src.w, h = src.h;
    std::vector<uint32_t> H((size_t)w * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t* s = src.row(y);
        for (int x = 0; x < w; ++x) {
            uint32_t acc = 0;
            for (int u = -3; u <= 3; ++u) acc += (uint32_t)k[u + 3] * s[reflect101(x + u, w)];
            H[(size_t)y * w + x] = acc;  // <= 255*256, fits ufixedpoint16
        }
    }
    dst.w = w, dst.h = h, dst.px.assign((size_t)w * h, 0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            uint64_t acc = 0;
            for (int v = -3; v <= 3; ++v)
                acc += (uint64_t)k[v + 3] * H[(size_t)reflect101(y + v, h) * w + x];
            dst.row(y)[x] = sat_u8((int)((acc + (1u << 15)) >> 16));
        }
}

// ------------------------------------------------------------------------------------------
// cv::FAST(img, kps, threshold, nonmax=true), TYPE_9_16 (OpenCV 4.2 features2d/src/fast.cpp:
// FAST_t<16>, cornerScore<16>, makeOffsets).  Called per cell at ORBextractor_old.cc:828,847.
const int kRing16[16][2] = {{0, 3},  {1, 3},  {2, 2},  {3, 1},  {3, 0},  {3, -1},
                            {2, -2}, {1, -3}, {0, -3}, {-1, -3}, {-2, -2}, {-3, -1},
                            {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

int corner_score16(const uint8_t* ptr, const int pixel[25], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[N];
    for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

void make_offsets(int pixel[25], int step) {
    for (int k = 0; k < 16; ++k) pixel[k] = kRing16[k][0] + kRing16[k][1] * step;
    for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
}

// img points at the ROI origin; rows/cols are the ROI size; step is the parent row stride.
void fast16(const uint8_t* img, int step, int cols, int rows, int threshold,
            std::vector<KeyPoint>& keypoints) {
    const int K = 8, N = 16 + K + 1;
    int pixel[25];
    make_offsets(pixel, step);
    keypoints.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t threshold_tab[512];
    for (int i = -255; i <= 255; i++)
        threshold_tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols < 1) return;
    std::vector<uint8_t> bufs(3 * (size_t)cols, 0);
    std::vector<int> cpb(3 * ((size_t)cols + 1), 0);
    uint8_t* buf[3] = {bufs.data(), bufs.data() + cols, bufs.data() + 2 * cols};
    int* cpbuf[3] = {cpb.data() + 1, cpb.data() + 1 + (cols + 1), cpb.data() + 1 + 2 * (cols + 1)};
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* tab = &threshold_tab[0] - v + 255;
                int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
                d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
                d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
                d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
                d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
                d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                score > curr[j] && score > curr[j + 1]) {
                KeyPoint kp;
                kp.x = (float)j, kp.y = (float)(i - 1), kp.size = 7.f, kp.angle = -1;
                kp.response = (float)score;
                keypoints.push_back(kp);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// cv::fastAtan2 (OpenCV 4.2 core/src/mathfuncs_core.simd.hpp atanImpl<float>), degrees.
const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// IC_Angle (ORBextractor_old.cc:78-105).
float ic_angle(const uint8_t* image, int step, float px, float py, const std::vector<int>& u_max) {
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = image + (size_t)cvRound(py) * step + cvRound(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = u_max[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// 0: cos / sin of computeOrbDescriptor as the reference source calls them (float overloads);
// 1: (float)cos((double)angle) -- only to measure how often the two differ (oracle_set_trig_double).
static int g_trig_double = 0;

// computeOrbDescriptor (ORBextractor_old.cc:108-148).
const float factorPI = (float)(M_PI / 180.f);
void orb_descriptor(const KeyPoint& kpt, const uint8_t* img, int step, const int* pattern,
                    uint8_t* desc) {
    float angle = (float)kpt.angle * factorPI;
    // `(float)cos(angle)` with a float angle under `using namespace std` (:68, :114-115) is the
    // float overload std::cos(float) = libm cosf; g_trig_double selects the double-evaluated
    // alternative for the deviation measurement of tests/test_oracle.py only
    float a, b;
    if (g_trig_double) {
        a = (float)std::cos((double)angle);
        b = (float)std::sin((double)angle);
    } else {
        a = (float)std::cos(angle);
        b = (float)std::sin(angle);
    }
    const uint8_t* center = img + (size_t)cvRound(kpt.y) * step + cvRound(kpt.x);
    auto get = [&](const int* p, int idx) {
        float px = (float)p[2 * idx], py = (float)p[2 * idx + 1];
        float rx = px * b + py * a;   // row offset
        float ry = px * a - py * b;   // column offset
        return (int)center[cvRound(rx) * step + cvRound(ry)];
    };
    const int* pat = pattern;
    for (int i = 0; i < 32; ++i, pat += 32) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
            int t0 = get(pat, 2 * bit), t1 = get(pat, 2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

// ------------------------------------------------------------------------------------------
// ExtractorNode / DistributeOctTree (ORBextractor_old.cc:482-555, 557-781; class at
// cpp/include/ORBextractor_old.h:33-43).
struct IPoint { int x = 0, y = 0; };
struct ExtractorNode {
    std::vector<KeyPoint> vKeys;
    IPoint UL, UR, BL, BR;
    std::list<ExtractorNode>::iterator lit;
    bool bNoMore = false;
    void DivideNode(ExtractorNode& n1, ExtractorNode& n2, ExtractorNode& n3, ExtractorNode& n4);
};

void ExtractorNode::DivideNode(ExtractorNode& n1, ExtractorNode& n2, ExtractorNode& n3,
                               ExtractorNode& n4) {
    const int halfX = (int)std::ceil(static_cast<float>(UR.x - UL.x) / 2);
    const int halfY = (int)std::ceil(static_cast<float>(BR.y - UL.y) / 2);
    n1.UL = UL;
    n1.UR = {UL.x + halfX, UL.y};
    n1.BL = {UL.x, UL.y + halfY};
    n1.BR = {UL.x + halfX, UL.y + halfY};
    n2.UL = n1.UR;
    n2.UR = UR;
    n2.BL = n1.BR;
    n2.BR = {UR.x, UL.y + halfY};
    n3.UL = n1.BL;
    n3.UR = n1.BR;
    n3.BL = BL;
    n3.BR = {n1.BR.x, BL.y};
    n4.UL = n3.UR;
    n4.UR = n2.BR;
    n4.BL = n3.BR;
    n4.BR = BR;
    for (size_t i = 0; i < vKeys.size(); i++) {
        const KeyPoint& kp = vKeys[i];
        if (kp.x < n1.UR.x) {
            if (kp.y < n1.BR.y) n1.vKeys.push_back(kp);
            else n3.vKeys.push_back(kp);
        } else if (kp.y < n1.BR.y)
            n2.vKeys.push_back(kp);
        else
            n4.vKeys.push_back(kp);
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

bool compareNodes(std::pair<int, ExtractorNode*>& e1, std::pair<int, ExtractorNode*>& e2) {
    if (e1.first < e2.first) return true;
    if (e1.first > e2.first) return false;
    return e1.second->UL.x < e2.second->UL.x;
}

void push_children(std::list<ExtractorNode>& lNodes, ExtractorNode* ch[4],
                   std::vector<std::pair<int, ExtractorNode*>>& vSize, int* nToExpand) {
    for (int c = 0; c < 4; ++c) {
        ExtractorNode& n = *ch[c];
        if (n.vKeys.size() > 0) {
            lNodes.push_front(n);
            if (n.vKeys.size() > 1) {
                if (nToExpand) (*nToExpand)++;
                vSize.push_back(std::make_pair((int)n.vKeys.size(), &lNodes.front()));
                lNodes.front().lit = lNodes.begin();
            }
        }
    }
}

std::vector<KeyPoint> distribute_octree(const std::vector<KeyPoint>& vToDistributeKeys,
                                        int minX, int maxX, int minY, int maxY, int N) {
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::list<ExtractorNode> lNodes;
    std::vector<ExtractorNode*> vpIniNodes(nIni);
    for (int i = 0; i < nIni; i++) {
        ExtractorNode ni;
        ni.UL = {(int)(hX * static_cast<float>(i)), 0};
        ni.UR = {(int)(hX * static_cast<float>(i + 1)), 0};
        ni.BL = {ni.UL.x, maxY - minY};
        ni.BR = {ni.UR.x, maxY - minY};
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (size_t i = 0; i < vToDistributeKeys.size(); i++) {
        const KeyPoint& kp = vToDistributeKeys[i];
        vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
    }
    auto lit = lNodes.begin();
    while (lit != lNodes.end()) {
        if (lit->vKeys.size() == 1) {
            lit->bNoMore = true;
            lit++;
        } else if (lit->vKeys.empty())
            lit = lNodes.erase(lit);
        else
            lit++;
    }
    bool bFinish = false;
    std::vector<std::pair<int, ExtractorNode*>> vSizeAndPointerToNode;
    while (!bFinish) {
        int prevSize = (int)lNodes.size();
        lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) {
                lit++;
                continue;
            }
            ExtractorNode n1, n2, n3, n4;
            lit->DivideNode(n1, n2, n3, n4);
            ExtractorNode* ch[4] = {&n1, &n2, &n3, &n4};
            push_children(lNodes, ch, vSizeAndPointerToNode, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                std::vector<std::pair<int, ExtractorNode*>> vPrev = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                std::sort(vPrev.begin(), vPrev.end(), compareNodes);
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    ExtractorNode n1, n2, n3, n4;
                    vPrev[j].second->DivideNode(n1, n2, n3, n4);
                    ExtractorNode* ch[4] = {&n1, &n2, &n3, &n4};
                    push_children(lNodes, ch, vSizeAndPointerToNode, nullptr);
                    lNodes.erase(vPrev[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<KeyPoint> vResultKeys;
    for (auto it = lNodes.begin(); it != lNodes.end(); it++) {
        std::vector<KeyPoint>& vNodeKeys = it->vKeys;
        KeyPoint* pKP = &vNodeKeys[0];
        float maxResponse = pKP->response;
        for (size_t k = 1; k < vNodeKeys.size(); k++)
            if (vNodeKeys[k].response > maxResponse) {
                pKP = &vNodeKeys[k];
                maxResponse = vNodeKeys[k].response;
            }
        vResultKeys.push_back(*pKP);
    }
    return vResultKeys;
}

// ------------------------------------------------------------------------------------------
// ORBextractor (ORBextractor_old.cc:411-471, 783-898, 1088-1191, canonical pyramid 1331-1356).
struct Extractor {
    int nfeatures;
    double scaleFactor;
    int nlevels, iniThFAST, minThFAST;
    std::vector<int> mnFeaturesPerLevel, umax, pattern;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    std::vector<Plane> mvImagePyramid;

    Extractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
        : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels),
          iniThFAST(_iniThFAST), minThFAST(_minThFAST) {
        mvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvScaleFactor[0] = 1.0f;
        mvLevelSigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
            mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
        }
        mvInvScaleFactor.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        for (int i = 0; i < nlevels; i++) {
            mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
            mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
        }
        mvImagePyramid.resize(nlevels);
        mnFeaturesPerLevel.resize(nlevels);
        float factor = (float)(1.0f / scaleFactor);
        float nDesiredFeaturesPerScale =
            nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
        int sumFeatures = 0;
        for (int level = 0; level < nlevels - 1; level++) {
            mnFeaturesPerLevel[level] = cvRound(nDesiredFeaturesPerScale);
            sumFeatures += mnFeaturesPerLevel[level];
            nDesiredFeaturesPerScale *= factor;
        }
        mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sumFeatures, 0);
        pattern = pattern_table();
        umax.resize(HALF_PATCH_SIZE + 1);
        int v, v0, vmax = cvFloor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
        int vmin = cvCeil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
        const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
        for (v = 0; v <= vmax; ++v) umax[v] = cvRound(std::sqrt(hp2 - v * v));
        for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    void ComputePyramid(const uint8_t* img, int w, int h, int stride) {
        for (int level = 0; level < nlevels; ++level) {
            float scale = mvInvScaleFactor[level];
            int sw = cvRound((float)w * scale), sh = cvRound((float)h * scale);
            Plane& P = mvImagePyramid[level];
            P.w = sw, P.h = sh, P.px.assign((size_t)sw * sh, 0);
            if (level != 0) {
                const Plane& S = mvImagePyramid[level - 1];
                resize_linear(S.px.data(), S.w, S.h, S.w, P.px.data(), sw, sh, sw);
            } else {
                for (int y = 0; y < h; ++y) memcpy(P.row(y), img + (size_t)y * stride, w);
            }
        }
    }

    // The per-cell FAST loop of ComputeKeyPointsOctTree (:787-874).
    std::vector<KeyPoint> LevelCandidates(const Plane& P, int* minBX, int* maxBX, int* minBY,
                                          int* maxBY) const {
        const float W = 35;
        const int minBorderX = EDGE_THRESHOLD - 3;
        const int minBorderY = minBorderX;
        const int maxBorderX = P.w - EDGE_THRESHOLD + 3;
        const int maxBorderY = P.h - EDGE_THRESHOLD + 3;
        *minBX = minBorderX, *maxBX = maxBorderX, *minBY = minBorderY, *maxBY = maxBorderY;
        std::vector<KeyPoint> vToDistributeKeys;
        const float width = (maxBorderX - minBorderX);
        const float height = (maxBorderY - minBorderY);
        const int nCols = (int)(width / W);
        const int nRows = (int)(height / W);
        const int wCell = (int)std::ceil(width / nCols);
        const int hCell = (int)std::ceil(height / nRows);
        for (int i = 0; i < nRows; i++) {
            const float iniY = minBorderY + i * hCell;
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = minBorderX + j * wCell;
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = maxBorderX;
                std::vector<KeyPoint> vKeysCell;
                const int y0 = (int)iniY, x0 = (int)iniX;
                const int rows = (int)maxY - y0, cols = (int)maxX - x0;
                const uint8_t* roi = P.px.data() + (size_t)y0 * P.w + x0;
                fast16(roi, P.w, cols, rows, iniThFAST, vKeysCell);
                if (vKeysCell.empty()) fast16(roi, P.w, cols, rows, minThFAST, vKeysCell);
                for (auto& kp : vKeysCell) {
                    kp.x += j * wCell;
                    kp.y += i * hCell;
                    vToDistributeKeys.push_back(kp);
                }
            }
        }
        return vToDistributeKeys;
    }

    void ComputeKeyPointsOctTree(std::vector<std::vector<KeyPoint>>& allKeypoints) {
        allKeypoints.resize(nlevels);
        for (int level = 0; level < nlevels; ++level) {
            int minBorderX, maxBorderX, minBorderY, maxBorderY;
            std::vector<KeyPoint> cand = LevelCandidates(mvImagePyramid[level], &minBorderX,
                                                         &maxBorderX, &minBorderY, &maxBorderY);
            std::vector<KeyPoint>& keypoints = allKeypoints[level];
            keypoints = distribute_octree(cand, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                          mnFeaturesPerLevel[level]);
            const int scaledPatchSize = (int)(PATCH_SIZE * mvScaleFactor[level]);
            for (auto& kp : keypoints) {
                kp.x += minBorderX;
                kp.y += minBorderY;
                kp.octave = level;
                kp.size = (float)scaledPatchSize;
            }
        }
        for (int level = 0; level < nlevels; ++level) {
            const Plane& P = mvImagePyramid[level];
            for (auto& kp : allKeypoints[level])
                kp.angle = ic_angle(P.px.data(), P.w, kp.x, kp.y, umax);
        }
    }
};

oracle_kp to_c(const KeyPoint& k) {
    oracle_kp o;
    o.x = k.x, o.y = k.y, o.size = k.size, o.angle = k.angle, o.response = k.response;
    o.octave = k.octave, o.class_id = k.class_id;
    return o;
}
KeyPoint from_c(const oracle_kp& o) {
    KeyPoint k;
    k.x = o.x, k.y = o.y, k.size = o.size, k.angle = o.angle, k.response = o.response;
    k.octave = o.octave, k.class_id = o.class_id;
    return k;
}

}  // namespace

// ============================================================================================
extern "C" {

int oracle_resize_simd_end(int width) { return simd_end(width); }
void oracle_blur_kernel(int32_t k[7]) {
    int kk[7];
    blur_kernel7(kk);
    for (int i = 0; i < 7; ++i) k[i] = kk[i];
}

void oracle_level_sizes(float scale_factor, int nlevels, int w, int h, int* lw, int* lh) {
    Extractor e(1000, scale_factor, nlevels, 20, 7);
    for (int l = 0; l < nlevels; ++l) {
        lw[l] = cvRound((float)w * e.mvInvScaleFactor[l]);
        lh[l] = cvRound((float)h * e.mvInvScaleFactor[l]);
    }
}

int oracle_pyramid(float scale_factor, int nlevels, const uint8_t* img, int w, int h, int stride,
                   uint8_t* out) {
    Extractor e(1000, scale_factor, nlevels, 20, 7);
    e.ComputePyramid(img, w, h, stride);
    size_t off = 0;
    for (int l = 0; l < nlevels; ++l) {
        memcpy(out + off, e.mvImagePyramid[l].px.data(), e.mvImagePyramid[l].px.size());
        off += e.mvImagePyramid[l].px.size();
    }
    return (int)off;
}

void oracle_resize(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                   int dstride) {
    resize_linear(src, sw, sh, sstride, dst, dw, dh, dstride);
}

void oracle_gaussian_blur(const uint8_t* src, int w, int h, uint8_t* dst) {
    Plane s, d;
    s.w = w, s.h = h, s.px.assign(src, src + (size_t)w * h);
    gaussian_blur(s, d);
    memcpy(dst, d.px.data(), (size_t)w * h);
}

int oracle_fast(const uint8_t* img, int stride, int x0, int y0, int cols, int rows, int th,
                oracle_kp* kps, int cap) {
    std::vector<KeyPoint> v;
    fast16(img + (size_t)y0 * stride + x0, stride, cols, rows, th, v);
    int n = (int)v.size();
    for (int i = 0; i < n && i < cap; ++i) kps[i] = to_c(v[i]);
    return n;
}

int oracle_corner_score(const uint8_t* img, int stride, int x, int y, int th) {
    int pixel[25];
    make_offsets(pixel, stride);
    return corner_score16(img + (size_t)y * stride + x, pixel, th);
}

int oracle_level_candidates(const uint8_t* lvl, int w, int h, int ini_th, int min_th,
                            oracle_kp* kps, int cap) {
    Extractor e(1000, 1.2f, 1, ini_th, min_th);
    Plane P;
    P.w = w, P.h = h, P.px.assign(lvl, lvl + (size_t)w * h);
    int a, b, c, d;
    std::vector<KeyPoint> v = e.LevelCandidates(P, &a, &b, &c, &d);
    int n = (int)v.size();
    for (int i = 0; i < n && i < cap; ++i) kps[i] = to_c(v[i]);
    return n;
}

int oracle_distribute_octree(const oracle_kp* keys, int n, int minX, int maxX, int minY, int maxY,
                             int N, oracle_kp* out, int cap) {
    std::vector<KeyPoint> v(n);
    for (int i = 0; i < n; ++i) v[i] = from_c(keys[i]);
    std::vector<KeyPoint> r = distribute_octree(v, minX, maxX, minY, maxY, N);
    int m = (int)r.size();
    for (int i = 0; i < m && i < cap; ++i) out[i] = to_c(r[i]);
    return m;
}

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }

float oracle_ic_angle(const uint8_t* img, int stride, int x, int y) {
    Extractor e(1000, 1.2f, 1, 20, 7);
    return ic_angle(img, stride, (float)x, (float)y, e.umax);
}

void oracle_orb_descriptor(const uint8_t* blurred, int stride, float x, float y, float angle,
                           uint8_t* desc32) {
    KeyPoint k;
    k.x = x, k.y = y, k.angle = angle;
    std::vector<int> pat = pattern_table();
    orb_descriptor(k, blurred, stride, pat.data(), desc32);
}

void oracle_umax(int* umax16) {
    Extractor e(1000, 1.2f, 1, 20, 7);
    for (int i = 0; i < 16; ++i) umax16[i] = e.umax[i];
}

void oracle_features_per_level(int nfeatures, float scale_factor, int nlevels, int* out) {
    Extractor e(nfeatures, scale_factor, nlevels, 20, 7);
    for (int i = 0; i < nlevels; ++i) out[i] = e.mnFeaturesPerLevel[i];
}

void oracle_scale_factors(float scale_factor, int nlevels, float* scale, float* inv_scale,
                          float* sigma2, float* inv_sigma2) {
    Extractor e(1000, scale_factor, nlevels, 20, 7);
    for (int i = 0; i < nlevels; ++i) {
        scale[i] = e.mvScaleFactor[i];
        inv_scale[i] = e.mvInvScaleFactor[i];
        sigma2[i] = e.mvLevelSigma2[i];
        inv_sigma2[i] = e.mvInvLevelSigma2[i];
    }
}

int oracle_extract_levels(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                          const uint8_t* img, int w, int h, int stride, oracle_kp* kps,
                          uint8_t* desc, int cap, int* lvl_count) {
    if (!img || w <= 0 || h <= 0) return -1;
    Extractor e(nfeatures, scale_factor, nlevels, ini_th, min_th);
    e.ComputePyramid(img, w, h, stride);
    std::vector<std::vector<KeyPoint>> all;
    e.ComputeKeyPointsOctTree(all);
    int off = 0;
    for (int level = 0; level < nlevels; ++level) {
        Plane blurred;
        gaussian_blur(e.mvImagePyramid[level], blurred);
        lvl_count[level] = (int)all[level].size();
        for (auto& kp : all[level]) {
            if (off >= cap) return -2;
            kps[off] = to_c(kp);
            orb_descriptor(kp, blurred.px.data(), blurred.w, e.pattern.data(), desc + 32 * off);
            ++off;
        }
    }
    return off;
}

int oracle_extract(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                   const uint8_t* img, int w, int h, int stride, int lap0, int lap1,
                   oracle_kp* out_kps, uint8_t* out_desc, int cap, int* n_out) {
    *n_out = 0;
    if (!img || w <= 0 || h <= 0) return -1;  // :1092-1093
    Extractor e(nfeatures, scale_factor, nlevels, ini_th, min_th);
    e.ComputePyramid(img, w, h, stride);
    std::vector<std::vector<KeyPoint>> allKeypoints;
    e.ComputeKeyPointsOctTree(allKeypoints);
    int nkeypoints = 0;
    for (int level = 0; level < nlevels; ++level) nkeypoints += (int)allKeypoints[level].size();
    if (nkeypoints > cap) return -2;
    *n_out = nkeypoints;
    int monoIndex = 0, stereoIndex = nkeypoints - 1;
    for (int level = 0; level < nlevels; ++level) {
        std::vector<KeyPoint>& keypoints = allKeypoints[level];
        int nkeypointsLevel = (int)keypoints.size();
        if (nkeypointsLevel == 0) continue;
        Plane workingMat;
        gaussian_blur(e.mvImagePyramid[level], workingMat);
        std::vector<uint8_t> desc((size_t)nkeypointsLevel * 32);
        for (int i = 0; i < nkeypointsLevel; ++i)
            orb_descriptor(keypoints[i], workingMat.px.data(), workingMat.w, e.pattern.data(),
                           desc.data() + 32 * i);
        float scale = e.mvScaleFactor[level];
        int i = 0;
        for (auto& kp : keypoints) {
            if (level != 0) {
                kp.x *= scale;
                kp.y *= scale;
            }
            int dst;
            if (kp.x >= lap0 && kp.x <= lap1) dst = stereoIndex--;
            else dst = monoIndex++;
            out_kps[dst] = to_c(kp);
            memcpy(out_desc + 32 * dst, desc.data() + 32 * i, 32);
            i++;
        }
    }
    return monoIndex;
}

int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    // SWAR popcount over 8 int32 words (ORBmatcher.cc:2107-2123).
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        uint32_t v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

// The CPU baseline's frames-parallel pool (SURVEY §8d mode 3): n_images frames of w x h (pitch w)
// extracted by `nthreads` std::threads, each taking the next frame from a shared counter; per-frame
// keypoint counts out.  Returns the total keypoint count (< 0 on an error).
long long oracle_extract_many(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                              const uint8_t* imgs, int n_images, int w, int h, int nthreads, int32_t* counts) {
    if (!imgs || n_images < 0 || nthreads < 1) return -1;
    std::atomic<int> next{0};
    std::atomic<long long> total{0};
    std::atomic<int> err{0};
    auto work = [&] {
        const int cap = 4 * nfeatures + 64 * nlevels + 4096;
        std::vector<oracle_kp> kps(cap);
        std::vector<uint8_t> desc((size_t)cap * 32);
        for (int i = next++; i < n_images; i = next++) {
            int n = 0;
            const int r = oracle_extract(nfeatures, scale_factor, nlevels, ini_th, min_th, imgs + (size_t)i * w * h, w,
                                         h, w, 0, 0, kps.data(), desc.data(), cap, &n);
            if (r < 0) err = r;
            if (counts) counts[i] = n;
            total += n;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    return err ? (long long)err : total.load();
}

void oracle_set_trig_double(int on) { g_trig_double = on ? 1 : 0; }

void oracle_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx1, int32_t* d1,
                 int32_t* idx2, int32_t* d2) {
    // cv::batchDistance(K=2, NORM_HAMMING) insertion rule; knnMatch drops idx<0 entries.
    for (int i = 0; i < nq; ++i) {
        int dist[2] = {INT_MAX, INT_MAX}, nidx[2] = {-1, -1};
        for (int j = 0; j < nt; ++j) {
            int d = oracle_descriptor_distance(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (d < dist[1]) {
                int k;
                for (k = 0; k >= 0 && dist[k] > d; k--) {
                    nidx[k + 1] = nidx[k];
                    dist[k + 1] = dist[k];
                }
                nidx[k + 1] = j;
                dist[k + 1] = d;
            }
        }
        idx1[i] = nidx[0], d1[i] = dist[0], idx2[i] = nidx[1], d2[i] = dist[1];
    }
}

void oracle_sort_nodes(const int32_t* size, const int32_t* ulx, int n, int32_t* perm) {
    std::vector<ExtractorNode> nodes(n);
    std::vector<std::pair<int, ExtractorNode*>> v(n);
    for (int i = 0; i < n; ++i) {
        nodes[i].UL.x = ulx[i];
        v[i] = std::make_pair((int)size[i], &nodes[i]);
    }
    std::sort(v.begin(), v.end(), compareNodes);
    for (int i = 0; i < n; ++i) perm[i] = (int32_t)(v[i].second - nodes.data());
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Frame::ComputeStereoMatches (cpp/src/Frame.cc:827-997), restated line by line for one rectified
// stereo frame.  kpsL/kpsR are the extractor outputs (mvKeys / mvKeysRight, level-0 coordinates),
// descL/descR their descriptors, pyrL/pyrR the UNBLURRED pyramids (mvImagePyramid, level l at
// pyr[l], lw[l] x lh[l], pitch lw[l]), scale/inv_scale = mvScaleFactors / mvInvScaleFactors.
// Writes mvuRight / mvDepth (-1 = no stereo match) and, for tests, the SAD distance of each
// accepted match in sad[] (-1 otherwise; entries later rejected by the median rule keep theirs).
// Float expressions are evaluated in source order without contraction (-ffp-contract=off).
void oracle_stereo_matches(const oracle_kp* kpsL, int nL, const uint8_t* descL, const oracle_kp* kpsR,
                           int nR, const uint8_t* descR, const uint8_t* const* pyrL,
                           const uint8_t* const* pyrR, const int* lw, const int* lh, int nlevels,
                           const float* scale, const float* inv_scale, float mbf, float mb,
                           float* uRight, float* depth, int32_t* sad) {
    (void)nlevels;
    for (int i = 0; i < nL; ++i) uRight[i] = -1.0f, depth[i] = -1.0f, sad[i] = -1;
    const int TH_HIGH = 100, TH_LOW = 50;       // ORBmatcher.cc:36-37
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
    const int nRows = lh[0];
    // :842-855 row table (rows outside the image are dropped: the reference writes past the
    // table there, which our keypoints never reach)
    std::vector<std::vector<size_t>> vRowIndices(nRows);
    for (int iR = 0; iR < nR; iR++) {
        const oracle_kp& kp = kpsR[iR];
        const float& kpY = kp.y;
        const float r = 2.0f * scale[kp.octave];
        const int maxr = (int)std::ceil(kpY + r);
        const int minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) vRowIndices[yi].push_back(iR);
    }
    const float minZ = mb;
    const float minD = 0;
    const float maxD = mbf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    for (int iL = 0; iL < nL; iL++) {
        const oracle_kp& kpL = kpsL[iL];
        const int& levelL = kpL.octave;
        const float& vL = kpL.y;
        const float& uL = kpL.x;
        const size_t row = (size_t)vL;
        if (row >= (size_t)nRows) continue;
        const std::vector<size_t>& vCandidates = vRowIndices[row];
        if (vCandidates.empty()) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        size_t bestIdxR = 0;
        const uint8_t* dL = descL + 32 * (size_t)iL;
        for (size_t iC = 0; iC < vCandidates.size(); iC++) {
            const size_t iR = vCandidates[iC];
            const oracle_kp& kpR = kpsR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float& uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = oracle_descriptor_distance(dL, descR + 32 * iR);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist < thOrbDist) {
            const float uR0 = kpsR[bestIdxR].x;
            const float scaleFactor = inv_scale[kpL.octave];
            const float scaleduL = std::round(kpL.x * scaleFactor);
            const float scaledvL = std::round(kpL.y * scaleFactor);
            const float scaleduR0 = std::round(uR0 * scaleFactor);
            const int w = 5;
            const int lvl = kpL.octave, W = lw[lvl], H = lh[lvl];
            const int r0 = (int)scaledvL - w, c0 = (int)scaleduL - w;
            int sadBest = INT_MAX;
            int bestincR = 0;
            const int L = 5;
            float vDists[2 * L + 1];
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= W) continue;
            // cv::Mat rowRange/colRange would assert outside the level; never reached here
            if (r0 < 0 || r0 + 2 * w + 1 > H || c0 < 0 || c0 + 2 * w + 1 > W || (int)scaleduR0 - L - w < 0) continue;
            for (int incR = -L; incR <= +L; incR++) {
                const int cr = (int)scaleduR0 + incR - w;
                int s = 0;  // cv::norm(IL, IR, NORM_L1): exact integer sum, returned as double
                for (int y = 0; y < 2 * w + 1; ++y)
                    for (int x = 0; x < 2 * w + 1; ++x)
                        s += std::abs((int)pyrL[lvl][(size_t)(r0 + y) * W + c0 + x] -
                                      (int)pyrR[lvl][(size_t)(r0 + y) * W + cr + x]);
                const float dist = (float)(double)s;
                if (dist < sadBest) {
                    sadBest = (int)dist;
                    bestincR = incR;
                }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[L + bestincR - 1];
            const float dist2 = vDists[L + bestincR];
            const float dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01;
                    bestuR = uL - 0.01;
                }
                depth[iL] = mbf / disparity;
                uRight[iL] = bestuR;
                sad[iL] = sadBest;
                vDistIdx.push_back(std::pair<int, int>(sadBest, iL));
            }
        }
    }
    if (vDistIdx.empty()) return;  // the reference reads vDistIdx[0] of an empty vector here
    std::sort(vDistIdx.begin(), vDistIdx.end());
    const float median = vDistIdx[vDistIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
        if (vDistIdx[i].first < thDist)
            break;
        else {
            uRight[vDistIdx[i].second] = -1;
            depth[vDistIdx[i].second] = -1;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Frame::UndistortKeyPoints (cpp/src/Frame.cc:763-796) -> cv::undistortPoints(src, dst, K, D,
// noArray(), K) [EXT: OpenCV 4.2 cvUndistortPointsInternal, TermCriteria(COUNT, 5, 0.01)], in
// double with the operation order of that function (identity tilt and rectification folded: the
// products with 1 / 0 they add are exact), no FMA contraction.  dist = k1 k2 p1 p2 [k3].
static void undistort_point(float px, float py, const float K[4], const double k[14], float* ox, float* oy) {
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    double x = px, y = py;
    const double u = x, v = y;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {  // undistortPoints.regression_14583
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // P = K, R = I: xx = fx*x + 0*y + cx, ww = 1/(0*x + 0*y + 1) = 1
    const double xx = fx * x + 0. * y + cx;
    const double yy = 0. * x + fy * y + cy;
    const double ww = 1. / (0. * x + 0. * y + 1.);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

static void dist_table(const float* dist, int ndist, double k[14]) {
    for (int i = 0; i < 14; ++i) k[i] = 0;
    for (int i = 0; i < ndist && i < 5; ++i) k[i] = dist[i];
}

void oracle_undistort_points(const float* xy, int n, const float K[4], const float* dist, int ndist, float* out) {
    double k[14];
    dist_table(dist, ndist, k);
    for (int i = 0; i < n; ++i) {
        if (ndist == 0 || dist[0] == 0.0f) {  // Frame.cc:765-769: mvKeysUn = mvKeys
            out[2 * i] = xy[2 * i];
            out[2 * i + 1] = xy[2 * i + 1];
        } else {
            undistort_point(xy[2 * i], xy[2 * i + 1], K, k, &out[2 * i], &out[2 * i + 1]);
        }
    }
}

// Frame::ComputeImageBounds (Frame.cc:798-825): the undistorted image corners.
void oracle_image_bounds(int cols, int rows, const float K[4], const float* dist, int ndist, float bounds[4]) {
    if (ndist > 0 && dist[0] != 0.0f) {
        const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float u[8];
        oracle_undistort_points(c, 4, K, dist, ndist, u);
        bounds[0] = std::min(u[0], u[4]);  // mnMinX
        bounds[1] = std::max(u[2], u[6]);  // mnMaxX
        bounds[2] = std::min(u[1], u[3]);  // mnMinY
        bounds[3] = std::max(u[5], u[7]);  // mnMaxY
    } else {
        bounds[0] = 0.0f;
        bounds[1] = (float)cols;
        bounds[2] = 0.0f;
        bounds[3] = (float)rows;
    }
}

// Frame::AssignFeaturesToGrid + PosInGrid (Frame.cc:405-436, 741-751), FRAME_GRID_COLS x ROWS =
// 64 x 48 (Frame.h:46-47), on undistorted points: cell[i] = posX * 48 + posY or -1;
// cell_start[64*48 + 1] / cell_idx: the mGrid[posX][posY] vectors, indices ascending.
void oracle_assign_grid(const float* xy_un, int n, const float bounds[4], int32_t* cell, int32_t* cell_start,
                        int32_t* cell_idx) {
    const int GC = 64, GR = 48;
    const float wInv = static_cast<float>(GC) / (bounds[1] - bounds[0]);
    const float hInv = static_cast<float>(GR) / (bounds[3] - bounds[2]);
    std::vector<std::vector<int>> grid((size_t)GC * GR);
    for (int i = 0; i < n; ++i) {
        const int posX = (int)std::round((xy_un[2 * i] - bounds[0]) * wInv);
        const int posY = (int)std::round((xy_un[2 * i + 1] - bounds[2]) * hInv);
        if (posX < 0 || posX >= GC || posY < 0 || posY >= GR) {
            cell[i] = -1;
            continue;
        }
        cell[i] = posX * GR + posY;
        grid[(size_t)posX * GR + posY].push_back(i);
    }
    int o = 0;
    for (int c = 0; c < GC * GR; ++c) {
        cell_start[c] = o;
        for (int i : grid[c]) cell_idx[o++] = i;
    }
    cell_start[GC * GR] = o;
}

// IDL SoA egress (see the header): the host-side restatement of what the device packs.
void oracle_pack_soa(const oracle_kp* kps, int n, int32_t* x, int32_t* y, int32_t* angle, int32_t* level) {
    for (int i = 0; i < n; ++i) {
        const float rad = (float)kps[i].angle * factorPI;
        const float a = (float)std::cos(rad), b = (float)std::sin(rad);  // as the descriptor
        const int c8 = (int)std::nearbyint(64.0f * a), s8 = (int)std::nearbyint(64.0f * b);
        x[i] = (int32_t)kps[i].x;
        y[i] = (int32_t)kps[i].y;
        angle[i] = (c8 & 0xFF) | ((s8 & 0xFF) << 8);
        level[i] = kps[i].octave;
    }
}

// ---- ORBmatcher::SearchByProjection (ORBmatcher.cc:44-214), pinhole frame ---------------------
namespace {

// Frame::GetFeaturesInArea (Frame.cc:673-735) on the CSR grid.
void features_in_area(const float* xy_un, const int32_t* octave, const float bounds[4], const int32_t* cs,
                      const int32_t* ci, float x, float y, float r, int minLevel, int maxLevel,
                      std::vector<int>& out) {
    out.clear();
    const float wInv = static_cast<float>(64) / (bounds[1] - bounds[0]);
    const float hInv = static_cast<float>(48) / (bounds[3] - bounds[2]);
    const int nMinCellX = std::max(0, (int)std::floor((x - bounds[0] - r) * wInv));
    if (nMinCellX >= 64) return;
    const int nMaxCellX = std::min(63, (int)std::ceil((x - bounds[0] + r) * wInv));
    if (nMaxCellX < 0) return;
    const int nMinCellY = std::max(0, (int)std::floor((y - bounds[2] - r) * hInv));
    if (nMinCellY >= 48) return;
    const int nMaxCellY = std::min(47, (int)std::ceil((y - bounds[2] + r) * hInv));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
            for (int j = cs[ix * 48 + iy]; j < cs[ix * 48 + iy + 1]; j++) {
                const int k = ci[j];
                if (bCheckLevels) {
                    if (octave[k] < minLevel) continue;
                    if (maxLevel >= 0 && octave[k] > maxLevel) continue;
                }
                const float distx = xy_un[2 * k] - x, disty = xy_un[2 * k + 1] - y;
                if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(k);
            }
}

}  // namespace

int oracle_search_by_projection(const oracle_map_point* mps, int nmp, const float* xy_un, const int32_t* octave,
                                const uint8_t* desc, const float* uRight, int n, const float bounds[4],
                                const int32_t* cell_start, const int32_t* cell_idx, const float* scale,
                                int nlevels, const uint8_t* kp_block, float th, float nnratio,
                                int far_points, float th_far, int32_t* match) {
    std::vector<uint8_t> blocked(n, 0);
    if (kp_block) std::copy(kp_block, kp_block + n, blocked.begin());
    for (int k = 0; k < n; ++k) match[k] = -1;
    const bool bFactor = th != 1.0;
    std::vector<int> cand;
    int nmatches = 0;
    for (int i = 0; i < nmp; ++i) {
        const oracle_map_point& mp = mps[i];
        if (!(mp.flags & ORACLE_MP_IN_VIEW)) continue;
        if (far_points && mp.depth > th_far) continue;
        if (mp.flags & ORACLE_MP_BAD) continue;
        const int lvl = mp.level;
        if (lvl < 0 || lvl >= nlevels) continue;  // PredictScale never leaves [0, nlevels)
        float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:216-222)
        if (bFactor) r *= th;
        const float rs = r * scale[lvl];
        features_in_area(xy_un, octave, bounds, cell_start, cell_idx, mp.proj_x, mp.proj_y, rs, lvl - 1, lvl, cand);
        if (cand.empty()) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int idx : cand) {
            if (blocked[idx]) continue;
            if (uRight && uRight[idx] > 0) {
                const float er = std::fabs(mp.proj_xr - uRight[idx]);
                if (er > r * scale[lvl]) continue;
            }
            const int dist = oracle_descriptor_distance(mp.desc, desc + (size_t)idx * 32);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = octave[idx];
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = octave[idx];
                bestDist2 = dist;
            }
        }
        if (bestDist <= 100) {  // TH_HIGH
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                match[bestIdx] = i;
                blocked[bestIdx] = (mp.flags & ORACLE_MP_HAS_OBS) ? 1 : 0;
                nmatches++;
            }
        }
    }
    return nmatches;
}

int oracle_search_by_projection2(const oracle_map_point* mps, int nmp, const float* xyL, const int32_t* octL,
                                 const uint8_t* descL, int nl, const int32_t* csL, const int32_t* ciL,
                                 const float* xyR, const int32_t* octR, const uint8_t* descR, int nr,
                                 const int32_t* csR, const int32_t* ciR, const float bounds[4],
                                 const int32_t* l2r, const int32_t* r2l, const float* scale, int nlevels,
                                 const uint8_t* kp_block, float th, float nnratio, int far_points,
                                 float th_far, int32_t* match) {
    const int n = nl + nr;
    std::vector<uint8_t> blocked(n, 0);  // mvpMapPoints[k] set with Observations() > 0
    if (kp_block) std::copy(kp_block, kp_block + n, blocked.begin());
    for (int k = 0; k < n; ++k) match[k] = -1;
    auto assign = [&](int k, int i, const oracle_map_point& mp) {
        match[k] = i;
        blocked[k] = (mp.flags & ORACLE_MP_HAS_OBS) ? 1 : 0;
    };
    const bool bFactor = th != 1.0;
    std::vector<int> cand;
    int nmatches = 0;
    for (int i = 0; i < nmp; ++i) {
        const oracle_map_point& mp = mps[i];
        if (!(mp.flags & ORACLE_MP_IN_VIEW) && !(mp.flags & ORACLE_MP_IN_VIEW_R)) continue;
        if (far_points && mp.depth > th_far) continue;
        if (mp.flags & ORACLE_MP_BAD) continue;
        if (mp.flags & ORACLE_MP_IN_VIEW) {
            const int lvl = mp.level;
            if (lvl >= 0 && lvl < nlevels) {
                float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;
                if (bFactor) r *= th;
                features_in_area(xyL, octL, bounds, csL, ciL, mp.proj_x, mp.proj_y, r * scale[lvl], lvl - 1, lvl, cand);
                if (!cand.empty()) {
                    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                    for (int idx : cand) {
                        if (blocked[idx]) continue;
                        const int dist = oracle_descriptor_distance(mp.desc, descL + (size_t)idx * 32);
                        if (dist < bestDist) {
                            bestDist2 = bestDist;
                            bestDist = dist;
                            bestLevel2 = bestLevel;
                            bestLevel = octL[idx];
                            bestIdx = idx;
                        } else if (dist < bestDist2) {
                            bestLevel2 = octL[idx];
                            bestDist2 = dist;
                        }
                    }
                    if (bestDist <= 100) {
                        if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;  // skips the right branch too
                        if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                            assign(bestIdx, i, mp);
                            if (l2r && l2r[bestIdx] != -1) {
                                assign(l2r[bestIdx] + nl, i, mp);
                                nmatches++;
                            }
                            nmatches++;
                        }
                    }
                }
            }
        }
        if (mp.flags & ORACLE_MP_IN_VIEW_R) {
            const int lvl = mp.level_r;
            if (lvl != -1 && lvl >= 0 && lvl < nlevels) {
                const float r = mp.view_cos_r > 0.998 ? 2.5f : 4.0f;
                features_in_area(xyR, octR, bounds, csR, ciR, mp.proj_xr, mp.proj_yr, r * scale[lvl], lvl - 1, lvl, cand);
                if (cand.empty()) continue;
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (int idx : cand) {
                    if (blocked[idx + nl]) continue;
                    const int dist = oracle_descriptor_distance(mp.desc, descR + (size_t)idx * 32);
                    if (dist < bestDist) {
                        bestDist2 = bestDist;
                        bestDist = dist;
                        bestLevel2 = bestLevel;
                        bestLevel = octR[idx];
                        bestIdx = idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = octR[idx];
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= 100) {
                    if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
                    if (r2l && r2l[bestIdx] != -1) {
                        assign(r2l[bestIdx], i, mp);
                        nmatches++;
                    }
                    assign(bestIdx + nl, i, mp);
                    nmatches++;
                }
            }
        }
    }
    return nmatches;
}
