// facade_test.cpp -- TEST: the C++ ORB_SLAM3::ORBextractor facade (include/orbslam3/ORBextractor.h)
// on the GPU vs the CPU oracle (oracle/build/liborb_oracle.so, loaded with dlopen as the checker).
// Built by `make facade_test`; run by tests/test_gpu_parity.py::test_cpp_facade.
#include <dlfcn.h>

#include <cstdint>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/orbslam3/ORBextractor.h"

typedef struct { float x, y, size, angle, response; int32_t octave, class_id; } okp;
typedef int (*oracle_extract_t)(int, float, int, int, int, const uint8_t*, int, int, int, int, int,
                                okp*, uint8_t*, int, int*);
typedef void (*oracle_knn2_t)(const uint8_t*, int, const uint8_t*, int, int32_t*, int32_t*, int32_t*, int32_t*);

static std::vector<uint8_t> texture(int w, int h, uint32_t seed) {
    std::vector<uint8_t> img((size_t)w * h);
    uint32_t s = seed;
    std::vector<int> coarse((w / 8 + 2) * (h / 8 + 2));
    for (auto& c : coarse) { s = s * 1664525u + 1013904223u; c = (s >> 24); }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            s = s * 1664525u + 1013904223u;
            const int c = coarse[(y / 8) * (w / 8 + 2) + x / 8];
            const int v = c + (int)((s >> 27) & 15) - 8 + ((x / 24 + y / 24) % 2 ? 40 : -40);
            img[(size_t)y * w + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    return img;
}

static int compare(const char* tag, const std::vector<cv::KeyPoint>& k, const cv::Mat& d, int mono,
                   const okp* rk, const uint8_t* rd, int rn, int rmono) {
    if ((int)k.size() != rn || mono != rmono) {
        printf("%s: count %zu vs %d, mono %d vs %d\n", tag, k.size(), rn, mono, rmono);
        return 1;
    }
    for (int i = 0; i < rn; ++i) {
        if (k[i].pt.x != rk[i].x || k[i].pt.y != rk[i].y || k[i].angle != rk[i].angle ||
            k[i].response != rk[i].response || k[i].octave != rk[i].octave || k[i].size != rk[i].size) {
            printf("%s: keypoint %d differs\n", tag, i);
            return 1;
        }
        if (std::memcmp(d.ptr<unsigned char>(i), rd + 32 * (size_t)i, 32)) {
            printf("%s: descriptor %d differs\n", tag, i);
            return 1;
        }
    }
    return 0;
}

static int compare_knn(const char* tag, const std::vector<uint16_t>& idx, const std::vector<uint16_t>& d1,
                       const std::vector<uint16_t>& d2, const int32_t* ri1, const int32_t* rd1, const int32_t* rd2,
                       int nq) {
    if ((int)idx.size() != nq || (int)d1.size() != nq || (int)d2.size() != nq) {
        printf("%s: %zu matches vs %d queries\n", tag, idx.size(), nq);
        return 1;
    }
    for (int i = 0; i < nq; ++i) {
        const uint16_t ei1 = (uint16_t)(int16_t)ri1[i];
        const uint16_t ed1 = (uint16_t)(rd1[i] > 32767 ? 32767 : rd1[i]), ed2 = (uint16_t)(rd2[i] > 32767 ? 32767 : rd2[i]);
        if (idx[i] != ei1 || d1[i] != ed1 || d2[i] != ed2) {
            printf("%s: match %d differs (%d %d %d vs %d %d %d)\n", tag, i, idx[i], d1[i], d2[i], ri1[i], rd1[i], rd2[i]);
            return 1;
        }
    }
    return 0;
}

// A test double of the headset's buffer: the facade only sees AHardwareBuffer* and calls the
// installed lock / unlock (ORB_SLAM3::SetAHardwareBufferAccess).
struct AHardwareBuffer {
    std::vector<uint8_t> pixels;
    int width = 0, height = 0, stride = 0;
    int locks = 0, unlocks = 0;
    bool locked = false;
};
static AHardwareBuffer g_buf;
static int test_ahb_lock(AHardwareBuffer* b, const uint8_t** data, int* w, int* h, int* stride) {
    if (b->locked) return -1;
    b->locked = true;
    ++b->locks;
    *data = b->pixels.data();
    *w = b->width;
    *h = b->height;
    *stride = b->stride;
    return 0;
}
static void test_ahb_unlock(AHardwareBuffer* b) {
    b->locked = false;
    ++b->unlocks;
}

int main(int argc, char** argv) {
    const char* oracle_path = argc > 1 ? argv[1] : "oracle/build/liborb_oracle.so";
    void* h = dlopen(oracle_path, RTLD_NOW);
    if (!h) { printf("cannot load oracle %s\n", oracle_path); return 2; }
    auto ox = (oracle_extract_t)dlsym(h, "oracle_extract");
    auto oknn = (oracle_knn2_t)dlsym(h, "oracle_knn2");
    if (!ox || !oknn) { printf("oracle symbols\n"); return 2; }
    // the eye geometry: 640x480 by default; 640 400 is the headset's (LynxHardwareAccelerator.h:20-21)
    const int W = argc > 3 ? atoi(argv[2]) : 640, H = argc > 3 ? atoi(argv[3]) : 480;
    std::vector<uint8_t> L = texture(W, H, 7), R = texture(W, H, 8);
    ORB_SLAM3::ORBextractor ex(2000, 1.2f, 8, 20, 7);
    if (ex.GetLevels() != 8 || ex.GetScaleFactors().size() != 8) { printf("getters\n"); return 1; }
    {   // the facades build on the caller's current HIP device (ORBGPU_DEVICE_CURRENT): on this
        // one-GPU process that is ordinal 0, and a context made the same way reports the same one
        orbgpu_params p{500, 1.2f, 4, 20, 7};
        orbgpu_ctx* c = nullptr;
        const int rc = orbgpu_create(&p, ORBGPU_DEVICE_CURRENT, 160, 120, 2, &c);
        const int dev = rc == ORBGPU_OK ? orbgpu_get_device(c) : rc;
        orbgpu_destroy(c);
        if (dev != 0) { printf("current-device context on %d\n", dev); return 1; }
        if (orbgpu_create(&p, 4096, 160, 120, 2, &c) != ORBGPU_ERR_NO_DEVICE) { printf("bad ordinal accepted\n"); return 1; }
    }
    cv::Mat im(H, W, CV_8U, L.data(), W), desc;
    std::vector<cv::KeyPoint> kps;
    std::vector<int> lap = {0, 1000};
    const int mono = ex(im, cv::Mat(), kps, desc, lap);
    std::vector<okp> rk(20000);
    std::vector<uint8_t> rd(20000 * 32);
    int rn = 0;
    int rmono = ox(2000, 1.2f, 8, 20, 7, L.data(), W, H, W, 0, 1000, rk.data(), rd.data(), 20000, &rn);
    int bad = compare("mono", kps, desc, mono, rk.data(), rd.data(), rn, rmono);
    // level sizes cvRound(W * invScale) (ComputePyramid :1336): 533 and 134 at 640x480
    const std::vector<float> inv = ex.GetInverseScaleFactors();
    if (ex.mvImagePyramid.size() != 8 || ex.mvImagePyramid[1].cols != (int)lrintf((float)W * inv[1]) ||
        ex.mvImagePyramid[7].rows != (int)lrintf((float)H * inv[7]) ||
        (W == 640 && H == 480 && (ex.mvImagePyramid[1].cols != 533 || ex.mvImagePyramid[7].rows != 134))) {
        printf("pyramid export\n");
        bad = 1;
    }
    // stereo forms: the side-by-side frame (ORBextractor.h:52-57) and two images; each returns
    // the frame id whose matches LynxHardwareAccelerator::BFMatchORB returns (Frame.cc:1164)
    std::vector<uint8_t> sbs((size_t)2 * W * H);
    for (int y = 0; y < H; ++y) {
        std::memcpy(sbs.data() + (size_t)y * 2 * W, L.data() + (size_t)y * W, W);
        std::memcpy(sbs.data() + (size_t)y * 2 * W + W, R.data() + (size_t)y * W, W);
    }
    cv::Mat frame(H, 2 * W, CV_8U, sbs.data(), 2 * W), ir(H, W, CV_8U, R.data(), W);
    std::vector<int> lapL = {300, 640}, lapR = {0, 340};
    std::vector<okp> rkl(20000), rkr(20000);
    std::vector<uint8_t> rdl(20000 * 32), rdr(20000 * 32);
    int rnl = 0, rnr = 0;
    const int rml = ox(2000, 1.2f, 8, 20, 7, L.data(), W, H, W, lapL[0], lapL[1], rkl.data(), rdl.data(), 20000, &rnl);
    const int rmr = ox(2000, 1.2f, 8, 20, 7, R.data(), W, H, W, lapR[0], lapR[1], rkr.data(), rdr.data(), 20000, &rnr);
    const int nq = rnl - rml;
    std::vector<int32_t> ri1(nq + 1), rd1(nq + 1), ri2(nq + 1), rd2(nq + 1);
    oknn(rdl.data() + 32 * (size_t)rml, nq, rdr.data() + 32 * (size_t)rmr, rnr - rmr, ri1.data(), rd1.data(),
         ri2.data(), rd2.data());
    int ids[2] = {0, 0};
    for (int form = 0; form < 2; ++form) {
        cv::Mat dl, dr;
        std::vector<cv::KeyPoint> kl, kr;
        int ml = -1, mr = -1;
        ids[form] = form == 0 ? ex(frame, kl, dl, lapL, kr, dr, lapR, ml, mr)
                              : ex(im, ir, kl, dl, lapL, kr, dr, lapR, ml, mr);
        const char* tag = form == 0 ? "sbs" : "pair";
        if (ids[form] <= 0) { printf("%s: frame id %d\n", tag, ids[form]); bad = 1; continue; }
        bad |= compare(tag, kl, dl, ml, rkl.data(), rdl.data(), rnl, rml);
        bad |= compare(tag, kr, dr, mr, rkr.data(), rdr.data(), rnr, rmr);
        std::vector<uint16_t> idx, d1, d2;
        ORB_SLAM3::LynxHardwareAccelerator::lynxHardwareAccelerator->BFMatchORB(
            ids[form], dr.rowRange(mr, dr.rows), dl.rowRange(ml, dl.rows), idx, d1, d2);
        bad |= compare_knn(tag, idx, d1, d2, ri1.data(), rd1.data(), rd2.data(), nq);
        if (ex.mvImagePyramid[0].cols != W) { printf("%s: pyramid\n", tag); bad = 1; }
    }
    if (ids[1] != ids[0] + 1) { printf("frame ids %d %d\n", ids[0], ids[1]); bad = 1; }
    // the AHardwareBuffer form, called as FrameAHB::ExtractORB does (FrameAHB.cc:168-177), on a
    // test double of the buffer with a padded row stride; locked once, unlocked once
    {
        const int stride = 2 * W + 64;
        g_buf.pixels.assign((size_t)stride * H, 0xEE);
        for (int y = 0; y < H; ++y) std::memcpy(g_buf.pixels.data() + (size_t)y * stride, sbs.data() + (size_t)y * 2 * W, 2 * W);
        g_buf.width = 2 * W;
        g_buf.height = H;
        g_buf.stride = stride;
        cv::Mat dl, dr;
        std::vector<cv::KeyPoint> kl, kr;
        int ml = -1, mr = -1;
        if (ex((AHardwareBuffer*)&g_buf, kl, dl, lapL, kr, dr, lapR, ml, mr) != -1) {  // no access installed
            printf("ahb: accepted without a lock function\n");
            bad = 1;
        }
        ORB_SLAM3::SetAHardwareBufferAccess({test_ahb_lock, test_ahb_unlock});
        const int id = ex((AHardwareBuffer*)&g_buf, kl, dl, lapL, kr, dr, lapR, ml, mr);
        if (id <= 0 || g_buf.locks != 1 || g_buf.unlocks != 1 || g_buf.locked) {
            printf("ahb: id %d locks %d unlocks %d\n", id, g_buf.locks, g_buf.unlocks);
            bad = 1;
        } else {
            bad |= compare("ahb", kl, dl, ml, rkl.data(), rdl.data(), rnl, rml);
            bad |= compare("ahb", kr, dr, mr, rkr.data(), rdr.data(), rnr, rmr);
            std::vector<uint16_t> idx, d1, d2;
            ORB_SLAM3::LynxHardwareAccelerator::lynxHardwareAccelerator->BFMatchORB(
                id, dr.rowRange(mr, dr.rows), dl.rowRange(ml, dl.rows), idx, d1, d2);
            bad |= compare_knn("ahb", idx, d1, d2, ri1.data(), rd1.data(), rd2.data(), nq);
        }
    }
    // a frame id that left the 3-frame cache: matched again on the device from the rows given
    {
        cv::Mat dl, dr;
        std::vector<cv::KeyPoint> kl, kr;
        int ml = 0, mr = 0;
        for (int k = 0; k < 3; ++k) ex(im, ir, kl, dl, lapL, kr, dr, lapR, ml, mr);
        std::vector<uint16_t> idx, d1, d2;
        ORB_SLAM3::LynxHardwareAccelerator::lynxHardwareAccelerator->BFMatchORB(
            ids[0], dr.rowRange(mr, dr.rows), dl.rowRange(ml, dl.rows), idx, d1, d2);
        bad |= compare_knn("stale id", idx, d1, d2, ri1.data(), rd1.data(), rd2.data(), nq);
    }
    cv::Mat d0 = desc.rowRange(0, 1), d1 = desc.rowRange(1, 2);
    const int dd = ORB_SLAM3::orbgpu::DescriptorDistance(d0, d1);
    int ref = 0;
    for (int b = 0; b < 32; ++b) ref += __builtin_popcount(d0.ptr<unsigned char>(0)[b] ^ d1.ptr<unsigned char>(0)[b]);
    if (dd != ref) { printf("DescriptorDistance %d vs %d\n", dd, ref); bad = 1; }
    cv::Mat empty;
    if (ex(empty, cv::Mat(), kps, desc, lap) != -1) bad = 1;
    printf(bad ? "FACADE FAIL %dx%d\n" : "FACADE OK %dx%d %zu keypoints\n", W, H, kps.size());
    return bad;
}
