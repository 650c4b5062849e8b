// facade_test.cpp -- TEST: the C++ ORB_SLAM3::ORBextractor facade (include/orbslam3/ORBextractor.h)
// on the GPU vs the CPU oracle (oracle/build/liborb_oracle.so, loaded with dlopen as the checker).
// Built by `make facade_test`; run by tests/test_gpu_parity.py::test_cpp_facade.
#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/orbslam3/ORBextractor.h"

typedef struct { float x, y, size, angle, response; int32_t octave, class_id; } okp;
typedef int (*oracle_extract_t)(int, float, int, int, int, const uint8_t*, int, int, int, int, int,
                                okp*, uint8_t*, int, int*);

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
        if (std::memcmp(d.ptr(i), rd + 32 * (size_t)i, 32)) {
            printf("%s: descriptor %d differs\n", tag, i);
            return 1;
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    const char* oracle_path = argc > 1 ? argv[1] : "oracle/build/liborb_oracle.so";
    void* h = dlopen(oracle_path, RTLD_NOW);
    if (!h) { printf("cannot load oracle %s\n", oracle_path); return 2; }
    auto ox = (oracle_extract_t)dlsym(h, "oracle_extract");
    const int W = 640, H = 480;
    std::vector<uint8_t> L = texture(W, H, 7), R = texture(W, H, 8);
    ORB_SLAM3::ORBextractor ex(2000, 1.2f, 8, 20, 7);
    if (ex.GetLevels() != 8 || ex.GetScaleFactors().size() != 8) { printf("getters\n"); return 1; }
    cv::Mat im(H, W, cv::CV_8U, L.data(), W), desc;
    std::vector<cv::KeyPoint> kps;
    std::vector<int> lap = {0, 1000};
    const int mono = ex(im, cv::Mat(), kps, desc, lap);
    std::vector<okp> rk(20000);
    std::vector<uint8_t> rd(20000 * 32);
    int rn = 0;
    int rmono = ox(2000, 1.2f, 8, 20, 7, L.data(), W, H, W, 0, 1000, rk.data(), rd.data(), 20000, &rn);
    int bad = compare("mono", kps, desc, mono, rk.data(), rd.data(), rn, rmono);
    if (ex.mvImagePyramid.size() != 8 || ex.mvImagePyramid[1].cols != 533 || ex.mvImagePyramid[7].rows != 134) {
        printf("pyramid export\n");
        bad = 1;
    }
    cv::Mat ir(H, W, cv::CV_8U, R.data(), W), dl, dr;
    std::vector<cv::KeyPoint> kl, kr;
    std::vector<int> lapL = {0, 0}, lapR = {100, 600};
    int ml = 0, mr = 0;
    ex(im, ir, kl, dl, lapL, kr, dr, lapR, ml, mr);
    rmono = ox(2000, 1.2f, 8, 20, 7, L.data(), W, H, W, 0, 0, rk.data(), rd.data(), 20000, &rn);
    bad |= compare("stereo-left", kl, dl, ml, rk.data(), rd.data(), rn, rmono);
    rmono = ox(2000, 1.2f, 8, 20, 7, R.data(), W, H, W, 100, 600, rk.data(), rd.data(), 20000, &rn);
    bad |= compare("stereo-right", kr, dr, mr, rk.data(), rd.data(), rn, rmono);
    int dd = ORB_SLAM3::ORBmatcher::DescriptorDistance(dl.rowRange(0, 1), dr.rowRange(0, 1));
    if (dd < 0 || dd > 256) bad = 1;
    cv::Mat empty;
    if (ex(empty, cv::Mat(), kps, desc, lap) != -1) bad = 1;
    printf(bad ? "FACADE FAIL\n" : "FACADE OK %zu keypoints\n", kps.size());
    return bad;
}
