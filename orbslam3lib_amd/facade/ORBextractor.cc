// ORBextractor.cc -- the ORB_SLAM3::ORBextractor facade over the C ABI (include/orbgpu.h).
//
// Compiled by the integrating project (with -DORBGPU_WITH_OPENCV and its OpenCV), or against
// include/orbslam3/cv_shim.h as in tests/cpp.  Mirrors cpp/src/ORBextractor_old.cc:411-471
// (ctor tables) and :1088-1191 (operator() output contract); the compute is liborbgpu.so.
#include "../../include/orbslam3/ORBextractor.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace ORB_SLAM3 {

static_assert(sizeof(orbgpu_keypoint) == 28, "cv::KeyPoint layout");

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST,
                           int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    mvImagePyramid.resize(nlevels);
    // Tables come from the library (same float/double arithmetic as :416-447); the context
    // itself is created lazily at the first image size, like LynxHardwareAccelerator.
    if (ensureContext(640, 480) != ORBGPU_OK)
        throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    orbgpu_get_scale_tables(mCtx, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                            mvInvLevelSigma2.data(), mnFeaturesPerLevel.data());
}

ORBextractor::~ORBextractor() { orbgpu_destroy(mCtx); }

int ORBextractor::ensureContext(int w, int h) {
    if (mCtx && w <= mCtxW && h <= mCtxH) return ORBGPU_OK;
    orbgpu_destroy(mCtx);
    mCtx = nullptr;
    orbgpu_params p{nfeatures, (float)scaleFactor, nlevels, iniThFAST, minThFAST};
    const int W = w > mCtxW ? w : mCtxW, H = h > mCtxH ? h : mCtxH;
    mStatus = orbgpu_create(&p, 0, W, H, 2, &mCtx);
    if (mStatus == ORBGPU_OK) mCtxW = W, mCtxH = H;
    return mStatus;
}

void ORBextractor::exportPyramid(int image) {
    if (!mbExportPyramid) return;
    for (int l = 0; l < nlevels; ++l) {
        int w = 0, h = 0;
        orbgpu_get_pyramid_level(mCtx, image, l, 0, nullptr, 0, &w, &h);
        mvImagePyramid[l].create(h, w, cv::CV_8U);
        orbgpu_get_pyramid_level(mCtx, image, l, 0, mvImagePyramid[l].ptr(0), (int)mvImagePyramid[l].step, &w, &h);
    }
}

static void to_cv(const std::vector<orbgpu_keypoint>& src, int n, std::vector<cv::KeyPoint>& dst) {
    dst.resize(n);
    for (int i = 0; i < n; ++i) {
        cv::KeyPoint& k = dst[i];
        k.pt.x = src[i].x;
        k.pt.y = src[i].y;
        k.size = src[i].size;
        k.angle = src[i].angle;
        k.response = src[i].response;
        k.octave = src[i].octave;
        k.class_id = src[i].class_id;
    }
}

int ORBextractor::operator()(cv::InputArray _image, cv::InputArray /*_mask*/,
                             std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors,
                             std::vector<int>& vLappingArea) {
    cv::Mat image = _image.getMat();
    if (image.empty()) return -1;  // :1092-1093
    if (image.type() != cv::CV_8UC1) return -1;
    if ((mStatus = ensureContext(image.cols, image.rows)) != ORBGPU_OK) return -1;
    const int cap = 8 * nfeatures + 64 * nlevels + 4096;
    mKps[0].resize(cap);
    std::vector<uint8_t> desc((size_t)cap * 32);
    int n = 0, mono = 0;
    const int lap0 = vLappingArea.size() > 0 ? vLappingArea[0] : 0;
    const int lap1 = vLappingArea.size() > 1 ? vLappingArea[1] : 0;
    mStatus = orbgpu_extract(mCtx, image.ptr(0), image.cols, image.rows, (int)image.step1(), lap0, lap1,
                             mKps[0].data(), desc.data(), cap, &n, &mono);
    if (mStatus != ORBGPU_OK) return -1;
    to_cv(mKps[0], n, _keypoints);
    if (n == 0) {
        _descriptors.release();  // :1120-1121
    } else {
        _descriptors.create(n, 32, cv::CV_8U);
        cv::Mat d = _descriptors.getMat();
        for (int i = 0; i < n; ++i) std::memcpy(d.ptr(i), desc.data() + 32 * (size_t)i, 32);
    }
    exportPyramid(0);
    return mono;
}

int ORBextractor::operator()(cv::InputArray left, cv::InputArray right,
                             std::vector<cv::KeyPoint>& kl, cv::OutputArray dl, std::vector<int>& lapL,
                             std::vector<cv::KeyPoint>& kr, cv::OutputArray dr, std::vector<int>& lapR,
                             int& monoLeft, int& monoRight) {
    cv::Mat L = left.getMat(), R = right.getMat();
    if (L.empty() || R.empty() || L.rows != R.rows || L.cols != R.cols || L.step1() != R.step1()) return -1;
    if ((mStatus = ensureContext(L.cols, L.rows)) != ORBGPU_OK) return -1;
    const int cap = 8 * nfeatures + 64 * nlevels + 4096;
    mKps[0].resize(cap);
    mKps[1].resize(cap);
    std::vector<uint8_t> d0((size_t)cap * 32), d1((size_t)cap * 32);
    int la[2] = {lapL.size() > 0 ? lapL[0] : 0, lapL.size() > 1 ? lapL[1] : 0};
    int ra[2] = {lapR.size() > 0 ? lapR[0] : 0, lapR.size() > 1 ? lapR[1] : 0};
    int nl = 0, nr = 0;
    mStatus = orbgpu_extract_stereo(mCtx, L.ptr(0), R.ptr(0), L.cols, L.rows, (int)L.step1(), la, ra,
                                    mKps[0].data(), d0.data(), &nl, &monoLeft, mKps[1].data(), d1.data(),
                                    &nr, &monoRight, cap);
    if (mStatus != ORBGPU_OK) return -1;
    to_cv(mKps[0], nl, kl);
    to_cv(mKps[1], nr, kr);
    struct { cv::Mat* m; std::vector<uint8_t>* d; int n; } outs[2] = {{&dl, &d0, nl}, {&dr, &d1, nr}};
    for (auto& o : outs) {
        if (o.n == 0) {
            o.m->release();
            continue;
        }
        o.m->create(o.n, 32, cv::CV_8U);
        for (int i = 0; i < o.n; ++i) std::memcpy(o.m->ptr(i), o.d->data() + 32 * (size_t)i, 32);
    }
    exportPyramid(0);
    return 0;
}

}  // namespace ORB_SLAM3
