// ORBextractor.cc -- the ORB_SLAM3::ORBextractor facade over the C ABI (include/orbgpu.h).
//
// Compiled by the integrating project (with -DORBGPU_WITH_OPENCV and its OpenCV), or against
// include/orbslam3/cv_shim.h as in tests/cpp; both modes see OpenCV's API shape (CV_8U macros,
// InputArray = const _InputArray&).  Mirrors cpp/src/ORBextractor_old.cc:411-471 (ctor tables)
// and :1088-1191 (operator() output contract), and cpp/src/ORBextractor.cc:118-165 (the stereo
// operator() over the accelerator session); the compute is liborbgpu.so.
#include "../../include/orbslam3/ORBextractor.h"

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#if defined(__ANDROID__)
#include <android/hardware_buffer.h>
#endif

namespace ORB_SLAM3 {

static_assert(sizeof(orbgpu_keypoint) == 28, "cv::KeyPoint layout");

namespace {
#if defined(__ANDROID__)
// ORBextractor.cc:133-147: describe, lock for CPU reads, unlock after the copy.  The frame is an
// 8-bit format, so the stride in pixels is the stride in bytes.
int ahb_lock_ndk(AHardwareBuffer* b, const uint8_t** data, int* w, int* h, int* stride) {
    AHardwareBuffer_Desc d = {};
    AHardwareBuffer_describe(b, &d);
    void* p = nullptr;
    if (AHardwareBuffer_lock(b, AHARDWAREBUFFER_USAGE_CPU_READ_OFTEN, -1, nullptr, &p) != 0 || !p) return -1;
    *data = static_cast<const uint8_t*>(p);
    *w = (int)d.width;
    *h = (int)d.height;
    *stride = (int)d.stride;
    return 0;
}
void ahb_unlock_ndk(AHardwareBuffer* b) { AHardwareBuffer_unlock(b, nullptr); }
AHardwareBufferAccess g_ahb{ahb_lock_ndk, ahb_unlock_ndk};
#else
AHardwareBufferAccess g_ahb{nullptr, nullptr};
#endif
std::mutex g_ahb_mutex;
}  // namespace

void SetAHardwareBufferAccess(const AHardwareBufferAccess& access) {
    std::lock_guard<std::mutex> g(g_ahb_mutex);
    g_ahb = access;
}

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
    // Tables come from the library (same float/double arithmetic as :416-447); the context grows
    // to the largest image seen.
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
    // the caller's current HIP device (a multi-camera process selects the GPU before constructing
    // the extractor), kept for later regrowths
    mStatus = orbgpu_create(&p, mDevice, W, H, 2, &mCtx);
    if (mStatus == ORBGPU_OK) mCtxW = W, mCtxH = H, mDevice = orbgpu_get_device(mCtx);
    return mStatus;
}

void ORBextractor::exportPyramid(int image) {
    if (!mbExportPyramid) return;
    for (int l = 0; l < nlevels; ++l) {
        int w = 0, h = 0;
        orbgpu_get_pyramid_level(mCtx, image, l, 0, nullptr, 0, &w, &h);
        mvImagePyramid[l].create(h, w, CV_8U);
        orbgpu_get_pyramid_level(mCtx, image, l, 0, mvImagePyramid[l].ptr<unsigned char>(0),
                                 (int)mvImagePyramid[l].step[0], &w, &h);
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
    if (_image.empty()) return -1;  // :1092-1093
    cv::Mat image = _image.getMat();
    if (image.type() != CV_8UC1) return -1;  // assert :1096
    if ((mStatus = ensureContext(image.cols, image.rows)) != ORBGPU_OK) return -1;
    const int cap = 8 * nfeatures + 64 * nlevels + 4096;
    mKps.resize(cap);
    mDesc.resize((size_t)cap * 32);
    int n = 0, mono = 0;
    const int lap0 = vLappingArea.size() > 0 ? vLappingArea[0] : 0;
    const int lap1 = vLappingArea.size() > 1 ? vLappingArea[1] : 0;
    mStatus = orbgpu_extract(mCtx, image.ptr<unsigned char>(0), image.cols, image.rows, (int)image.step[0], lap0,
                             lap1, mKps.data(), mDesc.data(), cap, &n, &mono);
    if (mStatus != ORBGPU_OK) return -1;
    to_cv(mKps, n, _keypoints);
    if (n == 0) {
        _descriptors.release();  // :1120-1121
    } else {
        _descriptors.create(n, 32, CV_8U);
        cv::Mat d = _descriptors.getMat();
        for (int i = 0; i < n; ++i) std::memcpy(d.ptr<unsigned char>(i), mDesc.data() + 32 * (size_t)i, 32);
    }
    exportPyramid(0);
    return mono;
}

LynxHardwareAccelerator* ORBextractor::accelerator(int width, int height) {
    // ORBextractor.cc:125-128: the session is created on first use (with this extractor's
    // parameters and geometry here, the DSP's were fixed)
    if (!LynxHardwareAccelerator::lynxHardwareAccelerator)
        LynxHardwareAccelerator::lynxHardwareAccelerator.reset(
            new LynxHardwareAccelerator(nfeatures, (float)scaleFactor, nlevels, iniThFAST, minThFAST, width, height));
    return LynxHardwareAccelerator::lynxHardwareAccelerator.get();
}

// Both eyes of the frame the accelerator holds, the stereo-row kNN2, the pyramid export.
int ORBextractor::extractStored(LynxHardwareAccelerator* acc, std::vector<cv::KeyPoint>& kl, cv::OutputArray dl,
                                std::vector<int>& lapL, std::vector<cv::KeyPoint>& kr, cv::OutputArray dr,
                                std::vector<int>& lapR, int& monoLeft, int& monoRight) {
    int nl = 0, nr = 0;
    const int id = acc->ExtractORB(nl, nr, kl, kr, dl, dr, lapL.size() > 0 ? lapL[0] : 0,
                                   lapL.size() > 1 ? lapL[1] : 0, lapR.size() > 0 ? lapR[0] : 0,
                                   lapR.size() > 1 ? lapR[1] : 0, monoLeft, monoRight);
    if (id < 0) return -1;
    if (mbExportPyramid) acc->ExportPyramid(0, mvImagePyramid);
    return id;
}

int ORBextractor::operator()(AHardwareBuffer* _image, std::vector<cv::KeyPoint>& kl, cv::OutputArray dl,
                             std::vector<int>& lapL, std::vector<cv::KeyPoint>& kr, cv::OutputArray dr,
                             std::vector<int>& lapR, int& monoLeft, int& monoRight) {
    AHardwareBufferAccess access;
    {
        std::lock_guard<std::mutex> g(g_ahb_mutex);
        access = g_ahb;
    }
    if (!_image || !access.lock || !access.unlock) {
        mStatus = ORBGPU_ERR_INVALID;
        return -1;
    }
    const uint8_t* data = nullptr;
    int width = 0, height = 0, stride = 0;
    if (access.lock(_image, &data, &width, &height, &stride) != 0 || !data) {
        mStatus = ORBGPU_ERR_INVALID;
        return -1;
    }
    // :136-137: each eye is half the buffer's width
    if (width < 2 || (width & 1) || height < 1 || stride < width) {
        access.unlock(_image);
        mStatus = ORBGPU_ERR_INVALID;
        return -1;
    }
    // :143 copies the frame to the accelerator and :146-148 unlock; the copy here may still be in
    // flight on the device queue when StoreInputBuffer returns, so the buffer stays locked until
    // the extraction (which waits for it) has returned
    int id = -1;
    try {
        LynxHardwareAccelerator* acc = accelerator(width / 2, height);
        acc->StoreInputBuffer(data, width / 2, height, stride);
        id = extractStored(acc, kl, dl, lapL, kr, dr, lapR, monoLeft, monoRight);
    } catch (const std::exception&) {
        mStatus = ORBGPU_ERR_HIP;
        id = -1;
    }
    access.unlock(_image);
    return id;
}

int ORBextractor::operator()(cv::InputArray _image, std::vector<cv::KeyPoint>& kl, cv::OutputArray dl,
                             std::vector<int>& lapL, std::vector<cv::KeyPoint>& kr, cv::OutputArray dr,
                             std::vector<int>& lapR, int& monoLeft, int& monoRight) {
    if (_image.empty()) return -1;
    cv::Mat sbs = _image.getMat();
    if (sbs.type() != CV_8UC1 || sbs.cols < 2 || (sbs.cols & 1)) return -1;
    const int W = sbs.cols / 2, H = sbs.rows;
    try {
        LynxHardwareAccelerator* acc = accelerator(W, H);
        acc->StoreInputBuffer(sbs.ptr<unsigned char>(0), W, H, (int)sbs.step[0]);
        return extractStored(acc, kl, dl, lapL, kr, dr, lapR, monoLeft, monoRight);
    } catch (const std::exception&) {
        mStatus = ORBGPU_ERR_HIP;
        return -1;
    }
}

int ORBextractor::operator()(cv::InputArray left, cv::InputArray right, std::vector<cv::KeyPoint>& kl,
                             cv::OutputArray dl, std::vector<int>& lapL, std::vector<cv::KeyPoint>& kr,
                             cv::OutputArray dr, std::vector<int>& lapR, int& monoLeft, int& monoRight) {
    if (left.empty() || right.empty()) return -1;
    cv::Mat L = left.getMat(), R = right.getMat();
    if (L.rows != R.rows || L.cols != R.cols || L.step[0] != R.step[0] || L.type() != CV_8UC1 ||
        R.type() != CV_8UC1)
        return -1;
    try {
        LynxHardwareAccelerator* acc = accelerator(L.cols, L.rows);
        int nl = 0, nr = 0;
        const int id = acc->ExtractORBPair(L.ptr<unsigned char>(0), R.ptr<unsigned char>(0), L.cols, L.rows,
                                           (int)L.step[0], nl, nr, kl, kr, dl, dr, lapL.size() > 0 ? lapL[0] : 0,
                                           lapL.size() > 1 ? lapL[1] : 0, lapR.size() > 0 ? lapR[0] : 0,
                                           lapR.size() > 1 ? lapR[1] : 0, monoLeft, monoRight);
        if (id < 0) return -1;
        if (mbExportPyramid) acc->ExportPyramid(0, mvImagePyramid);
        return id;
    } catch (const std::exception&) {
        mStatus = ORBGPU_ERR_HIP;
        return -1;
    }
}

}  // namespace ORB_SLAM3
