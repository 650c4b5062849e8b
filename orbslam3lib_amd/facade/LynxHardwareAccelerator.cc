// LynxHardwareAccelerator.cc -- the accelerator session over the C ABI (include/orbgpu.h).
//
// Replaces cpp/src/LynxHardwareAcceleration/LynxHardwareAccelerator.cpp (FastRPC session, rpcmem
// buffers, 3-slot match cache).  One liborbgpu context (two images: the eyes of one frame) holds
// the frame on the device; ExtractORB runs the extraction of both eyes and the stereo-row kNN2
// as one submission (orbgpu_run_batch_match) and keeps the matches in the slot of its frame id,
// as :134-213 do with matchingCache*.
#include "../../include/orbslam3/LynxHardwareAcceleration/LynxHardwareAccelerator.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace ORB_SLAM3 {

std::unique_ptr<LynxHardwareAccelerator> LynxHardwareAccelerator::lynxHardwareAccelerator;

namespace {

void to_cv(const std::vector<orbgpu_keypoint>& src, int n, std::vector<cv::KeyPoint>& dst) {
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

void to_mat(const std::vector<uint8_t>& d, int n, cv::OutputArray out) {
    out.create(n, 32, CV_8U);
    if (n == 0) return;
    cv::Mat m = out.getMat();
    for (int i = 0; i < n; ++i) std::memcpy(m.ptr<unsigned char>(i), d.data() + 32 * (size_t)i, 32);
}

// the FastRPC result layout's int16 fields read as uint16 (Frame.cc:1161): absent second match
// -> index 0xFFFF, distances clamped to 32767 (orbgpu.h, orbgpu_pack_soa)
uint16_t idx16(int32_t i) { return (uint16_t)(int16_t)(i < 0 ? -1 : i); }
uint16_t dist16(int32_t d) { return (uint16_t)(d > 32767 ? 32767 : d); }

std::vector<uint8_t> rows(const cv::Mat& m) {
    std::vector<uint8_t> v((size_t)m.rows * 32);
    for (int i = 0; i < m.rows; ++i) std::memcpy(v.data() + 32 * (size_t)i, m.ptr<unsigned char>(i), 32);
    return v;
}

}  // namespace

LynxHardwareAccelerator::LynxHardwareAccelerator()
    : LynxHardwareAccelerator(2000, 1.2f, 8, 20, 7, DEFAULT_WIDTH, DEFAULT_HEIGHT) {}

LynxHardwareAccelerator::LynxHardwareAccelerator(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
                                                 int minThFAST, int width, int height) {
    mParams = orbgpu_params{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
    if (ensure(width, height) != ORBGPU_OK)
        throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
}

LynxHardwareAccelerator::~LynxHardwareAccelerator() { orbgpu_destroy(mCtx); }

int LynxHardwareAccelerator::ensure(int w, int h) const {
    if (mCtx && w <= mWidth && h <= mHeight) return ORBGPU_OK;
    orbgpu_destroy(mCtx);
    mCtx = nullptr;
    const int W = w > mWidth ? w : mWidth, H = h > mHeight ? h : mHeight;
    const int r = orbgpu_create(&mParams, mDevice, W, H, 2, &mCtx);  // the caller's current device
    if (r == ORBGPU_OK) mWidth = W, mHeight = H, mDevice = orbgpu_get_device(mCtx);
    return r;
}

void LynxHardwareAccelerator::StoreInputBuffer(const uint8_t* frameData) const {
    StoreInputBuffer(frameData, DEFAULT_WIDTH, DEFAULT_HEIGHT, 2 * DEFAULT_WIDTH);
}

void LynxHardwareAccelerator::StoreInputBuffer(const uint8_t* frameData, int width, int height, int stride) const {
    std::lock_guard<std::mutex> g(mMutex);
    if (ensure(width, height) != ORBGPU_OK) throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    if (orbgpu_upload_sbs(mCtx, frameData, 1, width, height, stride) != ORBGPU_OK)
        throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    mFrameW = width;
    mFrameH = height;
}

int LynxHardwareAccelerator::finish(int& nl, int& nr, std::vector<cv::KeyPoint>& kl, std::vector<cv::KeyPoint>& kr,
                                    cv::OutputArray& dl, cv::OutputArray& dr, int& monoLeft, int& monoRight) {
    int32_t counts[2] = {0, 0};
    if (orbgpu_download_counts(mCtx, 2, counts, nullptr) != ORBGPU_OK) return -1;
    const int cap = (counts[0] > counts[1] ? counts[0] : counts[1]) + 1;
    std::vector<orbgpu_keypoint> k((size_t)cap);
    std::vector<uint8_t> d((size_t)cap * 32);
    int* n[2] = {&nl, &nr};
    int* mono[2] = {&monoLeft, &monoRight};
    std::vector<cv::KeyPoint>* kout[2] = {&kl, &kr};
    const cv::_OutputArray* dout[2] = {&dl, &dr};
    for (int e = 0; e < 2; ++e) {
        if (orbgpu_download_result(mCtx, e, k.data(), d.data(), cap, n[e], mono[e]) != ORBGPU_OK) return -1;
        to_cv(k, *n[e], *kout[e]);
        to_mat(d, *n[e], *dout[e]);
    }
    const int nq = nl - monoLeft > 0 ? nl - monoLeft : 0;
    std::vector<int32_t> i1((size_t)nq + 1), d1((size_t)nq + 1), i2((size_t)nq + 1), d2((size_t)nq + 1);
    int got = 0;
    if (orbgpu_download_matches(mCtx, 0, i1.data(), d1.data(), i2.data(), d2.data(), nq + 1, &got) != ORBGPU_OK)
        return -1;
    ++mFrameCounter;
    CacheSlot& s = mCache[mFrameCounter % MATCHING_CACHE_SIZE];
    s.frame = mFrameCounter;
    s.indices.resize(got);
    s.dist1.resize(got);
    s.dist2.resize(got);
    for (int i = 0; i < got; ++i) {
        s.indices[i] = idx16(i1[i]);
        s.dist1[i] = dist16(d1[i]);
        s.dist2[i] = dist16(d2[i]);
    }
    return mFrameCounter;
}

int LynxHardwareAccelerator::ExtractORB(int& nl, int& nr, std::vector<cv::KeyPoint>& kl, std::vector<cv::KeyPoint>& kr,
                                        cv::OutputArray& dl, cv::OutputArray& dr, int l0, int l1, int r0, int r1,
                                        int& monoLeft, int& monoRight) {
    std::lock_guard<std::mutex> g(mMutex);
    if (mFrameW <= 0) return -1;  // nothing stored
    const int32_t laps[4] = {l0, l1, r0, r1};
    if (orbgpu_run_batch_match(mCtx, 2, mFrameW, mFrameH, laps, 1, nullptr) != ORBGPU_OK) return -1;
    return finish(nl, nr, kl, kr, dl, dr, monoLeft, monoRight);
}

int LynxHardwareAccelerator::ExtractORBPair(const uint8_t* left, const uint8_t* right, int width, int height,
                                            int stride, int& nl, int& nr, std::vector<cv::KeyPoint>& kl,
                                            std::vector<cv::KeyPoint>& kr, cv::OutputArray& dl, cv::OutputArray& dr,
                                            int l0, int l1, int r0, int r1, int& monoLeft, int& monoRight) {
    std::lock_guard<std::mutex> g(mMutex);
    if (!left || !right || width <= 0 || height <= 0 || stride < width) return -1;
    if (ensure(width, height) != ORBGPU_OK) return -1;
    // both eyes as batch images 0 / 1: one upload, one device pass, the stereo-row matches after
    mStage.resize(2 * (size_t)width * height);
    for (int y = 0; y < height; ++y) {
        std::memcpy(mStage.data() + (size_t)y * width, left + (size_t)y * stride, width);
        std::memcpy(mStage.data() + ((size_t)height + y) * width, right + (size_t)y * stride, width);
    }
    const int32_t laps[4] = {l0, l1, r0, r1};
    if (orbgpu_upload_images(mCtx, mStage.data(), 2, width, height, width) != ORBGPU_OK) return -1;
    mFrameW = width;
    mFrameH = height;
    if (orbgpu_run_batch_match(mCtx, 2, width, height, laps, 1, nullptr) != ORBGPU_OK) return -1;
    return finish(nl, nr, kl, kr, dl, dr, monoLeft, monoRight);
}

void LynxHardwareAccelerator::BFMatchORB(int id, const cv::Mat& leftDescriptors, const cv::Mat& rightDescriptors,
                                         std::vector<uint16_t>& indices, std::vector<uint16_t>& dist1,
                                         std::vector<uint16_t>& dist2) const {
    std::lock_guard<std::mutex> g(mMutex);
    const CacheSlot& s = mCache[((id % MATCHING_CACHE_SIZE) + MATCHING_CACHE_SIZE) % MATCHING_CACHE_SIZE];
    if (id > 0 && s.frame == id && (int)s.indices.size() == rightDescriptors.rows) {
        indices = s.indices;
        dist1 = s.dist1;
        dist2 = s.dist2;
        return;
    }
    // not (or no longer) cached: match the rows given on the device
    const int nq = rightDescriptors.rows, nt = leftDescriptors.rows;
    std::vector<uint8_t> q = rows(rightDescriptors), t = rows(leftDescriptors);
    std::vector<int32_t> i1((size_t)nq + 1), d1((size_t)nq + 1), i2((size_t)nq + 1), d2((size_t)nq + 1);
    if (orbgpu_match_knn2(mCtx, q.data(), nq, t.data(), nt, i1.data(), d1.data(), i2.data(), d2.data()) != ORBGPU_OK)
        throw std::runtime_error(std::string("orbgpu: ") + orbgpu_last_error());
    indices.resize(nq);
    dist1.resize(nq);
    dist2.resize(nq);
    for (int i = 0; i < nq; ++i) {
        indices[i] = idx16(i1[i]);
        dist1[i] = dist16(d1[i]);
        dist2[i] = dist16(d2[i]);
    }
}

int LynxHardwareAccelerator::ExportPyramid(int eye, std::vector<cv::Mat>& pyramid) const {
    std::lock_guard<std::mutex> g(mMutex);
    pyramid.resize(mParams.nlevels);
    for (int l = 0; l < mParams.nlevels; ++l) {
        int w = 0, h = 0;
        int r = orbgpu_get_pyramid_level(mCtx, eye, l, 0, nullptr, 0, &w, &h);
        if (r != ORBGPU_OK) return r;
        pyramid[l].create(h, w, CV_8U);
        r = orbgpu_get_pyramid_level(mCtx, eye, l, 0, pyramid[l].ptr<unsigned char>(0), (int)pyramid[l].step[0],
                                     &w, &h);
        if (r != ORBGPU_OK) return r;
    }
    return ORBGPU_OK;
}

}  // namespace ORB_SLAM3
