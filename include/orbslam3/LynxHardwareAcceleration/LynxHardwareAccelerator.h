// LynxHardwareAccelerator.h -- the reference's accelerator singleton, backed by the MI355X front-end.
//
// Same class, members and call shapes as cpp/include/LynxHardwareAcceleration/
// LynxHardwareAccelerator.h:29-52 (the Hexagon DSP session), so the reference's callers compile
// unchanged with this header first on the include path:
//   * ORBextractor.cc:125-164 (the stereo operator()): make_unique<LynxHardwareAccelerator>(),
//     StoreInputBuffer(side-by-side Y8 frame), ExtractORB(...) -> frame id;
//   * Frame.cc:1163-1164 (ComputeStereoFishEyeMatches): BFMatchORB(mnIdMatchingData,
//     stereoDescRight, stereoDescLeft, indices, dist1, dist2) -> the kNN2 of the frame's stereo
//     rows, computed on the device in the same pass as the extraction.
// Differences from the DSP session, on purpose: keypoints are the exact
// ORBextractor keypoints (float coordinates, exact angle, size, response), the counts are not
// decremented by one, and BFMatchORB returns exactly one entry per query row.  All compute is
// liborbgpu.so (include/orbgpu.h); a frame id that has left the 3-frame match cache is matched
// again on the device from the descriptors given.
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

#include "../../orbgpu.h"
#include "../cv_shim.h"

#ifndef DEFAULT_WIDTH
#define DEFAULT_WIDTH (640)   // per-eye width of the side-by-side frame (LynxHardwareAccelerator.h:20)
#endif
#ifndef DEFAULT_HEIGHT
#define DEFAULT_HEIGHT (400)  // (LynxHardwareAccelerator.h:21)
#endif
#ifndef MAX_POINTS
#define MAX_POINTS 20000
#endif

namespace ORB_SLAM3 {

constexpr int MATCHING_CACHE_SIZE = 3;  // frames whose matches stay fetchable (reference :31)

class LynxHardwareAccelerator {
public:
    static LynxHardwareAccelerator& GetInstance() {
        static LynxHardwareAccelerator instance;
        return instance;
    }
    static std::unique_ptr<LynxHardwareAccelerator> lynxHardwareAccelerator;

    // The DSP session's geometry (DEFAULT_WIDTH x DEFAULT_HEIGHT per eye) and the ORB-SLAM3 EuRoC
    // parameters; the second form takes the extractor's own.  Throws std::runtime_error when no
    // gfx950 device or liborbgpu context is available (no CPU fallback).
    LynxHardwareAccelerator();
    LynxHardwareAccelerator(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                            int width = DEFAULT_WIDTH, int height = DEFAULT_HEIGHT);
    ~LynxHardwareAccelerator();
    LynxHardwareAccelerator(const LynxHardwareAccelerator&) = delete;
    LynxHardwareAccelerator& operator=(const LynxHardwareAccelerator&) = delete;

    // Copies one side-by-side Y8 frame (2 * width x height bytes, row stride 2 * width) in.
    void StoreInputBuffer(const uint8_t* frameData) const;
    // Same, any geometry / row stride (e.g. a locked AHardwareBuffer's stride).
    void StoreInputBuffer(const uint8_t* frameData, int width, int height, int stride) const;

    // Extracts both eyes of the stored frame and matches the stereo rows ([mono, n) of each eye,
    // Frame.cc:1144-1148) left -> right.  Returns the frame id for BFMatchORB (> 0), or -1 on an
    // error (orbgpu_last_error()).
    int ExtractORB(int& leftKeypointsCount, int& rightKeypointsCount, std::vector<cv::KeyPoint>& leftKeyPoints,
                   std::vector<cv::KeyPoint>& rightKeyPoints, cv::OutputArray& leftDescriptors,
                   cv::OutputArray& rightDescriptors, int vLappingLeft0, int vLappingLeft1,
                   int vLappingRight0, int vLappingRight1, int& monoLeft, int& monoRight);
    // Same on two separate images (the rectified pinhole pair), row stride `stride`.
    int ExtractORBPair(const uint8_t* left, const uint8_t* right, int width, int height, int stride,
                       int& leftKeypointsCount, int& rightKeypointsCount, std::vector<cv::KeyPoint>& leftKeyPoints,
                       std::vector<cv::KeyPoint>& rightKeyPoints, cv::OutputArray& leftDescriptors,
                       cv::OutputArray& rightDescriptors, int vLappingLeft0, int vLappingLeft1,
                       int vLappingRight0, int vLappingRight1, int& monoLeft, int& monoRight);

    // For frame nIdMatchingData: per row i of rightDescriptors (the query: Frame.cc passes the
    // left stereo rows second) the best train row of leftDescriptors (the right stereo rows),
    // and the best / second-best Hamming distances (65535 = no second row).
    void BFMatchORB(int nIdMatchingData, const cv::Mat& leftDescriptors, const cv::Mat& rightDescriptors,
                    std::vector<uint16_t>& indices, std::vector<uint16_t>& dist1, std::vector<uint16_t>& dist2) const;

    // The last frame's (unblurred) pyramid of eye 0 / 1 (ORBextractor::mvImagePyramid).
    int ExportPyramid(int eye, std::vector<cv::Mat>& pyramid) const;

    orbgpu_ctx* context() const { return mCtx; }

private:
    int ensure(int width, int height) const;
    int finish(int& leftKeypointsCount, int& rightKeypointsCount, std::vector<cv::KeyPoint>& leftKeyPoints,
               std::vector<cv::KeyPoint>& rightKeyPoints, cv::OutputArray& leftDescriptors,
               cv::OutputArray& rightDescriptors, int& monoLeft, int& monoRight);

    struct CacheSlot {
        int frame = 0;
        std::vector<uint16_t> indices, dist1, dist2;
    };
    orbgpu_params mParams{};
    mutable orbgpu_ctx* mCtx = nullptr;
    mutable int mDevice = ORBGPU_DEVICE_CURRENT;  // the device current at construction
    mutable int mWidth = 0, mHeight = 0;  // context capacity, per eye
    mutable int mFrameW = 0, mFrameH = 0;  // geometry of the stored frame
    std::vector<uint8_t> mStage;           // host staging of ExtractORBPair
    int mFrameCounter = 0;
    CacheSlot mCache[MATCHING_CACHE_SIZE];
    mutable std::mutex mMutex;
};

}  // namespace ORB_SLAM3
