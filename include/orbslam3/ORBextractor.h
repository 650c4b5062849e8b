// ORBextractor.h -- source-compatible ORB_SLAM3::ORBextractor backed by the MI355X front-end.
//
// Same public surface as the reference's CPU extractor (cpp/include/ORBextractor_old.h:45-116):
// the 5-parameter ctor, operator()(image, mask, keypoints, descriptors, vLappingArea) returning
// monoIndex, the scale getters and the public mvImagePyramid, plus the stereo entry point of the
// DSP-backed extractor (cpp/include/ORBextractor.h:52-57) taking two images instead of an
// AHardwareBuffer.  ORBmatcher::DescriptorDistance (cpp/include/ORBmatcher.h:44) is provided as
// a static helper.  Everything computes on the GPU through include/orbgpu.h; Tracking / Frame
// code compiles unchanged against it.
#pragma once
#include <vector>

#include "../orbgpu.h"
#include "cv_shim.h"

namespace ORB_SLAM3 {

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
    ~ORBextractor();
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // Compute the ORB features and descriptors on an image (mask is ignored, as in the
    // reference).  Returns the number of keypoints outside vLappingArea (written first); the
    // lapping-area keypoints follow in reverse order.  -1 on an empty image.
    int operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                   cv::OutputArray _descriptors, std::vector<int>& vLappingArea);

    // Stereo form: both eyes in one device pass (ORBextractor.h:52-57 semantics).
    int operator()(cv::InputArray left, cv::InputArray right, std::vector<cv::KeyPoint>& keypointsLeft,
                   cv::OutputArray descriptorsLeft, std::vector<int>& vLappingAreaLeft,
                   std::vector<cv::KeyPoint>& keypointsRight, cv::OutputArray descriptorsRight,
                   std::vector<int>& vLappingAreaRight, int& monoLeft, int& monoRight);

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    // Filled after every call (Frame::ComputeStereoMatches reads it); set
    // mbExportPyramid = false to skip the device->host copy when nobody reads it.
    std::vector<cv::Mat> mvImagePyramid;
    bool mbExportPyramid = true;

    // Device, image-size limits and status of the underlying context.
    int lastStatus() const { return mStatus; }

protected:
    int ensureContext(int width, int height);
    void exportPyramid(int image);

    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;

    orbgpu_ctx* mCtx = nullptr;
    int mCtxW = 0, mCtxH = 0;
    int mStatus = 0;
    std::vector<orbgpu_keypoint> mKps[2];
};

class ORBmatcher {
public:
    // Bit-count Hamming distance of two 32-byte descriptors (ORBmatcher.cc:2107-2123).
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
        return orbgpu_descriptor_distance(a.ptr(0), b.ptr(0));
    }
};

}  // namespace ORB_SLAM3
