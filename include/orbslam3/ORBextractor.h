// ORBextractor.h -- source-compatible ORB_SLAM3::ORBextractor backed by the MI355X front-end.
//
// Same public surface as the reference's CPU extractor (cpp/include/ORBextractor_old.h:45-116):
// the 5-parameter ctor, operator()(image, mask, keypoints, descriptors, vLappingArea) returning
// monoIndex, the scale getters and the public mvImagePyramid; plus the stereo entry point of the
// DSP-backed extractor (cpp/include/ORBextractor.h:52-57), which returns the frame id whose
// matches LynxHardwareAccelerator::BFMatchORB fetches (Frame.cc:1164).  The stereo form takes
// the AHardwareBuffer itself (as FrameAHB.cc:176 passes it), the side-by-side Y8 frame as a
// cv::Mat (2W x H), or two images.
// ORBmatcher stays the reference's own class (cpp/include/ORBmatcher.h:37-44); its
// DescriptorDistance body can call orbgpu::DescriptorDistance below.
// Everything computes on the GPU through include/orbgpu.h.
#pragma once
#include <cstdint>
#include <vector>

#include "../orbgpu.h"
#include "LynxHardwareAcceleration/LynxHardwareAccelerator.h"
#include "cv_shim.h"

// <android/hardware_buffer.h>'s opaque buffer type: only pointers to it cross this header.
struct AHardwareBuffer;

namespace ORB_SLAM3 {

// How the AHardwareBuffer form of operator() reads a buffer (ORBextractor.cc:133-147 does
// AHardwareBuffer_describe + AHardwareBuffer_lock(CPU_READ_OFTEN), then unlocks once the frame is
// copied): lock maps the side-by-side Y8 frame for reading and reports its full width (both eyes),
// height and row stride in bytes, returning 0 on success; unlock releases it.  Under __ANDROID__
// the default is exactly those NDK calls; elsewhere there is no default and the caller installs one
// (a camera SDK's buffer type, a test double).
struct AHardwareBufferAccess {
    int (*lock)(AHardwareBuffer* buffer, const uint8_t** data, int* width, int* height, int* stride);
    void (*unlock)(AHardwareBuffer* buffer);
};
void SetAHardwareBufferAccess(const AHardwareBufferAccess& access);

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
    ~ORBextractor();
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // Compute the ORB features and descriptors on an image (mask is ignored, as in the
    // reference).  Returns the number of keypoints outside vLappingArea (written first); the
    // lapping-area keypoints follow in reverse order.  -1 on an empty image (:1092-1093) or a
    // device error (lastStatus()).
    int operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                   cv::OutputArray _descriptors, std::vector<int>& vLappingArea);

    // Stereo form of the headset (ORBextractor.h:52-57, ORBextractor.cc:118-165; called by
    // FrameAHB::ExtractORB, FrameAHB.cc:176): the AHardwareBuffer holds one side-by-side Y8 frame,
    // left eye in columns [0, W), right eye in [W, 2W).  It is locked (SetAHardwareBufferAccess),
    // copied to the device and unlocked, then both eyes and the stereo-row kNN2 run in one device
    // pass; returns the frame id (for LynxHardwareAccelerator::BFMatchORB), -1 on an error (no
    // lock function, lock failure, odd width, device error: lastStatus()).
    int operator()(AHardwareBuffer* _image, std::vector<cv::KeyPoint>& _keypointsLeft,
                   cv::OutputArray _descriptorsLeft, std::vector<int>& vLappingAreaLeft,
                   std::vector<cv::KeyPoint>& _keypointsRight, cv::OutputArray _descriptorsRight,
                   std::vector<int>& vLappingAreaRight, int& monoLeft, int& monoRight);

    // Same with the side-by-side frame as an image (2W x H).
    int operator()(cv::InputArray _image, std::vector<cv::KeyPoint>& _keypointsLeft,
                   cv::OutputArray _descriptorsLeft, std::vector<int>& vLappingAreaLeft,
                   std::vector<cv::KeyPoint>& _keypointsRight, cv::OutputArray _descriptorsRight,
                   std::vector<int>& vLappingAreaRight, int& monoLeft, int& monoRight);

    // Same on two separate images of one rectified pair.
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

    // Status of the last call (orbgpu status code, 0 = OK).
    int lastStatus() const { return mStatus; }

protected:
    int ensureContext(int width, int height);
    void exportPyramid(int image);
    LynxHardwareAccelerator* accelerator(int width, int height);
    int extractStored(LynxHardwareAccelerator* acc, std::vector<cv::KeyPoint>& kl, cv::OutputArray dl,
                      std::vector<int>& lapL, std::vector<cv::KeyPoint>& kr, cv::OutputArray dr,
                      std::vector<int>& lapR, int& monoLeft, int& monoRight);

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
    // the HIP device current when the extractor was built (ORBGPU_DEVICE_CURRENT); a context
    // regrown for a larger image stays on it
    int mDevice = ORBGPU_DEVICE_CURRENT;
    int mStatus = 0;
    std::vector<orbgpu_keypoint> mKps;
    std::vector<uint8_t> mDesc;
};

namespace orbgpu {
// ORBmatcher::DescriptorDistance (ORBmatcher.cc:2107-2123) on two 32-byte descriptor rows.
inline int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
    return orbgpu_descriptor_distance(a.ptr<unsigned char>(0), b.ptr<unsigned char>(0));
}
}  // namespace orbgpu

}  // namespace ORB_SLAM3
