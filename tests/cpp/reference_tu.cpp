// reference_tu.cpp -- TEST (compile-only): a translation unit shaped like the reference's callers of
// the front-end, compiled against include/orbslam3 with OpenCV's API (tests/cpp/opencv_api or the
// real headers) to show they build unchanged:
//   * Frame.cc:24,26 include ORBextractor.h and ORBmatcher.h together -- ORBmatcher stays the
//     reference's own class (declared here with its shape from ORBmatcher.h:37-44);
//   * the CPU extractor call of Frame::ExtractORB (ORBextractor_old.h:56-57) and the stereo call of
//     FrameAHB::ExtractORB (FrameAHB.cc:168-177, AHardwareBuffer* in) returning mnIdMatchingData;
//   * Frame::ComputeStereoFishEyeMatches' fetch of the matches (Frame.cc:1161-1164);
//   * ComputeStereoMatches' read of mvImagePyramid (Frame.cc:834).
#include <opencv2/opencv.hpp>
#include <vector>

#include "ORBextractor.h"

namespace ORB_SLAM3 {

class ORBmatcher {  // the reference's class (ORBmatcher.h:37-44), declarations only
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true);
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);
    static const int TH_LOW;
    static const int TH_HIGH;
};

// ORBmatcher.cc:2107 as INTEGRATION.md §2 has it: the body calls the library
int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
    return orbgpu::DescriptorDistance(a, b);
}

struct FrameLike {
    ORBextractor* mpORBextractorLeft = nullptr;
    std::vector<cv::KeyPoint> mvKeys, mvKeysRight;
    cv::Mat mDescriptors, mDescriptorsRight;
    int monoLeft = 0, monoRight = 0, mnIdMatchingData = 0;

    void ExtractORB(int flag, const cv::Mat& im, const int x0, const int x1) {
        std::vector<int> vLapping = {x0, x1};
        if (flag == 0) monoLeft = (*mpORBextractorLeft)(im, cv::Mat(), mvKeys, mDescriptors, vLapping);
    }
    // FrameAHB::ExtractORB (FrameAHB.cc:168-177) as the reference writes it
    void ExtractORB(AHardwareBuffer* imagesBuffer, const int x0, const int x1, const int x0_1, const int x0_2) {
        std::vector<int> vLapping_left = {x0, x1};
        std::vector<int> vLapping_right = {x0_1, x0_2};
        monoLeft = 0;
        monoRight = 0;
        mnIdMatchingData = (*mpORBextractorLeft)(imagesBuffer, mvKeys, mDescriptors, vLapping_left, mvKeysRight,
                                                 mDescriptorsRight, vLapping_right, monoLeft, monoRight);
    }
    void ExtractORBStereo(const cv::Mat& sideBySide, int x0, int x1, int x0_1, int x0_2) {
        std::vector<int> vLapping_left = {x0, x1};
        std::vector<int> vLapping_right = {x0_1, x0_2};
        mnIdMatchingData = (*mpORBextractorLeft)(sideBySide, mvKeys, mDescriptors, vLapping_left, mvKeysRight,
                                                 mDescriptorsRight, vLapping_right, monoLeft, monoRight);
    }
    int ComputeStereoFishEyeMatches() {
        cv::Mat stereoDescLeft = mDescriptors.rowRange(monoLeft, mDescriptors.rows);
        cv::Mat stereoDescRight = mDescriptorsRight.rowRange(monoRight, mDescriptorsRight.rows);
        std::vector<uint16_t> indices, dist1, dist2;
        LynxHardwareAccelerator::lynxHardwareAccelerator->BFMatchORB(mnIdMatchingData, stereoDescRight,
                                                                     stereoDescLeft, indices, dist1, dist2);
        int good = 0;
        for (int i = 0; i < stereoDescLeft.rows; i++)
            if (dist1[i] != 0 && dist1[i] < 70) ++good;
        return good + ORBmatcher::DescriptorDistance(stereoDescLeft.row(0), stereoDescRight.row(0));
    }
    int PyramidRows(int level) { return mpORBextractorLeft->mvImagePyramid[level].rows; }
};

}  // namespace ORB_SLAM3
