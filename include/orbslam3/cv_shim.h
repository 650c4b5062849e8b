// cv_shim.h -- the few OpenCV types the ORB front-end facade touches, for builds without OpenCV.
//
// With real OpenCV (the ORB-SLAM3 build), define ORBGPU_WITH_OPENCV before including
// ORBextractor.h and the facade uses cv::Mat / cv::KeyPoint / cv::InputArray directly.  This shim
// keeps the same field layout (cv::KeyPoint = 28 bytes) so results can be memcpy'd either way.
#pragma once
#ifdef ORBGPU_WITH_OPENCV
#include <opencv2/core/core.hpp>
#else
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace cv {

enum { CV_8U = 0, CV_8UC1 = 0 };

struct Point2f {
    float x = 0, y = 0;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};

// Minimal owning/non-owning 8-bit single-channel matrix.
class Mat {
public:
    int rows = 0, cols = 0;
    size_t step = 0;
    uint8_t* data = nullptr;
    Mat() = default;
    Mat(int r, int c, int /*type*/ = CV_8U) { create(r, c, CV_8U); }
    Mat(int r, int c, int /*type*/, void* ext, size_t st = 0)
        : rows(r), cols(c), step(st ? st : (size_t)c), data(static_cast<uint8_t*>(ext)) {}
    void create(int r, int c, int /*type*/ = CV_8U) {
        if (r == rows && c == cols && data && own_) return;
        own_ = std::make_shared<std::vector<uint8_t>>((size_t)r * c);
        rows = r;
        cols = c;
        step = (size_t)c;
        data = own_->data();
    }
    void release() { *this = Mat(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return CV_8UC1; }
    size_t step1() const { return step; }
    Mat getMat() const { return *this; }
    uint8_t* ptr(int r = 0) { return data + (size_t)r * step; }
    const uint8_t* ptr(int r = 0) const { return data + (size_t)r * step; }
    Mat rowRange(int a, int b) const { return Mat(b - a, cols, CV_8U, data + (size_t)a * step, step); }
    Mat clone() const {
        Mat m(rows, cols);
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols; ++c) m.data[(size_t)r * m.step + c] = data[(size_t)r * step + c];
        return m;
    }

private:
    std::shared_ptr<std::vector<uint8_t>> own_;
};

using InputArray = const Mat&;
using OutputArray = Mat&;

}  // namespace cv
#endif
