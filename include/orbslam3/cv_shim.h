// cv_shim.h -- the few OpenCV 4.x types the ORB front-end facade touches, for builds without OpenCV.
//
// With real OpenCV (the ORB-SLAM3 build) define ORBGPU_WITH_OPENCV and the facade uses OpenCV's own
// cv::Mat / cv::KeyPoint / cv::_InputArray.  Without it this shim stands in, with OpenCV's API
// shape so the facade source is the same in both modes:
//   * CV_8U / CV_8UC1 are macros (opencv2/core/hal/interface.h), not cv:: names;
//   * cv::InputArray / cv::OutputArray are `const _InputArray&` / `const _OutputArray&`, whose
//     getMat / create / release / empty are const members (opencv2/core/mat.hpp);
//   * cv::Mat::step is a MatStep (step[0] = bytes per row), ptr<T>(row) is a template;
//   * cv::KeyPoint keeps its 28-byte layout (pt, size, angle, response, octave, class_id).
#pragma once
#ifdef ORBGPU_WITH_OPENCV
#include <opencv2/core/core.hpp>
#else
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#ifndef CV_8U
#define CV_8U 0
#endif
#ifndef CV_8UC1
#define CV_8UC1 0
#endif

namespace cv {

typedef unsigned char uchar;

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

struct MatStep {  // Mat::step: step[0] = bytes per row, converts to size_t like OpenCV's
    size_t p[2] = {0, 1};
    size_t operator[](int i) const { return p[i]; }
    size_t& operator[](int i) { return p[i]; }
    operator size_t() const { return p[0]; }
};

// Minimal owning/non-owning 8-bit single-channel matrix (reference-counted like cv::Mat).
class Mat {
public:
    int rows = 0, cols = 0;
    MatStep step;
    uchar* data = nullptr;
    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(int r, int c, int /*type*/, void* ext, size_t st = 0) : rows(r), cols(c), data(static_cast<uchar*>(ext)) {
        step[0] = st ? st : (size_t)c;
    }
    void create(int r, int c, int /*type*/) {
        if (r == rows && c == cols && data && own_.use_count() == 1) return;
        own_ = std::make_shared<std::vector<uchar>>((size_t)r * c);
        rows = r;
        cols = c;
        step[0] = (size_t)c;
        data = own_->data();
    }
    void release() { *this = Mat(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return CV_8UC1; }
    size_t step1() const { return step[0]; }
    bool isContinuous() const { return step[0] == (size_t)cols || rows <= 1; }
    template <class T = uchar>
    T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step[0]); }
    template <class T = uchar>
    const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + (size_t)r * step[0]); }
    Mat rowRange(int a, int b) const {
        Mat m(b - a, cols, CV_8U, data + (size_t)a * step[0], step[0]);
        m.own_ = own_;
        return m;
    }
    Mat clone() const {
        Mat m(rows, cols, CV_8U);
        for (int r = 0; r < rows; ++r) std::memcpy(m.ptr(r), ptr(r), (size_t)cols);
        return m;
    }

private:
    std::shared_ptr<std::vector<uchar>> own_;
};

// The proxies OpenCV functions take (cv::_InputArray / cv::_OutputArray over a Mat).
class _InputArray {
public:
    _InputArray() = default;
    _InputArray(const Mat& m) : m_(const_cast<Mat*>(&m)) {}
    Mat getMat(int /*idx*/ = -1) const { return m_ ? *m_ : Mat(); }
    bool empty() const { return !m_ || m_->empty(); }
    int type(int /*idx*/ = -1) const { return CV_8UC1; }

protected:
    Mat* m_ = nullptr;
};

class _OutputArray : public _InputArray {
public:
    _OutputArray() = default;
    _OutputArray(Mat& m) : _InputArray(m) {}
    void create(int rows, int cols, int type, int /*i*/ = -1, bool /*allowTransposed*/ = false,
                int /*fixedDepthMask*/ = 0) const {
        if (m_) m_->create(rows, cols, type);
    }
    void release() const {
        if (m_) m_->release();
    }
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;

inline InputArray noArray() {
    static _InputArray none;
    return none;
}

}  // namespace cv
#endif
