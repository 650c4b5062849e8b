// opencv_api/opencv2/core/core.hpp -- TEST: declaration-only restatement of the OpenCV 4.2 API
// surface the C++ facade and its callers touch (opencv2/core/hal/interface.h, core/types.hpp,
// core/mat.hpp).  No definitions: it exists so `g++ -fsyntax-only -DORBGPU_WITH_OPENCV` checks the
// facade against OpenCV's real shapes, where the build's own shim could hide a mismatch:
//   * CV_8U / CV_8UC1 are preprocessor macros (cv::CV_8U does not exist);
//   * InputArray / OutputArray are const references to the _InputArray / _OutputArray proxies
//     (not Mat&), whose getMat / create / release / empty are const members;
//   * Mat::step is a MatStep; Mat::ptr has plain and template overloads.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

typedef unsigned char uchar;
typedef unsigned short ushort;

#define CV_CN_SHIFT 3
#define CV_DEPTH_MAX (1 << CV_CN_SHIFT)
#define CV_8U 0
#define CV_MAT_DEPTH_MASK (CV_DEPTH_MAX - 1)
#define CV_MAT_DEPTH(flags) ((flags) & CV_MAT_DEPTH_MASK)
#define CV_MAKETYPE(depth, cn) (CV_MAT_DEPTH(depth) + (((cn) - 1) << CV_CN_SHIFT))
#define CV_8UC1 CV_MAKETYPE(CV_8U, 1)

namespace cv {

template <typename _Tp>
class Point_ {
public:
    Point_();
    Point_(_Tp _x, _Tp _y);
    _Tp x, y;
};
typedef Point_<float> Point2f;
typedef Point_<int> Point;

class KeyPoint {
public:
    KeyPoint();
    KeyPoint(Point2f _pt, float _size, float _angle = -1, float _response = 0, int _octave = 0, int _class_id = -1);
    Point2f pt;
    float size;
    float angle;
    float response;
    int octave;
    int class_id;
};

struct MatStep {
    MatStep();
    size_t operator[](int i) const;
    size_t& operator[](int i);
    operator size_t() const;
    size_t* p;
    size_t buf[2];
};

class Mat {
public:
    enum { AUTO_STEP = 0 };
    Mat();
    Mat(int rows, int cols, int type);
    Mat(int rows, int cols, int type, void* data, size_t step = AUTO_STEP);
    Mat(const Mat& m);
    ~Mat();
    Mat& operator=(const Mat& m);
    Mat row(int y) const;
    Mat rowRange(int startrow, int endrow) const;
    Mat clone() const;
    void create(int rows, int cols, int type);
    void release();
    bool empty() const;
    bool isContinuous() const;
    int type() const;
    size_t step1(int i = 0) const;
    uchar* ptr(int i0 = 0);
    const uchar* ptr(int i0 = 0) const;
    template <typename _Tp> _Tp* ptr(int i0 = 0);
    template <typename _Tp> const _Tp* ptr(int i0 = 0) const;
    int flags;
    int dims;
    int rows, cols;
    uchar* data;
    MatStep step;
};

class _InputArray {
public:
    _InputArray();
    _InputArray(const Mat& m);
    Mat getMat(int idx = -1) const;
    bool empty() const;
    int type(int i = -1) const;
    int rows(int i = -1) const;
    int cols(int i = -1) const;
};

class _OutputArray : public _InputArray {
public:
    enum DepthMask { DEPTH_MASK_8U = 1 << CV_8U };
    _OutputArray();
    _OutputArray(Mat& m);
    void create(int rows, int cols, int type, int i = -1, bool allowTransposed = false,
                DepthMask fixedDepthMask = static_cast<DepthMask>(0)) const;
    void release() const;
    Mat& getMatRef(int i = -1) const;
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;
InputArray noArray();

}  // namespace cv
