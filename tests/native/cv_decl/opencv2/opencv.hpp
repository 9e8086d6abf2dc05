// Declaration-only subset of the OpenCV 4.x API that the reference's
// include/ORBextractor.h and adapters/orbslam3/ORBextractor.cc use, with
// OpenCV's own signatures (core/types.hpp, core/mat.hpp, core/hal/interface.h).
// Test infrastructure for the adapter against the reference header
// (tests/test_adapter.py: `g++ -fsyntax-only`; tests/test_gpu_adapter.py: the
// adapter linked with tests/native/cv_min.cpp, a minimal test-only
// implementation of this subset, into a program run on the GPU).  It stands in
// for no part of the reference itself.
#pragma once
#include <cstddef>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5
#define CV_32FC1 5
#define CV_64F 6

namespace cv {
typedef unsigned char uchar;
template <typename T> class Point_ {
public:
    Point_();
    Point_(T x, T y);
    Point_& operator*=(T s);
    T x, y;
};
typedef Point_<int> Point2i;
typedef Point_<float> Point2f;
typedef Point_<double> Point2d;
typedef Point2i Point;
template <typename T> class Point3_ {
public:
    Point3_();
    Point3_(T x, T y, T z);
    T x, y, z;
};
typedef Point3_<float> Point3f;
typedef Point3_<double> Point3d;
template <typename T> class Size_ {
public:
    Size_(T w, T h);
    T width, height;
};
typedef Size_<int> Size;

class KeyPoint {
public:
    Point2f pt;
    float size;
    float angle;
    float response;
    int octave;
    int class_id;
};

struct MatStep {
    size_t operator[](int i) const;
    size_t buf[2];
};

class _OutputArray;
class Mat {
public:
    Mat();
    Mat(int rows, int cols, int type);
    Mat(int rows, int cols, int type, void* data, size_t step = 0);
    Mat(const Mat& m);
    Mat& operator=(const Mat& m);
    ~Mat();
    void create(int rows, int cols, int type);
    Mat rowRange(int startrow, int endrow) const;
    Mat row(int y) const;
    Mat clone() const;
    void copyTo(const _OutputArray& m) const;
    void release();
    bool empty() const;
    int type() const;
    bool isContinuous() const;
    size_t elemSize() const;
    size_t total() const;
    uchar* ptr(int i0 = 0);
    const uchar* ptr(int i0 = 0) const;
    template <typename T> T* ptr(int i0 = 0);
    template <typename T> const T* ptr(int i0 = 0) const;
    template <typename T> T& at(int i0, int i1);
    template <typename T> const T& at(int i0, int i1) const;
    template <typename T> T& at(int i0);
    template <typename T> const T& at(int i0) const;
    int flags, dims, rows, cols;
    uchar* data;
    MatStep step;
    void* u;   // the shared buffer (OpenCV: UMatData*)
};

class _InputArray {
public:
    _InputArray(const Mat& m);
    Mat getMat(int idx = -1) const;
    bool empty() const;
protected:
    int flags;
    void* obj;
};
class _OutputArray : public _InputArray {
public:
    _OutputArray(Mat& m);
    _OutputArray(const Mat& m);
    void create(int rows, int cols, int type, int i = -1, bool allowTransposed = false, int fixedDepthMask = 0) const;
    void release() const;
    Mat& getMatRef(int i = -1) const;
};
typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;
}  // namespace cv
