// Minimal test-only implementation of the OpenCV subset declared in
// tests/native/cv_decl/opencv2/opencv.hpp: 8-bit single-channel matrices with
// a shared, reference-counted buffer (copies share data, rowRange views,
// create() reallocates only when the shape changes), and the InputArray /
// OutputArray wrappers over a Mat.  Enough to run the drop-in extractor
// adapter (adapters/orbslam3/ORBextractor.cc) in tests/test_gpu_adapter.py;
// not OpenCV and not part of the product.
#include <opencv2/opencv.hpp>

#include <atomic>
#include <cstring>
#include <vector>

namespace cv {
namespace {
struct Block {
    std::atomic<int> ref{1};
    std::vector<uchar> buf;
};
void retain(void* u) { if (u) ++static_cast<Block*>(u)->ref; }
void drop(void* u) { if (u && --static_cast<Block*>(u)->ref == 0) delete static_cast<Block*>(u); }
}  // namespace

template <typename T> Point_<T>::Point_() : x(0), y(0) {}
template <typename T> Point_<T>::Point_(T x_, T y_) : x(x_), y(y_) {}
template <typename T> Point_<T>& Point_<T>::operator*=(T s) { x *= s; y *= s; return *this; }
template class Point_<float>;
template class Point_<int>;

size_t MatStep::operator[](int i) const { return buf[i]; }

Mat::Mat() : flags(0), dims(0), rows(0), cols(0), data(nullptr), step(), u(nullptr) { step.buf[0] = step.buf[1] = 0; }
Mat::Mat(int r, int c, int type) : Mat() { create(r, c, type); }
Mat::Mat(const Mat& m) : flags(m.flags), dims(m.dims), rows(m.rows), cols(m.cols), data(m.data), step(m.step), u(m.u) {
    retain(u);
}
Mat& Mat::operator=(const Mat& m) {
    if (this != &m) {
        retain(m.u);
        drop(u);
        flags = m.flags; dims = m.dims; rows = m.rows; cols = m.cols; data = m.data; step = m.step; u = m.u;
    }
    return *this;
}
Mat::~Mat() { drop(u); }
void Mat::create(int r, int c, int type) {
    if (u && rows == r && cols == c && type == CV_8U) return;
    release();
    Block* b = new Block();
    b->buf.assign((size_t)r * c, 0);
    u = b;
    flags = CV_8U; dims = 2; rows = r; cols = c;
    data = b->buf.data();
    step.buf[0] = (size_t)c; step.buf[1] = 1;
}
Mat Mat::rowRange(int r0, int r1) const {
    Mat m(*this);
    m.rows = r1 - r0;
    m.data = data + (size_t)r0 * step.buf[0];
    return m;
}
Mat Mat::row(int y) const { return rowRange(y, y + 1); }
Mat Mat::clone() const {
    Mat m(rows, cols, CV_8U);
    for (int y = 0; y < rows; ++y) std::memcpy(m.data + (size_t)y * m.step.buf[0], data + (size_t)y * step.buf[0], cols);
    return m;
}
void Mat::copyTo(const _OutputArray& o) const {
    o.create(rows, cols, CV_8U);
    Mat& d = o.getMatRef();
    for (int y = 0; y < rows; ++y) std::memcpy(d.data + (size_t)y * d.step.buf[0], data + (size_t)y * step.buf[0], cols);
}
void Mat::release() {
    drop(u);
    u = nullptr; data = nullptr; rows = cols = 0; dims = 0;
    step.buf[0] = step.buf[1] = 0;
}
bool Mat::empty() const { return data == nullptr || rows == 0 || cols == 0; }
int Mat::type() const { return CV_8U; }

_InputArray::_InputArray(const Mat& m) : flags(0), obj(const_cast<Mat*>(&m)) {}
Mat _InputArray::getMat(int) const { return *static_cast<Mat*>(obj); }
bool _InputArray::empty() const { return static_cast<Mat*>(obj)->empty(); }
_OutputArray::_OutputArray(Mat& m) : _InputArray(m) {}
_OutputArray::_OutputArray(const Mat& m) : _InputArray(m) {}
void _OutputArray::create(int r, int c, int type, int, bool, int) const { static_cast<Mat*>(obj)->create(r, c, type); }
void _OutputArray::release() const { static_cast<Mat*>(obj)->release(); }
Mat& _OutputArray::getMatRef(int) const { return *static_cast<Mat*>(obj); }
}  // namespace cv
