// TEST DOUBLE — not OpenCV. OpenCV is absent from this image, so include/dofs_cv.hpp is compiled against this
// minimal stand-in of the few cv:: types the adapter touches (Mat with rows / cols / step / type / ptr,
// Point_, Matx33f) to check that the adapter compiles and converts correctly. It is used only by
// tests/cv_adapter/test_cv_adapter.cpp; a real host builds the adapter against its own OpenCV.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#define CV_32S 4
#define CV_32FC2 13

namespace cv {
template <class T>
struct Point_ {
    T x, y;
    Point_() : x(0), y(0) {}
    Point_(T a, T b) : x(a), y(b) {}
};
using Point2f = Point_<float>;
using Point2i = Point_<int>;

struct Matx33f {
    float val[9];
    Matx33f() {
        for (float& v : val) v = 0.f;
    }
    float operator()(int r, int c) const { return val[3 * r + c]; }
};

class Mat {
public:
    int rows = 0, cols = 0, dims = 2;
    size_t step = 0;
    unsigned char* data = nullptr;
    Mat() {}
    Mat(int r, int c, int type) : rows(r), cols(c), t_(type) {
        step = (size_t)c * (type == CV_32FC2 ? 8 : 4);
        buf_ = std::make_shared<std::vector<unsigned char>>(step * (size_t)r);
        data = buf_->data();
    }
    int type() const { return t_; }
    template <class T>
    T* ptr(int y = 0) {
        return reinterpret_cast<T*>(data + step * (size_t)y);
    }
    template <class T>
    const T* ptr(int y = 0) const {
        return reinterpret_cast<const T*>(data + step * (size_t)y);
    }
    Mat clone() const {
        Mat m(rows, cols, t_);
        *m.buf_ = *buf_;
        return m;
    }

private:
    int t_ = 0;
    std::shared_ptr<std::vector<unsigned char>> buf_;
};
}  // namespace cv
