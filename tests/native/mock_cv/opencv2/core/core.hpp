// Minimal stand-in for the parts of OpenCV core that include/orbgpu_cv.hpp uses, so the shim can be
// compiled and exercised on the CPU (OpenCV is absent from this image).  Test infrastructure only:
// 8-bit single-channel matrices with shared storage, views by Rect / row ranges, KeyPoint.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_Assert(e) \
    do {             \
        if (!(e)) throw std::runtime_error("CV_Assert: " #e); \
    } while (0)

namespace cv {

struct Rect {
    int x, y, width, height;
    Rect(int x_, int y_, int w_, int h_) : x(x_), y(y_), width(w_), height(h_) {}
};

struct KeyPoint {
    struct { float x, y; } pt;
    float size, angle, response;
    int octave, class_id;
    KeyPoint() = default;
    KeyPoint(float x, float y, float s, float a, float r, int o, int c)
        : pt{x, y}, size(s), angle(a), response(r), octave(o), class_id(c) {}
};

class Mat {
public:
    int rows = 0, cols = 0;
    size_t step = 0;
    uint8_t* data = nullptr;

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    void create(int r, int c, int /*type*/) {
        if (buf_ && buf_.use_count() == 1 && r == rows && c == cols && (size_t)c == step) return;
        buf_ = std::make_shared<std::vector<uint8_t>>((size_t)r * c);
        rows = r, cols = c, step = c, data = buf_->data();
    }
    int type() const { return CV_8UC1; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    void release() { *this = Mat(); }
    Mat operator()(const Rect& rc) const {
        Mat v = *this;
        v.data = data + (size_t)rc.y * step + rc.x;
        v.rows = rc.height, v.cols = rc.width;
        return v;
    }
    Mat rowRange(int a, int b) const { return (*this)(Rect(0, a, cols, b - a)); }
    Mat colRange(int a, int b) const { return (*this)(Rect(a, 0, b - a, rows)); }
    uint8_t at(int r, int c) const { return data[(size_t)r * step + c]; }
    void copyTo(class _OutputArray dst) const;
    long use_count() const { return buf_.use_count(); }

private:
    std::shared_ptr<std::vector<uint8_t>> buf_;
};

class _InputArray {
public:
    _InputArray(const Mat& m) : m_(&m) {}
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }

private:
    const Mat* m_;
};
using InputArray = const _InputArray&;

class _OutputArray {
public:
    _OutputArray(Mat& m) : m_(&m) {}
    void release() const { m_->release(); }
    Mat& getMatRef() const { return *m_; }

private:
    Mat* m_;
};
using OutputArray = const _OutputArray&;

inline void Mat::copyTo(_OutputArray dst) const {
    Mat& d = dst.getMatRef();
    d.create(rows, cols, CV_8U);
    for (int r = 0; r < rows; ++r) std::memcpy(d.data + (size_t)r * d.step, data + (size_t)r * step, cols);
}

}  // namespace cv
