// Test stub (NOT OpenCV): the handful of cv:: types the reference's call sites and
// the drop-in headers touch, so tests/dropin/dropin_calls.cpp compiles in this
// image, which has no OpenCV.  Written for the test; the layouts that matter
// (cv::KeyPoint = 28 bytes; Mat data / step / rows / cols) follow OpenCV's.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_32F 5

namespace cv {

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
    Point2f &operator*=(float s) { x *= s; y *= s; return *this; }
};

struct KeyPoint {
    Point2f pt;
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
    KeyPoint() = default;
    KeyPoint(Point2f p, float sz, float a = -1, float r = 0, int o = 0, int c = -1)
        : pt(p), size(sz), angle(a), response(r), octave(o), class_id(c) {}
};

struct MatStep {
    size_t s[2] = {0, 1};
    size_t operator[](int i) const { return s[i]; }
    operator size_t() const { return s[0]; }
};

class Mat {
public:
    int rows = 0, cols = 0;
    uint8_t *data = nullptr;
    MatStep step;
    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    void create(int r, int c, int type) {
        const size_t es = type == CV_32F ? 4 : 1;
        buf_ = std::make_shared<std::vector<uint8_t>>((size_t)r * c * es);
        rows = r;
        cols = c;
        elem_ = es;
        step.s[0] = (size_t)c * es;
        data = buf_->data();
    }
    void release() { *this = Mat(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    Mat clone() const {
        Mat m;
        if (empty()) return m;
        m.create(rows, cols, elem_ == 4 ? CV_32F : CV_8U);
        for (int y = 0; y < rows; y++) std::memcpy(m.data + y * m.step[0], data + y * step[0], cols * elem_);
        return m;
    }
    Mat row(int i) const {  // a 1 x cols view
        Mat m = *this;
        m.rows = 1;
        m.data = data + (size_t)i * step[0];
        return m;
    }
    template <class T>
    T *ptr(int r = 0) { return reinterpret_cast<T *>(data + (size_t)r * step[0]); }
    template <class T>
    const T *ptr(int r = 0) const { return reinterpret_cast<const T *>(data + (size_t)r * step[0]); }

private:
    std::shared_ptr<std::vector<uint8_t>> buf_;
    size_t elem_ = 1;
};

class _InputArray {
public:
    _InputArray(const Mat &m) : m_(&m) {}
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }

private:
    const Mat *m_;
};
class _OutputArray {
public:
    _OutputArray(Mat &m) : m_(&m) {}
    void create(int r, int c, int type) const { m_->create(r, c, type); }
    Mat getMat() const { return *m_; }
    void release() const { m_->release(); }

private:
    Mat *m_;
};
typedef const _InputArray &InputArray;
typedef const _OutputArray &OutputArray;

}  // namespace cv
