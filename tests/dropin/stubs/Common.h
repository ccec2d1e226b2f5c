// Test stub of the reference's include/Common.h (NOT Eigen / Sophus): the few
// vector / pose types and operations the reference's call sites and the
// drop-in headers use, in float, so the drop-in test builds in this image
// (no Eigen, no Sophus, no OpenCV).  Written for the test.
#pragma once
#include <cmath>
#include <list>
#include <map>
#include <set>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

namespace Eigen {

struct Vector2f {
    float v[2] = {0.f, 0.f};
    Vector2f() = default;
    Vector2f(float x, float y) { v[0] = x; v[1] = y; }
    float &operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
    Vector2f operator*(float s) const { return Vector2f(v[0] * s, v[1] * s); }
};

struct Vector3f {
    float v[3] = {0.f, 0.f, 0.f};
    Vector3f() = default;
    Vector3f(float x, float y, float z) { v[0] = x; v[1] = y; v[2] = z; }
    float &operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
    Vector3f operator+(const Vector3f &o) const { return Vector3f(v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2]); }
    Vector3f operator-(const Vector3f &o) const { return Vector3f(v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]); }
    float norm() const { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
};

struct Matrix3f {
    float m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    float &operator()(int r, int c) { return m[3 * r + c]; }
    float operator()(int r, int c) const { return m[3 * r + c]; }
    Vector3f operator*(const Vector3f &p) const {
        return Vector3f(m[0] * p[0] + m[1] * p[1] + m[2] * p[2], m[3] * p[0] + m[4] * p[1] + m[5] * p[2],
                        m[6] * p[0] + m[7] * p[1] + m[8] * p[2]);
    }
    Matrix3f transpose() const {
        Matrix3f t;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) t.m[3 * r + c] = m[3 * c + r];
        return t;
    }
};
inline Matrix3f operator*(int s, const Matrix3f &a) {
    Matrix3f t;
    for (int i = 0; i < 9; i++) t.m[i] = (float)s * a.m[i];
    return t;
}

template <class T, int R, int C>
struct Matrix {
    T d[R * C];
    T &operator()(int r, int c) { return d[r * C + c]; }
    T operator()(int r, int c) const { return d[r * C + c]; }
};

struct Quaternionf {
    float w_ = 1.f, x_ = 0.f, y_ = 0.f, z_ = 0.f;
    Quaternionf() = default;
    Quaternionf(float w, float x, float y, float z) : w_(w), x_(x), y_(y), z_(z) {}
    float w() const { return w_; }
    float x() const { return x_; }
    float y() const { return y_; }
    float z() const { return z_; }
    Quaternionf operator*(const Quaternionf &b) const {
        return Quaternionf(w_ * b.w_ - x_ * b.x_ - y_ * b.y_ - z_ * b.z_, w_ * b.x_ + x_ * b.w_ + y_ * b.z_ - z_ * b.y_,
                           w_ * b.y_ + y_ * b.w_ + z_ * b.x_ - x_ * b.z_, w_ * b.z_ + z_ * b.w_ + x_ * b.y_ - y_ * b.x_);
    }
    Quaternionf conjugate() const { return Quaternionf(w_, -x_, -y_, -z_); }
    Vector3f rotate(const Vector3f &v) const {  // v + 2w (u x v) + 2 u x (u x v)
        const float uv0 = 2 * (y_ * v[2] - z_ * v[1]), uv1 = 2 * (z_ * v[0] - x_ * v[2]), uv2 = 2 * (x_ * v[1] - y_ * v[0]);
        return Vector3f(v[0] + w_ * uv0 + (y_ * uv2 - z_ * uv1), v[1] + w_ * uv1 + (z_ * uv0 - x_ * uv2),
                        v[2] + w_ * uv2 + (x_ * uv1 - y_ * uv0));
    }
    Matrix3f toRotationMatrix() const {
        Matrix3f R;
        const Vector3f c0 = rotate(Vector3f(1, 0, 0)), c1 = rotate(Vector3f(0, 1, 0)), c2 = rotate(Vector3f(0, 0, 1));
        for (int r = 0; r < 3; r++) {
            R.m[3 * r + 0] = c0[r];
            R.m[3 * r + 1] = c1[r];
            R.m[3 * r + 2] = c2[r];
        }
        return R;
    }
};

}  // namespace Eigen

namespace Sophus {

struct SE3f {
    typedef Eigen::Vector3f Point;
    Eigen::Quaternionf q;
    Eigen::Vector3f t;
    SE3f() = default;
    SE3f(const Eigen::Quaternionf &q_, const Point &t_) : q(q_), t(t_) {}
    SE3f operator*(const SE3f &o) const { return SE3f(q * o.q, q.rotate(o.t) + t); }
    Point operator*(const Point &p) const { return q.rotate(p) + t; }
    SE3f inverse() const {
        const Eigen::Quaternionf qi = q.conjugate();
        const Point ti = qi.rotate(t);
        return SE3f(qi, Point(-ti[0], -ti[1], -ti[2]));
    }
    const Eigen::Quaternionf &unit_quaternion() const { return q; }
    const Point &translation() const { return t; }
    Eigen::Matrix3f rotationMatrix() const { return q.toRotationMatrix(); }
};

}  // namespace Sophus

namespace DBoW2 {
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
typedef std::map<NodeId, std::vector<unsigned int>> FeatureVector;
typedef std::map<WordId, WordValue> BowVector;
}  // namespace DBoW2

namespace ygz {
class ORBVocabulary;  // TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary.h): only its address is used
}  // namespace ygz

namespace ygz {
using namespace std;
using cv::Mat;
using Eigen::Matrix3f;
using Eigen::Vector2f;
using Eigen::Vector3f;
using Sophus::SE3f;
}  // namespace ygz
