// Test model only — NOT part of the adapter.
//
// The smallest subset of Eigen 3, Sophus and OpenCV that the reference's Map / KeyFrame / MapPoint /
// Frame / Settings headers expose through the members the adapter calls (Modules/Map/*.h,
// Modules/Mapping/Frame.h, Modules/System/Settings.h), so that adapter/src/*.cc compiles and runs
// in this image, which has none of those libraries.  In the reference tree the adapter is compiled
// against the real headers instead; it uses only calls that exist there with the same meaning:
//   Eigen:   Vector3f/Vector3d/Vector2f (x(), y(), z(), operator(), cast<T>(), norm()),
//            Quaternionf/Quaterniond (ctor (w, x, y, z), x() y() z() w(), cast<T>())
//   Sophus:  SE3f (ctor (Quaternionf, Vector3f), unit_quaternion(), translation(), inverse())
//   OpenCV:  cv::KeyPoint (pt.x, pt.y, octave), cv::Point2f
//
// Arithmetic that reaches the solver follows the restatements the native library already pins:
// SO3 construction from a quaternion normalizes in float by the reciprocal of its norm, and the
// inverse is the conjugate with -(R^T t) by Eigen's quaternion-vector product — exactly
// deftri_global_insert (csrc/deformation.cpp), so that a map driven through this model and a map
// driven through the native outer loop hold the same global-transformation entries bit for bit.
#pragma once

#include <cmath>
#include <cstddef>

namespace Eigen {

template <typename S, int N>
struct Vec {
    S v[N];
    Vec() : v{} {}
    template <int M = N, typename = typename std::enable_if<M == 2>::type>
    Vec(S a, S b) : v{a, b} {}
    template <int M = N, typename = typename std::enable_if<M == 3>::type>
    Vec(S a, S b, S c) : v{a, b, c} {}
    S &operator()(int i) { return v[i]; }
    S operator()(int i) const { return v[i]; }
    S &operator[](int i) { return v[i]; }
    S operator[](int i) const { return v[i]; }
    S x() const { return v[0]; }
    S y() const { return v[1]; }
    template <int M = N, typename = typename std::enable_if<(M >= 3)>::type>
    S z() const { return v[2]; }
    S *data() { return v; }
    const S *data() const { return v; }
    static constexpr int size() { return N; }
    template <typename T>
    Vec<T, N> cast() const {
        Vec<T, N> r;
        for (int i = 0; i < N; i++) r.v[i] = (T)v[i];
        return r;
    }
    S squaredNorm() const {
        S s = 0;
        for (int i = 0; i < N; i++) s += v[i] * v[i];
        return s;
    }
    S norm() const { return std::sqrt(squaredNorm()); }
    Vec operator-(const Vec &o) const {
        Vec r;
        for (int i = 0; i < N; i++) r.v[i] = v[i] - o.v[i];
        return r;
    }
    Vec operator+(const Vec &o) const {
        Vec r;
        for (int i = 0; i < N; i++) r.v[i] = v[i] + o.v[i];
        return r;
    }
    Vec operator*(S s) const {
        Vec r;
        for (int i = 0; i < N; i++) r.v[i] = v[i] * s;
        return r;
    }
};

using Vector2f = Vec<float, 2>;
using Vector3f = Vec<float, 3>;
using Vector3d = Vec<double, 3>;

template <typename S>
struct Quaternion {
    S qx, qy, qz, qw;
    Quaternion() : qx(0), qy(0), qz(0), qw(1) {}
    Quaternion(S w, S x, S y, S z) : qx(x), qy(y), qz(z), qw(w) {}   // Eigen's (w, x, y, z) order
    S x() const { return qx; }
    S y() const { return qy; }
    S z() const { return qz; }
    S w() const { return qw; }
    template <typename T>
    Quaternion<T> cast() const { return Quaternion<T>((T)qw, (T)qx, (T)qy, (T)qz); }
    Quaternion conjugate() const { return Quaternion(qw, -qx, -qy, -qz); }
    // q * v, Eigen's _transformVector: uv = 2 (q.vec() x v); v + w uv + q.vec() x uv
    Vec<S, 3> operator*(const Vec<S, 3> &p) const {
        S uv[3] = {qy * p[2] - qz * p[1], qz * p[0] - qx * p[2], qx * p[1] - qy * p[0]};
        for (S &u : uv) u += u;
        const S cx[3] = {qy * uv[2] - qz * uv[1], qz * uv[0] - qx * uv[2], qx * uv[1] - qy * uv[0]};
        Vec<S, 3> r;
        for (int k = 0; k < 3; k++) r[k] = (p[k] + qw * uv[k]) + cx[k];
        return r;
    }
};

using Quaternionf = Quaternion<float>;
using Quaterniond = Quaternion<double>;

}  // namespace Eigen

namespace Sophus {

template <typename S>
class SO3 {
public:
    SO3() = default;
    explicit SO3(const Eigen::Quaternion<S> &q) : q_(q) {
        const S n2 = ((q_.qx * q_.qx + q_.qy * q_.qy) + q_.qz * q_.qz) + q_.qw * q_.qw;
        const S inv = S(1) / std::sqrt(n2);
        q_.qx *= inv;
        q_.qy *= inv;
        q_.qz *= inv;
        q_.qw *= inv;
    }
    const Eigen::Quaternion<S> &unit_quaternion() const { return q_; }
    SO3 inverse() const {
        SO3 r;
        r.q_ = q_.conjugate();
        return r;
    }
    Eigen::Vec<S, 3> operator*(const Eigen::Vec<S, 3> &p) const { return q_ * p; }

private:
    Eigen::Quaternion<S> q_;
};

template <typename S>
class SE3 {
public:
    SE3() = default;
    SE3(const Eigen::Quaternion<S> &q, const Eigen::Vec<S, 3> &t) : so3_(q), t_(t) {}
    SE3(const SO3<S> &r, const Eigen::Vec<S, 3> &t) : so3_(r), t_(t) {}
    const Eigen::Quaternion<S> &unit_quaternion() const { return so3_.unit_quaternion(); }
    const Eigen::Vec<S, 3> &translation() const { return t_; }
    const SO3<S> &so3() const { return so3_; }
    SE3 inverse() const {
        const SO3<S> ri = so3_.inverse();
        Eigen::Vec<S, 3> ti = ri * t_;
        for (int k = 0; k < 3; k++) ti[k] = -ti[k];
        return SE3(ri, ti);
    }
    Eigen::Vec<S, 3> operator*(const Eigen::Vec<S, 3> &p) const { return so3_ * p + t_; }

private:
    SO3<S> so3_;
    Eigen::Vec<S, 3> t_;
};

using SO3f = SO3<float>;
using SE3f = SE3<float>;

}  // namespace Sophus

namespace cv {
struct Point2f {
    float x = 0.f, y = 0.f;
};
struct KeyPoint {
    Point2f pt;
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
};
}  // namespace cv
