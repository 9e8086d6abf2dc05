// Declaration-only subset of Sophus (the reference vendors it under
// Thirdparty/Sophus; its implementation needs Eigen, which this image lacks)
// for the syntax check of adapters/orbslam3/ORBmatcher_searches.cc against the
// reference's headers (tests/test_adapter.py): SE3 / SO3 / Sim3 with the
// member functions those headers and the adapter call, Sophus's own
// signatures.  Nothing is defined; the check never links.  Test
// infrastructure; it stands in for no part of the reference itself.
#pragma once
#include "../eigen3/Eigen/Dense"

namespace Sophus {
template <class S, int Opt = 0>
class SO3 {
public:
    typedef S Scalar;
    SO3();
    SO3(const Eigen::Matrix<S, 3, 3>& R);
    SO3(const Eigen::Quaternion<S>& q);
    Eigen::Matrix<S, 3, 3> matrix() const;
    SO3 inverse() const;
    Eigen::Quaternion<S> unit_quaternion() const;
    Eigen::Matrix<S, 3, 1> log() const;
    static SO3 exp(const Eigen::Matrix<S, 3, 1>& w);
    static Eigen::Matrix<S, 3, 3> hat(const Eigen::Matrix<S, 3, 1>& w);
    template <class T> SO3<T> cast() const;
    SO3 operator*(const SO3&) const;
    Eigen::Matrix<S, 3, 1> operator*(const Eigen::Matrix<S, 3, 1>&) const;
};
typedef SO3<float> SO3f;
typedef SO3<double> SO3d;

template <class S, int Opt = 0>
class SE3 {
public:
    typedef S Scalar;
    SE3();
    SE3(const SO3<S>& R, const Eigen::Matrix<S, 3, 1>& t);
    SE3(const Eigen::Matrix<S, 3, 3>& R, const Eigen::Matrix<S, 3, 1>& t);
    SE3(const Eigen::Quaternion<S>& q, const Eigen::Matrix<S, 3, 1>& t);
    explicit SE3(const Eigen::Matrix<S, 4, 4>& T);
    SE3 inverse() const;
    Eigen::Matrix<S, 3, 1>& translation();
    const Eigen::Matrix<S, 3, 1>& translation() const;
    SO3<S>& so3();
    const SO3<S>& so3() const;
    Eigen::Matrix<S, 3, 3> rotationMatrix() const;
    Eigen::Quaternion<S> unit_quaternion() const;
    Eigen::Matrix<S, 4, 4> matrix() const;
    Eigen::Matrix<S, 3, 4> matrix3x4() const;
    Eigen::Matrix<S, 6, 1> log() const;
    static SE3 exp(const Eigen::Matrix<S, 6, 1>& a);
    template <class T> SE3<T> cast() const;
    S* data();
    const S* data() const;
    SE3 operator*(const SE3&) const;
    Eigen::Matrix<S, 3, 1> operator*(const Eigen::Matrix<S, 3, 1>&) const;
};
typedef SE3<float> SE3f;
typedef SE3<double> SE3d;
}  // namespace Sophus
