// Declaration-only subset of Sophus (see se3.hpp): Sim3.
#pragma once
#include "se3.hpp"
namespace Sophus {
template <class S>
class RxSO3 {
public:
    RxSO3();
    S scale() const;
    Eigen::Matrix<S, 3, 3> rotationMatrix() const;
    Eigen::Matrix<S, 3, 3> matrix() const;
};
template <class S, int Opt = 0>
class Sim3 {
public:
    typedef S Scalar;
    Sim3();
    Sim3(const RxSO3<S>& sR, const Eigen::Matrix<S, 3, 1>& t);
    Sim3(const Eigen::Quaternion<S>& q, const Eigen::Matrix<S, 3, 1>& t);
    Sim3 inverse() const;
    S scale() const;
    Eigen::Matrix<S, 3, 3> rotationMatrix() const;
    Eigen::Quaternion<S> quaternion() const;
    Eigen::Matrix<S, 3, 1>& translation();
    const Eigen::Matrix<S, 3, 1>& translation() const;
    RxSO3<S>& rxso3();
    const RxSO3<S>& rxso3() const;
    Eigen::Matrix<S, 4, 4> matrix() const;
    template <class T> Sim3<T> cast() const;
    Sim3 operator*(const Sim3&) const;
    Eigen::Matrix<S, 3, 1> operator*(const Eigen::Matrix<S, 3, 1>&) const;
};
typedef Sim3<float> Sim3f;
typedef Sim3<double> Sim3d;
}  // namespace Sophus
