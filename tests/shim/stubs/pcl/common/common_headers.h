// Stand-in for <pcl/common/common_headers.h>, which brings Eigen into the aicp interfaces:
// the two Eigen types of the interface signatures, with the members the shims use
// (Matrix4f::data() column-major like Eigen's default storage, Isometry3d::translation()).
#pragma once
#include "../point_types.h"

namespace Eigen {
struct Matrix4f {
  float m[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  float* data() { return m; }
  const float* data() const { return m; }
  float& operator()(int r, int c) { return m[c * 4 + r]; }
  static Matrix4f Identity() { return Matrix4f(); }
};
struct Vector3d {
  double v[3] = {0, 0, 0};
  double& operator()(int i) { return v[i]; }
  double operator()(int i) const { return v[i]; }
};
struct Isometry3d {
  Vector3d t;
  Vector3d& translation() { return t; }
  const Vector3d& translation() const { return t; }
};
}  // namespace Eigen
