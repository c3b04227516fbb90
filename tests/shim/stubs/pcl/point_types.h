// Stand-in for PCL's point types (PCL is not in this image): only the memory layout and the
// members the shims touch. pcl::PointXYZ is 16 B (x, y, z, pad), PointXYZRGB 32 B, and
// PointXYZRGBNormal 48 B, with x, y, z first in every row, as in PCL 1.8.
#pragma once
#include <stdint.h>

#include <cstddef>
#include <vector>

namespace pcl {
struct alignas(16) PointXYZ {
  float x = 0, y = 0, z = 0, pad = 1;
};
struct alignas(16) PointXYZRGB {
  float x = 0, y = 0, z = 0, pad = 1;
  float rgb = 0, pad2[3] = {0, 0, 0};
};
struct alignas(16) PointXYZRGBNormal {
  float x = 0, y = 0, z = 0, pad = 1;
  float normal_x = 0, normal_y = 0, normal_z = 0, pad3 = 0;
  float rgb = 0, curvature = 0, pad4[2] = {0, 0};
};
static_assert(sizeof(PointXYZ) == 16 && sizeof(PointXYZRGB) == 32 && sizeof(PointXYZRGBNormal) == 48,
              "PCL point layouts");

template <class PointT>
struct PointCloud {
  std::vector<PointT> points;
  uint32_t width = 0, height = 1;
  size_t size() const { return points.size(); }
  void resize(size_t n) {
    points.resize(n);
    width = (uint32_t)n;
    height = 1;
  }
};
}  // namespace pcl
