// Stand-in restating the interface of aicp_core/include/aicp_overlap/abstract_overlapper.hpp:13-19
// (computeOverlap with the poses taken by value, getOverlap; `using namespace octomap`).
#pragma once
#include "octomap/ColorOcTree.h"
#include "octomap/octomap.h"
#include "pcl/common/common_headers.h"
#include "pcl/point_types.h"

using namespace octomap;

namespace aicp {
class AbstractOverlapper {
 public:
  virtual ColorOcTree* computeOverlap(pcl::PointCloud<pcl::PointXYZ>& ref_cloud,
                                      pcl::PointCloud<pcl::PointXYZ>& read_cloud, Eigen::Isometry3d ref_pose,
                                      Eigen::Isometry3d read_pose, ColorOcTree* reading_tree) = 0;
  virtual float getOverlap() = 0;
};
}  // namespace aicp
