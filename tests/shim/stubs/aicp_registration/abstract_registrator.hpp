// Stand-in restating the interface of aicp_core/include/aicp_registration/abstract_registrator.hpp:8-19
// (pure virtual registerClouds over PointXYZ / PointXYZRGB / PointXYZRGBNormal clouds,
// getInitializedReading, getOutputReading, updateConfigParams; no virtual destructor), so the
// drop-in shim compiles against the same declarations in this image, which has no PCL / Eigen.
#pragma once
#include <string>

#include "pcl/common/common_headers.h"
#include "pcl/point_types.h"

namespace aicp {
class AbstractRegistrator {
 public:
  virtual void registerClouds(pcl::PointCloud<pcl::PointXYZ>& cloud_ref, pcl::PointCloud<pcl::PointXYZ>& cloud_read,
                              Eigen::Matrix4f& final_transform) = 0;
  virtual void registerClouds(pcl::PointCloud<pcl::PointXYZRGB>& cloud_ref,
                              pcl::PointCloud<pcl::PointXYZRGB>& cloud_read, Eigen::Matrix4f& final_transform) = 0;
  virtual void registerClouds(pcl::PointCloud<pcl::PointXYZRGBNormal>& cloud_ref,
                              pcl::PointCloud<pcl::PointXYZRGBNormal>& cloud_read,
                              Eigen::Matrix4f& final_transform) = 0;
  virtual void getInitializedReading(pcl::PointCloud<pcl::PointXYZ>& initialized_reading) = 0;
  virtual void getOutputReading(pcl::PointCloud<pcl::PointXYZ>& out_read_cloud) = 0;
  virtual void updateConfigParams(std::string config_name) = 0;
};
}  // namespace aicp
