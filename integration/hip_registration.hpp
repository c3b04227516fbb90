// hip_registration.hpp — drop-in AbstractRegistrator / AbstractOverlapper over libaicp_hip.so.
//
// A maintainer of aicp_core adds this header next to pointmatcher_registration.hpp and one
// `else if (parameters.type == "HIP")` branch to each factory:
//   aicp::HipRegistration  implements aicp::AbstractRegistrator
//                          (aicp_core/include/aicp_registration/abstract_registrator.hpp:8-19)
//   aicp::HipOverlapper    implements aicp::AbstractOverlapper
//                          (aicp_core/include/aicp_overlap/abstract_overlapper.hpp:13-19)
// The compute goes through the C-ABI of include/aicp_hip.h only. tests/shim/ compiles this
// header against stand-in declarations of the two interfaces (tests/test_shim.py).
//
// Behaviour kept from the reference:
//   - registerClouds(PointXYZ) / (PointXYZRGB): counts = cloud.width (cloudIO.cpp:83), xyz
//     read in place at the point stride (16 / 32 B), identity initial transform
//     (pointmatcher_registration.cpp:104-111), T written column-major into the Matrix4f.
//   - registerClouds(PointXYZRGBNormal) is a no-op, as the reference's body is commented out
//     (pointmatcher_registration.cpp:36-45).
//   - PM::ConvergenceError / TransformationError are not caught in App (app.cpp:210): the shim
//     throws std::runtime_error for AICP_ERR_CONVERGENCE / AICP_ERR_TRANSFORMATION.
//   - A missing chain file exits the process (pointmatcher_registration.cpp:59-64).
//   - getOutputReading = T * reading (pointmatcher_registration.cpp:128-131).
//   - computeOverlap: sensor origins = pose translations (octrees_overlap.cpp:184,229-230),
//     resolution read as float (yaml_configurator.cpp:81); App ignores the returned tree
//     (app.cpp:132-135), so nullptr is returned.
//
// Ownership. AbstractRegistrator / AbstractOverlapper declare no virtual destructor, and the
// factories return std::unique_ptr to the base, so deleting a shim skips its members'
// destructors: HipRegistration's RegistrationParams strings and the reading copy (read_xyz_),
// HipOverlapper's OverlapParams. That leaks those host allocations once per registrator, as the
// reference's PointmatcherRegistration leaks its DataPoints members the same way. App creates
// one of each per process (app.cpp:32-34), so this is bounded; a maintainer removes it upstream
// by adding `virtual ~AbstractRegistrator() = default;` (and the same to AbstractOverlapper).
// Device memory is not involved: the HIP context is one per process (hip_shared_ctx).
#ifndef AICP_HIP_REGISTRATION_HPP_
#define AICP_HIP_REGISTRATION_HPP_

#include <cstdlib>
#include <fstream>
#include <iostream>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "aicp_hip.h"
#include "aicp_overlap/abstract_overlapper.hpp"
#include "aicp_overlap/common.hpp"
#include "aicp_registration/abstract_registrator.hpp"
#include "aicp_registration/common.hpp"

namespace aicp {

// The process-wide device context (App calls both interfaces from its one worker thread,
// app.cpp:528-550). Throws std::runtime_error when no HIP device is usable.
inline aicp_hip_ctx* hip_shared_ctx() {
  static std::mutex mu;
  static aicp_hip_ctx* ctx = nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!ctx) {
    const char* dev = std::getenv("AICP_HIP_DEVICE");
    const int rc = aicp_hip_create(dev ? std::atoi(dev) : 0, &ctx);
    if (rc != AICP_OK) {
      ctx = nullptr;
      throw std::runtime_error("aicp_hip_create failed (" + std::to_string(rc) + "): no usable HIP device");
    }
  }
  return ctx;
}

inline void hip_throw_on_error(int rc) {
  if (rc == AICP_OK) return;
  const std::string msg = aicp_hip_last_error(hip_shared_ctx());
  if (rc == AICP_ERR_CONVERGENCE) throw std::runtime_error("ConvergenceError: " + msg);
  if (rc == AICP_ERR_TRANSFORMATION) throw std::runtime_error("TransformationError: " + msg);
  throw std::runtime_error("aicp_hip error " + std::to_string(rc) + ": " + msg);
}

class HipRegistration : public AbstractRegistrator {
 public:
  HipRegistration() = default;
  explicit HipRegistration(const RegistrationParams& params) : params_(params) {}

  // pointmatcher_registration.hpp:52-54: only the path is stored; the chain is read when
  // registering (App rewrites the ratio into the file before every call, app.cpp:194-205)
  void updateConfigParams(std::string config_name) override {
    params_.pointmatcher.configFileName.clear();
    params_.pointmatcher.configFileName.append(config_name);
  }

  void registerClouds(pcl::PointCloud<pcl::PointXYZ>& cloud_ref, pcl::PointCloud<pcl::PointXYZ>& cloud_read,
                      Eigen::Matrix4f& final_transform) override {
    run(first_x(cloud_ref), cloud_ref.width, sizeof(pcl::PointXYZ), first_x(cloud_read), cloud_read.width,
        sizeof(pcl::PointXYZ), final_transform);
  }

  void registerClouds(pcl::PointCloud<pcl::PointXYZRGB>& cloud_ref, pcl::PointCloud<pcl::PointXYZRGB>& cloud_read,
                      Eigen::Matrix4f& final_transform) override {
    // fromPCLToDataPoints keeps x, y, z only: the 32-B rows are read in place
    run(first_x(cloud_ref), cloud_ref.width, sizeof(pcl::PointXYZRGB), first_x(cloud_read), cloud_read.width,
        sizeof(pcl::PointXYZRGB), final_transform);
  }

  void registerClouds(pcl::PointCloud<pcl::PointXYZRGBNormal>&, pcl::PointCloud<pcl::PointXYZRGBNormal>&,
                      Eigen::Matrix4f&) override {
    // the reference's body is commented out (pointmatcher_registration.cpp:36-45): a no-op
  }

  // initialized_reading_ is only set by applyInitialization, which never runs in App (its
  // initialTransform is never parsed): the reference returns the reading itself
  void getInitializedReading(pcl::PointCloud<pcl::PointXYZ>& initialized_reading) override {
    std::cout << "[Pointmatcher] Reading cloud not initialized here." << std::endl;
    to_cloud(read_xyz_, initialized_reading);  // pointmatcher_registration.hpp:37-45
  }

  void getOutputReading(pcl::PointCloud<pcl::PointXYZ>& out_read_cloud) override {
    const size_t n = read_xyz_.size() / 3;
    std::vector<float> out(3 * n);
    if (n) hip_throw_on_error(aicp_hip_transform(hip_shared_ctx(), T_, read_xyz_.data(), n, 12, out.data()));
    to_cloud(out, out_read_cloud);
  }

  const aicp_icp_stats& lastStats() const { return stats_; }

  // &points[0].x, or nullptr for an empty cloud (points[0] of an empty vector is undefined);
  // the C-ABI rejects a null cloud with AICP_ERR_INVALID, which throws below
  template <class P>
  static const float* first_x(const pcl::PointCloud<P>& c) {
    return c.points.empty() ? nullptr : &c.points[0].x;
  }

 private:
  static void to_cloud(const std::vector<float>& xyz, pcl::PointCloud<pcl::PointXYZ>& out) {
    const size_t n = xyz.size() / 3;
    out.points.resize(n);
    for (size_t i = 0; i < n; ++i) {
      out.points[i].x = xyz[3 * i];
      out.points[i].y = xyz[3 * i + 1];
      out.points[i].z = xyz[3 * i + 2];
    }
    out.width = (uint32_t)n;
    out.height = 1;
  }

  // applyConfig (pointmatcher_registration.cpp:48-68), then the dimension check is implicit
  // (xyz rows) and the registration itself (:92-133)
  void run(const float* ref, uint32_t n_ref, size_t ref_stride, const float* read, uint32_t n_read,
           size_t read_stride, Eigen::Matrix4f& final_transform) {
    const std::string& path = params_.pointmatcher.configFileName;
    if (path.empty())  // icp_.setDefault(): libpointmatcher's default chain is not this core's
      throw std::runtime_error("aicp_hip: no ICP chain file (libpointmatcher's default chain is unsupported)");
    if (!std::ifstream(path.c_str()).good()) {
      std::cerr << "[Pointmatcher] Cannot open config file " << path << std::endl;
      std::exit(1);
    }
    const int prc = aicp_hip_parse_pm_yaml(path.c_str(), &cfg_);
    if (prc != AICP_OK)  // loadFromYaml throws on a chain it cannot build
      throw std::runtime_error("aicp_hip: invalid or unsupported ICP chain in " + path);
    aicp_pair p{};
    p.ref = ref;
    p.n_ref = n_ref;
    p.ref_stride = ref_stride;
    p.read = read;
    p.n_read = n_read;
    p.read_stride = read_stride;
    p.init_T = nullptr;  // identity (pointmatcher_registration.cpp:104-109 never fires in App)
    hip_throw_on_error(aicp_hip_register(hip_shared_ctx(), &cfg_, &p, final_transform.data(), &stats_));
    std::cout << "[Pointmatcher] Accepted matches (inliers): " << stats_.inlier_ratio * 100 << " %" << std::endl;
    for (int k = 0; k < 16; ++k) T_[k] = final_transform.data()[k];
    read_xyz_.resize(3 * (size_t)n_read);  // the reading as registered (out_read_cloud_ source)
    const char* b = reinterpret_cast<const char*>(read);
    for (uint32_t i = 0; i < n_read; ++i) {
      const float* q = reinterpret_cast<const float*>(b + i * read_stride);
      read_xyz_[3 * i] = q[0];
      read_xyz_[3 * i + 1] = q[1];
      read_xyz_[3 * i + 2] = q[2];
    }
  }

  RegistrationParams params_;
  aicp_icp_config cfg_{};
  aicp_icp_stats stats_{};
  float T_[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  std::vector<float> read_xyz_;
};

class HipOverlapper : public AbstractOverlapper {
 public:
  explicit HipOverlapper(const OverlapParams& params) : params_(params) {}

  // abstract_overlapper.hpp:15-17: poses by value, as declared
  ColorOcTree* computeOverlap(pcl::PointCloud<pcl::PointXYZ>& ref_cloud, pcl::PointCloud<pcl::PointXYZ>& read_cloud,
                              Eigen::Isometry3d ref_pose, Eigen::Isometry3d read_pose,
                              ColorOcTree* /*reading_tree*/) override {
    aicp_pair p{};
    p.ref = HipRegistration::first_x(ref_cloud);
    p.n_ref = ref_cloud.width;
    p.ref_stride = sizeof(pcl::PointXYZ);
    p.read = HipRegistration::first_x(read_cloud);
    p.n_read = read_cloud.width;
    p.read_stride = sizeof(pcl::PointXYZ);
    for (int k = 0; k < 3; ++k) {
      p.ref_origin[k] = ref_pose.translation()(k);
      p.read_origin[k] = read_pose.translation()(k);
    }
    const double res = (double)(float)params_.octree_based.octomapResolution;
    hip_throw_on_error(aicp_hip_overlap(hip_shared_ctx(), &p, res, &overlap_));
    return nullptr;
  }

  float getOverlap() override { return overlap_; }

 private:
  OverlapParams params_;
  float overlap_ = -1.f;
};

}  // namespace aicp

#endif  // AICP_HIP_REGISTRATION_HPP_
