// shim_main.cpp — drives integration/hip_registration.hpp through the aicp factories, the way
// App does (app.cpp:32-34, 132-135, 205-210), compiled against tests/shim/stubs (PCL / Eigen /
// octomap stand-ins and the restated aicp interfaces) and linked with libaicp_hip.so.
//
//   shim_main cpu <chain.yaml>
//       no device needed: factories, overload set, config handling, error paths
//   shim_main gpu <chain.yaml> <ref.bin> <read.bin> <ox oy oz> <rx ry rz>
//       registration + overlap through the shims; prints "T <16 floats col-major>",
//       "T_rgb ...", "overlap <pct>", "out <n> <x0 y0 z0>"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <vector>

#include "hip_registration.hpp"

namespace aicp {
// registration.hpp:9-19 with the branch INTEGRATION.md §4 adds
static std::unique_ptr<AbstractRegistrator> create_registrator(const RegistrationParams& parameters) {
  std::unique_ptr<AbstractRegistrator> registrator;
  if (parameters.type == "Pointmatcher") {
    // PointmatcherRegistration: not built here (libpointmatcher is absent)
  } else if (parameters.type == "HIP") {
    registrator = std::unique_ptr<AbstractRegistrator>(new HipRegistration(parameters));
  } else if (parameters.type == "GICP") {
  } else {
    std::cerr << "Invalid registration type " << parameters.type << "." << std::endl;
  }
  return registrator;
}
// overlap.hpp:9-19 with the HIP branch
static std::unique_ptr<AbstractOverlapper> create_overlapper(const OverlapParams& parameters) {
  std::unique_ptr<AbstractOverlapper> overlapper;
  if (parameters.type == "HIP") overlapper = std::unique_ptr<AbstractOverlapper>(new HipOverlapper(parameters));
  return overlapper;
}
}  // namespace aicp

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

static std::vector<float> load_xyz(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::vector<float> v;
  float x;
  while (f.read(reinterpret_cast<char*>(&x), 4)) v.push_back(x);
  return v;
}

template <class P>
static pcl::PointCloud<P> cloud_of(const std::vector<float>& xyz) {
  pcl::PointCloud<P> c;
  c.resize(xyz.size() / 3);
  for (size_t i = 0; i < c.size(); ++i) {
    c.points[i].x = xyz[3 * i];
    c.points[i].y = xyz[3 * i + 1];
    c.points[i].z = xyz[3 * i + 2];
  }
  return c;
}

static int cpu_mode(const char* chain) {
  RegistrationParams rp;
  rp.type = "HIP";
  auto reg = aicp::create_registrator(rp);
  if (!reg) return fail("factory did not create the HIP registrator");
  RegistrationParams bad;
  bad.type = "Nope";
  if (aicp::create_registrator(bad)) return fail("unknown type must give nullptr");
  OverlapParams op;
  op.type = "HIP";
  op.octree_based.octomapResolution = 0.2;
  if (!aicp::create_overlapper(op)) return fail("factory did not create the HIP overlapper");
  // no chain file yet: libpointmatcher's setDefault chain is refused before any device call
  pcl::PointCloud<pcl::PointXYZ> a = cloud_of<pcl::PointXYZ>({0, 0, 0, 1, 0, 0, 0, 1, 0});
  Eigen::Matrix4f T;
  bool threw = false;
  try {
    reg->registerClouds(a, a, T);
  } catch (const std::runtime_error& e) {
    threw = std::strstr(e.what(), "no ICP chain file") != nullptr;
  }
  if (!threw) return fail("empty chain must throw");
  // XYZRGBNormal: the reference's no-op, T untouched
  pcl::PointCloud<pcl::PointXYZRGBNormal> n3;
  n3.resize(3);
  T(0, 3) = 42.f;
  reg->registerClouds(n3, n3, T);
  if (T(0, 3) != 42.f) return fail("XYZRGBNormal overload must leave T untouched");
  reg->updateConfigParams(chain);
  aicp_icp_config cfg;
  if (aicp_hip_parse_pm_yaml(chain, &cfg) != AICP_OK) return fail("chain parse");
  std::printf("cpu ok: knn %d eps %.2f ratio %.2f maxIter %d\n", cfg.knn_normals, cfg.nn_epsilon, cfg.trimmed_ratio,
              cfg.max_iter);
  return 0;
}

static int gpu_mode(int argc, char** argv) {
  if (argc < 11) return fail("usage");
  const std::vector<float> ref = load_xyz(argv[3]), read = load_xyz(argv[4]);
  RegistrationParams rp;
  rp.type = "HIP";
  auto reg = aicp::create_registrator(rp);
  reg->updateConfigParams(argv[2]);  // App::computeRegistration, app.cpp:205
  auto ref_c = cloud_of<pcl::PointXYZ>(ref), read_c = cloud_of<pcl::PointXYZ>(read);
  Eigen::Matrix4f T;
  reg->registerClouds(ref_c, read_c, T);  // app.cpp:210
  auto ref_rgb = cloud_of<pcl::PointXYZRGB>(ref), read_rgb = cloud_of<pcl::PointXYZRGB>(read);
  Eigen::Matrix4f T_rgb;
  reg->registerClouds(ref_rgb, read_rgb, T_rgb);
  pcl::PointCloud<pcl::PointXYZ> out;
  reg->getOutputReading(out);
  OverlapParams op;
  op.type = "HIP";
  op.octree_based.octomapResolution = 0.2;
  auto ovl = aicp::create_overlapper(op);
  Eigen::Isometry3d ref_pose, read_pose;
  for (int k = 0; k < 3; ++k) {
    ref_pose.translation()(k) = std::atof(argv[5 + k]);
    read_pose.translation()(k) = std::atof(argv[8 + k]);
  }
  ovl->computeOverlap(ref_c, read_c, ref_pose, read_pose, nullptr);  // app.cpp:132-135
  // an empty cloud: no points[0] access, the C-ABI's AICP_ERR_INVALID surfaces as an exception
  pcl::PointCloud<pcl::PointXYZ> empty;
  Eigen::Matrix4f T_empty;
  bool threw = false;
  try {
    reg->registerClouds(empty, read_c, T_empty);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  if (!threw) return fail("empty reference must throw");
  threw = false;
  try {
    ovl->computeOverlap(ref_c, empty, ref_pose, read_pose, nullptr);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  if (!threw) return fail("empty reading in the overlap must throw");
  std::printf("T");
  for (int k = 0; k < 16; ++k) std::printf(" %.9g", T.data()[k]);
  std::printf("\nT_rgb");
  for (int k = 0; k < 16; ++k) std::printf(" %.9g", T_rgb.data()[k]);
  std::printf("\noverlap %.9g\n", ovl->getOverlap());
  std::printf("out %zu %.9g %.9g %.9g\n", out.size(), out.points[0].x, out.points[0].y, out.points[0].z);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && !std::strcmp(argv[1], "cpu")) return cpu_mode(argv[2]);
  if (argc >= 3 && !std::strcmp(argv[1], "gpu")) {
    try {
      return gpu_mode(argc, argv);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "exception: %s\n", e.what());
      return 2;
    }
  }
  return fail("usage: shim_main cpu|gpu <chain.yaml> ...");
}
