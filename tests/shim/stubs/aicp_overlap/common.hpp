// Stand-in restating OverlapParams (aicp_core/include/aicp_overlap/common.hpp:7-14).
#pragma once
#include <string>

struct OverlapParams {
  std::string type;
  std::string loadPosesFromFile;
  struct OctreeOverlapParams {
    double octomapResolution;
  } octree_based;
};
