// kdtree_host.hpp — host libnabo-order kd-tree (tools only: the library builds trees on the device,
// kernels_tree.hip) emitting the device node layout.
//
// Same splitting rule as libnabo's KDTreeUnbalancedPtInLeavesImplicitBoundsStackOpt::
// buildNodes (configured by KDTreeMatcher at icp_autotuned_default.yaml:27-30):
// widest box dimension, midpoint clamped to the points' bounds, two-pass partition
// (< cut, then <= cut), leftCount rule, bucket size 8, preorder node numbering.
#pragma once
#include <stdint.h>

#include <vector>

namespace aicp {

struct HostTree {
  std::vector<uint32_t> nodes;   // 4 words per node (see aicp_common.hpp)
  std::vector<int32_t> parent;   // per node
  std::vector<int32_t> perm;     // bucket position -> input index
  int32_t depth = 0;
};

// pts: packed xyz (stride 3 floats). Throws nothing; n >= 1.
void build_kdtree_host(const float* pts, int64_t n, int bucket, HostTree& out);

}  // namespace aicp
