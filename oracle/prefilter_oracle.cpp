// prefilter_oracle.cpp — TEST INFRASTRUCTURE ONLY (see aicp_oracle.h).
//
// CPU restatement of aicp_core's pre-filter regionGrowingUniformPlaneSegmentationFilter
// (aicp_core/src/utils/filteringUtils.cpp:5-45; second overload :51-103), i.e. three PCL stages:
//
//   VoxelGrid<PointXYZ> leaf 0.08      pcl-1.8.1 filters/impl/voxel_grid.hpp  (applyFilter)
//   NormalEstimation<PointXYZ> k = 30  pcl-1.8.1 features/impl/normal_3d.hpp  (computeFeature,
//                                      computePointNormal), common/impl/centroid.hpp
//                                      (computeMeanAndCovarianceMatrix), common/impl/eigen.hpp
//                                      (eigen33, computeRoots, computeRoots2),
//                                      features/normal_3d.h (flipNormalTowardsViewpoint)
//   RegionGrowing<PointXYZ, Normal>    pcl-1.8.1 segmentation/impl/region_growing.hpp
//                                      (extract, findPointNeighbours,
//                                      applySmoothRegionGrowingAlgorithm, growRegion,
//                                      validatePoint, assembleRegions)
//
// PCL (1.8.1, the ROS melodic version the reference builds against) is not vendored in the
// reference and is absent from this image; the stages are restated from its published source.
// PARITY UNPINNED: the reference holds no fixture for this path. Where PCL's result depends
// on unspecified behaviour this restatement fixes a rule, and the device path follows the
// same rule:
//   - VoxelGrid sorts (voxel index, point) pairs with std::sort on the index only (not
//     stable): the summation order inside a voxel is unspecified. Here: input order.
//   - FLANN returns equal-distance neighbours in visit order. Here: neighbours sorted by
//     (squared distance, index). The neighbour SET is libnabo's exact kNN (eps 0, self
//     included), the same set as FLANN's exact search except for ties at the k-th distance.
//   - RegionGrowing's second search (k = 15) is the first 15 of that sorted list.
//   - Seeds are sorted by curvature with std::sort (ties unspecified). Here: (curvature,
//     index), NaN curvature last.
//   - atan2 / cos / sin of computeRoots run in double and are rounded to float (the float
//     libm results of the reference's platform are within an ulp of that).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <queue>
#include <utility>
#include <vector>

#include "aicp_oracle.h"

namespace {

struct V3 {
  float x, y, z;
};

// computeRoots2 (eigen.hpp): roots of x^2 - b x + c with roots(0) = 0. `b * b - 4.0 * c` is
// a float product minus a double, rounded to float.
void roots2(float b, float c, float r[3]) {
  r[0] = 0.f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.f) d = 0.f;
  const float sd = std::sqrt(d);
  r[2] = 0.5f * (b + sd);
  r[1] = 0.5f * (b - sd);
}

// computeRoots (eigen.hpp): the three eigenvalues of a symmetric 3x3 (row-major m), ascending
void roots3(const float m[9], float r[3]) {
  const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
  const float c0 = m00 * m11 * m22 + 2.f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 - m22 * m01 * m01;
  const float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
  const float c2 = m00 + m11 + m22;
  if (std::fabs(c0) < std::numeric_limits<float>::epsilon()) {
    roots2(c2, c1, r);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = std::sqrt(3.f);
  const float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.f) a_over_3 = 0.f;
  const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.f) q = 0.f;
  const float rho = std::sqrt(-a_over_3);
  const float theta = (float)std::atan2((double)std::sqrt(-q), (double)half_b) * s_inv3;
  const float cos_t = (float)std::cos((double)theta);
  const float sin_t = (float)std::sin((double)theta);
  r[0] = c2_over_3 + 2.f * rho * cos_t;
  r[1] = c2_over_3 - rho * (cos_t + s_sqrt3 * sin_t);
  r[2] = c2_over_3 - rho * (cos_t - s_sqrt3 * sin_t);
  if (r[0] >= r[1]) std::swap(r[0], r[1]);
  if (r[1] >= r[2]) {
    std::swap(r[1], r[2]);
    if (r[0] >= r[1]) std::swap(r[0], r[1]);
  }
  if (r[0] <= 0.f) roots2(c2, c1, r);
}

// Eigen's unrolled 3-term sum: a0 + (a1 + a2)
inline float sum3(float a0, float a1, float a2) { return a0 + (a1 + a2); }
inline V3 cross(const float* a, const float* b) {
  return V3{a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
inline float sqnorm(const V3& v) { return sum3(v.x * v.x, v.y * v.y, v.z * v.z); }

// eigen33 (eigen.hpp): smallest eigenvalue and its eigenvector
void eigen33(const float cov[9], float* eigenvalue, V3* vec) {
  float scale = 0.f;
  for (int i = 0; i < 9; ++i) scale = std::max(scale, std::fabs(cov[i]));
  if (scale <= std::numeric_limits<float>::min()) scale = 1.f;
  float s[9];
  for (int i = 0; i < 9; ++i) s[i] = cov[i] / scale;
  float ev[3];
  roots3(s, ev);
  *eigenvalue = ev[0] * scale;
  s[0] -= ev[0];
  s[4] -= ev[0];
  s[8] -= ev[0];
  const V3 v1 = cross(s, s + 3), v2 = cross(s, s + 6), v3 = cross(s + 3, s + 6);
  const float l1 = sqnorm(v1), l2 = sqnorm(v2), l3 = sqnorm(v3);
  V3 v;
  float l;
  if (l1 >= l2 && l1 >= l3) {
    v = v1;
    l = l1;
  } else if (l2 >= l1 && l2 >= l3) {
    v = v2;
    l = l2;
  } else {
    v = v3;
    l = l3;
  }
  const float sl = std::sqrt(l);
  *vec = V3{v.x / sl, v.y / sl, v.z / sl};
}

// computePointNormal + flipNormalTowardsViewpoint for one point: nb = neighbour ids in order
void point_normal(const std::vector<V3>& P, const int32_t* nb, int cnt, const V3& p, const float vp[3], float out[4]) {
  const float nan = std::numeric_limits<float>::quiet_NaN();
  if (cnt < 3) {
    out[0] = out[1] = out[2] = out[3] = nan;
    return;
  }
  float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < cnt; ++j) {
    const V3& q = P[nb[j]];
    a[0] += q.x * q.x;
    a[1] += q.x * q.y;
    a[2] += q.x * q.z;
    a[3] += q.y * q.y;
    a[4] += q.y * q.z;
    a[5] += q.z * q.z;
    a[6] += q.x;
    a[7] += q.y;
    a[8] += q.z;
  }
  for (int i = 0; i < 9; ++i) a[i] /= (float)cnt;
  float cov[9];
  cov[0] = a[0] - a[6] * a[6];
  cov[1] = a[1] - a[6] * a[7];
  cov[2] = a[2] - a[6] * a[8];
  cov[4] = a[3] - a[7] * a[7];
  cov[5] = a[4] - a[7] * a[8];
  cov[8] = a[5] - a[8] * a[8];
  cov[3] = cov[1];
  cov[6] = cov[2];
  cov[7] = cov[5];
  float lambda;
  V3 n;
  eigen33(cov, &lambda, &n);
  const float eig_sum = cov[0] + cov[4] + cov[8];
  const float curv = eig_sum != 0.f ? std::fabs(lambda / eig_sum) : 0.f;
  const float vx = vp[0] - p.x, vy = vp[1] - p.y, vz = vp[2] - p.z;
  const float cos_theta = vx * n.x + vy * n.y + vz * n.z;
  if (cos_theta < 0.f) n = V3{-n.x, -n.y, -n.z};
  out[0] = n.x;
  out[1] = n.y;
  out[2] = n.z;
  out[3] = curv;
}

}  // namespace

extern "C" int ao_prefilter(const float* pts, int64_t n, int64_t stride_floats, const ao_prefilter_params* prm,
                            float* sampled, int32_t* labels, int64_t* n_sampled, int64_t* n_clusters, float* out,
                            int64_t* n_out) {
  if (!prm || !n_sampled || !n_clusters || !n_out || n < 0 || (n > 0 && (!pts || stride_floats < 3))) return 2;
  *n_sampled = *n_clusters = *n_out = 0;
  // ---- VoxelGrid::applyFilter ----
  std::vector<V3> P;
  {
    const float inv = 1.f / prm->leaf;  // inverse_leaf_size_ = Array4f::Ones() / leaf_size_
    float lo[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
                   std::numeric_limits<float>::max()};
    float hi[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(),
                   -std::numeric_limits<float>::max()};
    int64_t n_fin = 0;
    bool all_finite = true;
    for (int64_t i = 0; i < n; ++i) {
      const float* p = pts + i * stride_floats;
      if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) {
        all_finite = false;
        continue;
      }
      ++n_fin;
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(lo[k], p[k]);
        hi[k] = std::max(hi[k], p[k]);
      }
    }
    if (n_fin == 0) return 0;
    const int64_t dx = (int64_t)((hi[0] - lo[0]) * inv) + 1, dy = (int64_t)((hi[1] - lo[1]) * inv) + 1,
                  dz = (int64_t)((hi[2] - lo[2]) * inv) + 1;
    if (dx * dy * dz > (int64_t)std::numeric_limits<int32_t>::max()) {
      // "Leaf size is too small for the input dataset": PCL returns the input unfiltered
      if (!all_finite) return 3;
      for (int64_t i = 0; i < n; ++i) {
        const float* p = pts + i * stride_floats;
        P.push_back(V3{p[0], p[1], p[2]});
      }
    } else {
      int32_t minb[3], divb[3];
      for (int k = 0; k < 3; ++k) {
        minb[k] = (int32_t)std::floor(lo[k] * inv);
        divb[k] = (int32_t)std::floor(hi[k] * inv) - minb[k] + 1;
      }
      const uint32_t mul1 = (uint32_t)divb[0], mul2 = (uint32_t)divb[0] * (uint32_t)divb[1];
      std::vector<std::pair<uint32_t, int64_t>> iv;
      iv.reserve((size_t)n_fin);
      for (int64_t i = 0; i < n; ++i) {
        const float* p = pts + i * stride_floats;
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
        uint32_t ijk[3];
        for (int k = 0; k < 3; ++k) ijk[k] = (uint32_t)(int32_t)(std::floor(p[k] * inv) - (float)minb[k]);
        iv.emplace_back(ijk[0] + ijk[1] * mul1 + ijk[2] * mul2, i);
      }
      std::stable_sort(iv.begin(), iv.end(),
                       [](const std::pair<uint32_t, int64_t>& a, const std::pair<uint32_t, int64_t>& b) {
                         return a.first < b.first;
                       });
      size_t b = 0;
      while (b < iv.size()) {
        size_t e = b + 1;
        while (e < iv.size() && iv[e].first == iv[b].first) ++e;
        const float* p0 = pts + iv[b].second * stride_floats;
        float c[3] = {p0[0], p0[1], p0[2]};
        for (size_t i = b + 1; i < e; ++i) {
          const float* p = pts + iv[i].second * stride_floats;
          for (int k = 0; k < 3; ++k) c[k] += p[k];
        }
        const float cntf = (float)(e - b);
        P.push_back(V3{c[0] / cntf, c[1] / cntf, c[2] / cntf});
        b = e;
      }
    }
  }
  const int64_t V = (int64_t)P.size();
  *n_sampled = V;
  // ---- NormalEstimation: kNN (exact, self included) sorted by (d2, id) ----
  const int k = (int)std::min<int64_t>(prm->normal_k, V);
  std::vector<int32_t> ids((size_t)V * std::max(k, 1));
  std::vector<float> d2((size_t)V * std::max(k, 1));
  if (k > 0) {
    std::vector<float> flat((size_t)V * 3);
    for (int64_t i = 0; i < V; ++i) {
      flat[3 * i] = P[i].x;
      flat[3 * i + 1] = P[i].y;
      flat[3 * i + 2] = P[i].z;
    }
    ao_tree* t = nullptr;
    if (ao_tree_build(flat.data(), V, 3, 8, &t) != 0) return 2;
    uint64_t tp = 0, tn = 0;
    const int rc = ao_tree_knn(t, flat.data(), V, 3, k, 0.f, 1, std::numeric_limits<float>::infinity(), ids.data(),
                               d2.data(), &tp, &tn);
    ao_tree_free(t);
    if (rc != 0) return 2;
    for (int64_t i = 0; i < V; ++i) {
      std::vector<std::pair<float, int32_t>> l;
      for (int j = 0; j < k; ++j)
        if (ids[i * k + j] >= 0) l.emplace_back(d2[i * k + j], ids[i * k + j]);
      std::sort(l.begin(), l.end());
      for (int j = 0; j < k; ++j) ids[i * k + j] = j < (int)l.size() ? l[j].second : -1;
    }
  }
  std::vector<float> N((size_t)V * 4);
  for (int64_t i = 0; i < V; ++i) {
    int cnt = 0;
    while (cnt < k && ids[i * k + cnt] >= 0) ++cnt;
    point_normal(P, ids.data() + i * k, cnt, P[i], prm->viewpoint, &N[4 * i]);
  }
  // ---- RegionGrowing::extract ----
  const int nn = (int)std::min<int64_t>(prm->neighbours, k);
  std::vector<int64_t> order((size_t)V);
  for (int64_t i = 0; i < V; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    const float ca = N[4 * a + 3], cb = N[4 * b + 3];
    const bool na = std::isnan(ca), nb = std::isnan(cb);
    if (na != nb) return nb;  // NaN last
    if (!na && ca != cb) return ca < cb;
    return a < b;
  });
  std::vector<int32_t> lab((size_t)V, -1);
  std::vector<int64_t> seg_size;
  int64_t done = 0, sc = 0;
  while (done < V) {
    // next seed: first unlabelled point in curvature order
    while (sc < V && lab[order[sc]] != -1) ++sc;
    if (sc >= V) break;
    const int64_t seed = order[sc];
    const int32_t segno = (int32_t)seg_size.size();
    std::queue<int64_t> q;
    q.push(seed);
    lab[seed] = segno;
    int64_t cnt = 1;
    while (!q.empty()) {
      const int64_t cur = q.front();
      q.pop();
      for (int j = 0; j < nn; ++j) {
        const int32_t y = ids[cur * k + j];
        if (y < 0) break;
        if (lab[y] != -1) continue;
        // validatePoint: |n_y . n_cur| < cos(theta) rejects (a NaN dot passes)
        const float* a = &N[4 * y];
        const float* b = &N[4 * cur];
        const float dot = std::fabs(sum3(a[0] * b[0], a[1] * b[1], a[2] * b[2]));
        if (dot < prm->cos_smoothness) continue;
        lab[y] = segno;
        ++cnt;
        if (!(a[3] > prm->curvature)) q.push(y);  // is_a_seed unless its curvature exceeds the threshold
      }
    }
    seg_size.push_back(cnt);
    done += cnt;
  }
  // assembleRegions + the size filter of extract(); clusters keep creation order, points
  // ascending index
  std::vector<int32_t> cid(seg_size.size(), -1);
  int64_t nc = 0;
  for (size_t s = 0; s < seg_size.size(); ++s)
    if (seg_size[s] >= prm->min_cluster && seg_size[s] <= prm->max_cluster) cid[s] = (int32_t)nc++;
  *n_clusters = nc;
  std::vector<int64_t> off((size_t)nc + 1, 0);
  for (size_t s = 0; s < seg_size.size(); ++s)
    if (cid[s] >= 0) off[cid[s] + 1] = seg_size[s];
  for (int64_t c = 0; c < nc; ++c) off[c + 1] += off[c];
  std::vector<int64_t> fill(off.begin(), off.end() - 1);
  for (int64_t i = 0; i < V; ++i) {
    const int32_t c = lab[i] >= 0 ? cid[lab[i]] : -1;
    if (labels) labels[i] = c;
    if (sampled) {
      float* s = sampled + 8 * i;
      s[0] = P[i].x;
      s[1] = P[i].y;
      s[2] = P[i].z;
      s[3] = N[4 * i + 3];
      s[4] = N[4 * i];
      s[5] = N[4 * i + 1];
      s[6] = N[4 * i + 2];
      s[7] = (float)c;
    }
    if (c >= 0 && out) {
      const int64_t o = fill[c]++;
      out[3 * o] = P[i].x;
      out[3 * o + 1] = P[i].y;
      out[3 * o + 2] = P[i].z;
    }
  }
  *n_out = nc ? off[nc] : 0;
  return 0;
}
