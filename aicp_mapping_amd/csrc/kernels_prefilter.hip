// kernels_prefilter.hip — aicp_core's pre-filter regionGrowingUniformPlaneSegmentationFilter
// (filteringUtils.cpp:5-45, second overload :51-103) on the device, SURVEY.md §8(f) rank 2:
//
//   VoxelGrid 0.08 m   k_pf_minmax -> k_pf_grid -> k_pf_keys -> radix sort (voxel index, point)
//                      -> k_pf_heads + scan -> k_pf_centroid (one thread per voxel, input order)
//   NormalEstimation   the device kd-tree of the sampled cloud (kernels_tree.hip), exact libnabo
//   k = 30             kNN (k_knn_ids, eps 0, self included), k_pf_normals: neighbours
//                      sorted by (d2, id), PCL's float covariance, eigen33 and viewpoint flip
//   RegionGrowing      k_pf_order (seed order: curvature, index), k_pf_edges (smoothness mask of
//   15 nbrs, 3 deg,    the 15 nearest), k_uf_* + k_rg_iter (min-label propagation, see below),
//   curvature 1.0      k_rg_phaseb, k_rg_extract* (clusters of 50..1e6 points, creation order)
//
// RegionGrowing as min-label propagation. PCL grows one region at a time from the unlabelled
// point of lowest curvature (applySmoothRegionGrowingAlgorithm), and growRegion adds a neighbour
// y of a queued point x when |n_x . n_y| >= cos(theta); y is queued unless its curvature
// exceeds the threshold ("prop" points are the ones that are queued). The region of a point y
// is therefore the first seed, in seed order, that reaches y through prop points: with
// label = seed-order position, label(y) = min over prop points s that reach y of order(s). (The
// minimal such s is itself a seed: an earlier seed reaching it would reach y through it.) That
// fixed point is computed by monotone atomic minima along the valid edges of prop points, with
// pointer jumping (label[x] = min(label[x], label[node(label[x])]), valid because the node of a
// label is a prop point reaching x). Plain propagation moves a label one kNN radius per pass, so a
// plane-wide region would take hundreds of passes; mutual edges (x -> y and y -> x, both prop)
// are first merged by union-find (k_uf_*), every member of such a component reaches every
// other, and k_rg_iter passes labels member <-> root as well as along the edges, which leaves a
// handful of passes for the one-way edges between components.
// Non-prop points that no prop point reaches (curvature above the threshold: rounding cases
// only, as PCL's curvature is <= 1/3) are seeds after every prop point and are grown one level
// by k_rg_phaseb in seed order. tests/test_prefilter.py checks the labels against the oracle's
// literal BFS (oracle/prefilter_oracle.cpp).
//
// Rules for what PCL leaves unspecified (the same in the oracle): voxel sums in input order,
// neighbours ordered by (d2, id), seed ties by index, NaN curvature last; atan2/cos/sin of
// computeRoots in double rounded to float. The library is built -ffp-contract=off, so every
// float expression below rounds like PCL's scalar code.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "aicp_common.hpp"
#include "kernels.hpp"

namespace aicp {
namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t f2ord(float f) {  // order-preserving float -> u32
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }
__device__ __forceinline__ bool finite3(const float4& p) {
  return isfinite(p.x) && isfinite(p.y) && isfinite(p.z);
}

// ---- VoxelGrid -------------------------------------------------------------------------------

// one block of 1024 threads per 64 Ki points; LDS reduction, one set of atomics per block (not
// per wave: the eight words are shared by the whole grid)
__global__ __launch_bounds__(1024) void k_pf_minmax(uint32_t n, const float4* __restrict__ pts, PfCtl* ctl) {
  __shared__ uint32_t red[16][8];
  uint32_t v[8] = {kInf, kInf, kInf, 0u, 0u, 0u, 0u, 0u};  // lo xyz, hi xyz, finite, non-finite
  for (uint32_t i = blockIdx.x * 1024u + threadIdx.x; i < n; i += gridDim.x * 1024u) {
    const float4 p = pts[i];
    if (!finite3(p)) {
      ++v[7];
      continue;
    }
    ++v[6];
    v[0] = min(v[0], f2ord(p.x));
    v[1] = min(v[1], f2ord(p.y));
    v[2] = min(v[2], f2ord(p.z));
    v[3] = max(v[3], f2ord(p.x));
    v[4] = max(v[4], f2ord(p.y));
    v[5] = max(v[5], f2ord(p.z));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t w = (uint32_t)__shfl_xor((int)v[k], o, 64);
      v[k] = k < 3 ? min(v[k], w) : (k < 6 ? max(v[k], w) : v[k] + w);
    }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave][k] = v[k];
  __syncthreads();
  if (threadIdx.x < 8) {
    const int k = threadIdx.x;
    uint32_t r = red[0][k];
    for (int w = 1; w < 16; ++w) r = k < 3 ? min(r, red[w][k]) : (k < 6 ? max(r, red[w][k]) : r + red[w][k]);
    if (k < 3) atomicMin(&ctl->lo[k], r);
    else if (k < 6) atomicMax(&ctl->hi[k - 3], r);
    else if (k == 6) atomicAdd(&ctl->n_fin, r);
    else atomicAdd(&ctl->n_bad, r);
  }
}

// VoxelGrid::applyFilter's grid: the int64 overflow test on truncated extents (PCL passes the
// cloud through unfiltered when dx * dy * dz exceeds INT32_MAX), min_b_ and divb_mul_
__global__ void k_pf_grid(PfCtl* ctl, float inv) {
  if (threadIdx.x != 0) return;
  ctl->inv = inv;
  if (ctl->n_fin == 0) return;
  float lo[3], hi[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = ord2f(ctl->lo[k]);
    hi[k] = ord2f(ctl->hi[k]);
  }
  const long long dx = (long long)((hi[0] - lo[0]) * inv) + 1, dy = (long long)((hi[1] - lo[1]) * inv) + 1,
                  dz = (long long)((hi[2] - lo[2]) * inv) + 1;
  ctl->passthrough = (dx * dy * dz > 2147483647ll) ? 1u : 0u;
  int32_t div[3];
  for (int k = 0; k < 3; ++k) {
    ctl->minb[k] = (int32_t)floorf(lo[k] * inv);
    div[k] = (int32_t)floorf(hi[k] * inv) - ctl->minb[k] + 1;
  }
  ctl->mul1 = (uint32_t)div[0];
  ctl->mul2 = (uint32_t)div[0] * (uint32_t)div[1];
}

__global__ __launch_bounds__(256) void k_pf_keys(uint32_t n, const float4* __restrict__ pts, const PfCtl* ctl,
                                                 uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const float4 p = pts[i];
  uint32_t key;
  if (ctl->passthrough) {
    key = i;
  } else if (!finite3(p)) {
    key = kInf;
  } else {
    const float inv = ctl->inv;
    const uint32_t i0 = (uint32_t)(int32_t)(floorf(p.x * inv) - (float)ctl->minb[0]);
    const uint32_t i1 = (uint32_t)(int32_t)(floorf(p.y * inv) - (float)ctl->minb[1]);
    const uint32_t i2 = (uint32_t)(int32_t)(floorf(p.z * inv) - (float)ctl->minb[2]);
    key = i0 + i1 * ctl->mul1 + i2 * ctl->mul2;
  }
  keys[i] = key;
  vals[i] = i;
}

__global__ __launch_bounds__(256) void k_pf_heads(uint32_t n, const uint32_t* __restrict__ keys,
                                                  uint32_t* __restrict__ flag) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys[i];
  flag[i] = (k != kInf && (i == 0 || keys[i - 1] != k)) ? 1u : 0u;
}

// one thread per voxel: centroid = first point, += the others in input order, /= count
__global__ __launch_bounds__(256) void k_pf_centroid(uint32_t n, const uint32_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ vals, const float4* __restrict__ pts,
                                                     const uint32_t* __restrict__ flag,
                                                     const uint32_t* __restrict__ vid, float4* __restrict__ out,
                                                     PfCtl* ctl) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  if (i == n - 1) ctl->n_vox = vid[i] + flag[i];
  if (!flag[i]) return;
  const uint32_t k = keys[i];
  const float4 p0 = pts[vals[i]];
  float cx = p0.x, cy = p0.y, cz = p0.z;
  uint32_t j = i + 1;
  for (; j < n && keys[j] == k; ++j) {
    const float4 p = pts[vals[j]];
    cx += p.x;
    cy += p.y;
    cz += p.z;
  }
  const float c = (float)(j - i);
  out[vid[i]] = make_float4(cx / c, cy / c, cz / c, 1.f);
}

// ---- NormalEstimation --------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_pf_inv(uint32_t V, const float4* __restrict__ bpts, uint32_t* __restrict__ inv) {
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j < V) inv[__float_as_uint(bpts[j].w)] = j;
}

// Correctly rounded float square root, as sqrtf on the host: measured on gfx950, __fsqrt_rn
// differs by one ulp on some inputs (tools/experiments/pf_eig_check.hip). The double square root rounded to
// float is the correctly rounded float result (53 >= 2 * 24 + 2 bits).
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }

__device__ __forceinline__ void roots2(float b, float c, float r[3]) {
  r[0] = 0.f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.f) d = 0.f;
  const float sd = sqrt_rn(d);
  r[2] = 0.5f * (b + sd);
  r[1] = 0.5f * (b - sd);
}

// computeRoots (PCL eigen.hpp), float, characteristic polynomial in closed form
__device__ __forceinline__ void roots3(const float m[9], float r[3]) {
  const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
  const float c0 = m00 * m11 * m22 + 2.f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 - m22 * m01 * m01;
  const float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
  const float c2 = m00 + m11 + m22;
  if (fabsf(c0) < 1.1920928955078125e-07f) {  // FLT_EPSILON
    roots2(c2, c1, r);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = sqrt_rn(3.f);
  const float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.f) a_over_3 = 0.f;
  const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.f) q = 0.f;
  const float rho = sqrt_rn(-a_over_3);
  const float theta = (float)atan2((double)sqrt_rn(-q), (double)half_b) * s_inv3;
  const float cos_t = (float)cos((double)theta);
  const float sin_t = (float)sin((double)theta);
  float r0 = c2_over_3 + 2.f * rho * cos_t;
  float r1 = c2_over_3 - rho * (cos_t + s_sqrt3 * sin_t);
  float r2 = c2_over_3 - rho * (cos_t - s_sqrt3 * sin_t);
  float t;
  if (r0 >= r1) { t = r0; r0 = r1; r1 = t; }
  if (r1 >= r2) {
    t = r1; r1 = r2; r2 = t;
    if (r0 >= r1) { t = r0; r0 = r1; r1 = t; }
  }
  r[0] = r0;
  r[1] = r1;
  r[2] = r2;
  if (r0 <= 0.f) roots2(c2, c1, r);
}

// eigen33 (PCL eigen.hpp): smallest eigenvalue and its eigenvector; Eigen's 3-term sums are
// a0 + (a1 + a2)
__device__ __forceinline__ void eigen33(const float cov[9], float& lambda, float& nx, float& ny, float& nz) {
  float scale = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i) scale = fmaxf(scale, fabsf(cov[i]));
  if (scale <= 1.17549435082228750797e-38f) scale = 1.f;  // FLT_MIN
  float s[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) s[i] = __fdiv_rn(cov[i], scale);
  float ev[3];
  roots3(s, ev);
  lambda = ev[0] * scale;
  s[0] -= ev[0];
  s[4] -= ev[0];
  s[8] -= ev[0];
  auto cross = [](const float* a, const float* b, float* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
  };
  float v1[3], v2[3], v3[3];
  cross(s, s + 3, v1);
  cross(s, s + 6, v2);
  cross(s + 3, s + 6, v3);
  const float l1 = v1[0] * v1[0] + (v1[1] * v1[1] + v1[2] * v1[2]);
  const float l2 = v2[0] * v2[0] + (v2[1] * v2[1] + v2[2] * v2[2]);
  const float l3 = v3[0] * v3[0] + (v3[1] * v3[1] + v3[2] * v3[2]);
  const float* v;
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
  const float sl = sqrt_rn(l);
  nx = __fdiv_rn(v[0], sl);
  ny = __fdiv_rn(v[1], sl);
  nz = __fdiv_rn(v[2], sl);
}

// One bucket position j: the K nearest (libnabo order, ties in visit order; given as bucket
// positions, d2 recomputed with libnabo's expression) sorted by (d2, sampled id),
// computePointNormal on them (computeMeanAndCovarianceMatrix's nine float sums in neighbour
// order, solvePlaneParameters), flipNormalTowardsViewpoint; then the seed-sort key (curvature,
// by sampled index) and the first `nnb` neighbours as bucket positions.
template <int K>
__global__ __launch_bounds__(256) void k_pf_normals(uint32_t V, int nnb, const float4* __restrict__ bpts,
                                                    const float4* __restrict__ sampled, const int32_t* __restrict__ ids,
                                                    const uint32_t* __restrict__ inv,
                                                    float vpx, float vpy, float vpz, float4* __restrict__ nrm,
                                                    int32_t* __restrict__ nbp, uint2* __restrict__ kth,
                                                    uint32_t* __restrict__ ckey, uint32_t* __restrict__ cval) {
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j >= V) return;
  const float4 p = bpts[j];
  float d[K];
  int32_t id[K];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const int32_t b = ids[(size_t)j * K + t];
    if (b < 0) {
      id[t] = 0x7fffffff;
      d[t] = __builtin_inff();
    } else {
      const float4 q = bpts[b];
      const float e0 = p.x - q.x, e1 = p.y - q.y, e2 = p.z - q.z;
      float dist = 0.f;
      dist += e0 * e0;
      dist += e1 * e1;
      dist += e2 * e2;
      d[t] = dist;
      id[t] = __float_as_int(q.w);
    }
  }
  // libnabo's list is ascending in d2 with ties in visit order: sort by (d2, id) only when a tie
  // is out of order (insertion sort on registers, compile-time indices only)
  bool ordered = true;
#pragma unroll
  for (int t = 1; t < K; ++t) ordered = ordered && (d[t - 1] < d[t] || (d[t - 1] == d[t] && id[t - 1] <= id[t]));
  if (!ordered)
#pragma unroll
  for (int a = 1; a < K; ++a)
#pragma unroll
    for (int b = a; b > 0; --b) {
      const bool sw = d[b] < d[b - 1] || (d[b] == d[b - 1] && id[b] < id[b - 1]);
      const float td = sw ? d[b - 1] : d[b];
      const int32_t ti = sw ? id[b - 1] : id[b];
      d[b - 1] = sw ? d[b] : d[b - 1];
      id[b - 1] = sw ? id[b] : id[b - 1];
      d[b] = td;
      id[b] = ti;
    }
  int cnt = 0;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f, a5 = 0.f, a6 = 0.f, a7 = 0.f, a8 = 0.f;
#pragma unroll
  for (int t = 0; t < K; ++t)
    if (id[t] != 0x7fffffff) {
      const float4 q = sampled[id[t]];
      a0 += q.x * q.x;
      a1 += q.x * q.y;
      a2 += q.x * q.z;
      a3 += q.y * q.y;
      a4 += q.y * q.z;
      a5 += q.z * q.z;
      a6 += q.x;
      a7 += q.y;
      a8 += q.z;
      ++cnt;
    }
  float nx, ny, nz, curv;
  if (cnt < 3) {
    nx = ny = nz = curv = __builtin_nanf("");
  } else {
    const float c = (float)cnt;
    a0 = __fdiv_rn(a0, c);
    a1 = __fdiv_rn(a1, c);
    a2 = __fdiv_rn(a2, c);
    a3 = __fdiv_rn(a3, c);
    a4 = __fdiv_rn(a4, c);
    a5 = __fdiv_rn(a5, c);
    a6 = __fdiv_rn(a6, c);
    a7 = __fdiv_rn(a7, c);
    a8 = __fdiv_rn(a8, c);
    float cov[9];
    cov[0] = a0 - a6 * a6;
    cov[1] = a1 - a6 * a7;
    cov[2] = a2 - a6 * a8;
    cov[4] = a3 - a7 * a7;
    cov[5] = a4 - a7 * a8;
    cov[8] = a5 - a8 * a8;
    cov[3] = cov[1];
    cov[6] = cov[2];
    cov[7] = cov[5];
    float lambda;
    eigen33(cov, lambda, nx, ny, nz);
    const float eig_sum = cov[0] + cov[4] + cov[8];
    curv = eig_sum != 0.f ? fabsf(__fdiv_rn(lambda, eig_sum)) : 0.f;
    const float vx = vpx - p.x, vy = vpy - p.y, vz = vpz - p.z;
    if (vx * nx + vy * ny + vz * nz < 0.f) {
      nx = -nx;
      ny = -ny;
      nz = -nz;
    }
  }
  nrm[j] = make_float4(nx, ny, nz, curv);
  // the last of the first nnb neighbours, (d2, sampled id): y is among x's nnb nearest iff
  // (d2(x, y), id y) <= kth[x] (the mutual-edge test of k_pf_edges)
  {
    const int last = (nnb < cnt ? nnb : cnt) - 1;
    uint2 k = make_uint2(0u, 0u);
#pragma unroll
    for (int t = 0; t < K; ++t)
      if (t == last) k = make_uint2(__float_as_uint(d[t]), (uint32_t)id[t]);
    kth[j] = k;
  }
#pragma unroll
  for (int t = 0; t < kPfMaxNbrs; ++t) {
    int32_t v = -1;
    if (t < K && t < nnb && t < cnt) v = (int32_t)inv[id[t < K ? t : 0]];
    nbp[(size_t)j * kPfMaxNbrs + t] = v;
  }
  const uint32_t sid = __float_as_uint(p.w);
  ckey[sid] = isnan(curv) ? kInf : f2ord(curv);
  cval[sid] = sid;
}

// seed order: node (bucket position) of each order position, and the order of each node
__global__ __launch_bounds__(256) void k_pf_rank(uint32_t V, const uint32_t* __restrict__ sorted_ids,
                                                 const uint32_t* __restrict__ inv, uint32_t* __restrict__ nob,
                                                 uint32_t* __restrict__ order_of) {
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= V) return;
  const uint32_t x = inv[sorted_ids[p]];
  nob[p] = x;
  order_of[x] = p;
}

// ---- RegionGrowing -----------------------------------------------------------------------------

// validatePoint's smoothness test per edge x -> y (|n_y . n_x| < cos rejects, a NaN dot passes)
// as a bit mask, bit 16 = prop (curvature not above the threshold); initial labels
__global__ __launch_bounds__(256) void k_pf_edges(uint32_t V, int nnb, const float4* __restrict__ bpts,
                                                  const float4* __restrict__ nrm, const int32_t* __restrict__ nbp,
                                                  const uint2* __restrict__ kth, const uint32_t* __restrict__ order_of,
                                                  float cos_thr, float curv_thr, uint32_t* __restrict__ em,
                                                  uint32_t* __restrict__ label) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= V) return;
  const float4 n = nrm[x];
  const float4 p = bpts[x];
  const bool prop = !(n.w > curv_thr);
  uint32_t m = 0, mm = 0;
  for (int t = 0; t < nnb; ++t) {
    const int32_t y = nbp[(size_t)x * kPfMaxNbrs + t];
    if (y < 0) break;
    const float4 ny = nrm[y];
    const float dot = fabsf(ny.x * n.x + (ny.y * n.y + ny.z * n.z));
    if (dot < cos_thr) continue;
    m |= 1u << t;
    // mutual: y prop too and x among y's nnb nearest, by y's (d2, id) order (d2 is symmetric)
    if (prop && !(ny.w > curv_thr)) {
      const float4 q = bpts[y];
      const float e0 = q.x - p.x, e1 = q.y - p.y, e2 = q.z - p.z;
      float d = 0.f;
      d += e0 * e0;
      d += e1 * e1;
      d += e2 * e2;
      const uint2 k = kth[y];
      const float kd = __uint_as_float(k.x);
      if (d < kd || (d == kd && __float_as_uint(p.w) <= k.y)) mm |= 1u << t;
    }
  }
  em[x] = m | (prop ? 1u << 16 : 0u) | (mm << 17);
  label[x] = prop ? order_of[x] : kInf;
}

// Union-find over mutual edges: x -> y and y -> x both valid, x and y both prop. Such points
// reach each other, so a component shares one label, and a label reaching any member reaches
// all of them: the propagation adds the member <-> root shortcuts (k_rg_iter), which turns the
// plane-wide wavefront of plain label propagation (one kNN radius per pass) into a few passes.
// par[v] <= v always (a root is hung under a smaller root).
// Plain (L1-cacheable) loads: every find ends at its root, and the root of a plane-wide
// component is one word read by every thread, which an L1-bypassing load turns into a hot
// spot in one L2 channel. A stale cached parent is always an older ancestor (parents only move
// up, par[v] <= v), so finds stay correct; a CAS that fails because its "root" was hooked in
// the meantime returns the real parent, and the hook continues from there (k_uf_hook), so a
// stale line never makes it spin.
__device__ __forceinline__ uint32_t uf_root(uint32_t* par, uint32_t x) {
  uint32_t p = par[x];
  while (p != x) {
    const uint32_t g = par[p];
    if (g == p) return p;
    par[x] = g;  // path halving; g is still an ancestor of x whatever other threads do
    x = p;
    p = g;
  }
  return x;
}

// atomicMin(&label[r], l) for the active lanes of a wave, one atomic per distinct r: the lanes
// of a big component all target its root, and per-lane atomics on one word serialise (the
// k_uf_compress of a 600 k-point cloud took 1.1 ms that way). Returns true if this lane's
// target decreased.
__device__ __forceinline__ bool wave_min_to(uint32_t* label, uint32_t r, uint32_t l, bool active) {
  bool dec = false;
  unsigned long long pending = __ballot(active);
  while (pending) {
    const int lead = __ffsll((long long)pending) - 1;
    const uint32_t r0 = (uint32_t)__shfl((int)r, lead, 64);
    const bool mine = active && r == r0;
    uint32_t m = mine ? l : kInf;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
    bool d = false;
    if ((int)(threadIdx.x & 63) == lead) d = m < atomicMin(&label[r0], m);
    d = __shfl((int)d, lead, 64) != 0;
    dec = dec || (mine && d);
    pending &= ~__ballot(mine);
  }
  return dec;
}

// tile-local union-find in LDS: the mutual edges inside each tile of 1024 consecutive bucket
// positions (a compact patch), flattened into par as global ids. The global hook then sees only
// the edges that cross tiles.
__device__ __forceinline__ uint32_t lds_root(uint32_t* lp, uint32_t x) {
  uint32_t p = lp[x];
  while (p != x) {
    const uint32_t g = lp[p];
    if (g == p) return p;
    lp[x] = g;
    x = p;
    p = g;
  }
  return x;
}
constexpr int kUfTile = 1024;
__global__ __launch_bounds__(kUfTile) void k_uf_tile(uint32_t V, int nnb, const int32_t* __restrict__ nbp,
                                                     const uint32_t* __restrict__ em, uint32_t* __restrict__ par) {
  __shared__ uint32_t lp[kUfTile];
  const uint32_t base = blockIdx.x * (uint32_t)kUfTile, x = base + threadIdx.x;
  lp[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint32_t mm = x < V ? em[x] >> 17 : 0u;
  for (int t = 0; t < nnb; ++t) {
    if (!((mm >> t) & 1u)) continue;
    const int32_t y = nbp[(size_t)x * kPfMaxNbrs + t];
    const uint32_t r = (uint32_t)y - base;
    if (y <= (int32_t)x || r >= (uint32_t)kUfTile) continue;
    uint32_t a = threadIdx.x, b = r;
    for (;;) {
      uint32_t ra = lds_root(lp, a), rb = lds_root(lp, b);
      if (ra == rb) break;
      if (ra < rb) {
        const uint32_t t2 = ra;
        ra = rb;
        rb = t2;
      }
      const uint32_t old = atomicCAS(&lp[ra], ra, rb);
      if (old == ra) break;
      a = old;
      b = rb;
    }
  }
  __syncthreads();
  if (x < V) par[x] = base + lds_root(lp, threadIdx.x);
}

// hook the mutual edges that cross tiles, each from its smaller end; roots are read through
// uf_root, so an edge inside one tree costs no CAS
__global__ __launch_bounds__(256) void k_uf_hook(uint32_t V, int nnb, const int32_t* __restrict__ nbp,
                                                 const uint32_t* __restrict__ em, uint32_t* par) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= V) return;
  const uint32_t mm = em[x] >> 17;
  if (!mm) return;
  for (int t = 0; t < nnb; ++t) {
    if (!((mm >> t) & 1u)) continue;
    const int32_t y = nbp[(size_t)x * kPfMaxNbrs + t];
    if (y <= (int32_t)x || (uint32_t)y / kUfTile == x / kUfTile) continue;  // once; tile edges are done
    uint32_t a = x, b = (uint32_t)y;
    for (;;) {
      uint32_t ra = uf_root(par, a), rb = uf_root(par, b);
      if (ra == rb) break;
      if (ra < rb) {
        const uint32_t t2 = ra;
        ra = rb;
        rb = t2;
      }
      const uint32_t old = atomicCAS(&par[ra], ra, rb);
      if (old == ra) break;
      a = old;  // ra was hooked meanwhile: continue from its real parent
      b = rb;
    }
  }
}

// components -> comp[x] (the root); each root starts at the smallest initial label of its members
__global__ __launch_bounds__(256) void k_uf_compress(uint32_t V, uint32_t* par, uint32_t* label) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  const bool in = x < V;
  uint32_t r = 0, l = kInf;
  if (in) {
    r = uf_root(par, x);
    par[x] = r;
    l = label[x];
  }
  wave_min_to(label, r, l, in && r != x && l != kInf);
}

// One pass of the propagation: prop x takes min(own, root's, pointer jump), gives it to its root,
// and pushes it along its valid edges to y and y's root. changed = 1 when any label decreased.
__global__ __launch_bounds__(256) void k_rg_iter(uint32_t V, int nnb, const int32_t* __restrict__ nbp,
                                                 const uint32_t* __restrict__ em, const uint32_t* __restrict__ nob,
                                                 const uint32_t* __restrict__ comp, uint32_t* label,
                                                 uint32_t* changed) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  int ch = 0;
  const uint32_t m = x < V ? em[x] : 0u;
  const bool prop = (m >> 16) & 1u;
  uint32_t r = 0, l = kInf, lr = kInf;
  if (prop) {
    r = comp[x];
    const uint32_t lx = label[x];
    lr = label[r];
    l = min(lx, lr);
    l = min(l, label[nob[l]]);
    if (l < lx && l < atomicMin(&label[x], l)) ch = 1;
  }
  if (wave_min_to(label, r, l, prop && l < lr)) ch = 1;
  if (prop) {
    for (int t = 0; t < nnb; ++t) {
      if (!((m >> t) & 1u)) continue;
      const int32_t y = nbp[(size_t)x * kPfMaxNbrs + t];
      if (l < label[y] && l < atomicMin(&label[y], l)) ch = 1;
      const uint32_t ry = comp[y];
      if (l < label[ry] && l < atomicMin(&label[ry], l)) ch = 1;
    }
  }
  if (__any(ch) && (threadIdx.x & 63) == 0) *changed = 1u;
}

// members adopt their root's final label (non-prop points are their own components)
__global__ __launch_bounds__(256) void k_rg_settle(uint32_t V, const uint32_t* __restrict__ comp, uint32_t* label) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= V) return;
  const uint32_t lr = label[comp[x]];
  if (lr < label[x]) label[x] = lr;
}

__global__ __launch_bounds__(256) void k_rg_count_inf(uint32_t V, const uint32_t* __restrict__ label, PfCtl* ctl) {
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  const bool f = x < V && label[x] == kInf;
  const unsigned long long b = __ballot(f);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&ctl->n_inf, (uint32_t)__popcll(b));
}

// a label load that bypasses the CU's vector L1 (another wave of the block may have stored it)
__device__ __forceinline__ uint32_t ld_label(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Seeds left after the propagation (non-prop points no prop point reaches), in seed order: each
// labels itself and its valid, still unlabelled neighbours (which are non-prop and not queued).
// One block; a chunk of order positions is scanned in parallel and only chunks holding such
// seeds are walked by one thread.
__global__ __launch_bounds__(256) void k_rg_phaseb(uint32_t V, int nnb, const int32_t* __restrict__ nbp,
                                                   const uint32_t* __restrict__ em, const uint32_t* __restrict__ nob,
                                                   uint32_t* label) {
  for (uint32_t b0 = 0; b0 < V; b0 += 256) {
    const uint32_t p = b0 + threadIdx.x;
    const bool f = p < V && ld_label(label + nob[p]) == kInf;
    if (__syncthreads_or(f) && threadIdx.x == 0) {
      const uint32_t e = min(V, b0 + 256u);
      for (uint32_t q = b0; q < e; ++q) {
        const uint32_t x = nob[q];
        if (ld_label(label + x) != kInf) continue;
        label[x] = q;
        const uint32_t m = em[x];
        for (int t = 0; t < nnb; ++t) {
          const int32_t y = nbp[(size_t)x * kPfMaxNbrs + t];
          if (y < 0) break;
          if (((m >> t) & 1u) && ld_label(label + y) == kInf) label[y] = q;
        }
      }
    }
    __syncthreads();
  }
}

// labels in sampled order (sort keys) and the identity values
__global__ __launch_bounds__(256) void k_rg_keys(uint32_t V, const uint32_t* __restrict__ label,
                                                 const uint32_t* __restrict__ inv, uint32_t* __restrict__ keys,
                                                 uint32_t* __restrict__ vals) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= V) return;
  keys[i] = label[inv[i]];
  vals[i] = i;
}

// after the (label, index) sort and the head scan: segment starts (and the end sentinel)
__global__ __launch_bounds__(256) void k_rg_segs(uint32_t V, const uint32_t* __restrict__ flag,
                                                 const uint32_t* __restrict__ segid, uint32_t* __restrict__ seg_start,
                                                 PfCtl* ctl) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= V) return;
  if (flag[i]) seg_start[segid[i]] = i;
  if (i == V - 1) {
    const uint32_t ns = segid[i] + flag[i];
    seg_start[ns] = V;
    ctl->n_seg = ns;
  }
}

// extract()'s size filter: keep = 1 per kept segment, kpts = its point count (for the scans)
__global__ __launch_bounds__(256) void k_rg_keep(uint32_t V, const uint32_t* __restrict__ seg_start, const PfCtl* ctl,
                                                 uint32_t min_size, uint32_t max_size, uint32_t* __restrict__ keep,
                                                 uint32_t* __restrict__ kpts) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= V) return;
  uint32_t k = 0, c = 0;
  if (s < ctl->n_seg) {
    c = seg_start[s + 1] - seg_start[s];
    k = (c >= min_size && c <= max_size) ? 1u : 0u;
  }
  keep[s] = k;
  kpts[s] = k ? c : 0u;
}

// kept points -> out (clusters in creation order, points ascending); cluster of every point
__global__ __launch_bounds__(256) void k_rg_scatter(uint32_t V, const uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ flag,
                                                    const uint32_t* __restrict__ heads_before,
                                                    const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ keep, const uint32_t* __restrict__ cid,
                                                    const uint32_t* __restrict__ koff, const float4* __restrict__ sampled,
                                                    float4* __restrict__ out, int32_t* __restrict__ cluster_of,
                                                    PfCtl* ctl) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= V) return;
  const uint32_t s = heads_before[i] + flag[i] - 1u;  // the exclusive head count is one past for non-heads
  const uint32_t v = vals[i];
  if (keep[s]) {
    out[koff[s] + (i - seg_start[s])] = sampled[v];
    cluster_of[v] = (int32_t)cid[s];
  } else {
    cluster_of[v] = -1;
  }
  if (i == V - 1) {
    const uint32_t ns = ctl->n_seg;
    ctl->n_clusters = ns ? cid[ns - 1] + keep[ns - 1] : 0u;
    ctl->n_out = ns ? koff[ns - 1] + (keep[ns - 1] ? seg_start[ns] - seg_start[ns - 1] : 0u) : 0u;
  }
}

inline unsigned blocks_for(uint32_t n) { return (n + 255u) / 256u; }

hipError_t scan_u32(hipStream_t s, void* temp, size_t bytes, const uint32_t* in, uint32_t* out, uint32_t n) {
  return rocprim::exclusive_scan(temp, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), s);
}
hipError_t sort_u32(hipStream_t s, void* temp, size_t bytes, const uint32_t* k0, uint32_t* k1, const uint32_t* v0,
                    uint32_t* v1, uint32_t n) {
  return rocprim::radix_sort_pairs(temp, bytes, k0, k1, v0, v1, n, 0, 32, s);
}

}  // namespace

size_t pf_temp_bytes(size_t n) {
  size_t a = 0, b = 0;
  (void)rocprim::exclusive_scan(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, n,
                                rocprim::plus<uint32_t>());
  (void)rocprim::radix_sort_pairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, n, 0, 32);
  return a > b ? a : b;
}

hipError_t launch_pf_voxel(hipStream_t s, uint32_t n, const float4* pts, float inv, PfCtl* ctl, const PfWork& w,
                           float4* sampled) {
  if (n == 0) return hipSuccess;
  k_pf_minmax<<<min((n + 65535u) / 65536u, 1024u), 1024, 0, s>>>(n, pts, ctl);
  k_pf_grid<<<1, 64, 0, s>>>(ctl, inv);
  k_pf_keys<<<blocks_for(n), 256, 0, s>>>(n, pts, ctl, w.k0, w.v0);
  hipError_t e = sort_u32(s, w.temp, w.temp_bytes, w.k0, w.k1, w.v0, w.v1, n);
  if (e != hipSuccess) return e;
  k_pf_heads<<<blocks_for(n), 256, 0, s>>>(n, w.k1, w.flag);
  e = scan_u32(s, w.temp, w.temp_bytes, w.flag, w.scan, n);
  if (e != hipSuccess) return e;
  k_pf_centroid<<<blocks_for(n), 256, 0, s>>>(n, w.k1, w.v1, pts, w.flag, w.scan, sampled, ctl);
  return hipGetLastError();
}

bool launch_pf_normals(hipStream_t s, uint32_t V, int k, int nnb, const float4* bpts, const float4* sampled,
                       const int32_t* ids, uint32_t* inv, const float vp[3], float4* nrm, int32_t* nbp, uint2* kth,
                       uint32_t* ckey, uint32_t* cval) {
  if (V == 0) return true;
  k_pf_inv<<<blocks_for(V), 256, 0, s>>>(V, bpts, inv);
  switch (k) {
    case 10: k_pf_normals<10><<<blocks_for(V), 256, 0, s>>>(V, nnb, bpts, sampled, ids, inv, vp[0], vp[1], vp[2], nrm, nbp, kth, ckey, cval); break;
    case 20: k_pf_normals<20><<<blocks_for(V), 256, 0, s>>>(V, nnb, bpts, sampled, ids, inv, vp[0], vp[1], vp[2], nrm, nbp, kth, ckey, cval); break;
    case 30: k_pf_normals<30><<<blocks_for(V), 256, 0, s>>>(V, nnb, bpts, sampled, ids, inv, vp[0], vp[1], vp[2], nrm, nbp, kth, ckey, cval); break;
    default: return false;
  }
  return true;
}

hipError_t launch_pf_order(hipStream_t s, uint32_t V, int nnb, const PfWork& w, const uint32_t* ckey,
                           const uint32_t* cval, const uint32_t* inv, const float4* bpts, const float4* nrm,
                           const int32_t* nbp, const uint2* kth, float cos_thr, float curv_thr, uint32_t* nob,
                           uint32_t* order_of, uint32_t* em, uint32_t* label) {
  if (V == 0) return hipSuccess;
  const hipError_t e = sort_u32(s, w.temp, w.temp_bytes, ckey, w.k1, cval, w.v1, V);
  if (e != hipSuccess) return e;
  k_pf_rank<<<blocks_for(V), 256, 0, s>>>(V, w.v1, inv, nob, order_of);
  k_pf_edges<<<blocks_for(V), 256, 0, s>>>(V, nnb, bpts, nrm, nbp, kth, order_of, cos_thr, curv_thr, em, label);
  return hipGetLastError();
}

void launch_rg_components(hipStream_t s, uint32_t V, int nnb, const int32_t* nbp, uint32_t* em, uint32_t* comp,
                          uint32_t* label) {
  if (!V) return;
  k_uf_tile<<<(V + kUfTile - 1) / kUfTile, kUfTile, 0, s>>>(V, nnb, nbp, em, comp);
  k_uf_hook<<<blocks_for(V), 256, 0, s>>>(V, nnb, nbp, em, comp);
  k_uf_compress<<<blocks_for(V), 256, 0, s>>>(V, comp, label);
}

void launch_rg_iter(hipStream_t s, uint32_t V, int nnb, const int32_t* nbp, const uint32_t* em, const uint32_t* nob,
                    const uint32_t* comp, uint32_t* label, uint32_t* changed) {
  if (V) k_rg_iter<<<blocks_for(V), 256, 0, s>>>(V, nnb, nbp, em, nob, comp, label, changed);
}

void launch_rg_settle(hipStream_t s, uint32_t V, const uint32_t* comp, uint32_t* label) {
  if (V) k_rg_settle<<<blocks_for(V), 256, 0, s>>>(V, comp, label);
}

void launch_rg_count_inf(hipStream_t s, uint32_t V, const uint32_t* label, PfCtl* ctl) {
  if (V) k_rg_count_inf<<<blocks_for(V), 256, 0, s>>>(V, label, ctl);
}

void launch_rg_phaseb(hipStream_t s, uint32_t V, int nnb, const int32_t* nbp, const uint32_t* em, const uint32_t* nob,
                      uint32_t* label) {
  if (V) k_rg_phaseb<<<1, 256, 0, s>>>(V, nnb, nbp, em, nob, label);
}

hipError_t launch_rg_extract(hipStream_t s, uint32_t V, uint32_t min_size, uint32_t max_size, const uint32_t* label,
                             const uint32_t* inv, const float4* sampled, const PfWork& w, float4* out,
                             int32_t* cluster_of, PfCtl* ctl) {
  if (V == 0) return hipSuccess;
  k_rg_keys<<<blocks_for(V), 256, 0, s>>>(V, label, inv, w.k0, w.v0);
  hipError_t e = sort_u32(s, w.temp, w.temp_bytes, w.k0, w.k1, w.v0, w.v1, V);
  if (e != hipSuccess) return e;
  k_pf_heads<<<blocks_for(V), 256, 0, s>>>(V, w.k1, w.flag);
  e = scan_u32(s, w.temp, w.temp_bytes, w.flag, w.scan, V);
  if (e != hipSuccess) return e;
  // seg_start: V + 1 words in k0 (free after the sort)
  uint32_t* seg_start = w.k0;
  k_rg_segs<<<blocks_for(V), 256, 0, s>>>(V, w.flag, w.scan, seg_start, ctl);
  // keep / kpts per segment, then their exclusive scans: cid (into v0), koff (into flag2)
  k_rg_keep<<<blocks_for(V), 256, 0, s>>>(V, seg_start, ctl, min_size, max_size, w.keep, w.kpts);
  e = scan_u32(s, w.temp, w.temp_bytes, w.keep, w.v0, V);
  if (e != hipSuccess) return e;
  e = scan_u32(s, w.temp, w.temp_bytes, w.kpts, w.koff, V);
  if (e != hipSuccess) return e;
  k_rg_scatter<<<blocks_for(V), 256, 0, s>>>(V, w.v1, w.flag, w.scan, seg_start, w.keep, w.v0, w.koff, sampled, out,
                                            cluster_of, ctl);
  return hipGetLastError();
}

}  // namespace aicp
