// kernels_overlap_sparse.hip — the overlap's key sets as sorted key lists, for batches whose
// dense voxel maps do not fit (a return kilometres away makes a key box of 10^12 voxels).
//
// Same sets as the dense path and as octomap (kernels_overlap.hip): every key of
// computeRayKeys(origin, p) plus p's own key, per cloud. Here each key is written out as a 64-bit
// word  cloud << 48 | k0 << 32 | k1 << 16 | k2  (cloud = overlap group, or G + pair for a reading),
// the words of all clouds are sorted together (rocprim radix sort), and:
//   |S_c|      = the distinct words of cloud c (a word differs from its predecessor);
//   |A ∩ B|    = the distinct words of reading p whose key is present under p's group
//                (binary search of group << 48 | key in the sorted array).
// Cost: 8 B per ray key written and sorted, where the dense path stores 1 byte per ray key into
// an L2-resident map; it is the fallback, not the default.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "aicp_common.hpp"
#include "kernels.hpp"

namespace aicp {

namespace {

constexpr int kKeyMax = 32768;

// coordToKeyChecked: the key exists iff floor(c / res) is in [-32768, 32768). (x86's int
// conversion of NaN or of a value beyond int range gives INT_MIN, which octomap's range test
// rejects; the test is written out here so NaN coordinates are rejected on the device too.)
__device__ __forceinline__ bool key_ok(double rf, float c, int& key) {
  const double f = floor(rf * (double)c);
  if (!(f >= -(double)kKeyMax && f < (double)kKeyMax)) return false;
  key = (int)f + kKeyMax;
  return true;
}

// computeRayKeys(origin, end) + the endpoint key, in k_ovl_mark's order and arithmetic
template <class Visit>
__device__ void ray_keys(double res, const double* org, float4 p4, Visit&& visit) {
  const float o[3] = {(float)org[0], (float)org[1], (float)org[2]};
  const float e[3] = {p4.x, p4.y, p4.z};
  const double rf = 1.0 / res;
  int ko[3], ke[3];
  const bool okO = key_ok(rf, o[0], ko[0]) && key_ok(rf, o[1], ko[1]) && key_ok(rf, o[2], ko[2]);
  const bool okE = key_ok(rf, e[0], ke[0]) && key_ok(rf, e[1], ke[1]) && key_ok(rf, e[2], ke[2]);
  if (okO && okE && !(ko[0] == ke[0] && ko[1] == ke[1] && ko[2] == ke[2])) {
    visit(ko[0], ko[1], ko[2]);
    float dir[3] = {e[0] - o[0], e[1] - o[1], e[2] - o[2]};
    const float nsq = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
    const float length = (float)sqrt((double)nsq);
    for (int i = 0; i < 3; ++i) dir[i] /= length;
    int step[3];
    double tMax[3], tDelta[3];
    int cur[3] = {ko[0], ko[1], ko[2]};
    for (int i = 0; i < 3; ++i) {
      step[i] = dir[i] > 0.0f ? 1 : (dir[i] < 0.0f ? -1 : 0);
      if (step[i] != 0) {
        double vb = (double(cur[i] - kKeyMax) + 0.5) * res;
        vb += (float)(step[i] * res * 0.5);
        tMax[i] = (vb - (double)o[i]) / (double)dir[i];
        tDelta[i] = res / (double)fabsf(dir[i]);
      } else {
        tMax[i] = 1.7976931348623157e308;
        tDelta[i] = 1.7976931348623157e308;
      }
    }
    const double len = (double)length;
    for (;;) {
      int dim;
      if (tMax[0] < tMax[1])
        dim = (tMax[0] < tMax[2]) ? 0 : 2;
      else
        dim = (tMax[1] < tMax[2]) ? 1 : 2;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i == dim) {
          cur[i] = (cur[i] + step[i]) & 0xFFFF;
          tMax[i] += tDelta[i];
        }
      if (cur[0] == ke[0] && cur[1] == ke[1] && cur[2] == ke[2]) break;
      const double dfo = fmin(fmin(tMax[0], tMax[1]), tMax[2]);
      if (dfo > len) break;
      visit(cur[0], cur[1], cur[2]);
    }
  }
  if (okE) visit(ke[0], ke[1], ke[2]);
}

__device__ __forceinline__ const float4* cloud_pts(const OvlCloud& c, const float4* ref, const float4* read) {
  return (c.side ? read : ref) + c.pts_off;
}

__global__ __launch_bounds__(256) void k_spo_count(const uint32_t* __restrict__ blk_cloud,
                                                   const uint32_t* __restrict__ blk_start,
                                                   const OvlCloud* __restrict__ clouds, const float4* __restrict__ ref,
                                                   const float4* __restrict__ read, double res,
                                                   uint32_t* __restrict__ cnt) {
  const OvlCloud& c = clouds[blk_cloud[blockIdx.x]];
  const uint32_t j = blk_start[blockIdx.x] + threadIdx.x;
  if (j >= c.n) return;
  uint32_t k = 0;
  ray_keys(res, c.origin, cloud_pts(c, ref, read)[j], [&](int, int, int) { ++k; });
  cnt[c.slot + j] = k;
}

__global__ __launch_bounds__(256) void k_spo_emit(const uint32_t* __restrict__ blk_cloud,
                                                  const uint32_t* __restrict__ blk_start,
                                                  const OvlCloud* __restrict__ clouds, const float4* __restrict__ ref,
                                                  const float4* __restrict__ read, double res,
                                                  const uint64_t* __restrict__ off, uint64_t* __restrict__ keys) {
  const uint32_t ci = blk_cloud[blockIdx.x];
  const OvlCloud& c = clouds[ci];
  const uint32_t j = blk_start[blockIdx.x] + threadIdx.x;
  if (j >= c.n) return;
  uint64_t o = off[c.slot + j];
  const uint64_t hi = (uint64_t)ci << 48;
  ray_keys(res, c.origin, cloud_pts(c, ref, read)[j], [&](int a, int b, int d) {
    keys[o++] = hi | ((uint64_t)a << 32) | ((uint64_t)b << 16) | (uint64_t)d;
  });
}

// distinct words per cloud (wave-aggregated atomics: sorted runs share their cloud)
__global__ __launch_bounds__(256) void k_spo_unique(const uint64_t* __restrict__ keys, uint64_t total,
                                                    unsigned long long* __restrict__ per_cloud) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < total;
  const uint64_t k = in ? keys[i] : 0;
  const bool uniq = in && (i == 0 || keys[i - 1] != k);
  const uint32_t cloud = (uint32_t)(k >> 48);
  const uint32_t c0 = __shfl(cloud, 0, 64);
  const bool same = __all(!in || cloud == c0);
  if (same) {
    const uint64_t m = __ballot(uniq);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&per_cloud[c0], (unsigned long long)__popcll(m));
  } else if (uniq) {
    atomicAdd(&per_cloud[cloud], 1ull);
  }
}

// |A ∩ B|: distinct words of reading clouds (>= n_groups) whose key is under the pair's group
__global__ __launch_bounds__(256) void k_spo_intersect(const uint64_t* __restrict__ keys, uint64_t total,
                                                       int n_groups, const PairDesc* __restrict__ pd,
                                                       unsigned long long* __restrict__ per_pair) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint64_t k = keys[i];
  if (i > 0 && keys[i - 1] == k) return;
  const uint32_t cloud = (uint32_t)(k >> 48);
  if ((int)cloud < n_groups) return;
  const int p = (int)cloud - n_groups;
  const uint64_t want = ((uint64_t)pd[p].ogroup << 48) | (k & 0xFFFFFFFFFFFFull);
  uint64_t lo = 0, hi = total;  // first position with keys[pos] >= want
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] < want)
      lo = mid + 1;
    else
      hi = mid;
  }
  if (lo < total && keys[lo] == want) atomicAdd(&per_pair[p], 1ull);
}

__global__ void k_spo_counts(int n_groups, int n_pairs, const unsigned long long* __restrict__ per_cloud,
                             const unsigned long long* __restrict__ per_pair, PairState* gst, PairState* st) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_groups) gst[i].ovl_counts[0] = per_cloud[i];
  if (i < n_pairs) {
    st[i].ovl_counts[1] = per_cloud[n_groups + i];
    st[i].ovl_counts[2] = per_pair[i];
  }
}

// ---- the stream's sorted-key overlap (sequence.cpp): one key list per side of a window ----
// The clouds of one side (a window's readings, or its reference) write their words
// cloud << 48 | key into a list of `cap` words, a host bound of the keys the rays can visit
// (no read-back of the true count: the stream stays free of host synchronisation); the words
// past the true total are padding (n_clouds << 48, sorted last, never counted).

// a cloud's origin written on the device: the reference's by k_seq_ref_points, a debug-mode
// reading's by k_debug_prep
__global__ void k_spo_origin(OvlCloud* c, const double* __restrict__ o) {
  if (threadIdx.x < 3) c->origin[threadIdx.x] = o[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_spo_emit_cap(const uint32_t* __restrict__ blk_cloud,
                                                      const uint32_t* __restrict__ blk_start,
                                                      const OvlCloud* __restrict__ clouds,
                                                      const float4* __restrict__ pts, double res,
                                                      const uint64_t* __restrict__ off, uint64_t cap,
                                                      uint64_t* __restrict__ keys, PairState* est) {
  const uint32_t ci = blk_cloud[blockIdx.x];
  const OvlCloud& c = clouds[ci];
  const uint32_t j = blk_start[blockIdx.x] + threadIdx.x;
  if (j >= c.n) return;
  uint64_t o = off[c.slot + j];
  const uint64_t hi = (uint64_t)ci << 48;
  bool over = false;
  ray_keys(res, c.origin, pts[c.pts_off + j], [&](int a, int b, int d) {
    if (o < cap)
      keys[o++] = hi | ((uint64_t)a << 32) | ((uint64_t)b << 16) | (uint64_t)d;
    else
      over = true;
  });
  if (over) atomicOr(&est[ci].ovl_err, 1);  // the host bound was wrong: reported, never written past
}

// words [total, cap) := pad, total = off[n - 1] + cnt[n - 1]
__global__ __launch_bounds__(256) void k_spo_pad(const uint64_t* __restrict__ off, const uint32_t* __restrict__ cnt,
                                                 uint32_t n, uint64_t cap, uint64_t pad, uint64_t* keys) {
  const uint64_t total = n ? off[n - 1] + cnt[n - 1] : 0;
  for (uint64_t i = total + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += (uint64_t)gridDim.x * blockDim.x)
    keys[i] = pad;
}

// distinct words per cloud of a padded sorted list
__global__ __launch_bounds__(256) void k_spo_unique_cap(const uint64_t* __restrict__ keys, uint64_t cap,
                                                        uint32_t n_clouds, unsigned long long* __restrict__ per_cloud) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t k = i < cap ? keys[i] : ~0ull;
  const uint32_t cloud = (uint32_t)(k >> 48);
  const bool uniq = cloud < n_clouds && (i == 0 || keys[i - 1] != k);
  const uint32_t c0 = __shfl(cloud, 0, 64);
  if (__all(cloud == c0)) {
    const uint64_t m = __ballot(uniq);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&per_cloud[c0], (unsigned long long)__popcll(m));
  } else if (uniq) {
    atomicAdd(&per_cloud[cloud], 1ull);
  }
}

// |A ∩ B| per reading: its distinct words whose key is in the reference's list (cloud 0)
__global__ __launch_bounds__(256) void k_spo_intersect_ref(const uint64_t* __restrict__ rk, uint64_t cap_r,
                                                           uint32_t n_read, const uint64_t* __restrict__ gk,
                                                           uint64_t cap_g, unsigned long long* __restrict__ per_pair) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap_r) return;
  const uint64_t k = rk[i];
  const uint32_t cloud = (uint32_t)(k >> 48);
  if (cloud >= n_read || (i > 0 && rk[i - 1] == k)) return;
  const uint64_t want = k & 0xFFFFFFFFFFFFull;
  uint64_t lo = 0, hi = cap_g;  // first position with gk[pos] >= want
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (gk[mid] < want)
      lo = mid + 1;
    else
      hi = mid;
  }
  if (lo < cap_g && gk[lo] == want) atomicAdd(&per_pair[(uint32_t)cloud], 1ull);
}

__global__ void k_spo_store(int n, const unsigned long long* __restrict__ v, PairState* st, int slot) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) st[i].ovl_counts[slot] = v[i];
}

__global__ void k_spo_zero(unsigned long long* v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = 0ull;
}

int key_end_bit(int n_clouds) {
  int b = 1;
  while ((1 << b) <= n_clouds) ++b;
  return 48 + b;
}

}  // namespace

size_t ovl_sparse_scan_bytes(size_t n_points) {
  size_t b = 0;
  (void)rocprim::exclusive_scan(nullptr, b, (const uint32_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, n_points,
                                rocprim::plus<uint64_t>());
  return b;
}
size_t ovl_sparse_sort_bytes(size_t n_keys) {
  size_t b = 0;
  (void)rocprim::radix_sort_keys(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr, n_keys, 0, 64);
  return b;
}

hipError_t launch_ovl_sparse_count(hipStream_t s, uint32_t n_blocks, const uint32_t* blk_cloud,
                                   const uint32_t* blk_start, const OvlCloud* clouds, const float4* ref,
                                   const float4* read, double res, uint32_t n_points, uint32_t* cnt, uint64_t* off,
                                   void* temp, size_t temp_bytes) {
  if (!n_blocks) return hipSuccess;
  k_spo_count<<<n_blocks, 256, 0, s>>>(blk_cloud, blk_start, clouds, ref, read, res, cnt);
  size_t b = temp_bytes;
  return rocprim::exclusive_scan(temp, b, cnt, off, (uint64_t)0, n_points, rocprim::plus<uint64_t>(), s);
}

hipError_t launch_ovl_sparse_sets(hipStream_t s, uint32_t n_blocks, const uint32_t* blk_cloud,
                                  const uint32_t* blk_start, const OvlCloud* clouds, const float4* ref,
                                  const float4* read, double res, const uint64_t* off, uint64_t n_keys,
                                  uint64_t* keys0, uint64_t* keys1, void* temp, size_t temp_bytes, int n_groups,
                                  int n_pairs, const PairDesc* pd, unsigned long long* per_cloud,
                                  unsigned long long* per_pair, PairState* gst, PairState* st) {
  (void)hipMemsetAsync(per_cloud, 0, (size_t)(n_groups + n_pairs) * 8, s);
  (void)hipMemsetAsync(per_pair, 0, (size_t)n_pairs * 8, s);
  if (n_keys) {
    k_spo_emit<<<n_blocks, 256, 0, s>>>(blk_cloud, blk_start, clouds, ref, read, res, off, keys0);
    size_t b = temp_bytes;
    const hipError_t e = rocprim::radix_sort_keys(temp, b, keys0, keys1, n_keys, 0, 64, s);
    if (e != hipSuccess) return e;
    const unsigned g = (unsigned)((n_keys + 255) / 256);
    k_spo_unique<<<g, 256, 0, s>>>(keys1, n_keys, per_cloud);
    k_spo_intersect<<<g, 256, 0, s>>>(keys1, n_keys, n_groups, pd, per_pair);
  }
  const int m = n_groups > n_pairs ? n_groups : n_pairs;
  k_spo_counts<<<(m + 63) / 64, 64, 0, s>>>(n_groups, n_pairs, per_cloud, per_pair, gst, st);
  return hipGetLastError();
}

size_t ovl_keys_temp_bytes(size_t n_points, size_t cap, int n_clouds) {
  size_t a = 0, b = 0;
  (void)rocprim::exclusive_scan(nullptr, a, (const uint32_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, n_points,
                                rocprim::plus<uint64_t>());
  (void)rocprim::radix_sort_keys(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr, cap, 0,
                                 key_end_bit(n_clouds));
  return a > b ? a : b;
}

hipError_t launch_ovl_keys(hipStream_t s, const OvlKeySide& k, const double* origin0, const float4* pts,
                           double res, PairState* st, int slot) {
  if (origin0) k_spo_origin<<<1, 64, 0, s>>>(k.clouds, origin0);
  if (k.n_blocks) {
    k_spo_count<<<k.n_blocks, 256, 0, s>>>(k.blk_cloud, k.blk_start, k.clouds, pts, pts, res, k.cnt);
    size_t b = k.temp_bytes;
    hipError_t e = rocprim::exclusive_scan(k.temp, b, k.cnt, k.off, (uint64_t)0, k.n_points,
                                           rocprim::plus<uint64_t>(), s);
    if (e != hipSuccess) return e;
    k_spo_emit_cap<<<k.n_blocks, 256, 0, s>>>(k.blk_cloud, k.blk_start, k.clouds, pts, res, k.off, k.cap, k.keys0,
                                              st);
  }
  const uint64_t pad = (uint64_t)k.n_clouds << 48;
  const uint64_t pb = (k.cap + 255) / 256;
  if (k.cap) k_spo_pad<<<(unsigned)(pb < 4096 ? pb : 4096), 256, 0, s>>>(k.off, k.cnt, k.n_points, k.cap, pad, k.keys0);
  k_spo_zero<<<(k.n_clouds + 63) / 64, 64, 0, s>>>(k.per_cloud, k.n_clouds);
  if (k.cap) {
    size_t b = k.temp_bytes;
    const hipError_t e =
        rocprim::radix_sort_keys(k.temp, b, k.keys0, k.keys1, k.cap, 0, key_end_bit(k.n_clouds), s);
    if (e != hipSuccess) return e;
    k_spo_unique_cap<<<(unsigned)((k.cap + 255) / 256), 256, 0, s>>>(k.keys1, k.cap, (uint32_t)k.n_clouds,
                                                                     k.per_cloud);
  }
  k_spo_store<<<(k.n_clouds + 63) / 64, 64, 0, s>>>(k.n_clouds, k.per_cloud, st, slot);
  return hipGetLastError();
}

hipError_t launch_ovl_keys_intersect(hipStream_t s, const OvlKeySide& rd, const OvlKeySide& ref,
                                     unsigned long long* per_pair, PairState* st) {
  k_spo_zero<<<(rd.n_clouds + 63) / 64, 64, 0, s>>>(per_pair, rd.n_clouds);
  if (rd.cap)
    k_spo_intersect_ref<<<(unsigned)((rd.cap + 255) / 256), 256, 0, s>>>(rd.keys1, rd.cap, (uint32_t)rd.n_clouds,
                                                                         ref.keys1, ref.cap, per_pair);
  k_spo_store<<<(rd.n_clouds + 63) / 64, 64, 0, s>>>(rd.n_clouds, per_pair, st, 2);
  return hipGetLastError();
}

}  // namespace aicp
