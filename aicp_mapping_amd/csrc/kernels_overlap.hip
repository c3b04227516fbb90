// kernels_overlap.hip — octree overlap of OctreesOverlap::computeOverlap on the device.
//
// Reference (aicp_core/src/overlap/octrees_overlap.cpp:29-72,113-241 + octomap):
// each cloud's known-voxel set S = every key of computeRayKeys(origin, p) (Amanatides-Woo,
// float direction, double tMax) plus every endpoint key; overlap% = min(|A∩B|/|A|,
// |A∩B|/|B|) * 100. octomap stores S in an octree, prunes and expands it; only the set matters.
//
// Device form: one byte per voxel of a padded key box per cloud, in 8 x 8 x 2 bricks of 128 B
// (aicp_common.hpp: ovl_index). Every ray key is a plain byte store of 1 -- concurrent writers store the same value, so no atomics and no
// read-before-write are needed. A reference cloud seen from one origin has one voxel set
// whatever reading it is paired with, so its map is built once per (reference, origin)
// group and shared by the pairs of a reference window; |A| is counted once per group, |B|
// per reading, and |A∩B| by looking every voxel of a reading's map up in its group's map.
// A 60 x 60 x 6 m scene at 0.2 m is ~2.7 M voxels = 2.7 MB per map (L2/MALL resident).
// (tools/experiments/microbench.hip: with 16 distinct pairs, check+atomicOr bitmaps ran 11x slower.)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "aicp_common.hpp"
#include "icp_math.hpp"
#include "kernels.hpp"

namespace aicp {

constexpr int kTreeMaxVal = 32768;

// coordToKeyChecked: the key exists iff floor(c / res) is in [-32768, 32768) (x86 converts NaN
// and out-of-range values to INT_MIN, which octomap's range test rejects; written out here so a
// NaN coordinate is rejected on the device as well, instead of converting to 0)
__device__ __forceinline__ bool key_checked(double rf, float c, int& key) {
  const double f = floor(rf * (double)c);
  if (!(f >= -(double)kTreeMaxVal && f < (double)kTreeMaxVal)) return false;
  key = (int)f + kTreeMaxVal;
  return true;
}

// sides: 1 = the reference origin, 2 = the reading origin
__global__ void k_ovl_init(int n_pairs, const PairDesc* __restrict__ pd, PairState* st, double res, int sides) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const double rf = 1.0 / res;
  int lo[3] = {1 << 30, 1 << 30, 1 << 30}, hi[3] = {-(1 << 30), -(1 << 30), -(1 << 30)};
  for (int side = 0; side < 2; ++side) {
    if (!((sides >> side) & 1)) continue;
    const double* o = side ? pd[p].read_origin : pd[p].ref_origin;
    int k[3];
    bool ok = true;
    for (int i = 0; i < 3; ++i) ok &= key_checked(rf, (float)o[i], k[i]);
    if (!ok) continue;
    for (int i = 0; i < 3; ++i) {
      lo[i] = min(lo[i], k[i]);
      hi[i] = max(hi[i], k[i]);
    }
  }
  for (int i = 0; i < 3; ++i) {
    st[p].ovl_bbox[i] = lo[i];
    st[p].ovl_bbox[3 + i] = hi[i];
    st[p].ovl_counts[i] = 0;
  }
  st[p].ovl_err = 0;
}

__global__ __launch_bounds__(256) void k_ovl_bbox(BlockMap m, const PairDesc* __restrict__ pd,
                                                  PairState* st, const float4* __restrict__ pts,
                                                  int side, double res) {
  const int pair = m.pair[blockIdx.x];
  const uint32_t j = m.start[blockIdx.x] + threadIdx.x;
  const PairDesc& d = pd[pair];
  const uint32_t n = side ? d.n_read : d.n_ref;
  const uint32_t off = side ? d.read_off : d.ref_off;
  const double rf = 1.0 / res;
  int lo[3] = {1 << 30, 1 << 30, 1 << 30}, hi[3] = {-(1 << 30), -(1 << 30), -(1 << 30)};
  if (j < n) {
    const float4 p = pts[off + j];
    int k[3];
    if (key_checked(rf, p.x, k[0]) && key_checked(rf, p.y, k[1]) && key_checked(rf, p.z, k[2]))
      for (int i = 0; i < 3; ++i) lo[i] = hi[i] = k[i];
  }
  // block reduction, then at most 6 atomics per block, skipped when they cannot change the box
  __shared__ int slo[3][4], shi[3][4];
  const int w = threadIdx.x >> 6;
  for (int i = 0; i < 3; ++i) {
    int a = lo[i], b = hi[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a = min(a, __shfl_xor(a, o, 64));
      b = max(b, __shfl_xor(b, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      slo[i][w] = a;
      shi[i][w] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int i = threadIdx.x;
    const int a = min(min(slo[i][0], slo[i][1]), min(slo[i][2], slo[i][3]));
    const int b = max(max(shi[i][0], shi[i][1]), max(shi[i][2], shi[i][3]));
    if (a <= b) {
      if (a < st[pair].ovl_bbox[i]) atomicMin(&st[pair].ovl_bbox[i], a);
      if (b > st[pair].ovl_bbox[3 + i]) atomicMax(&st[pair].ovl_bbox[3 + i], b);
    }
  }
}

// computeRayKeys(origin, end) + endpoint key, marking bits of one bitmap.
// kFilter: a workgroup-local direct-mapped cache in LDS of the voxel indices its lanes have
// stored skips repeats (maps of < 2^32 voxels). Every store leaves L2 (MI355X_MICROARCH.md: "all
// bytes leave L2 every pass"), and the ~100 ray steps per point fall on far fewer distinct
// voxels; a skipped store is always one that a lane of the workgroup has already issued, so
// the map is the same union. C5 (r04, rocprofv3 + PMC WRITE_SIZE per dispatch): reference side
// 111 -> 66 GB, reading side 17.5 -> 13.9 GB, time equal (24.0 vs 23.5 ms average). The batch
// path (many clouds) uses it; the stream's window (6 clouds, latency-bound walks) does not: there
// the cache's LDS round trip per step made the launch slower (C2: 182 against 162 us). Measured
// and not kept: groups of 8 voxel bytes loaded and only the zero ones stored (WRITE_SIZE 109 ->
// 19.6 GB, but 24.6 -> 30.5 ms: the loads' latency enters the walk).
constexpr int kMarkCache = 4096;
template <bool kFilter>
__global__ __launch_bounds__(256) void k_ovl_mark(BlockMap m, const PairDesc* __restrict__ pd,
                                                  const OvlDesc* __restrict__ od, PairState* st,
                                                  const float4* __restrict__ pts, int side, double res,
                                                  uint8_t* maps) {
  __shared__ uint32_t cache[kFilter ? kMarkCache : 1];
  if constexpr (kFilter) {
    for (int i = threadIdx.x; i < kMarkCache; i += 256) cache[i] = 0xFFFFFFFFu;
    __syncthreads();
  }
  // grid-stride over the map's blocks (a launch may use fewer workgroups than blocks: the stream's
  // reference-side marks run beside the critical kd-tree build, launch_ovl_mark's max_blocks)
  for (uint32_t mb = blockIdx.x; mb < m.n_blocks; mb += gridDim.x) {
  const int pair = m.pair[mb];
  if (pair < 0) continue;  // (padding block of an XCD-dealt map)
  const uint32_t j = m.start[mb] + threadIdx.x;
  const PairDesc& d = pd[pair];
  const uint32_t n = side ? d.n_read : d.n_ref;
  if (j >= n) continue;
  const uint32_t off = side ? d.read_off : d.ref_off;
  const OvlDesc& ov = od[pair];
  uint8_t* bm = maps + ov.off;
  const int mn0 = ov.min[0], mn1 = ov.min[1], mn2 = ov.min[2];
  const int dm0 = ov.dim[0], dm1 = ov.dim[1], dm2 = ov.dim[2];
  bool err = false;
  const bool filt = kFilter && (uint64_t)dm0 * (uint64_t)dm1 * (uint64_t)dm2 < (1ull << 32);
  auto put = [&](int64_t idx) {
    if (filt) {
      const uint32_t v = (uint32_t)idx;
      const uint32_t slot = (v * 2654435761u) >> 20;  // 12 bits
      if (cache[slot] == v) return;
      bm[idx] = 1;
      cache[slot] = v;
      return;
    }
    bm[idx] = 1;
  };
  auto mark = [&](int k0, int k1, int k2) {
    const int a = k0 - mn0, b = k1 - mn1, c = k2 - mn2;
    if ((unsigned)a >= (unsigned)dm0 || (unsigned)b >= (unsigned)dm1 || (unsigned)c >= (unsigned)dm2) {
      err = true;
      return;
    }
    put((int64_t)ovl_index((uint32_t)a, (uint32_t)b, (uint32_t)c, (uint32_t)dm1, (uint32_t)dm2));
  };
  const double* org = side ? d.read_origin : d.ref_origin;
  const float o[3] = {(float)org[0], (float)org[1], (float)org[2]};
  const float4 p4 = pts[off + j];
  const float e[3] = {p4.x, p4.y, p4.z};
  const double rf = 1.0 / res;
  int ko[3], ke[3];
  const bool okO = key_checked(rf, o[0], ko[0]) && key_checked(rf, o[1], ko[1]) &&
                   key_checked(rf, o[2], ko[2]);
  const bool okE = key_checked(rf, e[0], ke[0]) && key_checked(rf, e[1], ke[1]) &&
                   key_checked(rf, e[2], ke[2]);
  if (okO && okE && !(ko[0] == ke[0] && ko[1] == ke[1] && ko[2] == ke[2])) {
    mark(ko[0], ko[1], ko[2]);
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
        double vb = (double(cur[i] - kTreeMaxVal) + 0.5) * res;
        vb += (float)(step[i] * res * 0.5);
        tMax[i] = (vb - (double)o[i]) / (double)dir[i];
        tDelta[i] = res / (double)fabsf(dir[i]);
      } else {
        tMax[i] = 1.7976931348623157e308;
        tDelta[i] = 1.7976931348623157e308;
      }
    }
    const double len = (double)length;
    // the box coordinates follow the walk (one bounds test on the axis that moved: the other two
    // are unchanged); the brick index is formed from them per step
    int rel[3] = {cur[0] - mn0, cur[1] - mn1, cur[2] - mn2};
    const int dims[3] = {dm0, dm1, dm2}, mins[3] = {mn0, mn1, mn2};
    // one step of the walk: false once it has ended (endpoint key, past the length, or bad)
    auto walk = [&](int64_t& out) -> bool {
      int dim;
      if (tMax[0] < tMax[1])
        dim = (tMax[0] < tMax[2]) ? 0 : 2;
      else
        dim = (tMax[1] < tMax[2]) ? 1 : 2;
      // cur[dim] = (cur[dim] + step[dim]) & 0xFFFF, on registers without dynamic indexing
      bool bad = false;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i == dim) {
          cur[i] = (cur[i] + step[i]) & 0xFFFF;
          tMax[i] += tDelta[i];
          rel[i] += step[i];
          // a key wrap (0xFFFF) or a walk leaving the padded box is reported, never stored
          bad = (cur[i] - mins[i]) != rel[i] || (unsigned)rel[i] >= (unsigned)dims[i];
        }
      if (cur[0] == ke[0] && cur[1] == ke[1] && cur[2] == ke[2]) return false;
      const double dfo = fmin(fmin(tMax[0], tMax[1]), tMax[2]);
      if (dfo > len) return false;
      if (bad) {
        err = true;
        return false;
      }
      out = (int64_t)ovl_index((uint32_t)rel[0], (uint32_t)rel[1], (uint32_t)rel[2], (uint32_t)dm1, (uint32_t)dm2);
      return true;
    };
    int64_t g;
    while (walk(g)) put(g);
  }
  if (okE) mark(ke[0], ke[1], ke[2]);
  if (err) atomicOr(&st[pair].ovl_err, 1);
  }
}

// popcounts: |A|, |B|, |A & B| (bpm workgroups per map, integer atomics -> deterministic).
// count_bpm: 64 per map for batches, more for a few maps (a single reading's ~3 MB map with 64
// workgroups took 57 us for the intersection, each thread walking 12 words of random lookups)
// Only the one-shot call of a single pair takes the wide form (wide = true): on the stream the
// counts run beside the window's kd-tree builds, and 409 workgroups per map there slowed the
// critical normals chain (ref -> normals 0.79-0.82 against 0.77 ms, r05 same-box A/B).
inline int count_bpm(int n_maps, bool wide) {
  return wide ? std::max(64, std::min(512, 2048 / std::max(1, n_maps))) : 64;
}

// the workgroup's sum of c added to *dst by one atomic (the counts of a map share one address:
// one atomic per wave was 2048 same-address atomics per map for the wide grid, ~20 us)
__device__ __forceinline__ void block_add_u64(unsigned long long c, unsigned long long* dst) {
  __shared__ unsigned long long wsum[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (t) atomicAdd(dst, t);
  }
}

// |S| of every map in od[]: byte sums (bytes are 0 or 1; maps 16-byte aligned and padded)
__global__ __launch_bounds__(256) void k_ovl_popcount(const OvlDesc* __restrict__ od, PairState* st, int slot,
                                                      const uint8_t* __restrict__ maps, int bpm) {
  const int m = blockIdx.x / bpm;
  const int sub = blockIdx.x % bpm;
  const OvlDesc& ov = od[m];
  const uint4* A = (const uint4*)(maps + ov.off);
  const uint64_t n16 = ov.bytes / 16;
  unsigned long long c = 0;
  for (uint64_t w = (uint64_t)sub * 256 + threadIdx.x; w < n16; w += (uint64_t)bpm * 256) {
    const uint4 a = A[w];
    c += __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w);
  }
  block_add_u64(c, (unsigned long long*)&st[m].ovl_counts[slot]);
}

// |A ∩ B|: every 16-byte word of a reading's map against the word holding the same voxels in its
// group's reference map (both boxes start on brick boundaries of the key lattice, so the word s of
// a brick covers the same keys in both); bytes are 0 or 1, so the popcount of the AND counts them
__global__ __launch_bounds__(256) void k_ovl_intersect(const PairDesc* __restrict__ pd,
                                                       const OvlDesc* __restrict__ od_read,
                                                       const OvlDesc* __restrict__ od_ref, PairState* st,
                                                       const uint8_t* __restrict__ maps, int bpm) {
  const int p = blockIdx.x / bpm;
  const int sub = blockIdx.x % bpm;
  const OvlDesc& rb = od_read[p];
  const OvlDesc& ra = od_ref[pd[p].ogroup];
  const uint4* B = (const uint4*)(maps + rb.off);
  const uint4* A = (const uint4*)(maps + ra.off);
  const uint64_t n16 = rb.bytes / 16;
  const uint32_t b1 = (uint32_t)rb.dim[1] / kOvlBrick1, b2 = (uint32_t)rb.dim[2] / kOvlBrick2;
  const uint32_t a0 = (uint32_t)ra.dim[0] / kOvlBrick0, a1 = (uint32_t)ra.dim[1] / kOvlBrick1,
                 a2 = (uint32_t)ra.dim[2] / kOvlBrick2;
  // the reading box's brick (0, 0, 0) in the reference box's bricks
  const int o0 = (rb.min[0] - ra.min[0]) / kOvlBrick0, o1 = (rb.min[1] - ra.min[1]) / kOvlBrick1,
            o2 = (rb.min[2] - ra.min[2]) / kOvlBrick2;
  constexpr uint32_t kWords = kOvlBrickBytes / 16;
  unsigned long long c = 0;
  for (uint64_t w = (uint64_t)sub * 256 + threadIdx.x; w < n16; w += (uint64_t)bpm * 256) {
    const uint4 b = B[w];
    if ((b.x | b.y | b.z | b.w) == 0) continue;
    const uint64_t brick = w / kWords;
    const uint32_t s = (uint32_t)(w % kWords);
    const uint32_t z = (uint32_t)(brick % b2);
    const uint64_t r = brick / b2;
    const uint32_t y = (uint32_t)(r % b1), x = (uint32_t)(r / b1);
    const int gx = (int)x + o0, gy = (int)y + o1, gz = (int)z + o2;
    if ((unsigned)gx >= a0 || (unsigned)gy >= a1 || (unsigned)gz >= a2) continue;
    const uint4 a = A[(((uint64_t)gx * a1 + (uint64_t)gy) * a2 + (uint64_t)gz) * kWords + s];
    c += __popc(a.x & b.x) + __popc(a.y & b.y) + __popc(a.z & b.z) + __popc(a.w & b.w);
  }
  block_add_u64(c, (unsigned long long*)&st[p].ovl_counts[2]);
}

__global__ void k_ovl_finish(int n_pairs, const PairDesc* __restrict__ pd, PairState* st,
                             const PairState* __restrict__ gst, int set_ratio) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  PairState& s = st[p];
  const PairState& g = gst[pd[p].ogroup];
  s.ovl_counts[0] = g.ovl_counts[0];
  if (g.ovl_err) s.ovl_err = 1;
  const float ov = (float)s.ovl_counts[2];
  const float a = ov / (float)s.ovl_counts[0];
  const float b = ov / (float)s.ovl_counts[1];
  const float mn = (b < a) ? b : a;  // std::min
  s.overlap = (float)(mn * 100.0);
  if (set_ratio) s.ratio = autotune_ratio_fast(s.overlap);
}

void launch_ovl_init(hipStream_t s, int n, const PairDesc* pd, PairState* st, double res, int sides) {
  if (n) k_ovl_init<<<(n + 63) / 64, 64, 0, s>>>(n, pd, st, res, sides);
}
void launch_ovl_bbox(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                     const float4* pts, int side, double res) {
  if (m.n_blocks) k_ovl_bbox<<<m.n_blocks, 256, 0, s>>>(m, pd, st, pts, side, res);
}
void launch_ovl_mark(hipStream_t s, BlockMap m, const PairDesc* pd, const OvlDesc* od, PairState* st,
                     const float4* pts, int side, double res, uint8_t* maps, bool filter, unsigned max_blocks) {
  if (!m.n_blocks) return;
  const unsigned g = max_blocks ? std::min<unsigned>(m.n_blocks, max_blocks) : m.n_blocks;
  if (filter)
    k_ovl_mark<true><<<g, 256, 0, s>>>(m, pd, od, st, pts, side, res, maps);
  else
    k_ovl_mark<false><<<g, 256, 0, s>>>(m, pd, od, st, pts, side, res, maps);
}
void launch_ovl_count(hipStream_t s, int n_pairs, int n_groups, const PairDesc* pd, const OvlDesc* od_read,
                      const OvlDesc* od_ref, PairState* st, PairState* gst, const uint8_t* maps) {
  const bool wide = n_pairs + n_groups <= 2;  // (the one-shot call of one pair)
  const int bg = count_bpm(n_groups, wide), bp = count_bpm(n_pairs, wide);
  k_ovl_popcount<<<n_groups * bg, 256, 0, s>>>(od_ref, gst, 0, maps, bg);
  k_ovl_popcount<<<n_pairs * bp, 256, 0, s>>>(od_read, st, 1, maps, bp);
  k_ovl_intersect<<<n_pairs * bp, 256, 0, s>>>(pd, od_read, od_ref, st, maps, bp);
}
void launch_ovl_popcount(hipStream_t s, int n, const OvlDesc* od, PairState* st, int slot, const uint8_t* maps,
                         bool wide) {
  if (n) k_ovl_popcount<<<n * count_bpm(n, wide), 256, 0, s>>>(od, st, slot, maps, count_bpm(n, wide));
}
void launch_ovl_intersect(hipStream_t s, int n_pairs, const PairDesc* pd, const OvlDesc* od_read, const OvlDesc* od_ref,
                          PairState* st, const uint8_t* maps, bool wide) {
  if (n_pairs)
    k_ovl_intersect<<<n_pairs * count_bpm(n_pairs, wide), 256, 0, s>>>(pd, od_read, od_ref, st, maps,
                                                                      count_bpm(n_pairs, wide));
}
void launch_ovl_finish(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const PairState* gst,
                       int set_ratio) {
  k_ovl_finish<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st, gst, set_ratio);
}

}  // namespace aicp
