// Oriented box crop of a resident map: getPointsInOrientedBox,
// aicp_core/src/utils/filteringUtils.cpp:619-637 (pcl::CropBox), as used by the
// localization-only mode to cut the reference out of the prior map (app.cpp:41-51).
//
// HBM-bound stream compaction, order-preserving like CropBox's index walk:
//   k_crop_count   one 1024-point tile per block: keep flags -> per-tile count
//   k_crop_scan    one block: exclusive scan of the tile counts (+ total)
//   k_crop_scatter the same flags again; ballot prefix inside each wave, LDS prefix over the
//                  4 waves, 4 rounds per tile in index order -> kept points at their rank.
// Algorithmic bytes: 2 x 16 B per input point (flags recomputed instead of stored) + 16 B per
// kept point + 8 B per tile. The 3x3 local-frame matrix is prepared on the host (kernels.hpp).
#include <cstring>

#include "kernels.hpp"

namespace aicp {
namespace {

constexpr int kCropThreads = 256;
constexpr int kCropTile = 1024;  // 4 rounds of 256

struct CropBoxArgs {
  float inv[9];  // row-major local-frame rotation (identity when CropBox would skip it)
  float t[3];    // translation subtracted first
  float mn, mx;
};

__device__ __forceinline__ bool crop_keep(const CropBoxArgs& a, float4 p) {
  if (!isfinite(p.x) || !isfinite(p.y) || !isfinite(p.z)) return false;
  const float x = __fsub_rn(p.x, a.t[0]), y = __fsub_rn(p.y, a.t[1]), z = __fsub_rn(p.z, a.t[2]);
  float l[3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
    l[r] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(a.inv[3 * r], x), __fmul_rn(a.inv[3 * r + 1], y)),
                               __fmul_rn(a.inv[3 * r + 2], z)),
                     0.f);
  return !(l[0] < a.mn || l[1] < a.mn || l[2] < a.mn || l[0] > a.mx || l[1] > a.mx || l[2] > a.mx);
}

__global__ __launch_bounds__(kCropThreads) void k_crop_count(int n, CropBoxArgs a, const float4* __restrict__ pts,
                                                             uint32_t* __restrict__ tile_cnt) {
  __shared__ uint32_t wsum[kCropThreads / 64];
  const int base = blockIdx.x * kCropTile;
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < kCropTile / kCropThreads; ++r) {
    const int i = base + r * kCropThreads + threadIdx.x;
    if (i < n && crop_keep(a, pts[i])) ++c;
  }
  // wave sum by xor shuffles, then the 4 wave sums through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// Single block of 1024 threads: exclusive scan of up to any number of tile counts, in chunks.
__device__ __forceinline__ void crop_scan_block(int n_tiles, const uint32_t* __restrict__ cnt,
                                                uint32_t* __restrict__ off, uint32_t* __restrict__ total) {
  __shared__ uint32_t wtot[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c0 = 0; c0 < n_tiles; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const uint32_t v = i < n_tiles ? cnt[i] : 0u;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    uint32_t wbase = carry;
    for (int q = 0; q < w; ++q) wbase += wtot[q];
    if (i < n_tiles) off[i] = wbase + incl - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = wbase + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ __launch_bounds__(1024) void k_crop_scan(int n_tiles, const uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ off, uint32_t* __restrict__ total) {
  crop_scan_block(n_tiles, cnt, off, total);
}
// one block per crop
__global__ __launch_bounds__(1024) void k_crop_scan_multi(int n_tiles, const uint32_t* __restrict__ cnt,
                                                          uint32_t* __restrict__ off, uint32_t* __restrict__ total) {
  const size_t o = (size_t)blockIdx.x * n_tiles;
  crop_scan_block(n_tiles, cnt + o, off + o, total + blockIdx.x);
}

__global__ __launch_bounds__(kCropThreads) void k_crop_scatter(int n, CropBoxArgs a, const float4* __restrict__ pts,
                                                               const uint32_t* __restrict__ tile_off,
                                                               float4* __restrict__ out) {
  __shared__ uint32_t wcnt[kCropThreads / 64];
  const int base = blockIdx.x * kCropTile;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t run = tile_off[blockIdx.x];
#pragma unroll 1
  for (int r = 0; r < kCropTile / kCropThreads; ++r) {
    const int i = base + r * kCropThreads + threadIdx.x;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    bool keep = false;
    if (i < n) {
      p = pts[i];
      keep = crop_keep(a, p);
    }
    const uint64_t m = __ballot(keep);
    const uint32_t below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t wb = run;
    for (int q = 0; q < w; ++q) wb += wcnt[q];
    if (keep) out[wb + below] = make_float4(p.x, p.y, p.z, 1.f);
    run += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
}

// Many crops of one map at once (one per reading of a localization batch): blockIdx.y = crop.
// Counts per (crop, tile), then one block per crop scans its tiles into offsets and a total.
__global__ __launch_bounds__(kCropThreads) void k_crop_count_multi(int n, const CropBoxArgs* __restrict__ args,
                                                                   const float4* __restrict__ pts,
                                                                   uint32_t* __restrict__ tile_cnt, int tiles) {
  __shared__ uint32_t wsum[kCropThreads / 64];
  const CropBoxArgs a = args[blockIdx.y];
  const int base = blockIdx.x * kCropTile;
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < kCropTile / kCropThreads; ++r) {
    const int i = base + r * kCropThreads + threadIdx.x;
    if (i < n && crop_keep(a, pts[i])) ++c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[(size_t)blockIdx.y * tiles + blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(kCropThreads) void k_crop_scatter_multi(int n, const CropBoxArgs* __restrict__ args,
                                                                     const float4* __restrict__ pts,
                                                                     const uint32_t* __restrict__ tile_off, int tiles,
                                                                     const uint32_t* __restrict__ base_of,
                                                                     float4* __restrict__ out) {
  __shared__ uint32_t wcnt[kCropThreads / 64];
  const CropBoxArgs a = args[blockIdx.y];
  const int base = blockIdx.x * kCropTile;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float4* o = out + base_of[blockIdx.y];
  uint32_t run = tile_off[(size_t)blockIdx.y * tiles + blockIdx.x];
#pragma unroll 1
  for (int r = 0; r < kCropTile / kCropThreads; ++r) {
    const int i = base + r * kCropThreads + threadIdx.x;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    bool keep = false;
    if (i < n) {
      p = pts[i];
      keep = crop_keep(a, p);
    }
    const uint64_t m = __ballot(keep);
    const uint32_t below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t wb = run;
    for (int q = 0; q < w; ++q) wb += wcnt[q];
    if (keep) o[wb + below] = make_float4(p.x, p.y, p.z, 1.f);
    run += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
}

}  // namespace

size_t crop_tiles(size_t n) { return (n + kCropTile - 1) / kCropTile; }
size_t crop_args_bytes() { return sizeof(CropBoxArgs); }

void pack_crop_args(const float inv[9], const float t[3], float mn, float mx, void* dst) {
  CropBoxArgs a;
  for (int q = 0; q < 9; ++q) a.inv[q] = inv[q];
  for (int q = 0; q < 3; ++q) a.t[q] = t[q];
  a.mn = mn;
  a.mx = mx;
  std::memcpy(dst, &a, sizeof(a));
}

void launch_crop_count_multi(hipStream_t s, int n, int n_crops, const void* args, const float4* pts,
                             uint32_t* tile_cnt, uint32_t* tile_off, uint32_t* totals) {
  const int tiles = (int)crop_tiles((size_t)n);
  if (!tiles || !n_crops) return;
  k_crop_count_multi<<<dim3(tiles, n_crops), kCropThreads, 0, s>>>(n, (const CropBoxArgs*)args, pts, tile_cnt, tiles);
  k_crop_scan_multi<<<n_crops, 1024, 0, s>>>(tiles, tile_cnt, tile_off, totals);
}

void launch_crop_scatter_multi(hipStream_t s, int n, int n_crops, const void* args, const float4* pts,
                               const uint32_t* tile_off, const uint32_t* base_of, float4* out) {
  const int tiles = (int)crop_tiles((size_t)n);
  if (!tiles || !n_crops) return;
  k_crop_scatter_multi<<<dim3(tiles, n_crops), kCropThreads, 0, s>>>(n, (const CropBoxArgs*)args, pts, tile_off, tiles,
                                                                    base_of, out);
}

void launch_crop_box(hipStream_t s, int n, const float inv[9], const float t[3], float mn, float mx,
                     const float4* pts, uint32_t* tile_cnt, uint32_t* tile_off, uint32_t* total,
                     float4* out) {
  CropBoxArgs a;
  for (int q = 0; q < 9; ++q) a.inv[q] = inv[q];
  for (int q = 0; q < 3; ++q) a.t[q] = t[q];
  a.mn = mn;
  a.mx = mx;
  const int tiles = (int)crop_tiles((size_t)n);
  if (tiles == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(uint32_t), s);
    return;
  }
  k_crop_count<<<tiles, kCropThreads, 0, s>>>(n, a, pts, tile_cnt);
  k_crop_scan<<<1, 1024, 0, s>>>(tiles, tile_cnt, tile_off, total);
  k_crop_scatter<<<tiles, kCropThreads, 0, s>>>(n, a, pts, tile_off, out);
}

}  // namespace aicp
