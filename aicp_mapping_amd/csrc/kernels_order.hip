// kernels_order.hip — spatial order of the reading points (queries) before the ICP loop.
//
// The nearest-neighbour search of a reading point does not depend on where the point sits in
// the reading array, and neither does anything else downstream: the trimmed select is a k-th
// value, the point-to-plane system is a sum (kept in double, summed per block in a fixed
// order), the overlap is a key set. So the batch may visit the readings in any order. The
// order it does visit them in decides how much the 64 lanes of a wave share: queries that are
// close in space descend through the same kd-tree nodes and scan the same buckets, so their
// 16-B loads coalesce into the same cache lines and their paths have similar lengths. A
// Morton (Z-order) sort of the points on 0.25 m cells, done once per batch, makes neighbouring
// slots neighbouring points whatever order the caller's scan came in (measured on MI355X: NN
// launch 803 us for the raster order of the synthetic scans, 1076 us shuffled, 734 us sorted).
//
// Key = pair index << 30 | 30-bit Morton code of the point's cell (10 bits per axis, the cell
// grid wraps every 256 m, which only costs locality). The stable radix sort keeps each pair's
// points inside the pair's own range [read_off, read_off + n_read) and makes the order
// deterministic.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "aicp_common.hpp"
#include "kernels.hpp"

namespace aicp {

namespace {

__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ __forceinline__ uint32_t cell10(float x) {
  return (uint32_t)__float2int_rd(x * 4.0f) & 0x3ffu;  // 0.25 m cells, wrapped
}

__global__ __launch_bounds__(256) void k_read_keys(BlockMap m, const PairDesc* __restrict__ pd,
                                                   const float4* __restrict__ raw,
                                                   uint64_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals) {
  const uint32_t b = blockIdx.x;
  const int pair = m.pair[b];
  const uint32_t j = m.start[b] + threadIdx.x;
  const PairDesc& d = pd[pair];
  if (j >= d.n_read) return;
  const uint32_t i = d.read_off + j;
  const float4 p = raw[i];
  const uint32_t z = spread3(cell10(p.x)) | (spread3(cell10(p.y)) << 1) | (spread3(cell10(p.z)) << 2);
  keys[i] = ((uint64_t)pair << 30) | z;
  vals[i] = i;
}

__global__ __launch_bounds__(256) void k_read_gather(uint32_t n, const uint32_t* __restrict__ idx,
                                                     const float4* __restrict__ raw,
                                                     float4* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) out[i] = raw[idx[i]];
}

int key_bits(int n_pairs) {
  int b = 0;
  while ((1 << b) < n_pairs) ++b;
  return 30 + b;
}

}  // namespace

size_t read_order_temp_bytes(size_t n, int n_pairs) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, key_bits(n_pairs));
  return bytes;
}

hipError_t launch_read_order(hipStream_t s, BlockMap m, int n_pairs, const PairDesc* pd, const float4* raw,
                             uint32_t total, uint64_t* keys0, uint64_t* keys1, uint32_t* vals0, uint32_t* vals1,
                             void* temp, size_t temp_bytes, float4* out) {
  if (!total || !m.n_blocks) return hipSuccess;
  k_read_keys<<<m.n_blocks, 256, 0, s>>>(m, pd, raw, keys0, vals0);
  size_t bytes = temp_bytes;
  const hipError_t e = rocprim::radix_sort_pairs(temp, bytes, keys0, keys1, vals0, vals1, total, 0,
                                                 key_bits(n_pairs), s);
  if (e != hipSuccess) return e;
  k_read_gather<<<(total + 255) / 256, 256, 0, s>>>(total, vals1, raw, out);
  return hipGetLastError();
}

}  // namespace aicp
