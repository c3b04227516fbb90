// kernels_tree.hip — reference centroid and libnabo-order kd-tree construction on the device.
//
// ICP::compute centres the reference on its mean and builds the matcher's kd-tree on it
// (SURVEY.md A.1 steps 2-3). The tree is libnabo's KDTreeUnbalancedPtInLeavesImplicitBounds-
// StackOpt::buildNodes (A.2): for a node over points [first, first + count) with box (mn, mx):
//   cd    = widest box dimension (first strict maximum), ideal = (mx[cd] + mn[cd]) / 2
//   cut   = clamp(ideal, min, max of the points' cd coordinate)
//   pass 1: Hoare partition of the range on (v < cut)        -> br1
//   pass 2: Hoare partition of [br1, count) on (v <= cut)    -> br2
//   left  = 1 if ideal < min; count - 1 if ideal > max; br1 if br1 > count/2;
//           br2 if br2 < count/2; count/2 otherwise
//   children [first, first + left) (box mx[cd] = cut) and the rest (box mn[cd] = cut);
//   a node with count <= bucket is a leaf (bucket = its point range).
// It is bit-for-bit the build of kdtree_host / the oracle, done level by level for all pairs
// and all nodes of a level at once:
//   - min/max and partition counts are wave-segmented reductions + atomics;
//   - a Hoare pass pairs the k-th misplaced element from the left of the boundary with the
//     k-th misplaced element from the right, so every element's destination follows from two
//     ranks, which one exclusive scan of the predicate over all positions provides (the
//     "prefix form" of the partition, checked against the sequential loop in
//     tests/test_oracle.py::test_partition_prefix_form_equals_hoare).
// Node numbering is preorder (left child = n + 1) without any traversal: a node v over
// positions [f, e) at depth d has preorder index d + #{nodes u : end(u) <= f}, because in a
// tree of nested ranges the nodes before v are exactly its d ancestors and the nodes
// entirely to its left. Every node adds 1 at its end position; one scan over positions
// gives all indices, and with the pairs' positions concatenated the same count also yields
// each pair's node offset.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "aicp_common.hpp"
#include "icp_math.hpp"
#include "kernels.hpp"

namespace aicp {

namespace {

__device__ __forceinline__ uint32_t ord_enc(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord_dec(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ float coord(const float4& p, int cd) {
  return cd == 0 ? p.x : (cd == 1 ? p.y : p.z);
}

// Inclusive segmented scan over the wave's lanes for runs of equal `key` (runs are
// contiguous because positions are sorted by segment). Returns true on the last lane of a
// run, which then holds the run's totals.
__device__ __forceinline__ bool wave_seg_minmax(int key, float& mn, float& mx) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int ko = __shfl_up(key, off, 64);
    const float a = __shfl_up(mn, off, 64);
    const float b = __shfl_up(mx, off, 64);
    if (lane >= off && ko == key) {
      mn = fminf(mn, a);
      mx = fmaxf(mx, b);
    }
  }
  const int kn = __shfl_down(key, 1, 64);
  return lane == 63 || kn != key;
}

// Whole-wave reductions (all 64 lanes active) on DPP row operations: quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror reduce each 16-lane row in registers; the four row results are
// combined from scalar readlanes. No LDS round trips (the ds_bpermute shuffles they replace
// cost ~6 dependent LDS-latency steps per reduction).
template <class T, class Op>
__device__ __forceinline__ T wave_reduce_dpp(T v, Op op) {
  static_assert(sizeof(T) == 4, "32-bit values");
  auto dpp = [](T x, int ctl) -> T {
    int i;
    __builtin_memcpy(&i, &x, 4);
    int r;
    switch (ctl) {
      case 0: r = __builtin_amdgcn_mov_dpp(i, 0xB1, 0xF, 0xF, false); break;
      case 1: r = __builtin_amdgcn_mov_dpp(i, 0x4E, 0xF, 0xF, false); break;
      case 2: r = __builtin_amdgcn_mov_dpp(i, 0x141, 0xF, 0xF, false); break;
      default: r = __builtin_amdgcn_mov_dpp(i, 0x140, 0xF, 0xF, false); break;
    }
    T y;
    __builtin_memcpy(&y, &r, 4);
    return y;
  };
  v = op(v, dpp(v, 0));
  v = op(v, dpp(v, 1));
  v = op(v, dpp(v, 2));
  v = op(v, dpp(v, 3));
  int i;
  __builtin_memcpy(&i, &v, 4);
  const int a = __builtin_amdgcn_readlane(i, 0), b = __builtin_amdgcn_readlane(i, 16),
            c = __builtin_amdgcn_readlane(i, 32), d = __builtin_amdgcn_readlane(i, 48);
  T ta, tb, tc, td;
  __builtin_memcpy(&ta, &a, 4);
  __builtin_memcpy(&tb, &b, 4);
  __builtin_memcpy(&tc, &c, 4);
  __builtin_memcpy(&td, &d, 4);
  return op(op(ta, tb), op(tc, td));
}
__device__ __forceinline__ float wave_min(float v) {
  return wave_reduce_dpp(v, [](float a, float b) { return fminf(a, b); });
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce_dpp(v, [](float a, float b) { return fmaxf(a, b); });
}

// Block-wide min/max of (mn, mx) for a block whose valid threads share one key; the result
// is valid on thread 0. 256-thread blocks.
__device__ __forceinline__ void block_minmax(float& mn, float& mx) {
  __shared__ float smn[4], smx[4];
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[w] = mn;
    smx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    mn = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
    mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  }
  __syncthreads();
}

__device__ __forceinline__ int pair_of_pos(const PairDesc* pd, int n_pairs, uint32_t s) {
  int lo = 0, hi = n_pairs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pd[mid].ref_off <= s) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// slot of a node: a leaf at its first position, an inner node at total + its split position
__device__ __forceinline__ void emit_event(NodeEvent* ev, uint8_t* valid, uint32_t* ecnt, uint32_t total,
                                           const NodeEvent& e) {
  const uint32_t slot = (e.cd == (int32_t)kLeaf) ? e.f : total + e.f + e.left;
  ev[slot] = e;
  valid[slot] = 1;
  atomicAdd(&ecnt[e.f + e.c], 1u);
}

__device__ __forceinline__ NodeEvent leaf_event(uint32_t f, uint32_t c, int depth, int pair, uint32_t pf, int pdepth) {
  NodeEvent e{};
  e.f = f;
  e.c = c;
  e.depth = depth;
  e.pair = pair;
  e.cd = (int32_t)kLeaf;
  e.parent_f = pf;
  e.parent_depth = pdepth;
  return e;
}

// cd and ideal of a box (kdtree_host.cpp / oracle: first strict maximum of the extents)
__device__ __forceinline__ void split_dim(const float* mn, const float* mx, int& cd, float& ideal) {
  cd = 0;
  float widest = 0.f;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float e = mx[d] - mn[d];
    if (e > widest) {
      widest = e;
      cd = d;
    }
  }
  const float a = cd == 0 ? mx[0] : (cd == 1 ? mx[1] : mx[2]);
  const float b = cd == 0 ? mn[0] : (cd == 1 ? mn[1] : mn[2]);
  ideal = (a + b) / 2;
}

__device__ __forceinline__ float seg_cut(const TreeSeg& s) {
  const float lo = ord_dec(s.lo), hi = ord_dec(s.hi);
  return s.ideal < lo ? lo : (s.ideal > hi ? hi : s.ideal);
}

// ---- single-pass scan (decoupled look-back) ---------------------------------------------------
// Exclusive scan of per-position counts over [0, n), written to X, in ONE launch: a tile of
// kLbTile positions per workgroup (tile order from an atomic ticket, so every tile's predecessors
// have started), its aggregate published at once, its inclusive prefix once the look-back over
// the predecessors' words (flag << 32 | value, one 64-bit word each) reaches an inclusive one.
// The counts are computed inside (a predicate: no flag array, no separate flag kernel). `st` holds the
// ticket and one word per tile, zeroed before the launch.
// A stalled look-back (impossible while tiles only wait on earlier tickets) gives up after a
// bounded spin, reports ctl->error 16 (the host then fails the call with AICP_ERR_HIP) and takes
// the slow path: the tile's wave 0 sums the predicate over every position before the tile itself
// (val is a pure function of inputs the scan does not write), so the prefix it writes and
// publishes is the exact one and no later kernel of the build indexes with a partial prefix.
// (r05 lost a box to the pattern "time out, then go on with what was there": a grid barrier that
// timed out and left garbage indices behind.) g_lb_force_stall (test hook,
// aicp_hip_test_force_scan_stall) sends every tile but the first down the slow path.
__device__ int g_lb_force_stall;
constexpr int kLbThreads = 256;
constexpr int kLbItems = 8;
constexpr uint32_t kLbTile = kLbThreads * kLbItems;
constexpr uint64_t kLbAgg = 1ull << 32, kLbIncl = 2ull << 32;

__host__ __device__ constexpr uint32_t lb_words(uint32_t n) { return (n + kLbTile - 1) / kLbTile + 1; }

template <class Val>
__device__ __forceinline__ void lookback_scan(uint32_t n, Val val, uint32_t* __restrict__ X, uint64_t* st,
                                              TreeCtl* ctl) {
  __shared__ uint32_t s_tile, s_excl, s_wsum[kLbThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) s_tile = atomicAdd(reinterpret_cast<unsigned int*>(st), 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  uint64_t* tw = st + 1;  // tile words
  const uint32_t i0 = tile * kLbTile + (uint32_t)t * kLbItems;
  uint32_t v[kLbItems];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kLbItems; ++j) {
    v[j] = i0 + j < n ? val(i0 + j) : 0u;
    sum += v[j];
  }
  // block exclusive prefix of the thread sums
  uint32_t x = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wsum[wv] = x;
  __syncthreads();
  uint32_t wbase = 0, agg = 0;
#pragma unroll
  for (int w = 0; w < kLbThreads / 64; ++w) {
    const uint32_t a = s_wsum[w];
    if (w < wv) wbase += a;
    agg += a;
  }
  const uint32_t texcl = wbase + x - sum;
  if (wv == 0) {
    uint32_t excl = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&tw[0], kLbIncl | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&tw[tile], kLbAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t top = (int64_t)tile - 1;  // the nearest predecessor not summed yet
      uint32_t spins = 0;
      bool stalled = __hip_atomic_load(&g_lb_force_stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      while (!stalled) {
        const int64_t idx = top - lane;
        const uint64_t w = idx >= 0 ? __hip_atomic_load(&tw[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : kLbIncl;
        const uint32_t flag = (uint32_t)(w >> 32);
        const uint64_t incl = __ballot(flag == 2), zero = __ballot(flag == 0);
        const int first = incl ? __ffsll((long long)incl) - 1 : 64;  // nearest inclusive word
        const uint64_t need = first == 64 ? ~0ull : ((2ull << first) - 1ull);
        if (zero & need) {  // a predecessor up to there has not published yet
          if (++spins > (1u << 22)) {
            stalled = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint32_t part = lane <= first ? (uint32_t)w : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
        excl += part;
        if (first < 64) break;
        top -= 64;
      }
      if (stalled) {  // the exact prefix the slow way (see above)
        if (lane == 0) atomicOr(&ctl->error, 16);
        uint32_t part = 0;
        const uint32_t end = min(tile * kLbTile, n);
        for (uint32_t i = (uint32_t)lane; i < end; i += 64) part += val(i);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
        excl = part;
      }
      if (lane == 0) __hip_atomic_store(&tw[tile], kLbIncl | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  uint32_t run = s_excl + texcl;
#pragma unroll
  for (int j = 0; j < kLbItems; ++j) {
    if (i0 + j < n) X[i0 + j] = run;
    run += v[j];
  }
}

// ---- centroid --------------------------------------------------------------------------------
// Exact order-independent sum: every coordinate as round(x * 2^40) in 128-bit two's complement
// (64-bit atomics with carry), so the result does not depend on the reduction order.
__device__ __forceinline__ void add128(uint64_t& lo, int64_t& hi, uint64_t lo2, int64_t hi2) {
  const uint64_t s = lo + lo2;
  hi = hi + hi2 + (s < lo ? 1 : 0);
  lo = s;
}

__device__ __forceinline__ void atomic_add128(uint64_t* w, uint64_t lo, int64_t hi) {
  const uint64_t old = atomicAdd((unsigned long long*)w, (unsigned long long)lo);
  const uint64_t carry = (old + lo < old) ? 1u : 0u;
  atomicAdd((unsigned long long*)(w + 1), (unsigned long long)((uint64_t)hi + carry));
}

// Per-pair reductions over the points use tiles of kTile positions per 256-thread block (8 per
// thread): a tile inside one pair (the common case) reduces in registers + LDS.
constexpr int kTileItems = 8;
constexpr uint32_t kTile = 256 * kTileItems;
inline unsigned tiles_of(size_t n) { return (unsigned)std::max<size_t>(1, (n + kTile - 1) / kTile); }

// The centroid sums: a tile inside one pair stores its 128-bit partials (part[6 * tile ..]) and
// k_tr_frames adds them per pair; a tile across pair boundaries adds its runs atomically into
// sums[6 * pair ..]. (With one atomic per word and tile, a C2 reference's 60 tiles took 40-56 us
// whenever the reading side's voxel marks ran beside it, r04 trace: same-address atomics wait
// behind the marks' stores at the memory side.)
__global__ __launch_bounds__(256) void k_tr_sum(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd,
                                                const float4* __restrict__ raw, uint64_t* sums, uint64_t* part) {
  __shared__ uint64_t slo[3][4];
  __shared__ int64_t shi[3][4];
  const uint32_t base = blockIdx.x * kTile;
  const uint32_t last = min(base + kTile - 1, total - 1);
  const int p_first = pair_of_pos(pd, n_pairs, base), p_last = pair_of_pos(pd, n_pairs, last);
  const bool uniform = p_first == p_last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t alo[3] = {0, 0, 0};
  int64_t ahi[3] = {0, 0, 0};
  for (int j = 0; j < kTileItems; ++j) {
    const uint32_t i = base + (uint32_t)j * 256 + threadIdx.x;
    const bool ok = i < total;
    const int pair = ok ? (uniform ? p_first : pair_of_pos(pd, n_pairs, i)) : -1;
    const float4 p = ok ? raw[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float c[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int64_t q = ok ? fixed40(c[d]) : 0;
      uint64_t lo = (uint64_t)q;
      int64_t hi = q < 0 ? -1 : 0;
      if (uniform) {
        add128(alo[d], ahi[d], lo, hi);
        continue;
      }
      // pair boundary inside the tile: segmented wave scan, one atomic pair per run
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int ko = __shfl_up(pair, off, 64);
        const uint64_t lo_o = __shfl_up(lo, off, 64);
        const int64_t hi_o = __shfl_up(hi, off, 64);
        if (lane >= off && ko == pair) add128(lo, hi, lo_o, hi_o);
      }
      const int kn = __shfl_down(pair, 1, 64);
      if (ok && (lane == 63 || kn != pair)) atomic_add128(sums + (size_t)pair * 6 + 2 * d, lo, hi);
    }
  }
  if (!uniform) return;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    uint64_t lo = alo[d];
    int64_t hi = ahi[d];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t lo_o = __shfl_xor(lo, off, 64);
      const int64_t hi_o = __shfl_xor(hi, off, 64);
      add128(lo, hi, lo_o, hi_o);
    }
    if (lane == 0) {
      slo[d][w] = lo;
      shi[d][w] = hi;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int d = threadIdx.x;
    uint64_t lo = slo[d][0];
    int64_t hi = shi[d][0];
    for (int k = 1; k < 4; ++k) add128(lo, hi, slo[d][k], shi[d][k]);
    part[(size_t)blockIdx.x * 6 + 2 * d] = lo;
    part[(size_t)blockIdx.x * 6 + 2 * d + 1] = (uint64_t)hi;
  }
}

// mean, T_refIn_refMean, T_refMean_dataIn = T_refIn_refMean^-1 * T0 (A.1 steps 2, 5);
// center == 0: the kernel-level kNN entry points build on the points as given. One wave per
// pair: the atomic sums of the boundary tiles plus the partials of the pair's own tiles (integer
// sums: the order does not matter).
__global__ __launch_bounds__(64) void k_tr_frames(int n_pairs, uint32_t total, PairDesc* pd, const uint64_t* sums,
                                                  const uint64_t* part, int center) {
  const int p = blockIdx.x;
  if (p >= n_pairs) return;
  PairDesc& d = pd[p];
  float mean[3] = {0.f, 0.f, 0.f};
  if (center) {
    const uint32_t ro = d.ref_off, re = d.ref_off + d.n_ref;
    const uint32_t t0 = (ro + kTile - 1) / kTile;  // the first tile starting inside the pair
    uint64_t lo[3] = {0, 0, 0};
    int64_t hi[3] = {0, 0, 0};
    for (uint32_t t = t0 + (uint32_t)threadIdx.x; (uint64_t)t * kTile < re; t += 64) {
      if (min((uint64_t)t * kTile + kTile, (uint64_t)total) > re) break;  // straddles the pair's end
#pragma unroll
      for (int k = 0; k < 3; ++k) add128(lo[k], hi[k], part[(size_t)t * 6 + 2 * k], (int64_t)part[(size_t)t * 6 + 2 * k + 1]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const uint64_t lo_o = __shfl_xor(lo[k], off, 64);
        const int64_t hi_o = __shfl_xor(hi[k], off, 64);
        add128(lo[k], hi[k], lo_o, hi_o);
      }
      add128(lo[k], hi[k], sums[p * 6 + 2 * k], (int64_t)sums[p * 6 + 2 * k + 1]);
      mean[k] = mean_from_fixed40(lo[k], (uint64_t)hi[k], d.n_ref);
    }
  }
  if (threadIdx.x != 0) return;
  float Tm[16], Tmi[16];
  ident4(Tm);
  ident4(Tmi);
  for (int k = 0; k < 3; ++k) {
    d.mean[k] = mean[k];
    Tm[12 + k] = d.mean[k];
    Tmi[12 + k] = -d.mean[k];
  }
  for (int k = 0; k < 16; ++k) d.Tmean[k] = Tm[k];
  mul4(Tmi, d.Tin, d.Tinit);
}

// The build's zeroed work space in one launch (instead of a memset per buffer): up to 6 regions,
// 16-byte words (every region is 16-byte aligned and has room up to its next multiple of 16), and
// the root segment boxes set empty (min at the largest encoding, max at the smallest).
struct ZeroJob {
  uint4* p[6];
  uint64_t n16[6];
};
__global__ __launch_bounds__(256) void k_tr_zero(ZeroJob job, int n_pairs, TreeSeg* seg) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
#pragma unroll
  for (int r = 0; r < 6; ++r)
    for (uint64_t i = g; i < job.n16[r]; i += stride) job.p[r][i] = make_uint4(0u, 0u, 0u, 0u);
  for (uint64_t p = g; p < (uint64_t)n_pairs; p += stride)
    for (int k = 0; k < 3; ++k) {
      seg[p].bmn[k] = 0xffffffffu;
      seg[p].bmx[k] = 0u;
    }
}

// root segment boxes start empty: min at the largest encoding, max at the smallest
__global__ void k_tr_init_boxes(int n_pairs, TreeSeg* seg) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  for (int k = 0; k < 3; ++k) {
    seg[p].bmn[k] = 0xffffffffu;
    seg[p].bmx[k] = 0u;
  }
}

// centred reference (w = local input id) into W0 and the bounding box of each pair's
// centred points. Level-0 segment of every pair = its index; pairs small enough for the wave
// subtree builder (or a single leaf, whose points are then final) leave the global levels.
__global__ __launch_bounds__(256) void k_tr_center(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd,
                                                   const float4* __restrict__ raw, float4* __restrict__ W,
                                                   int32_t* __restrict__ segof, TreeSeg* seg,
                                                   float4* __restrict__ bpts, int bucket, uint32_t mid_max) {
  const uint32_t base = blockIdx.x * kTile;
  const uint32_t last = min(base + kTile - 1, total - 1);
  const int p_first = pair_of_pos(pd, n_pairs, base), p_last = pair_of_pos(pd, n_pairs, last);
  const bool uniform = p_first == p_last;
  float amn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float amx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int j = 0; j < kTileItems; ++j) {
    const uint32_t i = base + (uint32_t)j * 256 + threadIdx.x;
    const bool ok = i < total;
    const int pair = ok ? (uniform ? p_first : pair_of_pos(pd, n_pairs, i)) : -1;
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
      const PairDesc& d = pd[pair];
      const float4 p = raw[i];
      c = make_float4(p.x - d.mean[0], p.y - d.mean[1], p.z - d.mean[2], __int_as_float((int32_t)(i - d.ref_off)));
      W[i] = c;
      segof[i] = d.n_ref <= mid_max ? -1 : pair;
      if (d.n_ref <= (uint32_t)bucket) bpts[i] = c;
    }
    const float v[3] = {c.x, c.y, c.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float mn = ok ? v[k] : __builtin_inff(), mx = ok ? v[k] : -__builtin_inff();
      if (uniform) {
        amn[k] = fminf(amn[k], mn);
        amx[k] = fmaxf(amx[k], mx);
        continue;
      }
      const bool lastl = wave_seg_minmax(pair, mn, mx);
      if (ok && lastl) {
        atomicMin(&seg[pair].bmn[k], ord_enc(mn));
        atomicMax(&seg[pair].bmx[k], ord_enc(mx));
      }
    }
  }
  if (!uniform) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    block_minmax(amn[k], amx[k]);
    // a cloud spans many tiles: skip the atomic when the box already holds the bound (a stale
    // read only lets an unnecessary atomic through)
    if (threadIdx.x == 0) {
      const uint32_t emn = ord_enc(amn[k]), emx = ord_enc(amx[k]);
      if (emn < seg[p_first].bmn[k]) atomicMin(&seg[p_first].bmn[k], emn);
      if (emx > seg[p_first].bmx[k]) atomicMax(&seg[p_first].bmx[k], emx);
    }
  }
}

// Level-0 segments from the boxes. A pair with n_ref <= bucket is one leaf (its points are
// final); one with n_ref <= kSubMax goes straight to the subtree builders, one with
// n_ref <= kMidMax to the mid-size builder.
__global__ void k_tr_roots(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd, TreeSeg* seg,
                           SubSeg* subs, SubSeg* mids, TreeCtl* ctl, NodeEvent* ev, uint8_t* valid, uint32_t* ecnt,
                           int bucket, uint32_t mid_max) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  TreeSeg& s = seg[p];
  const PairDesc& d = pd[p];
  s.first = d.ref_off;
  s.count = d.n_ref;
  s.pair = p;
  s.depth = 0;
  s.parent_f = 0;
  s.parent_depth = -1;
  for (int k = 0; k < 3; ++k) {
    s.mn[k] = ord_dec(s.bmn[k]);
    s.mx[k] = ord_dec(s.bmx[k]);
  }
  split_dim(s.mn, s.mx, s.cd, s.ideal);
  // the points' extent along cd: the box is the points' own at the root (level 0 needs no
  // k_tr_minmax)
  s.lo = s.bmn[s.cd];
  s.hi = s.bmx[s.cd];
  if (d.n_ref <= mid_max) {
    if (d.n_ref <= (uint32_t)bucket) {
      emit_event(ev, valid, ecnt, total, leaf_event(d.ref_off, d.n_ref, 0, p, 0, -1));
    } else {
      const uint32_t si = atomicAdd(d.n_ref <= (uint32_t)kSubMax ? &ctl->n_small : &ctl->n_mid, 1u);
      SubSeg& g = (d.n_ref <= (uint32_t)kSubMax ? subs : mids)[si];
      g.f = d.ref_off;
      g.c = d.n_ref;
      g.pair = p;
      g.depth = 0;
      for (int k = 0; k < 3; ++k) {
        g.mn[k] = s.mn[k];
        g.mx[k] = s.mx[k];
      }
      g.parent_f = 0;
      g.parent_depth = -1;
    }
    s.count = 0;  // not split by the global levels
  }
  if (p == 0) ctl->nseg[0] = (uint32_t)n_pairs;
}

// ---- one global level ------------------------------------------------------------------------
// ---- one global level ------------------------------------------------------------------------
// X1 = exclusive scan of the pass-1 predicate (v < cut) over positions [0, total]
__global__ __launch_bounds__(kLbThreads) void k_tr_scan1(uint32_t total, const int32_t* __restrict__ segof,
                                                        const float4* __restrict__ W, const TreeSeg* __restrict__ seg,
                                                        uint32_t* __restrict__ X, uint64_t* st, TreeCtl* ctl) {
  lookback_scan(
      total + 1,
      [&](uint32_t i) -> uint32_t {
        if (i >= total) return 0u;
        const int s = segof[i];
        return (s >= 0 && coord(W[i], seg[s].cd) < seg_cut(seg[s])) ? 1u : 0u;
      },
      X, st, ctl);
}

// X = exclusive scan of c[0, n)
__global__ __launch_bounds__(kLbThreads) void k_tr_scan_counts(uint32_t n, const uint32_t* __restrict__ c,
                                                              uint32_t* __restrict__ X, uint64_t* st, TreeCtl* ctl) {
  lookback_scan(n, [&](uint32_t i) -> uint32_t { return c[i]; }, X, st, ctl);
}

// The partner of the element at local position li directly, without the position arrays: the
// k-th misplaced element from the left pairs with the k-th from the right, so the partner of a
// misplaced-left element is the (nmr - 1 - k)-th predicate element of [br, count) and the partner
// of a misplaced-right one the k-th non-predicate element of [lo_b, br); both are found by binary
// search over the monotone counts X (L2-resident) instead of a scatter kernel and a kernel
// boundary.
__device__ __forceinline__ uint32_t hoare_partner(uint32_t li, bool pred, uint32_t f, uint32_t lo_b, uint32_t br,
                                                  uint32_t count, const uint32_t* __restrict__ X) {
  if (li < br) {
    if (pred) return li;
    const uint32_t k = (li - lo_b) - (X[f + li] - X[f + lo_b]);
    const uint32_t xb = X[f + br], nmr = X[f + count] - xb;
    const uint32_t target = xb + (nmr - 1 - k);  // smallest q in (br, count] with X[f + q] > target
    uint32_t lo = br + 1, hi = count;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (X[f + mid] > target) hi = mid;
      else lo = mid + 1;
    }
    return lo - 1;
  }
  if (!pred) return li;
  const uint32_t xb = X[f + br];
  const uint32_t k = (X[f + count] - xb) - 1 - (X[f + li] - xb);
  const uint32_t x0 = X[f + lo_b];  // smallest q in (lo_b, br] with #non-predicate in [lo_b, q) > k
  uint32_t lo = lo_b + 1, hi = br;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((mid - lo_b) - (X[f + mid] - x0) > k) hi = mid;
    else lo = mid + 1;
  }
  return lo - 1;
}

// pass 1: move every element to its place, and write the pass-2 predicate at the new place
__global__ __launch_bounds__(256) void k_tr_move1(uint32_t total, const int32_t* __restrict__ segof,
                                                  const float4* __restrict__ W, TreeSeg* seg,
                                                  const uint32_t* __restrict__ X, float4* __restrict__ W1,
                                                  uint32_t* __restrict__ flag2) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > total) return;
  if (i == total) {
    flag2[i] = 0;
    return;
  }
  const int s = segof[i];
  if (s < 0) {
    flag2[i] = 0;
    return;
  }
  const TreeSeg& g = seg[s];
  const float4 p = W[i];
  const float v = coord(p, g.cd), cut = seg_cut(g);
  const uint32_t f = g.first, li = i - f;
  const uint32_t br1 = X[f + g.count] - X[f];
  uint32_t p1 = hoare_partner(li, v < cut, f, 0, br1, g.count, X);
  if (p1 >= g.count) p1 = li;  // unreachable for a consistent scan; keeps stores in range
  W1[f + p1] = p;
  flag2[f + p1] = (p1 >= br1 && v == cut) ? 1u : 0u;
  if (li == 0) seg[s].br1 = br1;
}

// split: left-count rule, node event of this segment, children: leaf events, subtree segments
// (count <= kSubMax), mid-size segments (<= kMidMax) or next-level segments
__device__ void tr_split_seg(uint32_t si, int level, int last, uint32_t total, TreeSeg* seg, TreeSeg* next,
                             SubSeg* subs, SubSeg* mids, TreeCtl* ctl, const uint32_t* __restrict__ X2,
                             NodeEvent* ev, uint8_t* valid, uint32_t* ecnt, int32_t* pair_depth, int bucket,
                             uint32_t max_seg, uint32_t mid_max) {
  TreeSeg& g = seg[si];
  if (g.count == 0) return;  // root handled elsewhere
  const uint32_t f = g.first, count = g.count;
  const float lo = ord_dec(g.lo), hi = ord_dec(g.hi);
  const float cut = seg_cut(g);
  const uint32_t br1 = g.br1, br2 = br1 + (X2[f + count] - X2[f]);
  uint32_t left;
  if (g.ideal < lo) left = 1;
  else if (g.ideal > hi) left = count - 1;
  else if (br1 > count / 2) left = br1;
  else if (br2 < count / 2) left = br2;
  else left = count / 2;
  g.br2 = br2;
  g.left = left;
  NodeEvent e{};
  e.f = f;
  e.c = count;
  e.depth = g.depth;
  e.pair = g.pair;
  e.cut_bits = __float_as_uint(cut);
  e.cd = g.cd;
  e.left = left;
  e.parent_f = g.parent_f;
  e.parent_depth = g.parent_depth;
  emit_event(ev, valid, ecnt, total, e);
  const int cdepth = g.depth + 1;
  if (pair_depth[g.pair] < cdepth) atomicMax(&pair_depth[g.pair], cdepth);
  for (int side = 0; side < 2; ++side) {
    const uint32_t cf = side ? f + left : f, cc = side ? count - left : left;
    float mn[3], mx[3];
    for (int k = 0; k < 3; ++k) {
      mn[k] = g.mn[k];
      mx[k] = g.mx[k];
    }
    if (side) mn[g.cd] = cut;
    else mx[g.cd] = cut;
    if (cc <= (uint32_t)bucket) {
      emit_event(ev, valid, ecnt, total, leaf_event(cf, cc, cdepth, g.pair, f, g.depth));
      g.child[side] = -1;
      continue;
    }
    if (cc <= mid_max || last) {  // last planned level: oversized ones too (global path)
      const bool mid = cc > (uint32_t)kSubMax && cc <= mid_max;
      if (cc > mid_max) atomicAdd(&ctl->n_big, 1u);
      const uint32_t ni = atomicAdd(mid ? &ctl->n_mid : &ctl->n_small, 1u);
      if (ni >= max_seg) {
        atomicOr(&ctl->error, 4);
        g.child[side] = -1;
        continue;
      }
      SubSeg& c = (mid ? mids : subs)[ni];
      c.f = cf;
      c.c = cc;
      c.pair = g.pair;
      c.depth = cdepth;
      for (int k = 0; k < 3; ++k) {
        c.mn[k] = mn[k];
        c.mx[k] = mx[k];
      }
      c.parent_f = f;
      c.parent_depth = g.depth;
      g.child[side] = -2;
      continue;
    }
    const uint32_t ni = atomicAdd(&ctl->nseg[level + 1], 1u);
    if (ni >= max_seg) {
      atomicOr(&ctl->error, 4);
      g.child[side] = -1;
      continue;
    }
    TreeSeg& c = next[ni];
    c.first = cf;
    c.count = cc;
    c.pair = g.pair;
    c.depth = cdepth;
    c.parent_f = f;
    c.parent_depth = g.depth;
    for (int k = 0; k < 3; ++k) {
      c.mn[k] = mn[k];
      c.mx[k] = mx[k];
    }
    split_dim(c.mn, c.mx, c.cd, c.ideal);
    c.lo = 0xffffffffu;
    c.hi = 0u;
    g.child[side] = (int32_t)ni;
  }
}

__global__ __launch_bounds__(256) void k_tr_split(int level, int last, uint32_t total, TreeSeg* seg, TreeSeg* next,
                                                  SubSeg* subs, SubSeg* mids, TreeCtl* ctl, const uint32_t* __restrict__ X2,
                                                  NodeEvent* ev, uint8_t* valid, uint32_t* ecnt,
                                                  int32_t* pair_depth, int bucket, uint32_t max_seg,
                                                  uint32_t mid_max) {
  const uint32_t si = blockIdx.x * blockDim.x + threadIdx.x;
  if (si >= ctl->nseg[level]) return;
  tr_split_seg(si, level, last, total, seg, next, subs, mids, ctl, X2, ev, valid, ecnt, pair_depth, bucket, max_seg,
               mid_max);
}

// The next level's segment boxes along their split dimensions (a min/max pass at the start of a
// level otherwise), folded into the move that assigns the points to those segments: each wave
// reduces per next-level segment (ballot over the lanes with the same key), the workgroup merges
// its few keys in LDS, and one atomic per key and workgroup goes to the segment.
constexpr int kMmKeys = 8;
__device__ __forceinline__ void move2_minmax(bool has, int key, float v, TreeSeg* next) {
  __shared__ int mk[kMmKeys];
  __shared__ uint32_t mlo[kMmKeys], mhi[kMmKeys];
  const int t = threadIdx.x, lane = t & 63;
  if (t < kMmKeys) {
    mk[t] = -1;
    mlo[t] = 0xffffffffu;
    mhi[t] = 0u;
  }
  __syncthreads();
  uint64_t act = __ballot(has);
  while (act) {
    const int leader = __ffsll((long long)act) - 1;
    const int k = __shfl(key, leader, 64);
    const bool m = has && key == k;
    const uint64_t mm = __ballot(m);
    uint32_t e = m ? ord_enc(v) : 0xffffffffu, f = m ? ord_enc(v) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      e = min(e, (uint32_t)__shfl_xor((int)e, o, 64));
      f = max(f, (uint32_t)__shfl_xor((int)f, o, 64));
    }
    if (lane == 0) {
      int slot = -1;
      for (int q = 0; q < kMmKeys && slot < 0; ++q) {
        const int old = atomicCAS(&mk[q], -1, k);
        if (old == -1 || old == k) slot = q;
      }
      if (slot >= 0) {
        atomicMin(&mlo[slot], e);
        atomicMax(&mhi[slot], f);
      } else {  // more keys than slots (not expected: a workgroup spans at most two parents)
        atomicMin(&next[k].lo, e);
        atomicMax(&next[k].hi, f);
      }
    }
    act &= ~mm;
  }
  __syncthreads();
  if (t < kMmKeys && mk[t] >= 0) {
    atomicMin(&next[mk[t]].lo, mlo[t]);
    atomicMax(&next[mk[t]].hi, mhi[t]);
  }
}

// pass 2 move; next level's segment map; points landing in leaves are final (bucket order);
// also the next level's segment boxes (move2_minmax)
__global__ __launch_bounds__(256) void k_tr_move2(uint32_t total, const int32_t* __restrict__ segof,
                                                  const float4* __restrict__ W1, const TreeSeg* __restrict__ seg,
                                                  const uint32_t* __restrict__ X2, float4* __restrict__ W2,
                                                  int32_t* __restrict__ segof_next, float4* __restrict__ bpts,
                                                  TreeSeg* next) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = i < total ? segof[i] : -1;
  bool has = false;  // the point lands in a next-level segment (key, coordinate mv)
  int key = -1;
  float mv = 0.f;
  if (s < 0) {
    if (i < total) segof_next[i] = -1;
  } else {
    const TreeSeg& g = seg[s];
    const float4 p = W1[i];
    const float v = coord(p, g.cd), cut = seg_cut(g);
    const uint32_t f = g.first, li = i - f;
    uint32_t p2 = li;
    if (li >= g.br1) {
      p2 = hoare_partner(li, v == cut, f, g.br1, g.br2, g.count, X2);
      if (p2 >= g.count) p2 = li;  // unreachable for a consistent scan; keeps stores in range
    }
    const uint32_t q = f + p2;
    W2[q] = p;
    const int32_t child = g.child[p2 < g.left ? 0 : 1];
    segof_next[q] = child >= 0 ? child : -1;
    if (child == -1) bpts[q] = p;  // leaf: final; -2: the wave subtree builder takes it from W
    if (child >= 0) {
      has = true;
      key = child;
      mv = coord(p, next[child].cd);
    }
  }
  move2_minmax(has, key, mv, next);  // every thread of the workgroup, once
}

// ---- wave subtree builder ----------------------------------------------------------------------
// One wave finishes the whole subtree of a segment of <= kSubMax points in LDS, depth first,
// with the same node rule; the Hoare passes use ballot/popcount ranks and swap each
// misplaced pair in place (the pairs are disjoint). All control flow is wave-uniform.
struct SubNode {
  uint32_t lf, lc;  // local first / count
  int32_t depth;
  float mn[3], mx[3];
  uint32_t pf;      // parent first (global)
  int32_t pdepth;
};

__device__ __forceinline__ uint32_t popc_lt(uint64_t m) {
  const int lane = threadIdx.x & 63;
  return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v) {
  return wave_reduce_dpp(v, [](uint32_t a, uint32_t b) { return a + b; });
}

// one Hoare pass over local [lo_b, end) with boundary br: elements with pred in [lo_b, br)
template <class PosT, class Pred>
__device__ __forceinline__ void wave_hoare(float4* pts, PosT* posA, PosT* posB, uint32_t lo_b, uint32_t br,
                                           uint32_t end, Pred pred) {
  const int lane = threadIdx.x & 63;
  uint32_t ra = 0, rb = 0;
  for (uint32_t jb = lo_b; jb < end; jb += 64) {
    const uint32_t j = jb + lane;
    const bool ok = j < end;
    const bool pr = ok && pred(pts[j]);
    const bool ml = ok && j < br && !pr, mr = ok && j >= br && pr;
    const uint64_t ma = __ballot(ml), mb = __ballot(mr);
    if (ml) posA[ra + popc_lt(ma)] = (PosT)j;
    if (mr) posB[rb + popc_lt(mb)] = (PosT)j;
    ra += (uint32_t)__popcll(ma);
    rb += (uint32_t)__popcll(mb);
  }
  __syncthreads();
  // the k-th misplaced element from the left swaps with the k-th misplaced from the right
  for (uint32_t k = lane; k < ra; k += 64) {
    const uint32_t a = posA[k], b = posB[rb - 1 - k];
    const float4 t = pts[a];
    pts[a] = pts[b];
    pts[b] = t;
  }
  __syncthreads();
}

// One segment's whole subtree, depth first, by one wave. pts = the segment's points (LDS copy,
// or the segment's range of bpts in place for an oversized segment), posA / posB = partition
// scratch of the segment's size (LDS, or the free per-level position arrays).
template <class PosT>
__device__ void subtree_build(const SubSeg& g, uint32_t total, float4* pts, PosT* posA, PosT* posB, SubNode* stk,
                              NodeEvent* ev, uint8_t* valid, uint32_t* ecnt, int32_t* pair_depth, int bucket) {
  const int lane = threadIdx.x;
  const uint32_t gf = g.f;
  SubNode nd;
  nd.lf = 0;
  nd.lc = g.c;
  nd.depth = g.depth;
  for (int k = 0; k < 3; ++k) {
    nd.mn[k] = g.mn[k];
    nd.mx[k] = g.mx[k];
  }
  nd.pf = g.parent_f;
  nd.pdepth = g.parent_depth;
  int sp = 0;
  int maxd = g.depth;
  for (;;) {
    if (nd.lc <= (uint32_t)bucket) {
      if (lane == 0) emit_event(ev, valid, ecnt, total, leaf_event(gf + nd.lf, nd.lc, nd.depth, g.pair, nd.pf, nd.pdepth));
      if (sp == 0) break;
      nd = stk[--sp];
      continue;
    }
    int cd;
    float ideal;
    split_dim(nd.mn, nd.mx, cd, ideal);
    const uint32_t a0 = nd.lf, end = nd.lf + nd.lc;
    float mn = __builtin_inff(), mx = -__builtin_inff();
    for (uint32_t j = a0 + lane; j < end; j += 64) {
      const float v = coord(pts[j], cd);
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
    const float lo = wave_min(mn), hi = wave_max(mx);
    const float cut = ideal < lo ? lo : (ideal > hi ? hi : ideal);
    uint32_t nl = 0, ne = 0;
    for (uint32_t j = a0 + lane; j < end; j += 64) {
      const float v = coord(pts[j], cd);
      nl += v < cut ? 1u : 0u;
      ne += v == cut ? 1u : 0u;
    }
    nl = wave_sum_u(nl);
    ne = wave_sum_u(ne);
    const uint32_t br1 = nl, br2 = nl + ne, count = nd.lc;
    wave_hoare(pts, posA, posB, a0, a0 + br1, end, [&](const float4& p) { return coord(p, cd) < cut; });
    if (ne) wave_hoare(pts, posA, posB, a0 + br1, a0 + br2, end, [&](const float4& p) { return coord(p, cd) == cut; });
    uint32_t left;
    if (ideal < lo) left = 1;
    else if (ideal > hi) left = count - 1;
    else if (br1 > count / 2) left = br1;
    else if (br2 < count / 2) left = br2;
    else left = count / 2;
    if (lane == 0) {
      NodeEvent e{};
      e.f = gf + nd.lf;
      e.c = count;
      e.depth = nd.depth;
      e.pair = g.pair;
      e.cut_bits = __float_as_uint(cut);
      e.cd = cd;
      e.left = left;
      e.parent_f = nd.pf;
      e.parent_depth = nd.pdepth;
      emit_event(ev, valid, ecnt, total, e);
    }
    SubNode L, R;
    L.lf = nd.lf;
    L.lc = left;
    R.lf = nd.lf + left;
    R.lc = count - left;
    L.depth = R.depth = nd.depth + 1;
    L.pf = R.pf = gf + nd.lf;
    L.pdepth = R.pdepth = nd.depth;
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // selects, not a dynamic store (keeps the node in registers)
      L.mn[k] = nd.mn[k];
      R.mx[k] = nd.mx[k];
      L.mx[k] = k == cd ? cut : nd.mx[k];
      R.mn[k] = k == cd ? cut : nd.mn[k];
    }
    if (L.depth > maxd) maxd = L.depth;
    if (sp >= kFarStack) break;  // deeper than the device stack: k_tr_emit reports it
    if (lane == 0) stk[sp] = R;
    ++sp;
    __syncthreads();
    nd = L;
  }
  __syncthreads();
  if (lane == 0 && pair_depth[g.pair] < maxd) atomicMax(&pair_depth[g.pair], maxd);
}

// ---- block subtree builder: the same nodes, level by level, one node per wave -----------------
// A segment's subtree has ~(count / bucket) nodes but only ~log2(count / bucket) levels: the
// waves of a block take the nodes of one level each (a node is still split by one wave with the
// same Hoare passes, so the swaps and the resulting order are the wave builder's), and a block
// barrier separates the levels. Far fewer dependent steps per segment than depth-first by one wave.
// waves per block, one node each per level. r04 kept 8 because 16 cost C5 13 %; builds of C5's
// size now finish with k_tr_subtree_lvl (TreeWork::lvl_min), so only the small builds (C2's
// references) run this kernel, and 16 waves take it from 72 to 59 us there (r06, same box, C3 /
// C4 / C5 unchanged; profiles/r06_log.md)
#ifndef AICP_SUBWAVES
#define AICP_SUBWAVES 16
#endif
constexpr int kSubWaves = AICP_SUBWAVES;
constexpr int kSubLevelCap = 256;  // nodes above bucket per level (<= kSubMax / (bucket + 1))

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// wave_hoare with wave-local synchronisation (the other waves of the block work on other nodes)
__device__ __forceinline__ void wave_hoare_w(float4* pts, uint16_t* posA, uint16_t* posB, uint32_t lo_b, uint32_t br,
                                             uint32_t end, int cd, float cut, bool eq) {
  const int lane = threadIdx.x & 63;
  uint32_t ra = 0, rb = 0;
  for (uint32_t jb = lo_b; jb < end; jb += 64) {
    const uint32_t j = jb + lane;
    const bool ok = j < end;
    bool pr = false;
    if (ok) {
      const float v = coord(pts[j], cd);
      pr = eq ? (v == cut) : (v < cut);
    }
    const bool ml = ok && j < br && !pr, mr = ok && j >= br && pr;
    const uint64_t ma = __ballot(ml), mb = __ballot(mr);
    if (ml) posA[ra + popc_lt(ma)] = (uint16_t)j;
    if (mr) posB[rb + popc_lt(mb)] = (uint16_t)j;
    ra += (uint32_t)__popcll(ma);
    rb += (uint32_t)__popcll(mb);
  }
  wave_sync_lds();
  for (uint32_t k = lane; k < ra; k += 64) {
    const uint32_t a = posA[k], b = posB[rb - 1 - k];
    const float4 t = pts[a];
    pts[a] = pts[b];
    pts[b] = t;
  }
  wave_sync_lds();
}

__global__ __launch_bounds__(64 * kSubWaves) void k_tr_subtree_blk(uint32_t total, const TreeCtl* __restrict__ ctl,
                                                                   const SubSeg* __restrict__ subs,
                                                                   const float4* __restrict__ W,
                                                                   float4* __restrict__ bpts, NodeEvent* ev,
                                                                   uint8_t* valid, uint32_t* ecnt,
                                                                   int32_t* pair_depth, int bucket) {
  __shared__ float4 pts[kSubMax];
  __shared__ uint16_t posA[kSubWaves][kSubMax / 2], posB[kSubWaves][kSubMax / 2];
  __shared__ SubNode lvl[2][kSubLevelCap];
  __shared__ uint32_t n_lvl[2];
  __shared__ int32_t maxd;
  const uint32_t n_small = ctl->n_small;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t si = blockIdx.x; si < n_small; si += gridDim.x) {
    __syncthreads();  // the previous segment's last LDS reads precede this one's loads
    const SubSeg g = subs[si];
    if (g.c > (uint32_t)kSubMax) continue;  // oversized: k_tr_subtree's global path
    const uint32_t gf = g.f;
    for (uint32_t j = threadIdx.x; j < g.c; j += blockDim.x) pts[j] = W[gf + j];
    if (threadIdx.x == 0) {
      SubNode& r = lvl[0][0];
      r.lf = 0;
      r.lc = g.c;
      r.depth = g.depth;
      for (int k = 0; k < 3; ++k) {
        r.mn[k] = g.mn[k];
        r.mx[k] = g.mx[k];
      }
      r.pf = g.parent_f;
      r.pdepth = g.parent_depth;
      n_lvl[0] = 1;
      n_lvl[1] = 0;
      maxd = g.depth;
    }
    __syncthreads();
    int cur = 0;
    for (;;) {
      const uint32_t n = n_lvl[cur];
      if (n == 0) break;
      for (uint32_t i = wv; i < n; i += kSubWaves) {
        const SubNode nd = lvl[cur][i];  // count > bucket (leaves are emitted when created)
        int cd;
        float ideal;
        split_dim(nd.mn, nd.mx, cd, ideal);
        const uint32_t a0 = nd.lf, end = nd.lf + nd.lc;
        float mn = __builtin_inff(), mx = -__builtin_inff();
        for (uint32_t j = a0 + lane; j < end; j += 64) {
          const float v = coord(pts[j], cd);
          mn = fminf(mn, v);
          mx = fmaxf(mx, v);
        }
        const float lo = wave_min(mn), hi = wave_max(mx);
        const float cut = ideal < lo ? lo : (ideal > hi ? hi : ideal);
        uint32_t nl = 0, ne = 0;
        for (uint32_t j = a0 + lane; j < end; j += 64) {
          const float v = coord(pts[j], cd);
          nl += v < cut ? 1u : 0u;
          ne += v == cut ? 1u : 0u;
        }
        nl = wave_sum_u(nl);
        ne = wave_sum_u(ne);
        const uint32_t br1 = nl, br2 = nl + ne, count = nd.lc;
        wave_hoare_w(pts, posA[wv], posB[wv], a0, a0 + br1, end, cd, cut, false);
        if (ne) wave_hoare_w(pts, posA[wv], posB[wv], a0 + br1, a0 + br2, end, cd, cut, true);
        uint32_t left;
        if (ideal < lo) left = 1;
        else if (ideal > hi) left = count - 1;
        else if (br1 > count / 2) left = br1;
        else if (br2 < count / 2) left = br2;
        else left = count / 2;
        if (lane == 0) {
          NodeEvent e{};
          e.f = gf + nd.lf;
          e.c = count;
          e.depth = nd.depth;
          e.pair = g.pair;
          e.cut_bits = __float_as_uint(cut);
          e.cd = cd;
          e.left = left;
          e.parent_f = nd.pf;
          e.parent_depth = nd.pdepth;
          emit_event(ev, valid, ecnt, total, e);
          atomicMax(&maxd, nd.depth + 1);
          for (int side = 0; side < 2; ++side) {
            SubNode c;
            c.lf = side ? nd.lf + left : nd.lf;
            c.lc = side ? count - left : left;
            c.depth = nd.depth + 1;
            c.pf = gf + nd.lf;
            c.pdepth = nd.depth;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              c.mn[k] = (side && k == cd) ? cut : nd.mn[k];
              c.mx[k] = (!side && k == cd) ? cut : nd.mx[k];
            }
            if (c.lc <= (uint32_t)bucket) {
              emit_event(ev, valid, ecnt, total, leaf_event(gf + c.lf, c.lc, c.depth, g.pair, c.pf, c.pdepth));
            } else {
              const uint32_t q = atomicAdd(&n_lvl[cur ^ 1], 1u);
              if (q < (uint32_t)kSubLevelCap) lvl[cur ^ 1][q] = c;
            }
          }
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        n_lvl[cur] = 0;
        if (n_lvl[cur ^ 1] > (uint32_t)kSubLevelCap) n_lvl[cur ^ 1] = kSubLevelCap;  // (bucket >= 4: never)
      }
      __syncthreads();
      cur ^= 1;
    }
    for (uint32_t j = threadIdx.x; j < g.c; j += blockDim.x) bpts[gf + j] = pts[j];
    if (threadIdx.x == 0 && pair_depth[g.pair] < maxd) atomicMax(&pair_depth[g.pair], maxd);
  }
}

// ---- level-synchronous subtree builder: every node of a level at once --------------------------
// The block builder above gives each node of a level to one wave, and its per-node work (box,
// events, children: lane 0 of a wave, wave-wide) dominated at scale: on C5 (1024 pairs, ~100k
// segments) k_tr_subtree_blk ran ~50 VALU + 28 SALU wave instructions per point (PMC, r04). Here
// one workgroup runs a segment's levels in lockstep: the point passes (min/max of the cut
// dimension, the two partition counts, the Hoare passes) go over all positions of the segment
// with wave-segmented reductions per node, and the per-node steps (cut dimension, left count,
// events, children) run one node per thread. The node rule, the Hoare pairing (the k-th
// misplaced element from the left of a node swaps with the k-th from its right, ranks from one
// block-wide scan of the two flags) and so the tree and the point order are the other
// builders'. Needs bucket >= 8 (a level of <= kSubMax points has <= kLvlCap nodes above it).
constexpr int kLvlThreads = 512;
constexpr int kLvlPer = kSubMax / kLvlThreads;
constexpr int kLvlCap = 128;
static_assert(kSubMax % kLvlThreads == 0 && kSubMax <= 65535, "positions fit 16 bits");

struct LvlNodes {  // one level's nodes (SoA in LDS): local first / count, box, parent first
  uint16_t f[kLvlCap], c[kLvlCap];
  float mn[3][kLvlCap], mx[3][kLvlCap];
  uint32_t pf[kLvlCap];
};

// inclusive segmented sum over the wave's lanes for runs of equal key (contiguous runs); true on
// the last lane of a run, which then holds the run's total
__device__ __forceinline__ bool wave_seg_sum(int key, uint32_t& v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int ko = __shfl_up(key, off, 64);
    const uint32_t a = __shfl_up(v, off, 64);
    if (lane >= off && ko == key) v += a;
  }
  const int kn = __shfl_down(key, 1, 64);
  return lane == 63 || kn != key;
}

// exclusive scan of the packed flags fl[u] (position u * kLvlThreads + t) over all positions of
// the segment into X, and X[n] = the total
__device__ __forceinline__ void lvl_scan(const uint32_t* fl, uint32_t* X, uint32_t (*wtot)[kLvlThreads / 64],
                                         uint32_t n) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t inc[kLvlPer];
#pragma unroll
  for (int u = 0; u < kLvlPer; ++u) {
    uint32_t x = fl[u];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    inc[u] = x;
    if (lane == 63) wtot[u][wv] = x;
  }
  __syncthreads();
  uint32_t base = 0;
#pragma unroll
  for (int u = 0; u < kLvlPer; ++u) {
    uint32_t b = base;
#pragma unroll
    for (int w = 0; w < kLvlThreads / 64; ++w) {
      if (w < wv) b += wtot[u][w];
      base += wtot[u][w];
    }
    const uint32_t p = (uint32_t)(u * kLvlThreads + t);
    if (p < n) X[p] = b + inc[u] - fl[u];
  }
  if (t == 0) X[n] = base;
}

#if AICP_ITER_PROF
// diagnostic builds: k_tr_subtree_lvl's phases summed over segments (thread 0, s_memrealtime
// ticks at 100 MHz): [0] load, [1] min/max, [2] counts, [3] Hoare passes, [4] nodes + events,
// [5] child map, [6] store, [7] levels, [8] segments, [9] points, [10] slowest segment
__device__ unsigned long long g_lvl_prof[12];
#define AICP_LP(k)                                                  \
  do {                                                              \
    if (threadIdx.x == 0) {                                         \
      const uint64_t now_ = __builtin_amdgcn_s_memrealtime();       \
      lp[k] += now_ - lp_t;                                         \
      lp_t = now_;                                                  \
    }                                                               \
  } while (0)
#else
#define AICP_LP(k) \
  do {             \
  } while (0)
#endif
__global__ __launch_bounds__(kLvlThreads, 8) void k_tr_subtree_lvl(uint32_t total, const TreeCtl* __restrict__ ctl,
                                                                const SubSeg* __restrict__ subs,
                                                                const float4* __restrict__ W, float4* __restrict__ bpts,
                                                                NodeEvent* ev, uint8_t* valid, uint32_t* ecnt,
                                                                int32_t* pair_depth, int bucket) {
  __shared__ float4 pts[kSubMax];
  __shared__ uint16_t nid[kSubMax];   // node (index in the level) of each position, 0xFFFF: done
  __shared__ uint16_t posB[kSubMax];  // misplaced-right positions of a pass, at node first + rank
  __shared__ uint32_t X[kSubMax + 1];
  __shared__ LvlNodes lv[2];
  __shared__ uint8_t ncd[kLvlCap];
  __shared__ float nideal[kLvlCap];
  __shared__ uint32_t nlo[kLvlCap], nhi[kLvlCap], ncnt[kLvlCap];  // ordered-int min / max; nl | ne << 16
  __shared__ uint16_t nleft[kLvlCap], nch[2][kLvlCap];
  __shared__ uint32_t wtot[kLvlPer][kLvlThreads / 64];
  __shared__ uint32_t n_next, any_eq;
  const int t = threadIdx.x;
  const uint32_t n_small = ctl->n_small;
#if AICP_ITER_PROF
  uint64_t lp[12] = {}, lp_t = __builtin_amdgcn_s_memrealtime(), lp_seg0 = 0;
#endif
  for (uint32_t si = blockIdx.x; si < n_small; si += gridDim.x) {
    __syncthreads();  // the previous segment's last LDS reads precede this one's loads
    const SubSeg g = subs[si];
    if (g.c > (uint32_t)kSubMax) continue;  // oversized: k_tr_subtree's global path
    const uint32_t gf = g.f, n = g.c;
#if AICP_ITER_PROF
    if (t == 0) {
      lp_t = lp_seg0 = __builtin_amdgcn_s_memrealtime();
      lp[8] += 1;
      lp[9] += n;
    }
#endif
    for (uint32_t j = t; j < n; j += kLvlThreads) {
      pts[j] = W[gf + j];
      nid[j] = 0;
    }
    if (t == 0) {
      lv[0].f[0] = 0;
      lv[0].c[0] = (uint16_t)n;
      for (int k = 0; k < 3; ++k) {
        lv[0].mn[k][0] = g.mn[k];
        lv[0].mx[k][0] = g.mx[k];
      }
      lv[0].pf[0] = g.parent_f;
    }
    int cur = 0;
    uint32_t nn = 1;  // nodes of the level (each above the bucket: leaves are emitted when created)
    int depth = g.depth, maxd = g.depth;
    for (;;) {
      LvlNodes& N = lv[cur];
      LvlNodes& M = lv[cur ^ 1];
      if ((uint32_t)t < nn) {
        float mn[3], mx[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          mn[k] = N.mn[k][t];
          mx[k] = N.mx[k][t];
        }
        int cd;
        float ideal;
        split_dim(mn, mx, cd, ideal);
        ncd[t] = (uint8_t)cd;
        nideal[t] = ideal;
        nlo[t] = 0xFFFFFFFFu;
        nhi[t] = 0u;
        ncnt[t] = 0u;
      }
      if (t == 0) {
        n_next = 0;
        any_eq = 0;
      }
      __syncthreads();
      AICP_LP(0);
      // the cut dimension's min / max per node
      int key[kLvlPer];
      float v[kLvlPer];
#pragma unroll
      for (int u = 0; u < kLvlPer; ++u) {
        const uint32_t p = (uint32_t)(u * kLvlThreads + t);
        const uint32_t i = p < n ? nid[p] : 0xFFFFu;
        key[u] = i == 0xFFFFu ? -1 : (int)i;
        v[u] = key[u] >= 0 ? coord(pts[p], ncd[i]) : 0.f;
        float a = key[u] >= 0 ? v[u] : __builtin_inff(), b = key[u] >= 0 ? v[u] : -__builtin_inff();
        if (wave_seg_minmax(key[u], a, b) && key[u] >= 0) {
          atomicMin(&nlo[key[u]], ord_enc(a));
          atomicMax(&nhi[key[u]], ord_enc(b));
        }
      }
      __syncthreads();
      AICP_LP(1);
      // the partition counts (v < cut, v == cut) per node
      float cut[kLvlPer];
#pragma unroll
      for (int u = 0; u < kLvlPer; ++u) {
        uint32_t x = 0;
        cut[u] = 0.f;
        if (key[u] >= 0) {
          const float lo = ord_dec(nlo[key[u]]), hi = ord_dec(nhi[key[u]]), id = nideal[key[u]];
          cut[u] = id < lo ? lo : (id > hi ? hi : id);
          x = v[u] < cut[u] ? 1u : (v[u] == cut[u] ? 0x10000u : 0u);
        }
        if (wave_seg_sum(key[u], x) && key[u] >= 0 && x) {
          atomicAdd(&ncnt[key[u]], x);
          if (x >> 16) any_eq = 1;
        }
      }
      __syncthreads();
      AICP_LP(2);
      // Hoare pass 1 over each node on (v < cut) with boundary nl, then (if a node has ties)
      // pass 2 over [nl, count) on (v == cut) with boundary nl + ne
      for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1 && !any_eq) break;
        uint32_t fl[kLvlPer];
#pragma unroll
        for (int u = 0; u < kLvlPer; ++u) {
          fl[u] = 0;
          const uint32_t p = (uint32_t)(u * kLvlThreads + t);
          if (key[u] >= 0) {
            const int i = key[u];
            const uint32_t loc = p - N.f[i], nl = ncnt[i] & 0xFFFFu, ne = ncnt[i] >> 16;
            if (pass == 1) v[u] = coord(pts[p], ncd[i]);  // (moved by pass 1)
            const bool pr = pass == 0 ? v[u] < cut[u] : v[u] == cut[u];
            const uint32_t lo_b = pass == 0 ? 0u : nl, br = pass == 0 ? nl : nl + ne;
            if (loc >= lo_b) fl[u] = (loc < br && !pr) ? 1u : ((loc >= br && pr) ? 0x10000u : 0u);
          }
        }
        lvl_scan(fl, X, wtot, n);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kLvlPer; ++u)
          if (fl[u] >> 16) {
            const uint32_t p = (uint32_t)(u * kLvlThreads + t), f0 = N.f[key[u]];
            posB[f0 + ((X[p] - X[f0]) >> 16)] = (uint16_t)p;
          }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kLvlPer; ++u)
          if (fl[u] & 0xFFFFu) {
            const uint32_t p = (uint32_t)(u * kLvlThreads + t), f0 = N.f[key[u]];
            const uint32_t k = (X[p] - X[f0]) & 0xFFFFu;
            const uint32_t rb = (X[f0 + N.c[key[u]]] - X[f0]) >> 16;
            const uint32_t b = posB[f0 + rb - 1 - k];
            const float4 a4 = pts[p];
            pts[p] = pts[b];
            pts[b] = a4;
          }
        __syncthreads();
      }
      AICP_LP(3);
      // per node: the left count, its event, the children (leaf events or next-level nodes)
      if ((uint32_t)t < nn) {
        const uint32_t count = N.c[t], nl = ncnt[t] & 0xFFFFu, ne = ncnt[t] >> 16;
        const float lo = ord_dec(nlo[t]), hi = ord_dec(nhi[t]), ideal = nideal[t];
        const float ct = ideal < lo ? lo : (ideal > hi ? hi : ideal);
        const int cd = ncd[t];
        const uint32_t br1 = nl, br2 = nl + ne;
        uint32_t left;
        if (ideal < lo) left = 1;
        else if (ideal > hi) left = count - 1;
        else if (br1 > count / 2) left = br1;
        else if (br2 < count / 2) left = br2;
        else left = count / 2;
        nleft[t] = (uint16_t)left;
        const uint32_t f0 = N.f[t];
        const int pdepth = depth == g.depth ? g.parent_depth : depth - 1;
        NodeEvent e{};
        e.f = gf + f0;
        e.c = count;
        e.depth = depth;
        e.pair = g.pair;
        e.cut_bits = __float_as_uint(ct);
        e.cd = cd;
        e.left = left;
        e.parent_f = N.pf[t];
        e.parent_depth = pdepth;
        emit_event(ev, valid, ecnt, total, e);
        for (int side = 0; side < 2; ++side) {
          const uint32_t cf = side ? f0 + left : f0, cc = side ? count - left : left;
          if (cc <= (uint32_t)bucket) {
            emit_event(ev, valid, ecnt, total, leaf_event(gf + cf, cc, depth + 1, g.pair, gf + f0, depth));
            nch[side][t] = 0xFFFFu;
          } else {
            const uint32_t q = atomicAdd(&n_next, 1u);
            M.f[q] = (uint16_t)cf;
            M.c[q] = (uint16_t)cc;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              M.mn[k][q] = (side && k == cd) ? ct : N.mn[k][t];
              M.mx[k][q] = (!side && k == cd) ? ct : N.mx[k][t];
            }
            M.pf[q] = gf + f0;
            nch[side][t] = (uint16_t)q;
          }
        }
      }
      __syncthreads();
      AICP_LP(4);
      // positions to their child nodes
#pragma unroll
      for (int u = 0; u < kLvlPer; ++u)
        if (key[u] >= 0) {
          const uint32_t p = (uint32_t)(u * kLvlThreads + t);
          nid[p] = nch[(p - N.f[key[u]]) < nleft[key[u]] ? 0 : 1][key[u]];
        }
      maxd = depth + 1;
      nn = n_next;
      __syncthreads();
      AICP_LP(5);
#if AICP_ITER_PROF
      if (t == 0) lp[7] += 1;
#endif
      if (nn == 0) break;
      cur ^= 1;
      ++depth;
    }
    for (uint32_t j = t; j < n; j += kLvlThreads) bpts[gf + j] = pts[j];
    if (t == 0 && pair_depth[g.pair] < maxd) atomicMax(&pair_depth[g.pair], maxd);
#if AICP_ITER_PROF
    AICP_LP(6);
    if (t == 0) lp[10] = max(lp[10], (unsigned long long)(lp_t - lp_seg0));
#endif
  }
#if AICP_ITER_PROF
  if (t == 0) {
    for (int k = 0; k < 10; ++k) atomicAdd(&g_lvl_prof[k], (unsigned long long)lp[k]);
    atomicMax(&g_lvl_prof[10], (unsigned long long)lp[10]);
  }
#endif
}

// ---- mid-size builder: one workgroup splits a segment of <= kMidMax points in LDS ----------------
// The global levels stop at kMidMax points (instead of kSubMax): a workgroup of kMidWaves waves loads the
// segment into LDS and splits its nodes above kSubMax points one after another with block-wide
// reductions and Hoare passes (the same node rule and the same swaps as the sequential loop: the
// k-th misplaced element from the left swaps with the k-th from the right), depth first; the
// pieces of <= kSubMax points go to the subtree builders, leaves are emitted at once.
// threads per workgroup: 512 (r06; 1024 before): a node's phases are barrier-bound, and with 8
// waves instead of 16 a C2 segment's k_tr_mid took 63 against 76 us (256 threads: 81 us)
#ifndef AICP_MIDTHREADS
#define AICP_MIDTHREADS 512
#endif
constexpr int kMidThreads = AICP_MIDTHREADS;
constexpr int kMidWaves = kMidThreads / 64;
constexpr int kMidStack = 32;
constexpr int kMidOut = 64;  // pieces of <= kSubMax points per mid segment (2 per split node > kSubMax)

static_assert(kMidMax < 65536, "k_tr_mid packs two counts of a node into one word");

#if AICP_ITER_PROF
// diagnostic builds: k_tr_mid's phases per segment (s_memrealtime ticks, 100 MHz): load, nodes,
// store, node count, segments, and the slowest segment's total
__device__ unsigned long long g_mid_prof[8];
#endif

// one Hoare pass over local [lo_b, end) with boundary br, the whole workgroup. A round covers
// kMidSub chunks of kMidThreads elements with one barrier: the per-wave counts of the round's
// chunks go to one of two count buffers (alternating rounds, so a round's writes never meet the
// previous round's reads), and the offsets follow the element order (chunk, then wave, then
// lane) -- the k-th misplaced element from the left still meets the k-th from the right.
constexpr int kMidSub = 4;
__device__ void mid_hoare(float4* pts, uint16_t* posA, uint16_t* posB, uint32_t (*sAB)[2][kMidSub][kMidWaves],
                          uint32_t lo_b, uint32_t br, uint32_t end, int cd, float cut, bool eq) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t ra = 0, rb = 0;
  int buf = 0;
  for (uint32_t jb = lo_b; jb < end; jb += kMidThreads * kMidSub, buf ^= 1) {
    uint64_t ma[kMidSub], mb[kMidSub];
#pragma unroll
    for (int u = 0; u < kMidSub; ++u) {
      const uint32_t j = jb + u * kMidThreads + t;
      const bool ok = j < end;
      bool pr = false;
      if (ok) {
        const float v = coord(pts[j], cd);
        pr = eq ? (v == cut) : (v < cut);
      }
      ma[u] = __ballot(ok && j < br && !pr);
      mb[u] = __ballot(ok && j >= br && pr);
      if (lane == 0) {
        sAB[buf][0][u][wv] = (uint32_t)__popcll(ma[u]);
        sAB[buf][1][u][wv] = (uint32_t)__popcll(mb[u]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kMidSub; ++u) {
      uint32_t oa = ra, ob = rb, ta = 0, tb = 0;
#pragma unroll
      for (int w = 0; w < kMidWaves; ++w) {
        const uint32_t x = sAB[buf][0][u][w], y = sAB[buf][1][u][w];
        if (w < wv) {
          oa += x;
          ob += y;
        }
        ta += x;
        tb += y;
      }
      const uint32_t j = jb + u * kMidThreads + t;
      if ((ma[u] >> lane) & 1) posA[oa + popc_lt(ma[u])] = (uint16_t)j;
      if ((mb[u] >> lane) & 1) posB[ob + popc_lt(mb[u])] = (uint16_t)j;
      ra += ta;
      rb += tb;
    }
  }
  __syncthreads();  // every position written
  for (uint32_t k = t; k < ra; k += kMidThreads) {
    const uint32_t a = posA[k], b = posB[rb - 1 - k];
    const float4 x = pts[a];
    pts[a] = pts[b];
    pts[b] = x;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kMidThreads) void k_tr_mid(uint32_t total, TreeCtl* ctl, const SubSeg* __restrict__ mids,
                                                        SubSeg* subs, float4* W, float4* __restrict__ bpts,
                                                        NodeEvent* ev, uint8_t* valid, uint32_t* ecnt,
                                                        int32_t* pair_depth, int bucket, uint32_t max_seg) {
  __shared__ float4 pts[kMidMax];
  __shared__ uint16_t posA[kMidMax / 2], posB[kMidMax / 2];
  __shared__ uint32_t sAB[2][2][kMidSub][kMidWaves];
  __shared__ float sMn[kMidWaves], sMx[kMidWaves];
  __shared__ uint32_t sU[kMidWaves];
  __shared__ SubNode stk[kMidStack];
  __shared__ SubSeg outq[kMidOut];  // the segment's pieces for the subtree builders, written at its end
  __shared__ int sp_s, nout_s;
  __shared__ int32_t maxd_s;
  const int t = threadIdx.x;
  const uint32_t n_mid = ctl->n_mid;
  for (uint32_t mi = blockIdx.x; mi < n_mid; mi += gridDim.x) {
    __syncthreads();  // the previous segment's last LDS reads precede this one's loads
    const SubSeg g = mids[mi];
    const uint32_t gf = g.f;
#if AICP_ITER_PROF
    const unsigned long long mp0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long mp1 = 0, mp2 = 0;
    unsigned int mp_nodes = 0;
#endif
    for (uint32_t j = t; j < g.c; j += kMidThreads) pts[j] = W[gf + j];
    if (t == 0) {
      SubNode& r = stk[0];
      r.lf = 0;
      r.lc = g.c;
      r.depth = g.depth;
      for (int k = 0; k < 3; ++k) {
        r.mn[k] = g.mn[k];
        r.mx[k] = g.mx[k];
      }
      r.pf = g.parent_f;
      r.pdepth = g.parent_depth;
      sp_s = 1;
      nout_s = 0;
      maxd_s = g.depth;
    }
    __syncthreads();
#if AICP_ITER_PROF
    mp1 = __builtin_amdgcn_s_memrealtime();
#endif
    for (;;) {
      const int sp = sp_s;
      if (sp == 0) break;
#if AICP_ITER_PROF
      ++mp_nodes;
#endif
      const SubNode nd = stk[sp - 1];  // count > kSubMax: split here
      __syncthreads();
      int cd;
      float ideal;
      split_dim(nd.mn, nd.mx, cd, ideal);
      const uint32_t a0 = nd.lf, end = nd.lf + nd.lc, count = nd.lc;
      float mn = __builtin_inff(), mx = -__builtin_inff();
      for (uint32_t j = a0 + t; j < end; j += kMidThreads) {
        const float v = coord(pts[j], cd);
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
      }
      // min and max in one barrier, then the two counts packed in one word (count <= kMidMax <
      // 2^16) in one more; sMn / sMx / sU are written again only after this node's later barriers
      mn = wave_min(mn);
      mx = wave_max(mx);
      if ((t & 63) == 0) {
        sMn[t >> 6] = mn;
        sMx[t >> 6] = mx;
      }
      __syncthreads();
      float lo = sMn[0], hi = sMx[0];
#pragma unroll
      for (int i = 1; i < kMidWaves; ++i) {
        lo = fminf(lo, sMn[i]);
        hi = fmaxf(hi, sMx[i]);
      }
      const float cut = ideal < lo ? lo : (ideal > hi ? hi : ideal);
      uint32_t nle = 0;
      for (uint32_t j = a0 + t; j < end; j += kMidThreads) {
        const float v = coord(pts[j], cd);
        nle += v < cut ? 1u : (v == cut ? 0x10000u : 0u);
      }
      nle = wave_sum_u(nle);
      if ((t & 63) == 0) sU[t >> 6] = nle;
      __syncthreads();
      nle = 0;
#pragma unroll
      for (int i = 0; i < kMidWaves; ++i) nle += sU[i];
      const uint32_t nl = nle & 0xffffu, ne = nle >> 16;
      const uint32_t br1 = nl, br2 = nl + ne;
      mid_hoare(pts, posA, posB, sAB, a0, a0 + br1, end, cd, cut, false);
      if (ne) mid_hoare(pts, posA, posB, sAB, a0 + br1, a0 + br2, end, cd, cut, true);
      uint32_t left;
      if (ideal < lo) left = 1;
      else if (ideal > hi) left = count - 1;
      else if (br1 > count / 2) left = br1;
      else if (br2 < count / 2) left = br2;
      else left = count / 2;
      if (t == 0) {
        NodeEvent e{};
        e.f = gf + nd.lf;
        e.c = count;
        e.depth = nd.depth;
        e.pair = g.pair;
        e.cut_bits = __float_as_uint(cut);
        e.cd = cd;
        e.left = left;
        e.parent_f = nd.pf;
        e.parent_depth = nd.pdepth;
        emit_event(ev, valid, ecnt, total, e);
        if (nd.depth + 1 > maxd_s) maxd_s = nd.depth + 1;
        int spn = sp - 1;
        for (int side = 0; side < 2; ++side) {
          SubNode c;
          c.lf = side ? nd.lf + left : nd.lf;
          c.lc = side ? count - left : left;
          c.depth = nd.depth + 1;
          c.pf = gf + nd.lf;
          c.pdepth = nd.depth;
          for (int k = 0; k < 3; ++k) {
            c.mn[k] = (side && k == cd) ? cut : nd.mn[k];
            c.mx[k] = (!side && k == cd) ? cut : nd.mx[k];
          }
          if (c.lc <= (uint32_t)bucket) {
            emit_event(ev, valid, ecnt, total, leaf_event(gf + c.lf, c.lc, c.depth, g.pair, c.pf, c.pdepth));
          } else if (c.lc <= (uint32_t)kSubMax) {
            // queued in LDS: one slot reservation per segment at its end instead of a returning
            // device atomic per piece on the workgroup's serial path
            if (nout_s >= kMidOut) {
              atomicOr(&ctl->error, 8);
              continue;
            }
            SubSeg& o = outq[nout_s++];
            o.f = gf + c.lf;
            o.c = c.lc;
            o.pair = g.pair;
            o.depth = c.depth;
            for (int k = 0; k < 3; ++k) {
              o.mn[k] = c.mn[k];
              o.mx[k] = c.mx[k];
            }
            o.parent_f = c.pf;
            o.parent_depth = c.pdepth;
          } else if (spn < kMidStack) {
            stk[spn++] = c;
          } else {
            atomicOr(&ctl->error, 8);
          }
        }
        sp_s = spn;
      }
      __syncthreads();
    }
    // points back: W for the subtree builders, bpts for the leaves emitted here (the subtree
    // builders overwrite their ranges of bpts)
#if AICP_ITER_PROF
    mp2 = __builtin_amdgcn_s_memrealtime();
#endif
    {  // the queued pieces: one reservation, then a copy by the first nout threads
      __shared__ uint32_t base_s;
      const int nout = nout_s;
      if (t == 0) base_s = nout ? atomicAdd(&ctl->n_small, (uint32_t)nout) : 0u;
      __syncthreads();
      const uint32_t base = base_s;
      if (t < nout) {
        if (base + (uint32_t)t < max_seg) subs[base + t] = outq[t];
        else atomicOr(&ctl->error, 4);
      }
    }
    for (uint32_t j = t; j < g.c; j += kMidThreads) {
      const float4 p = pts[j];
      W[gf + j] = p;
      bpts[gf + j] = p;
    }
    if (t == 0 && pair_depth[g.pair] < maxd_s) atomicMax(&pair_depth[g.pair], maxd_s);
#if AICP_ITER_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      const unsigned long long mp3 = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&g_mid_prof[0], mp1 - mp0);
      atomicAdd(&g_mid_prof[1], mp2 - mp1);
      atomicAdd(&g_mid_prof[2], mp3 - mp2);
      atomicAdd(&g_mid_prof[3], (unsigned long long)mp_nodes);
      atomicAdd(&g_mid_prof[4], 1ull);
      atomicMax(&g_mid_prof[5], mp3 - mp0);
      atomicMax(&g_mid_prof[6], (unsigned long long)mp_nodes);
    }
#endif
  }
}

// Grid-stride over the small segments (the grid does not depend on their count, which only
// the device knows). A segment above kSubMax points -- left over when the planned number of
// global levels was too small for the data -- is finished in place in global memory with the
// same routine: slower, same tree.
__global__ __launch_bounds__(64) void k_tr_subtree(uint32_t total, const TreeCtl* __restrict__ ctl,
                                                   const SubSeg* __restrict__ subs, const float4* __restrict__ W,
                                                   float4* __restrict__ bpts, uint32_t* __restrict__ posL,
                                                   uint32_t* __restrict__ posR, NodeEvent* ev, uint8_t* valid,
                                                   uint32_t* ecnt, int32_t* pair_depth, int bucket, int blk_done) {
  __shared__ float4 pts[kSubMax];
  __shared__ uint16_t posA[kSubMax / 2], posB[kSubMax / 2];
  __shared__ SubNode stk[kFarStack];
  const uint32_t n_small = ctl->n_small;
  const int lane = threadIdx.x;
  for (uint32_t si = blockIdx.x; si < n_small; si += gridDim.x) {
    __syncthreads();  // the previous segment's last LDS reads precede this one's loads
    const SubSeg g = subs[si];
    const uint32_t gf = g.f;
    if (g.c <= (uint32_t)kSubMax) {
      if (blk_done) continue;  // built by k_tr_subtree_blk
      for (uint32_t j = lane; j < g.c; j += 64) pts[j] = W[gf + j];
      __syncthreads();
      subtree_build<uint16_t>(g, total, pts, posA, posB, stk, ev, valid, ecnt, pair_depth, bucket);
      for (uint32_t j = lane; j < g.c; j += 64) bpts[gf + j] = pts[j];
    } else {
      for (uint32_t j = lane; j < g.c; j += 64) bpts[gf + j] = W[gf + j];
      __syncthreads();
      subtree_build<uint32_t>(g, total, bpts + gf, posL + gf, posR + gf, stk, ev, valid, ecnt, pair_depth, bucket);
    }
  }
}

// ---- node records --------------------------------------------------------------------------
// the node records from the events, and (threads < n_pairs, formerly k_tr_desc) each pair's node
// range and depth in its descriptor: fields no event reads
__global__ __launch_bounds__(256) void k_tr_emit(uint32_t total, const NodeEvent* __restrict__ ev,
                                                 const uint8_t* __restrict__ valid, const uint32_t* __restrict__ S,
                                                 PairDesc* pd, uint4* __restrict__ nodes, TreeCtl* ctl, int n_pairs,
                                                 const int32_t* __restrict__ pair_depth) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (uint32_t)n_pairs) {
    PairDesc& d = pd[i];
    d.node_off = S[d.ref_off + 1];
    d.n_nodes = S[d.ref_off + d.n_ref + 1] - d.node_off;
    d.tree_depth = pair_depth[i];
    if (d.tree_depth >= kFarStack) atomicOr(&ctl->error, 1);
  }
  if (i >= 2 * total || !valid[i]) return;
  const NodeEvent e = ev[i];
  const uint32_t ro = pd[e.pair].ref_off;
  const uint32_t base = S[ro + 1];  // nodes of earlier pairs (all end at or before ref_off)
  const uint32_t pre = (uint32_t)e.depth + S[e.f + 1];
  const uint32_t par = e.parent_depth < 0 ? 0xffffffffu : (uint32_t)e.parent_depth + S[e.parent_f + 1] - base;
  uint4 r;
  if (e.cd == (int32_t)kLeaf) {
    r = make_uint4(e.c, kLeaf | ((e.f - ro) << 2), par, (uint32_t)e.depth);
  } else {
    const uint32_t right = (uint32_t)e.depth + 1 + S[e.f + e.left + 1] - base;
    r = make_uint4(e.cut_bits, (uint32_t)e.cd | (right << 2), par, (uint32_t)e.depth);
  }
  if (pre >= 2 * total + 2) {
    atomicOr(&ctl->error, 2);
    return;
  }
  nodes[pre] = r;
}

// Pairs sharing a reference cloud share its centroid, kd-tree and normals (built once per
// reference): copy the reference's fields into the pair descriptors;
// T_refMean_dataIn depends on the pair's own initial transform.
__global__ void k_pairs_from_refs(int n_pairs, PairDesc* pd, const PairDesc* __restrict__ rd) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  PairDesc& d = pd[p];
  const PairDesc& r = rd[d.ref_id];
  d.node_off = r.node_off;
  d.n_nodes = r.n_nodes;
  d.tree_depth = r.tree_depth;
  d.tl_off = r.tl_off;
  d.tl_cap = r.tl_cap;
  float Tmi[16];
  ident4(Tmi);
  for (int k = 0; k < 3; ++k) {
    d.mean[k] = r.mean[k];
    Tmi[12 + k] = -r.mean[k];
  }
  for (int k = 0; k < 16; ++k) d.Tmean[k] = r.Tmean[k];
  mul4(Tmi, d.Tin, d.Tinit);
}

// normals computed in the raw tree's bucket order -> the matcher tree's bucket order, through
// the input id each point carries in w
__global__ __launch_bounds__(256) void k_inv_perm(int n_refs, uint32_t total, const PairDesc* __restrict__ rd,
                                                  const float4* __restrict__ bpts, uint32_t* __restrict__ inv) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  const uint32_t ro = rd[pair_of_pos(rd, n_refs, j)].ref_off;
  inv[ro + (uint32_t)__float_as_int(bpts[j].w)] = j;
}

__global__ __launch_bounds__(256) void k_scatter_normals(int n_refs, uint32_t total, const PairDesc* __restrict__ rd,
                                                         const float4* __restrict__ bpts_raw,
                                                         const float4* __restrict__ nrm_raw,
                                                         const uint32_t* __restrict__ inv, float4* __restrict__ bnrm) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  const uint32_t ro = rd[pair_of_pos(rd, n_refs, j)].ref_off;
  bnrm[inv[ro + (uint32_t)__float_as_int(bpts_raw[j].w)]] = nrm_raw[j];
}

// what: 1 = the reference's degenerate-normal count (needs SurfaceNormal), 2 = the initial
// transform's rigidity check (needs only the pair frames; before the first active list)
__global__ void k_pairs_degenerate(int n_pairs, const PairDesc* __restrict__ pd, PairState* st,
                                   const PairState* __restrict__ rst, int what) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  if (what & 1) st[p].degenerate = rst[pd[p].ref_id].degenerate;
  // ICP::compute applies T_refMean_dataIn to the reading first: RigidTransformation's
  // checkParameters throws TransformationError for a non-rigid initial transform
  if ((what & 2) && !rigid_ok(pd[p].Tinit)) {
    st[p].status = 5;
    st[p].active = 0;
  }
}

inline unsigned grid_of(size_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

size_t tree_scan_temp_bytes(size_t n) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, n,
                                rocprim::plus<uint32_t>());
  return bytes;
}


// ---- treelets: the matcher tree in two-level, pointer-light records (Trav2C) ----------------
// The nodes at even depth are treelet roots. Treelet T = a root v and its two children, in one
// 16-byte record {slot v, slot L, slot R, meta}: an inner slot holds the cut (float bits), a leaf
// slot count << 28 | bucket start; meta = cd_v | cd_L << 2 | cd_R << 4 | base << 6 (cd 3 = leaf).
// The (up to four) treelets rooted at v's grandchildren LL, LR, RL, RR sit at base + 0..3, so no
// child pointer is stored. Slot 0 of a reference is the root's treelet; a treelet that has
// grandchildren gets its block of 4 at base = 1 + 4 * rank, rank = its position among such
// treelets in preorder (one scan), so every treelet's index follows from its grandparent's base
// without a level-by-level pass. link[T].x = the node id (treelet << 2 | slot) of the parent of
// T's root, -1 for the root treelet (the climb's step out of a treelet); link[T].y = the same for
// the parent treelet (two treelets ahead). Indices are local to the reference (PairDesc::tl_off,
// for tl and link).
__device__ __forceinline__ int ref_of_node(const PairDesc* __restrict__ rd, int n_refs, uint32_t g) {
  int lo = 0, hi = n_refs - 1;  // the reference owning node g (node_off ascending)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rd[mid].node_off <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ bool tl_has_block(const uint4* __restrict__ nd, uint32_t v) {
  const uint4 a = nd[v];
  if ((a.w & 1u) || (a.y & 3u) == kLeaf) return false;  // odd depth or leaf: no treelet block
  const uint4 L = nd[v + 1], R = nd[a.y >> 2];
  return (L.y & 3u) != kLeaf || (R.y & 3u) != kLeaf;
}

// rank = exclusive scan over the node records [0, n) of "has a block of grandchild treelets"
// (tl_has_block), the flag computed inside the single-pass look-back scan (one launch instead of
// a flag kernel and rocprim's two)
__global__ __launch_bounds__(kLbThreads) void k_tl_scan(int n_refs, uint32_t n, const PairDesc* __restrict__ rd,
                                                       const uint4* __restrict__ nodes, uint32_t* __restrict__ rank,
                                                       uint64_t* st, TreeCtl* ctl) {
  const uint32_t total = rd[n_refs - 1].node_off + rd[n_refs - 1].n_nodes;
  lookback_scan(
      n,
      [&](uint32_t g) -> uint32_t {
        if (g >= total) return 0u;
        const PairDesc& r = rd[ref_of_node(rd, n_refs, g)];
        return tl_has_block(nodes + r.node_off, g - r.node_off) ? 1u : 0u;
      },
      rank, st, ctl);
}

__device__ __forceinline__ uint32_t tl_slot(const uint4& a) {
  return (a.y & 3u) == kLeaf ? (a.x << 28) | (a.y >> 2) : a.x;
}

__device__ __forceinline__ void tl_check_ref(const PairDesc& r, const uint32_t* __restrict__ rank, int bucket,
                                             TreeCtl* ctl);
// the records; threads < n_refs also run k_tl_check's test for reference g
__global__ __launch_bounds__(256) void k_tl_build(int n_refs, uint32_t cap, const PairDesc* __restrict__ rd,
                                                  const uint4* __restrict__ nodes, const uint32_t* __restrict__ rank,
                                                  uint4* __restrict__ tl, uint2* __restrict__ link, int bucket,
                                                  TreeCtl* ctl) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g < (uint32_t)n_refs) tl_check_ref(rd[g], rank, bucket, ctl);
  const uint32_t total = rd[n_refs - 1].node_off + rd[n_refs - 1].n_nodes;
  if (g >= total || g >= cap) return;
  const PairDesc& r = rd[ref_of_node(rd, n_refs, g)];
  const uint4* nd = nodes + r.node_off;
  const uint32_t v = g - r.node_off;
  const uint4 a = nd[v];
  if (a.w & 1u) return;  // odd depth: a slot of its parent's treelet
  const uint32_t r0 = rank[r.node_off];
  auto base_of = [&](uint32_t u) { return 1u + 4u * (rank[r.node_off + u] - r0); };
  // treelet of an even-depth node u: 0 for the root, else its grandparent's base + k with
  // k = 2 * (parent is the grandparent's right child) + (u is its parent's right child)
  auto id_of = [&](uint32_t u) -> uint32_t {
    if (u == 0) return 0u;
    const uint32_t p = nd[u].z, gp = nd[p].z;
    return base_of(gp) + 2u * (p != gp + 1 ? 1u : 0u) + (u != p + 1 ? 1u : 0u);
  };
  const uint32_t id = id_of(v);
  if (id >= r.tl_cap) return;  // tl_check_ref reports it
  // parent of a treelet root u as a node id: the grandparent's treelet, slot of the parent
  auto up_of = [&](uint32_t u) -> uint32_t {
    if (u == 0) return 0xffffffffu;
    const uint32_t p = nd[u].z, gp = nd[p].z;
    return id_of(gp) << 2 | (p != gp + 1 ? 2u : 1u);
  };
  // link = {parent of this treelet's root, parent of the parent treelet's root}: the climb
  // names two treelets ahead (kernels_icp.hip, AICP_NN_CLIMB4)
  const uint32_t up = up_of(v);
  link[r.tl_off + id] = make_uint2(up, v == 0 ? 0xffffffffu : up_of(nd[a.z].z));  // nd[a.z].z: the grandparent, root of the parent treelet
  uint4 rec = make_uint4(tl_slot(a), 0u, 0u, a.y & 3u);
  if ((a.y & 3u) != kLeaf) {
    const uint4 L = nd[v + 1], R = nd[a.y >> 2];
    rec.y = tl_slot(L);
    rec.z = tl_slot(R);
    rec.w |= ((L.y & 3u) << 2) | ((R.y & 3u) << 4);
    if ((L.y & 3u) != kLeaf || (R.y & 3u) != kLeaf) rec.w |= base_of(v) << 6;
  }
  tl[r.tl_off + id] = rec;
}

// treelets used per reference within its allotment and addressable by the 26-bit base field;
// leaf slots need count < 16 and bucket starts < 2^28
__device__ __forceinline__ void tl_check_ref(const PairDesc& r, const uint32_t* __restrict__ rank, int bucket,
                                             TreeCtl* ctl) {
  const uint32_t used = 1u + 4u * (rank[r.node_off + r.n_nodes] - rank[r.node_off]);
  if (used > r.tl_cap || used >= (1u << 26) || bucket > 15 || r.n_ref >= (1u << 28)) atomicOr(&ctl->error, 4);
}

hipError_t launch_treelets(hipStream_t s, int n_refs, uint32_t cap, const PairDesc* rd, const uint4* nodes,
                           int bucket, uint32_t* rank, uint4* tl, uint2* link, const TreeWork& w) {
  if (n_refs <= 0 || cap == 0) return hipSuccess;
  TreeCtl* ctl = w.ctl;
  // the scan's look-back words: the two strides after the build's own (lb_bytes), zeroed with
  // them by launch_tree_prepare; cap + 1 = 2 * points + 3 records need at most two strides
  if (lb_words(cap + 1) > 2 * w.lb_stride) return hipErrorInvalidValue;
  uint64_t* st = w.lb + (size_t)(2 * kFarStack + 1) * w.lb_stride;
  k_tl_scan<<<(cap + 1 + kLbTile - 1) / kLbTile, kLbThreads, 0, s>>>(n_refs, cap + 1, rd, nodes, rank, st, ctl);
  k_tl_build<<<std::max(grid_of(cap), grid_of((size_t)n_refs)), 256, 0, s>>>(n_refs, cap, rd, nodes, rank, tl, link,
                                                                            bucket, ctl);
  return hipGetLastError();
}
void launch_pairs_from_refs(hipStream_t s, int n_pairs, PairDesc* pd, const PairDesc* rd) {
  k_pairs_from_refs<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, rd);
}
void launch_normals_to_matcher(hipStream_t s, int n_refs, uint32_t total, const PairDesc* rd, const float4* bpts,
                               const float4* bpts_raw, const float4* nrm_raw, uint32_t* inv, float4* bnrm) {
  if (!total) return;
  k_inv_perm<<<grid_of(total), 256, 0, s>>>(n_refs, total, rd, bpts, inv);
  k_scatter_normals<<<grid_of(total), 256, 0, s>>>(n_refs, total, rd, bpts_raw, nrm_raw, inv, bnrm);
}
void launch_pairs_degenerate(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const PairState* rst) {
  k_pairs_degenerate<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st, rst, 3);
}
void launch_pairs_degenerate_part(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const PairState* rst,
                                  int what) {
  k_pairs_degenerate<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st, rst, what);
}

// look-back words of every scan of a build: two per global level, the node count scan and (two
// strides) the matcher treelets' scan
size_t lb_stride_words(uint32_t total) { return lb_words(total + 2); }
uint32_t tree_mid_max() { return (uint32_t)kMidMax; }
size_t tree_sum_tiles(size_t n) { return tiles_of(n); }
// k_tr_subtree_lvl from this many points of a build (C5: 61 M); smaller builds are latency-bound
// and keep k_tr_subtree_blk (r04: C2 2620 against 2479 clouds/s with the level builder).
// aicp_hip_options::tree_lvl_min sets it (TreeWork::lvl_min; the equivalence test builds small
// trees both ways).
hipError_t set_lb_force_stall(int on) {
  const int v = on ? 1 : 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lb_force_stall), &v, sizeof(v));
}
size_t lb_bytes(uint32_t total) { return (size_t)(2 * kFarStack + 3) * lb_stride_words(total) * 8; }

hipError_t launch_tree_prepare(hipStream_t s, int n_pairs, uint32_t total, PairDesc* pd, const float4* raw,
                               int center, const TreeWork& w, float4* bpts, int bucket, int part) {
  // part 1: what does not read the points (the zeroed work space; without centring also the
  // frames), so a stream can run it before it waits for them; part 2: the rest; 0: all
  const bool first = part != 2, rest = part != 1;
  const bool frames_first = !center;
  ZeroJob z{};
  const size_t bytes[6] = {(size_t)n_pairs * 6 * sizeof(uint64_t), sizeof(TreeCtl), ((size_t)total + 2) * 4,
                           2 * (size_t)total, (size_t)n_pairs * 4, lb_bytes(total)};
  void* ptr[6] = {w.sums, w.ctl, w.ecnt, w.valid, w.pair_depth, w.lb};
  uint64_t most = 0;
  for (int r = 0; r < 6; ++r) {
    z.p[r] = reinterpret_cast<uint4*>(ptr[r]);
    z.n16[r] = (bytes[r] + 15) / 16;
    most = std::max<uint64_t>(most, z.n16[r]);
  }
  uint64_t* tpart = w.sums + (size_t)n_pairs * 6;  // tile partials (TreeWork::sums)
  if (first) {
    k_tr_zero<<<(unsigned)std::min<uint64_t>(1024, std::max<uint64_t>(1, (most + 255) / 256)), 256, 0, s>>>(
        z, n_pairs, w.seg[0]);
    if (frames_first) k_tr_frames<<<n_pairs, 64, 0, s>>>(n_pairs, total, pd, w.sums, tpart, center);
  }
  if (!rest) return hipGetLastError();
  if (center) k_tr_sum<<<tiles_of(total), 256, 0, s>>>(n_pairs, total, pd, raw, w.sums, tpart);
  if (!frames_first) k_tr_frames<<<n_pairs, 64, 0, s>>>(n_pairs, total, pd, w.sums, tpart, center);
  k_tr_center<<<tiles_of(total), 256, 0, s>>>(n_pairs, total, pd, raw, w.W[0], w.segof[0], w.seg[0], bpts, bucket,
                                             w.mid_max);
  k_tr_roots<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, total, pd, w.seg[0], w.subs, w.mids, w.ctl, w.ev, w.valid, w.ecnt,
                                                  bucket, w.mid_max);
  return hipGetLastError();
}

hipError_t launch_tree_level(hipStream_t s, int level, uint32_t total, const TreeWork& w, float4* bpts,
                             int bucket, bool last) {
  const int a = level & 1, b = a ^ 1;
  TreeSeg* seg = w.seg[a];
  TreeSeg* next = w.seg[b];
  const unsigned gp = grid_of(total), gp1 = grid_of((size_t)total + 1);
  // segments at this level: at most n_pairs << level and at most total / kSubMax
  const unsigned gs = grid_of(std::min<size_t>(w.max_seg, (size_t)w.n_pairs << std::min(level, 20)));
  const uint32_t nt1 = lb_words(total + 1) - 1;  // tiles of a scan over [0, total]
  uint64_t* st1 = w.lb + (size_t)(2 * level) * w.lb_stride;
  uint64_t* st2 = st1 + w.lb_stride;
  // level 0: the roots' boxes (k_tr_center); later levels: the previous level's move2 (move2_minmax)
  k_tr_scan1<<<nt1, kLbThreads, 0, s>>>(total, w.segof[a], w.W[0], seg, w.X1, st1, w.ctl);
  k_tr_move1<<<gp1, 256, 0, s>>>(total, w.segof[a], w.W[0], seg, w.X1, w.W[1], w.flag);
  k_tr_scan_counts<<<nt1, kLbThreads, 0, s>>>(total + 1, w.flag, w.X2, st2, w.ctl);
  k_tr_split<<<gs, 256, 0, s>>>(level, last ? 1 : 0, total, seg, next, w.subs, w.mids, w.ctl, w.X2, w.ev, w.valid,
                                w.ecnt, w.pair_depth, bucket, (uint32_t)w.max_seg, w.mid_max);
  k_tr_move2<<<gp, 256, 0, s>>>(total, w.segof[a], w.W[1], seg, w.X2, w.W[0], w.segof[b], bpts, next);
  return hipGetLastError();
}

// grid: an upper bound of the small-segment count (<= total / (bucket + 1) + pairs), capped;
// the kernel strides over the device-side count
hipError_t launch_tree_subtrees(hipStream_t s, uint32_t total, const TreeWork& w, float4* bpts, int bucket) {
  const size_t bound = std::min<size_t>(w.max_seg, (size_t)total / (size_t)(bucket + 1) + (size_t)w.n_pairs + 1);
  const bool blk = bucket >= 4;  // level widths fit kSubLevelCap
  if (bucket >= 8 && total >= w.lvl_min) {  // level widths fit kLvlCap
    const unsigned gl = (unsigned)std::max<size_t>(1, std::min<size_t>(bound, 2048));
    k_tr_subtree_lvl<<<gl, kLvlThreads, 0, s>>>(total, w.ctl, w.subs, w.W[0], bpts, w.ev, w.valid, w.ecnt,
                                                 w.pair_depth, bucket);
  } else if (blk) {
    const unsigned gb = (unsigned)std::max<size_t>(1, std::min<size_t>(bound, 2048));
    k_tr_subtree_blk<<<gb, 64 * kSubWaves, 0, s>>>(total, w.ctl, w.subs, w.W[0], bpts, w.ev, w.valid, w.ecnt,
                                                   w.pair_depth, bucket);
  }
  // oversized segments (a planned build that was too shallow), or every segment without blk
  const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>(bound, blk ? 256 : 16384));
  k_tr_subtree<<<g, 64, 0, s>>>(total, w.ctl, w.subs, w.W[0], bpts, w.posL, w.posR, w.ev, w.valid, w.ecnt,
                                w.pair_depth, bucket, blk ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_tree_mid(hipStream_t s, uint32_t total, const TreeWork& w, float4* bpts, int bucket) {
  // grid: an upper bound of the mid-size segment count, capped (the kernel strides over the
  // device-side count)
  const size_t bound = std::min<size_t>(w.max_seg, (size_t)total / (size_t)(kSubMax + 1) + (size_t)w.n_pairs + 1);
  const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>(bound, 1024));
  k_tr_mid<<<g, kMidThreads, 0, s>>>(total, w.ctl, w.mids, w.subs, w.W[0], bpts, w.ev, w.valid, w.ecnt, w.pair_depth,
                                     bucket, (uint32_t)w.max_seg);
  return hipGetLastError();
}

void tree_prof_dump() {
#if AICP_ITER_PROF
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mid_prof), sizeof(h)) == hipSuccess && h[4])
    fprintf(stderr,
            "[tree prof] k_tr_mid per segment: load %.2f us, nodes %.2f us (%.2f nodes), store %.2f us; "
            "slowest segment %.2f us, most nodes %llu, segments %llu\n",
            h[0] / 100.0 / h[4], h[1] / 100.0 / h[4], (double)h[3] / h[4], h[2] / 100.0 / h[4], h[5] / 100.0, h[6],
            h[4]);
  unsigned long long l[12];
  if (hipMemcpyFromSymbol(l, HIP_SYMBOL(g_lvl_prof), sizeof(l)) == hipSuccess && l[8]) {
    fprintf(stderr,
            "[tree prof] k_tr_subtree_lvl per segment (%llu segments, %.1f points, %.2f levels): load %.2f, "
            "minmax %.2f, counts %.2f, passes %.2f, nodes %.2f, child map %.2f, store %.2f us; slowest %.2f us\n",
            l[8], (double)l[9] / l[8], (double)l[7] / l[8], l[0] / 100.0 / l[8], l[1] / 100.0 / l[8],
            l[2] / 100.0 / l[8], l[3] / 100.0 / l[8], l[4] / 100.0 / l[8], l[5] / 100.0 / l[8],
            l[6] / 100.0 / l[8], l[10] / 100.0);
    unsigned long long z[12] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lvl_prof), z, sizeof(z));
  }
#endif
}

hipError_t launch_tree_finish(hipStream_t s, int n_pairs, uint32_t total, PairDesc* pd, const TreeWork& w,
                              uint4* nodes) {
  // S[p] = #nodes with end < p  (exclusive scan over end positions 0..total+1)
  k_tr_scan_counts<<<lb_words(total + 2) - 1, kLbThreads, 0, s>>>(total + 2, w.ecnt, w.X1,
                                                                    w.lb + (size_t)(2 * kFarStack) * w.lb_stride, w.ctl);
  k_tr_emit<<<std::max(grid_of(2 * (size_t)total), grid_of((size_t)n_pairs)), 256, 0, s>>>(
      total, w.ev, w.valid, w.X1, pd, nodes, w.ctl, n_pairs, w.pair_depth);
  return hipGetLastError();
}

}  // namespace aicp
