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

__device__ __forceinline__ int pair_of_pos(const PairDesc* pd, int n_pairs, uint32_t s) {
  int lo = 0, hi = n_pairs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pd[mid].ref_off <= s) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void emit_event(TreeCtl* ctl, NodeEvent* ev, uint32_t* ecnt, const NodeEvent& e) {
  const uint32_t i = atomicAdd(&ctl->n_events, 1u);
  ev[i] = e;
  atomicAdd(&ecnt[e.f + e.c], 1u);
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
  ideal = (mx[cd] + mn[cd]) / 2;
}

__device__ __forceinline__ float seg_cut(const TreeSeg& s) {
  const float lo = ord_dec(s.lo), hi = ord_dec(s.hi);
  return s.ideal < lo ? lo : (s.ideal > hi ? hi : s.ideal);
}

// ---- centroid --------------------------------------------------------------------------------
// Exact order-independent sum: every coordinate as round(x * 2^40) in 128-bit two's complement
// (two 64-bit atomics with carry), so the result does not depend on the reduction order.
__global__ __launch_bounds__(256) void k_tr_sum(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd,
                                                const float4* __restrict__ raw, uint64_t* sums) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < total;
  const int pair = ok ? pair_of_pos(pd, n_pairs, i) : -1;
  const float4 p = ok ? raw[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float c[3] = {p.x, p.y, p.z};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int64_t q = ok ? fixed40(c[d]) : 0;
    // segmented 128-bit sum over the wave: (lo, hi) with carry
    uint64_t lo = (uint64_t)q;
    int64_t hi = q < 0 ? -1 : 0;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int ko = __shfl_up(pair, off, 64);
      const uint64_t lo_o = __shfl_up(lo, off, 64);
      const int64_t hi_o = __shfl_up(hi, off, 64);
      if (lane >= off && ko == pair) {
        const uint64_t s = lo + lo_o;
        hi = hi + hi_o + (s < lo ? 1 : 0);
        lo = s;
      }
    }
    const int kn = __shfl_down(pair, 1, 64);
    if (ok && (lane == 63 || kn != pair)) {
      uint64_t* w = sums + (size_t)pair * 6 + 2 * d;
      const uint64_t old = atomicAdd((unsigned long long*)w, (unsigned long long)lo);
      const uint64_t carry = (old + lo < old) ? 1u : 0u;
      atomicAdd((unsigned long long*)(w + 1), (unsigned long long)((uint64_t)hi + carry));
    }
  }
}

// mean, T_refIn_refMean, T_refMean_dataIn = T_refIn_refMean^-1 * T0 (A.1 steps 2, 5);
// center == 0: the kernel-level kNN entry points build on the points as given.
__global__ void k_tr_frames(int n_pairs, PairDesc* pd, const uint64_t* sums, int center) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  PairDesc& d = pd[p];
  float Tm[16], Tmi[16];
  ident4(Tm);
  ident4(Tmi);
  for (int k = 0; k < 3; ++k) {
    d.mean[k] = center ? mean_from_fixed40(sums[p * 6 + 2 * k], sums[p * 6 + 2 * k + 1], d.n_ref) : 0.f;
    Tm[12 + k] = d.mean[k];
    Tmi[12 + k] = -d.mean[k];
  }
  for (int k = 0; k < 16; ++k) d.Tmean[k] = Tm[k];
  mul4(Tmi, d.Tin, d.Tinit);
}

// centred reference (w = local input id) into W0; the root segment of every pair; whole-cloud
// bounding box of the centred points; a pair with n_ref <= bucket is one leaf.
__global__ __launch_bounds__(256) void k_tr_center(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd,
                                                   const float4* __restrict__ raw, float4* __restrict__ W,
                                                   float4* __restrict__ bpts, int32_t* __restrict__ segof,
                                                   TreeSeg* seg, int bucket) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < total;
  const int pair = ok ? pair_of_pos(pd, n_pairs, i) : -1;
  float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    const PairDesc& d = pd[pair];
    const float4 p = raw[i];
    c = make_float4(p.x - d.mean[0], p.y - d.mean[1], p.z - d.mean[2], __int_as_float((int32_t)(i - d.ref_off)));
    W[i] = c;
    const bool leaf = d.n_ref <= (uint32_t)bucket;
    if (leaf) bpts[i] = c;
    segof[i] = leaf ? -1 : pair;
  }
  const float v[3] = {c.x, c.y, c.z};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float mn = v[k], mx = v[k];
    const bool last = wave_seg_minmax(pair, mn, mx);
    if (ok && last) {
      atomicMin(&seg[pair].bmn[k], ord_enc(mn));
      atomicMax(&seg[pair].bmx[k], ord_enc(mx));
    }
  }
}

// root segments (level 0, index = pair) from the boxes; single-leaf roots emit their event
__global__ void k_tr_roots(int n_pairs, const PairDesc* __restrict__ pd, TreeSeg* seg, TreeCtl* ctl,
                           NodeEvent* ev, uint32_t* ecnt, int bucket) {
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
  s.lo = 0xffffffffu;
  s.hi = 0u;
  if (d.n_ref <= (uint32_t)bucket) {
    NodeEvent e{};
    e.f = d.ref_off;
    e.c = d.n_ref;
    e.depth = 0;
    e.pair = p;
    e.cd = (int32_t)kLeaf;
    e.parent_depth = -1;
    emit_event(ctl, ev, ecnt, e);
    s.count = 0;  // not split
  }
  if (p == 0) ctl->nseg[0] = (uint32_t)n_pairs;
}

// ---- one level ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tr_minmax(uint32_t total, const int32_t* __restrict__ segof,
                                                   const float4* __restrict__ W, TreeSeg* seg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = i < total ? segof[i] : -1;
  float v = 0.f;
  if (s >= 0) v = coord(W[i], seg[s].cd);
  float mn = v, mx = v;
  const bool last = wave_seg_minmax(s, mn, mx);
  if (s >= 0 && last) {
    atomicMin(&seg[s].lo, ord_enc(mn));
    atomicMax(&seg[s].hi, ord_enc(mx));
  }
}

// pass-1 predicate (v < cut); position `total` stays 0
__global__ __launch_bounds__(256) void k_tr_flag1(uint32_t total, const int32_t* __restrict__ segof,
                                                  const float4* __restrict__ W, const TreeSeg* __restrict__ seg,
                                                  uint32_t* __restrict__ flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > total) return;
  uint32_t f = 0;
  if (i < total) {
    const int s = segof[i];
    if (s >= 0) f = coord(W[i], seg[s].cd) < seg_cut(seg[s]) ? 1u : 0u;
  }
  flag[i] = f;
}

// Destination of the element at local position li in a Hoare pass over [lo_b, count) with
// boundary br (elements satisfying the predicate end up in [lo_b, br)), given the exclusive
// scan X of the predicate: X[f + j] = #satisfying in [f, f + j).
struct HoareRanks {
  // misplaced-left rank (ascending) or misplaced-right rank (descending), -1 if in place
  __device__ static int32_t rank(uint32_t li, bool pred, uint32_t f, uint32_t lo_b, uint32_t br, uint32_t count,
                                 const uint32_t* X, bool& left_side) {
    if (li < br) {
      left_side = true;
      if (pred) return -1;
      return (int32_t)((li - lo_b) - (X[f + li] - X[f + lo_b]));  // non-satisfying in [lo_b, li)
    }
    left_side = false;
    if (!pred) return -1;
    const uint32_t kl = X[f + li] - X[f + br];
    const uint32_t nmr = X[f + count] - X[f + br];
    return (int32_t)(nmr - 1 - kl);
  }
};

// partner positions of the misplaced elements of a pass
__global__ __launch_bounds__(256) void k_tr_pos(uint32_t total, int pass, const int32_t* __restrict__ segof,
                                                const float4* __restrict__ W, const TreeSeg* __restrict__ seg,
                                                const uint32_t* __restrict__ X, uint32_t* __restrict__ posL,
                                                uint32_t* __restrict__ posR) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int s = segof[i];
  if (s < 0) return;
  const TreeSeg& g = seg[s];
  const float v = coord(W[i], g.cd), cut = seg_cut(g);
  const uint32_t f = g.first, li = i - f;
  uint32_t lo_b, br;
  bool pred;
  if (pass == 1) {
    lo_b = 0;
    br = X[f + g.count] - X[f];
    pred = v < cut;
  } else {
    lo_b = g.br1;
    br = g.br1 + (X[f + g.count] - X[f]);
    if (li < lo_b) return;
    pred = v == cut;  // v <= cut within [br1, count)
  }
  bool left;
  const int32_t k = HoareRanks::rank(li, pred, f, lo_b, br, g.count, X, left);
  if (k < 0 || (uint32_t)k >= g.count) return;
  (left ? posL : posR)[f + k] = li;
}

// pass 1: move every element to its place, and write the pass-2 predicate at the new place
__global__ __launch_bounds__(256) void k_tr_move1(uint32_t total, const int32_t* __restrict__ segof,
                                                  const float4* __restrict__ W, TreeSeg* seg,
                                                  const uint32_t* __restrict__ X, const uint32_t* __restrict__ posL,
                                                  const uint32_t* __restrict__ posR, float4* __restrict__ W1,
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
  bool left;
  const int32_t k = HoareRanks::rank(li, v < cut, f, 0, br1, g.count, X, left);
  uint32_t p1 = k < 0 ? li : (left ? posR[f + k] : posL[f + k]);
  if (p1 >= g.count) p1 = li;  // unreachable for a consistent scan; keeps stores in range
  W1[f + p1] = p;
  flag2[f + p1] = (p1 >= br1 && v == cut) ? 1u : 0u;
  if (li == 0) seg[s].br1 = br1;
}

// split: left-count rule, node event of this segment, children (leaf events or next-level
// segments)
__global__ __launch_bounds__(256) void k_tr_split(int level, TreeSeg* seg, TreeSeg* next, TreeCtl* ctl,
                                                  const uint32_t* __restrict__ X2, NodeEvent* ev, uint32_t* ecnt,
                                                  int32_t* pair_depth, int bucket, uint32_t max_seg) {
  const uint32_t si = blockIdx.x * blockDim.x + threadIdx.x;
  if (si >= ctl->nseg[level]) return;
  TreeSeg& g = seg[si];
  if (g.count == 0) return;  // single-leaf root
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
  emit_event(ctl, ev, ecnt, e);
  const int cdepth = g.depth + 1;
  atomicMax(&pair_depth[g.pair], cdepth);
  for (int side = 0; side < 2; ++side) {
    const uint32_t cf = side ? f + left : f, cc = side ? count - left : left;
    if (cc <= (uint32_t)bucket) {
      NodeEvent l{};
      l.f = cf;
      l.c = cc;
      l.depth = cdepth;
      l.pair = g.pair;
      l.cd = (int32_t)kLeaf;
      l.parent_f = f;
      l.parent_depth = g.depth;
      emit_event(ctl, ev, ecnt, l);
      g.child[side] = -1;
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
      c.mn[k] = g.mn[k];
      c.mx[k] = g.mx[k];
    }
    if (side) c.mn[g.cd] = cut;
    else c.mx[g.cd] = cut;
    split_dim(c.mn, c.mx, c.cd, c.ideal);
    c.lo = 0xffffffffu;
    c.hi = 0u;
    g.child[side] = (int32_t)ni;
  }
}

// pass 2 move; next level's segment map; points landing in leaves are final (bucket order)
__global__ __launch_bounds__(256) void k_tr_move2(uint32_t total, const int32_t* __restrict__ segof,
                                                  const float4* __restrict__ W1, const TreeSeg* __restrict__ seg,
                                                  const uint32_t* __restrict__ X2, const uint32_t* __restrict__ posL,
                                                  const uint32_t* __restrict__ posR, float4* __restrict__ W2,
                                                  int32_t* __restrict__ segof_next, float4* __restrict__ bpts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int s = segof[i];
  if (s < 0) {
    segof_next[i] = -1;
    return;
  }
  const TreeSeg& g = seg[s];
  const float4 p = W1[i];
  const float v = coord(p, g.cd), cut = seg_cut(g);
  const uint32_t f = g.first, li = i - f;
  uint32_t p2 = li;
  if (li >= g.br1) {
    bool left;
    const int32_t k = HoareRanks::rank(li, v == cut, f, g.br1, g.br2, g.count, X2, left);
    if (k >= 0) p2 = left ? posR[f + k] : posL[f + k];
    if (p2 >= g.count) p2 = li;  // unreachable for a consistent scan; keeps stores in range
  }
  const uint32_t q = f + p2;
  W2[q] = p;
  const int32_t child = g.child[p2 < g.left ? 0 : 1];
  segof_next[q] = child;
  if (child < 0) bpts[q] = p;
}

// ---- node records --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tr_emit(TreeCtl* ctl, const NodeEvent* __restrict__ ev,
                                                 const uint32_t* __restrict__ S, const PairDesc* __restrict__ pd,
                                                 uint4* __restrict__ nodes, uint32_t cap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ctl->n_events || i >= cap) return;
  const NodeEvent e = ev[i];
  const uint32_t ro = pd[e.pair].ref_off;
  const uint32_t base = S[ro + 1];  // nodes of earlier pairs (all end at or before ref_off)
  const uint32_t pre = (uint32_t)e.depth + S[e.f + 1];
  const uint32_t par = e.parent_depth < 0 ? 0xffffffffu : (uint32_t)e.parent_depth + S[e.parent_f + 1] - base;
  uint4 r;
  if (e.cd == (int32_t)kLeaf) {
    r = make_uint4(e.c, kLeaf | ((e.f - ro) << 2), par, 0u);
  } else {
    const uint32_t right = (uint32_t)e.depth + 1 + S[e.f + e.left + 1] - base;
    r = make_uint4(e.cut_bits, (uint32_t)e.cd | (right << 2), par, 0u);
  }
  if (pre >= cap) {
    atomicOr(&ctl->error, 2);
    return;
  }
  nodes[pre] = r;
}

__global__ void k_tr_desc(int n_pairs, PairDesc* pd, const uint32_t* __restrict__ S,
                          const int32_t* __restrict__ pair_depth, TreeCtl* ctl) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  PairDesc& d = pd[p];
  d.node_off = S[d.ref_off + 1];
  d.n_nodes = S[d.ref_off + d.n_ref + 1] - d.node_off;
  d.tree_depth = pair_depth[p];
  if (d.tree_depth >= kFarStack) atomicOr(&ctl->error, 1);
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

inline unsigned grid_of(size_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

size_t tree_scan_temp_bytes(size_t n) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, n,
                                rocprim::plus<uint32_t>());
  return bytes;
}

static hipError_t scan_u32(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, size_t n) {
  size_t bytes = temp_bytes;
  return rocprim::exclusive_scan(temp, bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), s);
}

hipError_t launch_tree_prepare(hipStream_t s, int n_pairs, uint32_t total, PairDesc* pd, const float4* raw,
                               int center, const TreeWork& w, float4* bpts, int bucket) {
  (void)hipMemsetAsync(w.sums, 0, (size_t)n_pairs * 6 * sizeof(uint64_t), s);
  (void)hipMemsetAsync(w.ctl, 0, sizeof(TreeCtl), s);
  (void)hipMemsetAsync(w.ecnt, 0, ((size_t)total + 2) * 4, s);
  (void)hipMemsetAsync(w.pair_depth, 0, (size_t)n_pairs * 4, s);
  if (center) k_tr_sum<<<grid_of(total), 256, 0, s>>>(n_pairs, total, pd, raw, w.sums);
  k_tr_frames<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, w.sums, center);
  k_tr_init_boxes<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, w.seg[0]);
  k_tr_center<<<grid_of(total), 256, 0, s>>>(n_pairs, total, pd, raw, w.W[0], bpts, w.segof[0], w.seg[0], bucket);
  k_tr_roots<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, w.seg[0], w.ctl, w.ev, w.ecnt, bucket);
  return hipGetLastError();
}

hipError_t launch_tree_level(hipStream_t s, int level, uint32_t total, const TreeWork& w, float4* bpts,
                             int bucket) {
  const int a = level & 1, b = a ^ 1;
  TreeSeg* seg = w.seg[a];
  TreeSeg* next = w.seg[b];
  const unsigned gp = grid_of(total), gp1 = grid_of((size_t)total + 1), gs = grid_of(w.max_seg);
  k_tr_minmax<<<gp, 256, 0, s>>>(total, w.segof[a], w.W[0], seg);
  k_tr_flag1<<<gp1, 256, 0, s>>>(total, w.segof[a], w.W[0], seg, w.flag);
  hipError_t e = scan_u32(s, w.scan_temp, w.scan_temp_bytes, w.flag, w.X1, (size_t)total + 1);
  if (e != hipSuccess) return e;
  k_tr_pos<<<gp, 256, 0, s>>>(total, 1, w.segof[a], w.W[0], seg, w.X1, w.posL, w.posR);
  k_tr_move1<<<gp1, 256, 0, s>>>(total, w.segof[a], w.W[0], seg, w.X1, w.posL, w.posR, w.W[1], w.flag);
  e = scan_u32(s, w.scan_temp, w.scan_temp_bytes, w.flag, w.X2, (size_t)total + 1);
  if (e != hipSuccess) return e;
  k_tr_split<<<gs, 256, 0, s>>>(level, seg, next, w.ctl, w.X2, w.ev, w.ecnt, w.pair_depth, bucket,
                                (uint32_t)w.max_seg);
  k_tr_pos<<<gp, 256, 0, s>>>(total, 2, w.segof[a], w.W[1], seg, w.X2, w.posL, w.posR);
  k_tr_move2<<<gp, 256, 0, s>>>(total, w.segof[a], w.W[1], seg, w.X2, w.posL, w.posR, w.W[0], w.segof[b], bpts);
  return hipGetLastError();
}

hipError_t launch_tree_finish(hipStream_t s, int n_pairs, uint32_t total, PairDesc* pd, const TreeWork& w,
                              uint4* nodes) {
  // S[p] = #nodes with end < p  (exclusive scan over end positions 0..total+1)
  hipError_t e = scan_u32(s, w.scan_temp, w.scan_temp_bytes, w.ecnt, w.X1, (size_t)total + 2);
  if (e != hipSuccess) return e;
  k_tr_emit<<<grid_of(2 * (size_t)total + 2), 256, 0, s>>>(w.ctl, w.ev, w.X1, pd, nodes, 2 * total + 2);
  k_tr_desc<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, w.X1, w.pair_depth, w.ctl);
  return hipGetLastError();
}

}  // namespace aicp
