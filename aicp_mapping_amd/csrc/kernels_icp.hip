// kernels_icp.hip — ICP hot path on CDNA4 (gfx950).
//
// Per ICP iteration (libpointmatcher ICP loop), for every pair of a
// batch at once, five launches and no host synchronisation:
//   k_active_list  compacts the pairs still iterating into the NN work space
//   k_icp_nn       persistent waves: transform by T_iter (fused) + libnabo-order approximate
//                  1-NN; a lane that finishes its query refills from a 64-query chunk of the
//                  work space, so far-descent tails do not hold whole waves
//   k_sel_*        exact k-th smallest d^2 (Matches::getDistsQuantile) by 3-digit radix select
//                  over the whole chip: digit-1 histograms per 1024 readings, then the bin's
//                  values compacted per pair and finished by one workgroup per pair
//   k_icp_reduce   TrimmedDist weights + getMatchedPoints gather + point-to-plane F, dot and the
//                  27-entry normal-equation sums in double from exact float products; DPP row
//                  sums + LDS, one deterministic partial row per workgroup (no atomics)
//   k_icp_update   fixed-order sum of the partial rows, 6x6 solve, AngleAxis update of T_iter,
//                  Counter + Differential checkers, per-pair active flag
// SurfaceNormal: k_knn_ids (persistent kNN, eps 0, ids only) + k_normals_from_ids (uniform
// covariance / eigen work per point).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <type_traits>
#include <cstdio>

#include <cstdlib>

#include "aicp_common.hpp"
#include "icp_math.hpp"
#include "kernels.hpp"

namespace aicp {

// ------------------------------------------------------------------------------------------
// k-NN traversal in libnabo recurseKnn order, resumable in rounds
// ------------------------------------------------------------------------------------------
// recurseKnn visits the near child first, then the far child if rd' = rd - off[cd]^2 +
// new_off^2 passes (rd' <= maxR2 && rd' * maxE2 < head). Along a run of near children rd and
// off do not change, so the far test of every level of a descent is evaluated during the
// descent itself; after the leaf the climb (through parent[]) is skipped when the smallest
// such rd' already fails -- the common case with epsilon = 3.16. A round = one descent, its
// bucket and the climb up to the next far child (or to the end of the query). Far descents
// push (far child, rd, off[cd], outer min, outer start); nesting <= tree depth < kFarStack.
template <int K>
struct Best {
  float v[K];  // ascending, head = v[K-1] (IndexHeapBruteForceVector)
  int32_t id[K];
};

template <int K>
__device__ __forceinline__ void best_init(Best<K>& b) {
#pragma unroll
  for (int i = 0; i < K; ++i) {
    b.v[i] = __builtin_inff();
    b.id[i] = -1;
  }
}

#ifndef AICP_BEST_NOCHAIN
#define AICP_BEST_NOCHAIN 1
#endif
template <int K>
__device__ __forceinline__ void best_replace(Best<K>& b, int32_t id, float val) {
#if AICP_BEST_NOCHAIN
  // the same insertion without the serial `placed` chain: with c(i) = v[i-1] > val (the list is
  // ascending, so c(i) implies c(i+1)), slot i takes v[i-1] when c(i), val when c(i+1) alone and
  // keeps v[i] otherwise -- equal values stay ahead of the new one, as in the loop below. Each
  // compare reads a slot not yet written (slots go downwards).
  bool cn = true;  // c(i+1); the last slot takes val unless shifted into
#pragma unroll
  for (int i = K - 1; i > 0; --i) {
    const bool ci = b.v[i - 1] > val;
    // v[i-1] <= v[i]: their median with val is v[i-1] below it, val between, v[i] above (the
    // caller passes val < v[K-1], finite)
    b.v[i] = __builtin_amdgcn_fmed3f(b.v[i - 1], b.v[i], val);
    b.id[i] = ci ? b.id[i - 1] : (cn ? id : b.id[i]);
    cn = ci;
  }
  if (cn) {
    b.v[0] = val;
    b.id[0] = id;
  }
  return;
#endif
  bool placed = false;
#pragma unroll
  for (int i = K - 1; i > 0; --i) {
    if (!placed) {
      if (b.v[i - 1] > val) {
        b.v[i] = b.v[i - 1];
        b.id[i] = b.id[i - 1];
      } else {
        b.v[i] = val;
        b.id[i] = id;
        placed = true;
      }
    }
  }
  if (!placed) {
    b.v[0] = val;
    b.id[0] = id;
  }
}

__device__ __forceinline__ float sel3(uint32_t cd, float a, float b, float c) {
  return cd == 0 ? a : (cd == 1 ? b : c);
}

// Far-descent stack: the only dynamically indexed state (private/scratch memory, touched only
// on far descents); kept apart from Trav so the rest of the traversal stays in registers.
// One 32-byte frame per far descent, so a push or pop moves 16-byte scratch words instead of
// seven separate dwords (NN launch -5 %).
struct FarFrame {
  int32_t F;
  float rd, old, mn;
  int32_t start, P, PP, pad;  // P: node whose far child began the frame, PP: its parent
};
struct FarStack {
  FarFrame f[kFarStack];
};
// the same frame in LDS, 24 bytes: P (node ids < 2^30) shares its word with cd
struct LdsFrame {
  int32_t Pcd;
  float rd, old, mn;
  int32_t start, PP;
};
// the NN kernel's LDS frame, 20 bytes (four per lane fit 20 KB per 256-lane block, 8 blocks per
// CU): PP (< 2^30) shares its word with cd; P itself is only compared with start, so its place is
// the sign bit of mn, set when P == start (a negative mn, possible by rounding, is stored as +0:
// both force the exact climb).
struct NnLdsFrame {
  int32_t PPcd;
  float rd, old;
  int32_t start;
  float mnf;
};
// Trav2C's frames past its LDS ones, in scratch in the same 20-byte layout (5 dwords per push
// and pop where FarFrame moves 8; scratch lines are written back to HBM through L2)
struct NnFarStack {
  NnLdsFrame f[kFarStack];
};
__device__ __forceinline__ void put_far(NnFarStack& fs, int32_t sp, const NnLdsFrame& g, const FarFrame&) {
  fs.f[sp] = g;
}
__device__ __forceinline__ void put_far(FarStack& fs, int32_t sp, const NnLdsFrame&, const FarFrame& f) {
  fs.f[sp] = f;
}

constexpr int kLeafBatch = 8;  // = libnabo's default bucket size
#ifndef AICP_NN_COOP
#define AICP_NN_COOP 0  // Trav2C: 1 = cooperative octet bucket scan, 0 = each lane scans its own bucket
#endif
#ifndef AICP_NN_PREFMIN
#define AICP_NN_PREFMIN 0  // Trav2C: per-depth running minimum of the far bounds in LDS (climb pruning; off: C2 -1 %, C4 +20 %)
#endif
[[maybe_unused]] constexpr int kPmDepth = 24;  // depths whose running minimum is kept (deeper levels climb unpruned)
#ifndef AICP_NN_POPCHK
#define AICP_NN_POPCHK 1  // Trav2C (CLIMB2): after a frame pop, skip the rest of the climb when no level above the frame's node can pass (per-depth prefix minima, one byte each, in LDS)
#endif
[[maybe_unused]] constexpr int kPopDepth = 16;  // depths whose prefix minimum is kept (frames deeper than this climb unchecked)
[[maybe_unused]] constexpr int kStartBits = 26;  // LDS frames keep P's depth above the start node id
#ifndef AICP_NN_CLIMB2
#define AICP_NN_CLIMB2 1  // Trav2C: climb one treelet (record + parent, up to two levels) per iteration
#endif
#ifndef AICP_NN_CLIMB4
#define AICP_NN_CLIMB4 0  // Trav2C (with CLIMB2): two treelets per climb round trip through the treelet links (measured 6 % slower: the extra records are mostly not needed)
#endif
#if AICP_NN_POPCHK && (!AICP_NN_CLIMB2 || AICP_NN_CLIMB4 || AICP_NN_PREFMIN)
#undef AICP_NN_POPCHK
#define AICP_NN_POPCHK 0  // the pop check belongs to the one-treelet climb
#endif
#ifndef AICP_NN_LDS_FRAMES
#define AICP_NN_LDS_FRAMES 3  // Trav2C: innermost far-descent frames kept in LDS (20 B each per lane; 4 measured no faster)
#endif
#ifndef AICP_KNN_LDS_FRAMES
#define AICP_KNN_LDS_FRAMES 6  // k_knn_ids (SurfaceNormal kNN): far frames per lane kept in LDS
#endif
constexpr int kKnnLdsFrames = AICP_KNN_LDS_FRAMES;

template <int K>
struct Trav {
  using Stack = FarStack;
  const uint4* nodes;
  const float4* pts;
  float q0, q1, q2;
  float off0, off1, off2, rd, minFar;
  int32_t n, start, sp;
  uint32_t tp, tn;
  Best<K> best;
  LdsFrame* lf = nullptr;  // innermost far frames in LDS (stride kNNBlock), nlf of them
  int32_t nlf = 0;

  __device__ __forceinline__ void bind(const uint4* nb, const float4* pb, uint32_t node_off, uint32_t ref_off) {
    nodes = nb + node_off;
    pts = pb + ref_off;
  }
  __device__ __forceinline__ float res_d2() const { return best.v[0]; }
  __device__ __forceinline__ int32_t res_id() const { return best.id[0]; }

  __device__ __forceinline__ void reset(float a, float b, float c) {
    q0 = a;
    q1 = b;
    q2 = c;
    off0 = off1 = off2 = rd = 0.f;
    n = start = sp = 0;
    tp = tn = 0;
    best_init<K>(best);
  }

  // one round (a descent, its bucket and the climb to the next far descent); true when done.
  // The climb follows the parent index stored in each node record (one load per level).
  __device__ __forceinline__ bool advance(FarStack& fs, float maxE2, float maxR2, const uint4*, const float4*) {
    minFar = __builtin_inff();
    // the descent reads the first 8 bytes of each record (cut, cd | right); the leaf's parent
    // is the node the descent came from (the climb reads whole records)
    const uint2* nodes2 = reinterpret_cast<const uint2*>(nodes);
    uint2 nd = nodes2[2 * n];
    int32_t pl = -1;
    while ((nd.y & 3u) != kLeaf) {
      const uint32_t cd = nd.y & 3u;
      const float no = sel3(cd, q0, q1, q2) - __uint_as_float(nd.x);
      const float oc = sel3(cd, off0, off1, off2);
      const float rdf = rd + (-oc * oc + no * no);
      minFar = fminf(minFar, rdf);
      pl = n;
      n = (no > 0.f) ? (int32_t)(nd.y >> 2) : n + 1;
      ++tn;
      nd = nodes2[2 * n];
    }
    if (pl < 0) pl = (int32_t)nodes[n].z;  // the descent started at a leaf
    {
      // bucket: the first kLeafBatch points are loaded before any is used (one round trip
      // instead of one per point), then scanned in order
      const uint32_t b0 = nd.y >> 2, cnt = nd.x;
      float3 P[kLeafBatch];
#pragma unroll
      for (int i = 0; i < kLeafBatch; ++i)
        if ((uint32_t)i < cnt) {
          const float4 p = pts[b0 + i];
          P[i] = make_float3(p.x, p.y, p.z);
        }
#pragma unroll
      for (int i = 0; i < kLeafBatch; ++i)
        if ((uint32_t)i < cnt) {
          const float d0 = q0 - P[i].x, d1 = q1 - P[i].y, d2 = q2 - P[i].z;
          float dist = 0.f;
          dist += d0 * d0;
          dist += d1 * d1;
          dist += d2 * d2;
          if (dist <= maxR2 && dist < best.v[K - 1]) best_replace<K>(best, (int32_t)(b0 + i), dist);
        }
      for (uint32_t i = kLeafBatch; i < cnt; ++i) {  // buckets larger than the default 8
        const float4 p = pts[b0 + i];
        const float d0 = q0 - p.x, d1 = q1 - p.y, d2 = q2 - p.z;
        float dist = 0.f;
        dist += d0 * d0;
        dist += d1 * d1;
        dist += d2 * d2;
        if (dist <= maxR2 && dist < best.v[K - 1]) best_replace<K>(best, (int32_t)(b0 + i), dist);
      }
      tp += cnt;
    }
    int32_t c = n, pc = pl;
    if (!(minFar <= maxR2 && minFar * maxE2 < best.v[K - 1])) c = start;
    for (;;) {
      if (c == start) {
        if (sp == 0) return true;
        --sp;
        FarFrame f;
        if (sp < nlf) {
          const LdsFrame g = lf[sp * kNNBlock];
          f = FarFrame{g.Pcd, g.rd, g.old, g.mn, g.start, g.Pcd & 0x3fffffff, g.PP, 0};
        } else {
          f = fs.f[sp];
        }
        const uint32_t pcd = (uint32_t)f.F >> 30;
        rd = f.rd;
        const float old = f.old;
        if (pcd == 0) off0 = old;
        else if (pcd == 1) off1 = old;
        else off2 = old;
        minFar = f.mn;
        start = f.start;
        c = f.P;
        pc = f.PP;
        if (!(minFar <= maxR2 && minFar * maxE2 < best.v[K - 1])) c = start;
        continue;
      }
      const int32_t p = pc;
      const uint4 pn = nodes[p];
      const uint32_t cd = pn.y & 3u;
      const float no = sel3(cd, q0, q1, q2) - __uint_as_float(pn.x);
      const float oc = sel3(cd, off0, off1, off2);
      const float rdf = rd + (-oc * oc + no * no);
      if (rdf <= maxR2 && rdf * maxE2 < best.v[K - 1]) {
        const int32_t far = (no > 0.f) ? p + 1 : (int32_t)(pn.y >> 2);
        if (sp < nlf) lf[sp * kNNBlock] = LdsFrame{(int32_t)((uint32_t)p | (cd << 30)), rd, oc, minFar, start, (int32_t)pn.z};
        else fs.f[sp] = FarFrame{(int32_t)((uint32_t)far | (cd << 30)), rd, oc, minFar, start, p, (int32_t)pn.z, 0};
        ++sp;
        if (cd == 0) off0 = no;
        else if (cd == 1) off1 = no;
        else off2 = no;
        rd = rdf;
        n = far;
        start = far;
        return false;
      }
      c = p;
      pc = (int32_t)pn.z;
    }
  }
};

// 1-NN (the ICP matcher) over the matcher tree's treelets (kernels_tree.hip: a node and its two
// children in one 16-byte record, the grandchildren's treelets at base + 0..3). A node is named
// by treelet << 2 | slot (slot 0 the treelet's root, 1 / 2 its left / right child), so the
// root is 0. One record load decides two levels of a descent; the climb steps inside a record
// without a load and into the parent treelet through ptl (loaded with the record). The records hold no parent, child or
// redundant copies (about 5 B per node against 32 B for two-level node records), so the trees
// of the references an XCD serves stay in its L2.
//
// The bucket scan is done by the wave cooperatively: lanes 8g..8g+7 (an "octet") read the 8
// points of one owner's bucket together -- one 128-byte run -- and compute their distances to
// the owner's query; a min over the octet (DPP) and the lowest lane holding it (ballot) give
// the owner the result of libnabo's in-order scan (first strictly smaller d^2 wins). Eight
// rounds serve the octet's eight owners. The split into descend() / (wave-wide bucket) /
// climb() keeps libnabo recurseKnn's visit order, far tests and counts.
// one 16-byte treelet record as a single dwordx4: the empty asm keeps the compiler from narrowing
// the load into the words used first plus a dependent load of the rest
__device__ __forceinline__ uint4 ld_rec(const uint4* p) {
  uint4 r = *p;
  asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w));
  return r;
}
// a record and its treelet's parent link in one round trip: both loads are issued before the
// empty asm makes the wave wait for them (ld_rec followed by a plain load would wait for the
// record first and send the link load after it, a second dependent round trip per climb step)
__device__ __forceinline__ uint4 ld_rec_up(const uint4* p, const uint2* l, int32_t& up) {
  uint32_t u = l->x;
  uint4 r = *p;
  asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w), "+v"(u));
  up = (int32_t)u;
  return r;
}

// Running minimum of far bounds: every bound is rd + (-off^2 + no^2) with |no| >= |off| (the
// region shrinks away from the query), so it is >= 0 and a signed integer minimum of the float
// bits is the float minimum (one v_min_i32, no NaN canonicalisation). A negative bound, if
// rounding ever produced one, only makes the minimum negative, i.e. forces the exact climb.
__device__ __forceinline__ float min_bound(float a, float b) {
  return __int_as_float(min(__float_as_int(a), __float_as_int(b)));
}

// One-byte lower bound of a non-negative float (the prefix minima of AICP_NN_POPCHK): code 0 is
// 0.0, code c >= 1 is the float with bits kPmBase + ((c - 1) << 21) (two mantissa bits), and a
// value always encodes to a code that decodes to <= itself (truncation, clamping at 255 only
// lowers it), so a failed far test on the decoded bound implies a failed test on the true one.
constexpr uint32_t kPmBase = 0x30000000u;  // 2^-31
__device__ __forceinline__ uint32_t pm_enc(float v) {
  const int32_t u = __float_as_int(v);
  const int32_t c = ((u - (int32_t)kPmBase) >> 21) + 1;
  return (uint32_t)min(max(c, 0), 255);
}
__device__ __forceinline__ float pm_dec(uint32_t c) {
  return c == 0 ? 0.f : __uint_as_float(kPmBase + ((c - 1u) << 21));
}

#if AICP_NN_POPCHK
// the NN kernel's one-byte prefix minima, depth-major: lane t of the block at [d * kNNBlock + t]
// (module scope, addressed from threadIdx.x at each use: the fetch, the descent and the climb
// all reach it, from the first round on)
__shared__ uint8_t g_pmb[kPopDepth * kNNBlock];
__device__ __forceinline__ uint8_t& pmb_at(int d) { return g_pmb[d * kNNBlock + threadIdx.x]; }
#endif

struct Trav2C {
#if AICP_NN_CLIMB2 && !AICP_NN_CLIMB4
  using Stack = NnFarStack;
#else
  using Stack = FarStack;
#endif
  const uint4* tlb;      // the batch's treelets (uniform: set per chunk)
  const uint2* ptlb;     // the batch's treelet links {parent of the root, parent of the parent treelet's root}
  uint32_t tlo;          // the pair's first treelet: one VGPR instead of two 64-bit pointers
  uint32_t pbase;        // the pair's first bucket point
  float q0, q1, q2;
  float noc0, noc1, noc2, rd, minFar;  // noc = -(off * off) per axis (libnabo's off[] enters only so)
  int32_t n, start, sp, pl;  // node ids; pl: parent of the node the last descent ended in
  int32_t dep;               // depth of n (descent) / of the node climbed from (climb)
  uint16_t* pm;              // this lane's prefix-minimum column in LDS (AICP_NN_PREFMIN)
  uint32_t lb0, lcnt;        // bucket of the leaf the last descent ended in
  NnLdsFrame* lf;            // this lane's LDS frames (AICP_NN_LDS_FRAMES, stride kNNBlock)
  uint32_t tp, tn;
  Best<1> best;

  __device__ __forceinline__ void bind(const uint4*, const uint2*, uint32_t tl_off, uint32_t ref_off) {
    tlo = tl_off;
    pbase = ref_off;
  }
  __device__ __forceinline__ void bind_batch(const uint4* t, const uint2* b) {  // wave-uniform
    tlb = t;
    ptlb = b;
  }
  // treelet T of the pair / its link: 32-bit byte offsets from the uniform bases (host-checked
  // to fit), so each address is one VGPR added to an SGPR pair
  __device__ __forceinline__ const uint4* trec(uint32_t T) const {
    return reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(tlb) + ((tlo + T) << 4));
  }
  __device__ __forceinline__ const uint2* tlink(uint32_t T) const {
    return reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(ptlb) + ((tlo + T) << 3));
  }
  __device__ __forceinline__ float res_d2() const { return best.v[0]; }
  __device__ __forceinline__ int32_t res_id() const { return best.id[0]; }

  __device__ __forceinline__ void reset(float a, float b, float c) {
    q0 = a;
    q1 = b;
    q2 = c;
    noc0 = noc1 = noc2 = rd = 0.f;
    n = start = sp = 0;
    pl = -1;
    dep = 0;
    tp = tn = 0;
    best_init<1>(best);
  }

  __device__ __forceinline__ static uint32_t slot_word(const uint4& r, uint32_t s) {
    return s == 0 ? r.x : (s == 1 ? r.y : r.z);
  }

  // one inner slot: fold its far bound into minFar, return true if the query goes right. With
  // AICP_NN_PREFMIN the running minimum after this level is kept per depth in LDS, rounded down
  // to bf16 (the upper half of the float bits, exact for the skip test's direction): the climb
  // then knows, before loading an ancestor, whether it or any level above it in this descent
  // can still pass the far test.
  __device__ __forceinline__ bool decide(uint32_t w, uint32_t cd) {
    const float no = sel3(cd, q0, q1, q2) - __uint_as_float(w);
    minFar = min_bound(minFar, rd + (sel3(cd, noc0, noc1, noc2) + no * no));
    ++tn;
#if AICP_NN_PREFMIN
    if (dep < kPmDepth) pm[dep * kNNBlock] = (uint16_t)(__float_as_uint(minFar) >> 16);
    ++dep;
#elif AICP_NN_POPCHK
    if (dep < kPopDepth) pmb_at(dep) = (uint8_t)pm_enc(minFar);
    ++dep;
#endif
    return no > 0.f;
  }

  // a descent from n: the root slot of each treelet, then the chosen child's slot, one record
  // load per two levels (a descent that starts at a child slot skips the first root step)
  __device__ __forceinline__ void descend() {
    minFar = __builtin_inff();
    uint32_t T = (uint32_t)n >> 2, s = (uint32_t)n & 3u;
    uint4 r = ld_rec(trec(T));
    uint32_t w = r.x, cd = r.w & 3u;
    if (s == 0 && cd != kLeaf) {
      s = decide(w, cd) ? 2u : 1u;
      pl = n;
      n = (int32_t)(T << 2 | s);
    }
    while (s != 0) {
      w = s == 1 ? r.y : r.z;
      cd = (r.w >> (2 * s)) & 3u;
      if (cd == kLeaf) break;
      const bool right = decide(w, cd);
      pl = n;
      T = (r.w >> 6) + 2 * (s - 1) + (right ? 1u : 0u);
      n = (int32_t)(T << 2);
      r = ld_rec(trec(T));
      w = r.x;
      cd = r.w & 3u;
      if (cd == kLeaf) break;
      s = decide(w, cd) ? 2u : 1u;
      pl = n;
      n = (int32_t)(T << 2 | s);
    }
    lb0 = w & 0x0FFFFFFFu;
    lcnt = w >> 28;
  }

  // the whole bucket by this lane (AICP_NN_COOP 0): the first kLeafBatch points loaded before
  // any is used, then scanned in order
  __device__ __forceinline__ void bucket_lane(const float4* __restrict__ pts, float maxR2) {
    float3 P[kLeafBatch];
#pragma unroll
    for (int i = 0; i < kLeafBatch; ++i)
      if ((uint32_t)i < lcnt) {
        const float4 p = pts[pbase + lb0 + i];
        P[i] = make_float3(p.x, p.y, p.z);
      }
#pragma unroll
    for (int i = 0; i < kLeafBatch; ++i)
      if ((uint32_t)i < lcnt) {
        const float d0 = q0 - P[i].x, d1 = q1 - P[i].y, d2 = q2 - P[i].z;
        float dist = 0.f;
        dist += d0 * d0;
        dist += d1 * d1;
        dist += d2 * d2;
        if (dist <= maxR2 && dist < best.v[0]) best_replace<1>(best, (int32_t)(lb0 + i), dist);
      }
    bucket_tail(pts, maxR2);
  }

  // bucket points beyond the first kLeafBatch (bucket sizes above libnabo's default 8), in order
  __device__ __forceinline__ void bucket_tail(const float4* __restrict__ pts, float maxR2) {
    for (uint32_t i = kLeafBatch; i < lcnt; ++i) {
      const float4 p = pts[pbase + lb0 + i];
      const float d0 = q0 - p.x, d1 = q1 - p.y, d2 = q2 - p.z;
      float dist = 0.f;
      dist += d0 * d0;
      dist += d1 * d1;
      dist += d2 * d2;
      if (dist <= maxR2 && dist < best.v[0]) best_replace<1>(best, (int32_t)(lb0 + i), dist);
    }
    tp += lcnt;
  }

#if AICP_NN_CLIMB2
  // far test of node p (slot s of record r, parent pp); on a pass: push the frame, start the far
  // descent and return true
  // dp: depth of p (AICP_NN_POPCHK: kept in the frame, the far descent starts at dp + 1)
  __device__ __forceinline__ bool far_push(Stack& fs, const uint4& r, int32_t p, uint32_t s, int32_t pp,
                                           float maxE2, float maxR2, int32_t dp = 0) {
    const uint32_t T = (uint32_t)p >> 2;
    const uint32_t w = slot_word(r, s), cd = (r.w >> (2 * s)) & 3u;
    const float no = sel3(cd, q0, q1, q2) - __uint_as_float(w);
    const float oc = sel3(cd, noc0, noc1, noc2);
    const float rdf = rd + (oc + no * no);
    if (!(rdf <= maxR2 && rdf * maxE2 < best.v[0])) return false;
    const uint32_t fr = no > 0.f ? 0u : 1u;  // far child = the left one when the query is right of the cut
    const int32_t far = s == 0 ? (int32_t)(T << 2 | (1u + fr)) : (int32_t)(((r.w >> 6) + 2 * (s - 1) + fr) << 2);
    // the innermost frames live in LDS (no scratch traffic: scratch frames are written back
    // to HBM through L2), deeper nesting in the scratch stack
#if AICP_NN_POPCHK
    const int32_t sdp = start | (dp << kStartBits);  // node ids < 2^kStartBits (host-checked)
#else
    const int32_t sdp = start;
#endif
    const NnLdsFrame frame{(int32_t)(((uint32_t)pp & 0x3fffffffu) | (cd << 30)), rd, oc, sdp,
                           __int_as_float(max(__float_as_int(minFar), 0) | (p == start ? (int32_t)0x80000000 : 0))};
    if (sp < AICP_NN_LDS_FRAMES) lf[sp * kNNBlock] = frame;
    else put_far(fs, sp, frame, FarFrame{(int32_t)((uint32_t)far | (cd << 30)), rd, oc, minFar, start, p, pp, dp});
    ++sp;
    const float nn = -no * no;
    if (cd == 0) noc0 = nn;
    else if (cd == 1) noc1 = nn;
    else noc2 = nn;
    rd = rdf;
    n = far;
    start = far;
    pl = p;
#if AICP_NN_POPCHK
    dep = dp + 1;
#endif
    return true;
  }

#if AICP_NN_CLIMB4
  // far tests of node p (slot s of record r) and, for a child slot, of the treelet root above
  // it: true on a far push; else c / pc advance to the highest node tested / its parent (stopping
  // at start)
  __device__ __forceinline__ bool climb_treelet(FarStack& fs, const uint4& r, int32_t p, int32_t rootpp, int32_t& c,
                                                int32_t& pc, float maxE2, float maxR2) {
    const uint32_t T = (uint32_t)p >> 2, s = (uint32_t)p & 3u;
    const int32_t root = (int32_t)(T << 2);
    if (far_push(fs, r, p, s, s != 0 ? root : rootpp, maxE2, maxR2)) return true;
    c = p;
    pc = s != 0 ? root : rootpp;
    if (s == 0 || c == start) return false;
    if (far_push(fs, r, root, 0, rootpp, maxE2, maxR2)) return true;
    c = root;
    pc = rootpp;
    return false;
  }

  // the climb two treelets (up to four levels) per round trip: the links {parent of the
  // treelet's root, parent of the parent treelet's root} name the next two treelets before
  // their records arrive. After a descent or a frame pop the first step knows only the node to
  // test, so it loads one record and its link.
  __device__ __forceinline__ bool climb(FarStack& fs, float maxE2, float maxR2) {
    int32_t c = n, pc = pl;
    int32_t px = 0;
    bool have_px = false;  // px: parent node of pc's treelet's root
    if (!(minFar <= maxR2 && minFar * maxE2 < best.v[0])) c = start;
    for (;;) {
      if (c == start) {
        if (sp == 0) return true;
        --sp;
        FarFrame f;
        if (sp < AICP_NN_LDS_FRAMES) {
          const NnLdsFrame g = lf[sp * kNNBlock];
          const int32_t mi = __float_as_int(g.mnf);
          f = FarFrame{g.PPcd, g.rd, g.old, __int_as_float(mi & 0x7fffffff), g.start, mi < 0 ? g.start : -2,
                       g.PPcd & 0x3fffffff, 0};
        } else {
          f = fs.f[sp];
        }
        const uint32_t pcd = (uint32_t)f.F >> 30;
        rd = f.rd;
        if (pcd == 0) noc0 = f.old;
        else if (pcd == 1) noc1 = f.old;
        else noc2 = f.old;
        minFar = f.mn;
        start = f.start;
        c = f.P;
        pc = f.PP;
        have_px = false;
        if (!(minFar <= maxR2 && minFar * maxE2 < best.v[0])) c = start;
        continue;
      }
      const uint32_t X = (uint32_t)pc >> 2;
      if (!have_px) {
        uint2 lk = *tlink(X);
        uint4 r = *trec(X);
        asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w), "+v"(lk.x), "+v"(lk.y));
        if (climb_treelet(fs, r, pc, (int32_t)lk.x, c, pc, maxE2, maxR2)) return false;
        px = (int32_t)lk.y;
        have_px = c != start;
        continue;
      }
      // pc in treelet X, px = parent of X's root in treelet Y (px < 0: X is the root treelet)
      // three independent loads, one wait
      const uint32_t Y = (uint32_t)max(px, 0) >> 2;
      uint2 ly = *tlink(Y);
      uint4 rx = *trec(X);
      uint4 ry = *trec(Y);
      asm volatile("" : "+v"(rx.x), "+v"(rx.y), "+v"(rx.z), "+v"(rx.w), "+v"(ry.x), "+v"(ry.y), "+v"(ry.z),
                   "+v"(ry.w), "+v"(ly.x), "+v"(ly.y));
      if (climb_treelet(fs, rx, pc, px, c, pc, maxE2, maxR2)) return false;
      if (c == start || px < 0) continue;  // px < 0: X's root is the tree root, so c == start there
      if (climb_treelet(fs, ry, px, (int32_t)ly.x, c, pc, maxE2, maxR2)) return false;
      px = (int32_t)ly.y;
    }
  }
#else
  // the climb one treelet per iteration: one record (and its root's parent) per round trip, the
  // node and, for a child slot, the treelet root above it.
  // With AICP_NN_POPCHK, dep tracks the depth of c: after a frame pop, the prefix minimum of the
  // far bounds from the frame's start down to P's parent (written by that descent and untouched
  // by the deeper far descents since) decides at once whether any level left to climb can pass.
  // The far tests it skips are ones the climb would have made and failed, so the visit order,
  // counts and result are unchanged.
  __device__ __forceinline__ bool climb(Stack& fs, float maxE2, float maxR2) {
    int32_t c = n, pc = pl;
    if (!(minFar <= maxR2 && minFar * maxE2 < best.v[0])) c = start;
    for (;;) {
      if (c == start) {
        if (sp == 0) return true;
        --sp;
        FarFrame f;
        {
          // the innermost frames from LDS, the deeper ones from scratch, both in one layout.
          // P only matters through P == start (the sign bit of mn); any other id != start will do
          NnLdsFrame g;
          if (sp < AICP_NN_LDS_FRAMES) g = lf[sp * kNNBlock];
          else g = fs.f[sp];
          const int32_t mi = __float_as_int(g.mnf);
#if AICP_NN_POPCHK
          const int32_t gs = g.start & ((1 << kStartBits) - 1);
          f = FarFrame{g.PPcd, g.rd, g.old, __int_as_float(mi & 0x7fffffff), gs, mi < 0 ? gs : -2,
                       g.PPcd & 0x3fffffff, (int32_t)((uint32_t)g.start >> kStartBits)};
#else
          f = FarFrame{g.PPcd, g.rd, g.old, __int_as_float(mi & 0x7fffffff), g.start, mi < 0 ? g.start : -2,
                       g.PPcd & 0x3fffffff, 0};
#endif
        }
        const uint32_t pcd = (uint32_t)f.F >> 30;
        rd = f.rd;
        if (pcd == 0) noc0 = f.old;
        else if (pcd == 1) noc1 = f.old;
        else noc2 = f.old;
        minFar = f.mn;
        start = f.start;
        c = f.P;
        pc = f.PP;
        if (!(minFar <= maxR2 && minFar * maxE2 < best.v[0])) c = start;
#if AICP_NN_POPCHK
        dep = f.pad;  // depth of P
        if (c != start && dep <= kPopDepth) {
          const float b = pm_dec(pmb_at(dep - 1));
          if (!(b <= maxR2 && b * maxE2 < best.v[0])) c = start;
        }
#endif
        continue;
      }
      const int32_t p = pc;
      const uint32_t T = (uint32_t)p >> 2, s = (uint32_t)p & 3u;
      int32_t rootpp;
      const uint4 r = ld_rec_up(trec(T), tlink(T), rootpp);
      const int32_t root = (int32_t)(T << 2);
      if (far_push(fs, r, p, s, s != 0 ? root : rootpp, maxE2, maxR2, dep - 1)) return false;
      c = p;
      pc = s != 0 ? root : rootpp;
#if AICP_NN_POPCHK
      --dep;
#endif
      if (s == 0 || c == start) continue;
      if (far_push(fs, r, root, 0, rootpp, maxE2, maxR2, dep - 1)) return false;
      c = root;
      pc = rootpp;
#if AICP_NN_POPCHK
      --dep;
#endif
    }
  }
#endif  // AICP_NN_CLIMB4
#else
#error "AICP_NN_CLIMB2=0: the one-node-per-step climb was removed in r05 (it no longer built)"
#endif
};

template <class E>
struct is_coop {
  static constexpr bool value = false;
};
template <>
struct is_coop<Trav2C> {
  static constexpr bool value = true;
};

// DPP row controls (gfx9): quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141;

__device__ __forceinline__ float octet_min(float v) {
  v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kDppXor1, 0xF, 0xF, false)));
  v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kDppXor2, 0xF, 0xF, false)));
  v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kDppHalfMirror, 0xF, 0xF, false)));
  return v;
}

// Wave-wide cooperative scan of the first kLeafBatch points of every active lane's bucket
// (Trav2C). Called by all 64 lanes in wave-uniform control flow; `act` = the lane has a
// bucket this round. xch = this wave's 64 exchange slots in LDS.
template <class Eng>
__device__ __forceinline__ void coop_bucket(Eng& t, bool act, const float4* __restrict__ pts, float maxR2,
                                            float4* xch) {
  const int lane = threadIdx.x & 63;
  const int oct = lane & ~7, i = lane & 7;
  const uint32_t cnt = act ? min(t.lcnt, (uint32_t)kLeafBatch) : 0u;
  xch[lane] = make_float4(t.q0, t.q1, t.q2, __uint_as_float(((t.pbase + t.lb0) << 4) | cnt));
  __builtin_amdgcn_wave_barrier();
  // only the owners' bucket words stay live across the loads; their queries are re-read from
  // LDS when used (keeps the kernel at <= 64 VGPRs, 8 waves/SIMD)
  float3 P[kLeafBatch];
#pragma unroll
  for (int j = 0; j < kLeafBatch; ++j) {
    const uint32_t w = __float_as_uint(xch[oct + j].w);
    if ((uint32_t)i < (w & 15u)) {
      const float4 p = pts[(w >> 4) + i];
      P[j] = make_float3(p.x, p.y, p.z);
    }
  }
  float res_d = __builtin_inff();
  uint32_t res_i = 0;
#pragma unroll
  for (int j = 0; j < kLeafBatch; ++j) {
    float dist = __builtin_inff();
    const float4 Q = xch[oct + j];
    if ((uint32_t)i < (__float_as_uint(Q.w) & 15u)) {
      const float d0 = Q.x - P[j].x, d1 = Q.y - P[j].y, d2 = Q.z - P[j].z;
      float d = 0.f;
      d += d0 * d0;
      d += d1 * d1;
      d += d2 * d2;
      if (d <= maxR2) dist = d;
    }
    const float m = octet_min(dist);
    const uint32_t hit = (uint32_t)(__ballot(dist == m) >> oct) & 0xFFu;
    if (i == j) {
      res_d = m;
      res_i = (uint32_t)__builtin_ctz(hit | 0x100u);
    }
  }
  __builtin_amdgcn_wave_barrier();  // every lane's reads of xch precede the next round's writes
  if (act && res_d < t.best.v[0]) best_replace<1>(t.best, (int32_t)(t.lb0 + res_i), res_d);
}

#if AICP_XCD_PROF
__device__ unsigned long long g_xcd_prof[64 * kXcdGroups * 2];
__device__ unsigned long long g_xcd_cost[64 * kXcdGroups];  // per launch slot and group: queries << 40 | sum tn + tp
#endif
#if AICP_QLAT_PROF
// [0, 256): query latency (pick-up to result, 1 us bins); [256, 512): completion time of the
// query after its wave's start (1 us bins); last bin of each half = overflow
__device__ unsigned long long g_qlat[512];
#endif
#if AICP_NN_PROF
__device__ unsigned long long g_nn_prof[8];
#endif
#if AICP_ITER_PROF
// per kernel k (0 hist_f, 1 compact_f, 2 reduce, 3 update_f): [4k] body sum, [4k+1] bodies,
// [4k+2] tail sum, [4k+3] tails (s_memrealtime ticks, 10 ns)
__device__ unsigned long long g_iter_prof[16];
#define AICP_IP_T0 const uint64_t ip_t0 = __builtin_amdgcn_s_memrealtime()
#define AICP_IP_BODY(k)                                                                          \
  do {                                                                                           \
    if (threadIdx.x == 0) {                                                                      \
      atomicAdd(&g_iter_prof[4 * (k)], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - ip_t0)); \
      atomicAdd(&g_iter_prof[4 * (k) + 1], 1ull);                                                \
    }                                                                                            \
  } while (0)
#define AICP_IP_TAIL0 const uint64_t ip_t1 = __builtin_amdgcn_s_memrealtime()
#define AICP_IP_TAIL(k)                                                                          \
  do {                                                                                           \
    if (threadIdx.x == 0) {                                                                      \
      atomicAdd(&g_iter_prof[4 * (k) + 2], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - ip_t1)); \
      atomicAdd(&g_iter_prof[4 * (k) + 3], 1ull);                                                \
    }                                                                                            \
  } while (0)
#else
#define AICP_IP_T0 \
  do {             \
  } while (0)
#define AICP_IP_BODY(k) \
  do {                  \
  } while (0)
#define AICP_IP_TAIL0 \
  do {                \
  } while (0)
#define AICP_IP_TAIL(k) \
  do {                  \
  } while (0)
#endif

// Persistent waves with XCD-affine work: the slot space [0, total) is cut into kXcdGroups
// contiguous ranges (64-slot aligned) and group g is served only by blocks with
// blockIdx % 8 == g, which the dispatcher places on one XCD (MI355X_MICROARCH.md, workgroup
// dispatch: speed only, never correctness -- any placement still processes every slot exactly
// once). Consecutive slots belong to the same pair, so each XCD's 4 MiB L2 holds the trees of
// ~P/8 pairs instead of all P. A wave takes 64-slot chunks (one returning atomic each) and hands
// their slots to the lanes that need work in lane order, so a lane starts a new query as soon as
// its previous one completes.
// r06: a group's range is cut into kHeads contiguous parts with a head each (one 64-byte line
// apiece). One head served all ~1024 waves of a group: a word takes ~88 returning atomics per us
// (MI355X_MICROARCH.md, "dequeue"), so the last wave of a full-chip launch got its first chunk
// ~12 us after the first. A wave starts at head (its index in the group) mod kHeads and, when
// that part is exhausted, moves to a part of the same group still open (the exhausted parts are
// bits of one more word): the work stays on the group's XCD and every chunk is still served
// exactly once. (Measured and not kept: each wave's first chunk dealt by its index, the heads
// serving only the rest -- 86.8 against 70.6 us per C2 launch: a wave that starts late, beside
// another stream's kernel, holds its dealt chunk back; with heads the early waves take it.)
//   on_chunk(base)      wave-uniform, once per chunk, before its slots are handed out
//   fetch(slot, eng)    initialises a lane's query; false: the slot has no work
//   done(slot, eng)     consumes the result
// ctr: kGroupCtrs * kXcdGroups counters at kCtrStride words, zero at the launch
__device__ __forceinline__ uint32_t head_lo(uint32_t lo, uint32_t hi, uint32_t h) {
  return h >= (uint32_t)kHeads ? hi : lo + ((uint32_t)(((uint64_t)(hi - lo) * h) / kHeads) & ~63u);
}
template <class Eng, class OnChunk, class Fetch, class Done>
__device__ __forceinline__ void persistent_xcd(uint32_t total, uint32_t* ctr, float maxE2, float maxR2,
                                               const uint4* __restrict__ nodes, const float4* __restrict__ pts,
                                               OnChunk&& on_chunk, Fetch&& fetch, Done&& done) {
  const int lane = threadIdx.x & 63;
  const uint32_t g = blockIdx.x % kXcdGroups;
  // group g serves slots [lo, hi) (its data stays in its XCD's L2). (Chunks dealt to the groups
  // round-robin instead measured equal on C2 windows, r03.)
  const uint32_t lo = (uint32_t)(((uint64_t)total * g) / kXcdGroups) & ~63u;
  const uint32_t hi = g + 1 == kXcdGroups ? total : (uint32_t)(((uint64_t)total * (g + 1)) / kXcdGroups) & ~63u;
  uint32_t* gctr = ctr + g * kGroupCtrs * kCtrStride;
  // this wave's head: consecutive waves of the group on different heads
  uint32_t h = ((blockIdx.x / kXcdGroups) * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kHeads;
  h = __builtin_amdgcn_readfirstlane(h);
  Eng t;
  typename Eng::Stack fs;
  bool has = false;
  uint32_t pool = 0, pool_end = 0, my = 0;
  bool exhausted = false;
#if AICP_NN_PROF
  uint64_t pf_t = __builtin_amdgcn_s_memtime(), pf_fill = 0, pf_desc = 0, pf_buck = 0, pf_climb = 0, pf_rounds = 0,
           pf_lanes = 0;
#define AICP_PF(acc)                                    \
  do {                                                  \
    const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
    acc += now_ - pf_t;                                 \
    pf_t = now_;                                        \
  } while (0)
#else
#define AICP_PF(acc) \
  do {               \
  } while (0)
#endif
  for (;;) {
    for (;;) {
      const uint64_t needm = __ballot(!has);
      if (needm == 0 || exhausted) break;
      if (pool >= pool_end) {
        uint32_t base = 0, end = 0;
        for (;;) {
          const uint32_t hl = head_lo(lo, hi, h);
          end = head_lo(lo, hi, h + 1);
          uint32_t b = 0;
          if (lane == 0) b = atomicAdd(gctr + h * kCtrStride, 64u);
          base = hl + __builtin_amdgcn_readfirstlane(b);
          if (base < end) break;
          // part h is exhausted: mark it, go on with the next part still open
          uint32_t m = 0;
          if (lane == 0) m = atomicOr(gctr + kHeads * kCtrStride, 1u << h);
          m = __builtin_amdgcn_readfirstlane(m) | (1u << h);
          if (m == (1u << kHeads) - 1u) {
            exhausted = true;
            break;
          }
          h = (uint32_t)__builtin_ctz(~m & ((1u << kHeads) - 1u));
        }
        if (exhausted) break;
        pool = base;
        pool_end = min(base + 64u, end);
        if constexpr (std::is_invocable_v<OnChunk, uint32_t, Eng&>) on_chunk(base, t);  // may set uniform engine state
        else on_chunk(base);
      }
      const uint32_t rank = (uint32_t)__popcll(needm & ((1ull << lane) - 1ull));
      const uint32_t avail = pool_end - pool;
      if (!has && rank < avail) {
        my = pool + rank;
        has = fetch(my, t);
      }
      pool += min(avail, (uint32_t)__popcll(needm));
    }
    if (__ballot(has) == 0) break;
    AICP_PF(pf_fill);
#if AICP_NN_PROF
    ++pf_rounds;
    pf_lanes += __popcll(__ballot(has));
#endif
    if constexpr (is_coop<Eng>::value) {
#if AICP_NN_PREFMIN
      __shared__ uint16_t pm_lds[kPmDepth * kNNBlock];
      t.pm = pm_lds + threadIdx.x;
#endif
      if (has) t.descend();
      AICP_PF(pf_desc);
#if AICP_NN_COOP
      __shared__ float4 xch_all[kNNBlock];
      coop_bucket(t, has, pts, maxR2, xch_all + (threadIdx.x & ~63));
#endif
      if (has) {
#if AICP_NN_COOP
        t.bucket_tail(pts, maxR2);
#else
        t.bucket_lane(pts, maxR2);
#endif
      }
      AICP_PF(pf_buck);
#if AICP_NN_LDS_FRAMES > 0
      {  // used by the climb only
        __shared__ NnLdsFrame lds_frames[AICP_NN_LDS_FRAMES * kNNBlock];
        t.lf = lds_frames + threadIdx.x;
      }
#endif
      if (has && t.climb(fs, maxE2, maxR2)) {
        done(my, t);
        has = false;
      }
      AICP_PF(pf_climb);
    } else {
      if (has && t.advance(fs, maxE2, maxR2, nodes, pts)) {
        done(my, t);
        has = false;
      }
    }
  }
#if AICP_NN_PROF
  if (lane == 0) {
    atomicAdd(&g_nn_prof[0], (unsigned long long)pf_fill);
    atomicAdd(&g_nn_prof[1], (unsigned long long)pf_desc);
    atomicAdd(&g_nn_prof[2], (unsigned long long)pf_buck);
    atomicAdd(&g_nn_prof[3], (unsigned long long)pf_climb);
    atomicAdd(&g_nn_prof[4], (unsigned long long)pf_rounds);
    atomicAdd(&g_nn_prof[5], (unsigned long long)pf_lanes);
  }
#endif
}

// ------------------------------------------------------------------------------------------
// setup kernels
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void block_map(const BlockMap& m, int& pair, uint32_t& local) {
  pair = m.pair[blockIdx.x];
  local = m.start[blockIdx.x] + threadIdx.x;
}

__global__ __launch_bounds__(256) void k_prepare_read(BlockMap m, const PairDesc* __restrict__ pd,
                                                      const float4* __restrict__ raw,
                                                      float4* __restrict__ out) {
  int pair;
  uint32_t j;
  block_map(m, pair, j);
  const PairDesc& d = pd[pair];
  if (j >= d.n_read) return;
  const float4 p = raw[d.read_off + j];
  float o[3];
  apply4(d.Tinit, p.x, p.y, p.z, o);
  out[d.read_off + j] = make_float4(o[0], o[1], o[2], 1.f);
}

__global__ __launch_bounds__(256) void k_gather_ref(BlockMap m, const PairDesc* __restrict__ pd,
                                                    const float4* __restrict__ raw,
                                                    const int32_t* __restrict__ perm,
                                                    float4* __restrict__ bpts) {
  int pair;
  uint32_t j;
  block_map(m, pair, j);
  const PairDesc& d = pd[pair];
  if (j >= d.n_ref) return;
  const int32_t id = perm[d.ref_off + j];
  const float4 p = raw[d.ref_off + id];
  bpts[d.ref_off + j] =
      make_float4(p.x - d.mean[0], p.y - d.mean[1], p.z - d.mean[2], __int_as_float(id));
}

__global__ void k_init_state(int n_pairs, const PairDesc* __restrict__ pd, PairState* st) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  PairState& s = st[p];
  ident4(s.T);
  s.limit = 0.f;
  s.ratio = pd[p].ratio;
  s.active = 1;
  s.status = 0;
  s.iters = 0;
  s.converged = 0;
  s.kept = 0;
  s.n_finite = 0;
  s.hist_count = 1;
  s.degenerate = 0;
  s.inlier_ratio = 0.f;
  s.overlap = -1.f;
  s.touched_pts = 0;
  s.touched_nodes = 0;
  for (int i = 0; i < 3; ++i) s.ovl_counts[i] = 0;
  s.ovl_err = 0;
  s.sel_b1 = 0;
  s.sel_r1 = 0;
  s.sel_miss = 0;
  quat_from_T(s.T, s.qh[0]);
  s.th[0][0] = s.th[0][1] = s.th[0][2] = 0.0;
}

// one workgroup (any size, whole waves): prefix of n_read over the pairs still active + zero the
// work counter
__device__ void active_list_body(int n_pairs, const PairDesc* __restrict__ pd, const PairState* __restrict__ st,
                                 ActiveList* al, uint32_t* ctr, uint32_t* host_n, uint64_t* done_sig,
                                 const uint64_t* ticket, float* outT, int src_pair) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t wcnt[16];
  __shared__ uint32_t carry_off, carry_cnt;
  __shared__ uint32_t r_off[1024];  // first slot of each entry of the current round
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nt = (int)blockDim.x, nw = nt >> 6;
  uint16_t* chunk = al_chunks(al);
  if (t == 0) carry_off = carry_cnt = 0;
  if (t < kXcdGroups * kGroupCtrs) ctr[t * kCtrStride] = 0;
  __syncthreads();
  for (int base = 0; base < n_pairs; base += nt) {
    const int p = base + t;
    const bool a = p < n_pairs && st[p].active;
    // each pair's slot range is padded to a multiple of 64: a 64-slot chunk of the NN work space
    // then belongs to one pair, whose parameters the wave keeps in scalar registers. (r04: each
    // XCD group serving the g-th eighth of every pair's Morton-ordered readings, so that a stream
    // window's XCD touches ~1/8 of the reference tree, measured equal on C2 (87 us per launch)
    // and 4 % slower on C5: the NN launch is bound by its queries' latency chains, not by L2 misses.)
    const uint32_t v = a ? (pd[p].n_read + 63u) & ~63u : 0u;
    uint32_t x = v, c = a ? 1u : 0u;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64), z = __shfl_up(c, off, 64);
      if (lane >= off) {
        x += y;
        c += z;
      }
    }
    if (lane == 63) {
      wsum[wave] = x;
      wcnt[wave] = c;
    }
    __syncthreads();
    const uint32_t e0 = carry_cnt, o0 = carry_off;  // this round's first entry and slot
    uint32_t bo = o0, bc = e0;
    for (int w = 0; w < wave; ++w) {
      bo += wsum[w];
      bc += wcnt[w];
    }
    uint32_t rn = 0, rs = 0;  // entries and slots of the whole round
    for (int w = 0; w < nw; ++w) {
      rn += wcnt[w];
      rs += wsum[w];
    }
    if (a) {
      const uint32_t e = bc + c - 1, o = bo + x - v;
      al->pair[e] = p;
      al->off[e] = o;
      const PairDesc& d = pd[p];
      al->ent[e] = NnEntry{o, d.n_read, d.read_off, d.tl_off, d.node_off, d.ref_off, p, 0u};
      r_off[e - e0] = o;
    }
    __syncthreads();
    // the chunk table of this round's entries: wave w fills entries w, w + nw, ...
    for (uint32_t i = (uint32_t)wave; i < rn; i += (uint32_t)nw) {
      const uint32_t c0 = r_off[i] >> 6, c1 = (i + 1 < rn ? r_off[i + 1] : o0 + rs) >> 6;
      for (uint32_t j = c0 + (uint32_t)lane; j < c1; j += 64) chunk[j] = (uint16_t)(e0 + i);
    }
    if (t == nt - 1) {
      carry_off = bo + x;
      carry_cnt = bc + c;
    }
    __syncthreads();
  }
  if (t == 0) {
    al->n = carry_cnt;
    al->total = carry_off;
    al->off[carry_cnt] = carry_off;
    // mapped host memory: the sequence's early-exit poll, read by the host without an event
    // (a system-scope store goes through to host memory; nothing else is published with it);
    // bit 31: pair src_pair is still active (the stream starts the next reference once it is not)
    const bool src_on = src_pair >= 0 && src_pair < n_pairs && st[src_pair].active;
    if (host_n)
      __hip_atomic_store(host_n, carry_cnt | (src_on ? 0x80000000u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // every pair has stopped: their corrections are final (k_finalize's arithmetic), and the
  // sequence's next reference, waiting on done_sig on another stream, may start now
  if (done_sig && carry_cnt == 0) {
    for (int p = t; p < n_pairs; p += nt) {
      float tmp[16];
      mul4(pd[p].Tmean, st[p].T, tmp);
      mul4(tmp, pd[p].Tinit, outT + 16 * (size_t)p);
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(done_sig, *ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(256) void k_active_list(int n_pairs, const PairDesc* __restrict__ pd,
                                                      const PairState* __restrict__ st,
                                                      ActiveList* al, uint32_t* ctr, uint32_t* host_n,
                                                      uint64_t* done_sig, const uint64_t* ticket, float* outT,
                                                      int src_pair) {
  active_list_body(n_pairs, pd, st, al, ctr, host_n, done_sig, ticket, outT, src_pair);
}

// The last workgroup to arrive at a per-pair (or per-group) counter runs the serial step that
// follows (fused ICP iteration, AICP_ICP_FUSE): every wave's stores complete, one lane releases
// them at agent scope and adds; the last one acquires before reading what the others wrote
// (cdna_hip_programming.md Guideline 16 / MI355X_MICROARCH.md: release fence, vmcnt wait, then
// the counter; acquire on the reading side). The counter is reset for the next launch.
__device__ __forceinline__ bool last_arrival(uint32_t* cnt, uint32_t n_expected) {
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = atomicAdd(cnt, 1u);
    const bool last = old + 1 == n_expected;
    if (last) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last ? 1u : 0u;
  }
  __syncthreads();
  return s_last != 0;
}

// ------------------------------------------------------------------------------------------
// SurfaceNormal: persistent kNN (ids) + uniform covariance / eigen pass
// ------------------------------------------------------------------------------------------
// slot = global reference index (bucket order, concatenated over pairs); pair by search over
// the pairs' ref_off (ascending).
__device__ __forceinline__ int pair_of_ref(const PairDesc* __restrict__ pd, int n_pairs, uint32_t s) {
  int lo = 0, hi = n_pairs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pd[mid].ref_off <= s) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <int K>
#ifndef AICP_KNN_WAVES
#define AICP_KNN_WAVES 0  // k_knn_ids: waves per SIMD to compile for (0: the compiler's choice)
#endif
#if AICP_KNN_WAVES > 0
#define AICP_KNN_ATTR __attribute__((amdgpu_waves_per_eu(AICP_KNN_WAVES)))
#else
#define AICP_KNN_ATTR
#endif
__global__ __launch_bounds__(256) AICP_KNN_ATTR void k_knn_ids(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd,
                                                 const uint4* __restrict__ nodes,
                                                 const int32_t* __restrict__ parent,
                                                 const float4* __restrict__ bpts,
                                                 int32_t* __restrict__ ids, uint32_t* ctr,
                                                 unsigned long long* touched) {
  // innermost far frames in LDS (the exact kNN nests far descents often; scratch frames are
  // written back to HBM): 4 blocks of 256 per CU at this kernel's VGPR count
  __shared__ LdsFrame knn_frames[(kKnnLdsFrames > 0 ? kKnnLdsFrames : 1) * kNNBlock];
  uint32_t tp = 0, tn = 0;
  int cur = -1;
  uint32_t cur_end = 0, cur_off = 0;
  persistent_xcd<Trav<K>>(
      total, ctr, 1.f, __builtin_inff(), nodes, bpts, [](uint32_t) {},
      [&](uint32_t s, Trav<K>& t) {
        if (cur < 0 || s < cur_off || s >= cur_end) {
          cur = pair_of_ref(pd, n_pairs, s);
          cur_off = pd[cur].ref_off;
          cur_end = cur_off + pd[cur].n_ref;
        }
        const PairDesc& d = pd[cur];
        t.nodes = nodes + d.node_off;
        t.pts = bpts + d.ref_off;
        const float4 q = bpts[s];
        t.reset(q.x, q.y, q.z);
        t.lf = knn_frames + threadIdx.x;
        t.nlf = kKnnLdsFrames;
        return true;
      },
      [&](uint32_t s, Trav<K>& t) {
#pragma unroll
        for (int i = 0; i < K; ++i) ids[(size_t)s * K + i] = (t.best.v[i] != __builtin_inff()) ? t.best.id[i] : -1;
        tp += t.tp;
        tn += t.tn;
      });
  if (touched) {  // touched points / inner nodes (the algorithmic bytes of the roofline), optional
    unsigned long long a = tp, b = tn;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o, 64);
      b += __shfl_xor(b, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&touched[0], a);
      atomicAdd(&touched[1], b);
    }
  }
}

// ---- k-NN of a tree's own points with one query per octet of lanes -------------------------
// libnabo recurseKnn (eps 0, the SurfaceNormal / pre-filter kNN) exactly as Trav<K>::advance
// walks it, but the traversal state is held identically by the 8 lanes of an octet and the
// k-best list (IndexHeapBruteForceVector, ascending, head = entry K-1) is spread over them:
// lane j holds entries [j*M, j*M + M). replaceHead's shift loop becomes, for every entry i at
// once, newA[i] = A[i-1] > v ? A[i-1] : (A[i] > v ? v : A[i]) (A[-1] = -inf), M selects per lane
// and one DPP move of the previous lane's last entry; for v >= head it changes nothing, so the
// `dist < head` test needs no broadcast. A bucket's points are loaded one per lane (one 128-byte
// run per octet) and their distances broadcast in order by ds_swizzle. Per query this issues a
// few hundred wave instructions with the octet's lanes all busy, against one lane doing K-long
// compare-shift chains: on a single 120k-point reference (the C2 stream's window) the kNN is
// bound by the longest query's latency, not by the chip's issue rate.
// far frames per query group kept in LDS (deeper ones in scratch): 24 per octet, 12 per quad
// (18 KB per 256-thread block either way: 8 blocks per CU)
template <int G>
struct GrpCfg {
  static constexpr int kFrames = G == 8 ? 24 : 12;
  static constexpr int kGroups = 256 / G;  // query groups per block
};

template <int K, int G>
struct OctBest {
  static constexpr int M = (K + G - 1) / G;
  float v[M];
  int32_t id[M];
};

__device__ __forceinline__ float oct_prev_f(float x) {  // lane l - 1's value (row_shr:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ int32_t oct_prev_i(int32_t x) {
  return __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
}
// lane (l & ~7) | I of the 32-lane half: ds_swizzle bit mode, and_mask 0x18, or_mask I
template <int I>
__device__ __forceinline__ float oct_bcast(float x) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x18 | (I << 5)));
}
// lane (l & ~3) | I: DPP quad_perm [I, I, I, I]
template <int I>
__device__ __forceinline__ float quad_bcast(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), I | (I << 2) | (I << 4) | (I << 6), 0xf, 0xf, false));
}
template <int I>
__device__ __forceinline__ float grp_bcast4(float x) { return quad_bcast<I>(x); }

template <int K, int G>
__device__ __forceinline__ void oct_insert(OctBest<K, G>& b, bool first_lane, float val, int32_t vid) {
  constexpr int M = OctBest<K, G>::M;
  float pv = oct_prev_f(b.v[M - 1]);
  int32_t pid = oct_prev_i(b.id[M - 1]);
  if (first_lane) pv = -__builtin_inff();
  float nv[M];
  int32_t ni[M];
  bool sh = pv > val;  // slot i's predecessor above val; pl of slot i is sh of slot i + 1
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const float a = i == 0 ? pv : b.v[i - 1];
    const int32_t ai = i == 0 ? pid : b.id[i - 1];
    const bool pl = b.v[i] > val;
    // a <= b.v[i] (ascending): the median of (a, b.v[i], val) is a if val < a, val if it lies
    // between, b.v[i] above (val is finite and not NaN: the caller filtered with `< head`)
    nv[i] = __builtin_amdgcn_fmed3f(a, b.v[i], val);
    ni[i] = sh ? ai : (pl ? vid : b.id[i]);
    sh = pl;
  }
#pragma unroll
  for (int i = 0; i < M; ++i) {
    b.v[i] = nv[i];
    b.id[i] = ni[i];
  }
}

// the distances of a bucket run of 8 points, in order, in every lane of the group: octets load
// one point per lane and broadcast by ds_swizzle; quads load two per lane (j, j + 4) and
// broadcast by DPP
template <int G>
__device__ __forceinline__ void grp_bucket_dists(const float4* __restrict__ pts, uint32_t base, uint32_t n, int j,
                                                 float q0, float q1, float q2, float (&dv)[8]) {
  auto dist_of = [&](uint32_t i) {
    float d = __builtin_inff();
    if (i < n) {
      const float4 p = pts[base + i];
      const float d0 = q0 - p.x, d1 = q1 - p.y, d2 = q2 - p.z;
      d = 0.f;
      d += d0 * d0;
      d += d1 * d1;
      d += d2 * d2;
    }
    return d;
  };
  if constexpr (G == 8) {
    const float d = dist_of((uint32_t)j);
    dv[0] = oct_bcast<0>(d);
    dv[1] = oct_bcast<1>(d);
    dv[2] = oct_bcast<2>(d);
    dv[3] = oct_bcast<3>(d);
    dv[4] = oct_bcast<4>(d);
    dv[5] = oct_bcast<5>(d);
    dv[6] = oct_bcast<6>(d);
    dv[7] = oct_bcast<7>(d);
  } else {
    const float da = dist_of((uint32_t)j), db = dist_of((uint32_t)j + 4);
    dv[0] = quad_bcast<0>(da);
    dv[1] = quad_bcast<1>(da);
    dv[2] = quad_bcast<2>(da);
    dv[3] = quad_bcast<3>(da);
    dv[4] = quad_bcast<0>(db);
    dv[5] = quad_bcast<1>(db);
    dv[6] = quad_bcast<2>(db);
    dv[7] = quad_bcast<3>(db);
  }
}

template <int K, int G>
__global__ __launch_bounds__(256) void k_knn_oct(int n_pairs, uint32_t total, const PairDesc* __restrict__ pd,
                                                 const uint4* __restrict__ nodes_all,
                                                 const float4* __restrict__ bpts, int32_t* __restrict__ ids,
                                                 unsigned long long* touched) {
  constexpr int M = OctBest<K, G>::M;
  constexpr int kHeadLane = (K - 1) / M, kHeadSlot = (K - 1) % M;
  constexpr int kFrames = GrpCfg<G>::kFrames, kGroups = GrpCfg<G>::kGroups;
  __shared__ LdsFrame oframes[kFrames * kGroups];
  const int lane = threadIdx.x & 63, j = lane & (G - 1), grp = threadIdx.x / G;  // grp: the block's group
  const uint32_t s = (blockIdx.x * 256u + threadIdx.x) / G;                          // the group's query
  const bool live = s < total;
  uint32_t tp = 0, tn = 0;
  if (live) {
    const int pair = pair_of_ref(pd, n_pairs, s);
    const PairDesc& d = pd[pair];
    const uint4* nodes = nodes_all + d.node_off;
    const float4* pts = bpts + d.ref_off;
    const float4 qq = bpts[s];
    const float q0 = qq.x, q1 = qq.y, q2 = qq.z;
    OctBest<K, G> best;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      best.v[i] = __builtin_inff();
      best.id[i] = -1;
    }
    float head = __builtin_inff();
    float off0 = 0.f, off1 = 0.f, off2 = 0.f, rd = 0.f, minFar;
    int32_t n = 0, start = 0, sp = 0;
    FarStack fs;
    LdsFrame* lf = oframes + grp;
    const uint2* nodes2 = reinterpret_cast<const uint2*>(nodes);
    for (;;) {
      // descent (Trav<K>::advance)
      minFar = __builtin_inff();
      uint2 nd = nodes2[2 * n];
      int32_t pl = -1;
      while ((nd.y & 3u) != kLeaf) {
        const uint32_t cd = nd.y & 3u;
        const float no = sel3(cd, q0, q1, q2) - __uint_as_float(nd.x);
        const float oc = sel3(cd, off0, off1, off2);
        const float rdf = rd + (-oc * oc + no * no);
        minFar = fminf(minFar, rdf);
        pl = n;
        n = (no > 0.f) ? (int32_t)(nd.y >> 2) : n + 1;
        ++tn;
        nd = nodes2[2 * n];
      }
      if (pl < 0) pl = (int32_t)nodes[n].z;
      // bucket: runs of 8 points, their distances in every lane of the group, in order
      {
        const uint32_t b0 = nd.y >> 2, cnt = nd.x;
        for (uint32_t c = 0; c < cnt; c += 8) {
          float dv[8];
          grp_bucket_dists<G>(pts, b0 + c, cnt - c, j, q0, q1, q2, dv);
          // candidates below the head as it stood before this run (libnabo's `dist < head`; a
          // candidate the earlier insertions of the run pushed above the head is a no-op)
          uint32_t m8 = 0;
#pragma unroll
          for (int i = 0; i < 8; ++i) m8 |= (dv[i] < head ? 1u : 0u) << i;
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if ((m8 >> i) & 1u) oct_insert<K, G>(best, j == 0, dv[i], (int32_t)(b0 + c + i));
          head = __shfl(best.v[kHeadSlot], (lane & ~(G - 1)) | kHeadLane, 64);
        }
        tp += cnt;
      }
      // climb to the next far descent (or the end of the query)
      int32_t cnode = n, pc = pl;
      bool done = false;
      if (!(minFar * 1.f < head)) cnode = start;
      for (;;) {
        if (cnode == start) {
          if (sp == 0) {
            done = true;
            break;
          }
          --sp;
          FarFrame f;
          if (sp < kFrames) {
            const LdsFrame g = lf[sp * kGroups];
            f = FarFrame{g.Pcd, g.rd, g.old, g.mn, g.start, g.Pcd & 0x3fffffff, g.PP, 0};
          } else {
            f = fs.f[sp];
          }
          const uint32_t pcd = (uint32_t)f.F >> 30;
          rd = f.rd;
          const float old = f.old;
          if (pcd == 0) off0 = old;
          else if (pcd == 1) off1 = old;
          else off2 = old;
          minFar = f.mn;
          start = f.start;
          cnode = f.P;
          pc = f.PP;
          if (!(minFar * 1.f < head)) cnode = start;
          continue;
        }
        const int32_t p = pc;
        const uint4 pn = nodes[p];
        const uint32_t cd = pn.y & 3u;
        const float no = sel3(cd, q0, q1, q2) - __uint_as_float(pn.x);
        const float oc = sel3(cd, off0, off1, off2);
        const float rdf = rd + (-oc * oc + no * no);
        if (rdf * 1.f < head) {
          const int32_t far = (no > 0.f) ? p + 1 : (int32_t)(pn.y >> 2);
          if (sp < kFrames) {
            if (j == 0)
              lf[sp * kGroups] = LdsFrame{(int32_t)((uint32_t)p | (cd << 30)), rd, oc, minFar, start, (int32_t)pn.z};
          } else {
            fs.f[sp] = FarFrame{(int32_t)((uint32_t)far | (cd << 30)), rd, oc, minFar, start, p, (int32_t)pn.z, 0};
          }
          ++sp;
          if (cd == 0) off0 = no;
          else if (cd == 1) off1 = no;
          else off2 = no;
          rd = rdf;
          n = far;
          start = far;
          break;
        }
        cnode = p;
        pc = (int32_t)pn.z;
      }
      if (done) break;
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int e = j * M + i;
      if (e < K) ids[(size_t)s * K + e] = best.v[i] != __builtin_inff() ? best.id[i] : -1;
    }
  }
  if (touched) {
    unsigned long long a = (live && j == 0) ? tp : 0, b = (live && j == 0) ? tn : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o, 64);
      b += __shfl_xor(b, o, 64);
    }
    if (lane == 0) {
      atomicAdd(&touched[0], a);
      atomicAdd(&touched[1], b);
    }
  }
}

template <int K>
__global__ __launch_bounds__(256) void k_normals_from_ids(int n_pairs, uint32_t total,
                                                          const PairDesc* __restrict__ pd, PairState* st,
                                                          const float4* __restrict__ bpts,
                                                          const int32_t* __restrict__ ids,
                                                          float4* __restrict__ bnrm) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= total) return;
  const int pair = pair_of_ref(pd, n_pairs, s);
  const float4* P = bpts + pd[pair].ref_off;
  int32_t nb[K];
#pragma unroll
  for (int i = 0; i < K; ++i) nb[i] = ids[(size_t)s * K + i];
  // d = neighbours with finite distance in heap order; mean; NN = d - mean; C = NN NN^T / k
  float sx = 0.f, sy = 0.f, sz = 0.f;
  int kk = 0;
#pragma unroll
  for (int i = 0; i < K; ++i)
    if (nb[i] >= 0) {
      const float4 p = P[nb[i]];
      sx += p.x;
      sy += p.y;
      sz += p.z;
      ++kk;
    }
  const float fk = (float)kk;
  const float mx = sx / fk, my = sy / fk, mz = sz / fk;
  double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
#pragma unroll
  for (int i = 0; i < K; ++i)
    if (nb[i] >= 0) {
      const float4 p = P[nb[i]];
      const double a = (double)(p.x - mx), b = (double)(p.y - my), c = (double)(p.z - mz);
      c00 += a * a;
      c01 += a * b;
      c02 += a * c;
      c11 += b * b;
      c12 += b * c;
      c22 += c * c;
    }
  const double C[9] = {c00 / kk, c01 / kk, c02 / kk, c01 / kk, c11 / kk,
                       c12 / kk, c02 / kk, c12 / kk, c22 / kk};
  float nrm[3];
  const bool dg = normal_from_cov(C, nrm);
  bnrm[s] = make_float4(nrm[0], nrm[1], nrm[2], 0.f);
  if (dg) atomicAdd(&st[pair].degenerate, 1);
}

// ------------------------------------------------------------------------------------------
// ICP iteration
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void apply_cols(const float4& c0, const float4& c1, const float4& c2, const float4& c3,
                                           float x, float y, float z, float& o0, float& o1, float& o2) {
  // same operation order as apply4: ((T(r,0) x + T(r,1) y) + T(r,2) z) + T(r,3)
  o0 = c0.x * x;
  o0 += c1.x * y;
  o0 += c2.x * z;
  o0 += c3.x;
  o1 = c0.y * x;
  o1 += c1.y * y;
  o1 += c2.y * z;
  o1 += c3.y;
  o2 = c0.z * x;
  o2 += c1.z * y;
  o2 += c2.z * z;
  o2 += c3.z;
}

// NN kernel: also stores the query's touch counts (inner nodes << 16 | bucket points, each
// saturated at 65535) for the reduce kernel to sum per pair without atomics.
template <class Eng>
#ifndef AICP_NN_WAVES
#define AICP_NN_WAVES 8  // waves per SIMD the NN kernel is compiled for (VGPR budget 512 / waves)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(AICP_NN_WAVES))) void k_icp_nn(
                                                const PairDesc* __restrict__ pd, const PairState* __restrict__ st,
                                                const ActiveList* __restrict__ al,
                                                const float4* __restrict__ read_c,
                                                const uint4* __restrict__ nodes,
                                                const int32_t* __restrict__ parent,
                                                const float4* __restrict__ bpts, const uint2* __restrict__ ptl,
                                                int32_t* __restrict__ match,
                                                float* __restrict__ d2out, uint32_t* __restrict__ touched,
                                                uint32_t* ctr, IcpParams prm) {
  const uint32_t total = al->total;
  if (total == 0) return;
#if AICP_XCD_PROF || AICP_QLAT_PROF
  const uint64_t xt0 = __builtin_amdgcn_s_memrealtime();
#endif
#if AICP_QLAT_PROF
  uint32_t qt0 = 0;
  __shared__ uint32_t qh[512];  // block-local histograms, flushed once at the end
  for (int i = threadIdx.x; i < 512; i += blockDim.x) qh[i] = 0;
  __syncthreads();
#endif
  // chunk context: wave-uniform (scalar registers)
  uint32_t c_lo = 0, c_n = 0, c_read = 0, c_node = 0, c_ref = 0;
  int c_pair = 0;
  uint32_t qidx = 0;
#if AICP_XCD_PROF
  uint64_t xc_cost = 0;  // this lane's queries and their inner nodes + bucket points
#endif
  persistent_xcd<Eng>(
      total, ctr, prm.maxE2, prm.maxR2, nodes, bpts,
      [&](uint32_t base, Eng& t) {
        if constexpr (std::is_same<Eng, Trav2C>::value) t.bind_batch(nodes, ptl);
        // the chunk's entry (u16 table, read as its aligned dword), then the entry: two
        // dependent scalar loads
        const uint32_t c = base >> 6;
        const uint32_t w2 = reinterpret_cast<const uint32_t*>(al_chunks(al))[c >> 1];
        const uint32_t e = __builtin_amdgcn_readfirstlane((w2 >> ((c & 1u) << 4)) & 0xffffu);
        const NnEntry& en = al->ent[e];
        c_pair = __builtin_amdgcn_readfirstlane(en.pair);
        c_lo = __builtin_amdgcn_readfirstlane(en.off);
        c_n = __builtin_amdgcn_readfirstlane(en.n_read);
        c_read = __builtin_amdgcn_readfirstlane(en.read_off);
        if constexpr (is_coop<Eng>::value) c_node = __builtin_amdgcn_readfirstlane(en.tl_off);
        else c_node = __builtin_amdgcn_readfirstlane(en.node_off);
        c_ref = __builtin_amdgcn_readfirstlane(en.ref_off);
      },
      [&](uint32_t s, Eng& t) {
        const uint32_t j = s - c_lo;
        if (j >= c_n) return false;  // padding slot
        if constexpr (is_coop<Eng>::value) t.bind(nodes, ptl, c_node, c_ref);
        else t.bind(nodes, bpts, c_node, c_ref);
        qidx = c_read + j;
        const float4 r = read_c[qidx];
        const float4* Tp = reinterpret_cast<const float4*>(st[c_pair].T);
        float q0, q1, q2;
        apply_cols(Tp[0], Tp[1], Tp[2], Tp[3], r.x, r.y, r.z, q0, q1, q2);
        t.reset(q0, q1, q2);
#if AICP_QLAT_PROF
        qt0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
        return true;
      },
      [&](uint32_t, Eng& t) {
        match[qidx] = t.res_id();
        d2out[qidx] = t.res_d2();
        touched[qidx] = (min(t.tn, 65535u) << 16) | min(t.tp, 65535u);
#if AICP_XCD_PROF
        xc_cost += (1ull << 40) + t.tn + t.tp;
#endif
#if AICP_QLAT_PROF
        const uint32_t qt1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
        atomicAdd(&qh[min((qt1 - qt0) / 100, 255u)], 1u);
        atomicAdd(&qh[256 + min((qt1 - (uint32_t)xt0) / 100, 255u)], 1u);
#endif
      });
#if AICP_QLAT_PROF
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += blockDim.x)
    if (qh[i]) atomicAdd(&g_qlat[i], (unsigned long long)qh[i]);
#endif
#if AICP_XCD_PROF
  // per launch slot and XCD group: earliest wave start, latest wave end (100 MHz clock)
  const uint64_t xt1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0 && prm.prof_slot < 64) {
    unsigned long long* r = g_xcd_prof + (prm.prof_slot * kXcdGroups + blockIdx.x % kXcdGroups) * 2;
    atomicMin(&r[0], (unsigned long long)xt0);
    atomicMax(&r[1], (unsigned long long)xt1);
  }
  {  // the block's query count and cost, one add per block
    __shared__ unsigned long long xc_sum;
    if (threadIdx.x == 0) xc_sum = 0;
    __syncthreads();
    atomicAdd(&xc_sum, (unsigned long long)xc_cost);
    __syncthreads();
    if (threadIdx.x == 0 && prm.prof_slot < 64)
      atomicAdd(&g_xcd_cost[prm.prof_slot * kXcdGroups + blockIdx.x % kXcdGroups], xc_sum);
  }
#endif
}

// rank k -> (bin, k - count before bin) over h[nb] (nb a multiple of the block size, whole
// waves); result in res[0..1]
__device__ void block_find_rank(const uint32_t* h, int nb, uint32_t k, uint32_t* res, uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = nb / (int)blockDim.x;
  uint32_t local = 0;
  for (int i = 0; i < per; ++i) local += h[t * per + i];
  uint32_t x = local;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  uint32_t before = 0;
  for (int w = 0; w < wave; ++w) before += wsum[w];
  const uint32_t excl = before + x - local;
  if (local && excl <= k && k < excl + local) {
    uint32_t run = excl;
    for (int i = 0; i < per; ++i) {
      const uint32_t c = h[t * per + i];
      if (k < run + c) {
        res[0] = (uint32_t)(t * per + i);
        res[1] = k - run;
        break;
      }
      run += c;
    }
  }
  __syncthreads();
}

constexpr uint32_t kInfBits = 0x7f800000u;

// ---- TrimmedDist limit = exact k-th smallest finite d2, k = (size_t)(float(n) * ratio)
// (getDistsQuantile), as a radix select on the float bits (non-negative floats
// order like their bit patterns) spread over the whole chip:
//   k_sel_hist    per 4096 readings: LDS histogram of digit 1 (bits 31..21) -> global
//   k_sel_find1   per pair: n = #finite, k, bin b1 holding rank k, rank r1 inside it
//   k_sel_compact per 4096 readings: the values of bin b1 -> per-pair candidate list
//   k_sel_final   per pair: digits 2 (bits 20..10) and 3 (bits 9..0) over the candidates
__global__ __launch_bounds__(256) void k_sel_hist(BlockMap m, const PairDesc* __restrict__ pd,
                                                  const PairState* __restrict__ st, const float* __restrict__ d2,
                                                  uint32_t* __restrict__ hist1) {
  const int pair = m.pair[blockIdx.x];
  if (!st[pair].active) return;
  __shared__ uint32_t h[2][kHistBins];  // one sub-histogram per wave pair (LDS atomic conflicts)
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2 * kHistBins / 256; ++i) (&h[0][0])[t + 256 * i] = 0;
  const PairDesc& d = pd[pair];
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  const uint32_t j0 = m.start[blockIdx.x];
  uint32_t v[kSelPerThread];
#pragma unroll
  for (int u = 0; u < kSelPerThread; ++u) {
    const uint32_t j = j0 + t + 256u * u;
    v[u] = j < d.n_read ? bits[j] : kInfBits;
  }
  __syncthreads();
  uint32_t* mine = h[t >> 7];
#pragma unroll
  for (int u = 0; u < kSelPerThread; ++u)
    if (v[u] != kInfBits) atomicAdd(&mine[v[u] >> 21], 1u);
  __syncthreads();
  uint32_t* g = hist1 + (size_t)pair * kHistBins;
#pragma unroll
  for (int i = 0; i < kHistBins / 256; ++i) {
    const int b = t + 256 * i;
    const uint32_t c = h[0][b] + h[1][b];
    if (c) atomicAdd(&g[b], c);
  }
}

// per pair (one workgroup, any size): n = #finite, k, bin b1 holding rank k, rank r1 inside it;
// the global histogram is read (atomics wrote it; agent-scope loads) and zeroed for the next
// iteration. Returns false when the pair stopped (no finite distance).
// LDS scratch of the select's serial tails, passed in by the kernel so that one allocation serves
// every phase (separate __shared__ arrays in each inlined body added up: k_sel_fused had 65.8 KB
// per workgroup and ran at 2 waves per SIMD)
struct SelLds {
  uint32_t* h;     // kHistBins
  uint32_t* wsum;  // 16
  uint32_t* res;   // 2
  uint32_t* cl;    // cl_cap candidates (the final select's LDS copy)
  uint32_t cl_cap;
};

__device__ bool sel_find1_body(PairState& s, uint32_t* __restrict__ g, const SelLds& L) {
  uint32_t* h = L.h;
  uint32_t* wsum = L.wsum;
  uint32_t* res = L.res;
  const int t = threadIdx.x, lane = t & 63, nt = (int)blockDim.x;
  uint32_t v = 0;
  // eight agent-scope loads in flight per thread (each is a fabric round trip), then the stores
  for (int i0 = 0; i0 < kHistBins; i0 += 8 * nt) {
    uint32_t c[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * nt + t;
      c[u] = i < kHistBins ? __hip_atomic_load(&g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * nt + t;
      if (i < kHistBins) {
        h[i] = c[u];
        g[i] = 0;  // ready for the next iteration
        v += c[u];
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) wsum[t >> 6] = v;
  __syncthreads();
  if (t == 0) {
    uint32_t n = 0;
    for (int w = 0; w < nt / 64; ++w) n += wsum[w];
    res[0] = n;
  }
  __syncthreads();
  const uint32_t n = res[0];
  __syncthreads();
  if (n == 0) {  // ConvergenceError("no outlier to filter")
    if (t == 0) {
      s.status = 1;
      s.active = 0;
    }
    return false;
  }
  const float ratio = s.ratio;
  uint32_t k;
  if (ratio == 1.0f) {
    k = n - 1;
  } else {
    const float kf = (float)n * ratio;
    k = (uint32_t)kf;
    if (k >= n) k = n - 1;
  }
  block_find_rank(h, kHistBins, k, res, wsum);
  if (t == 0) {
    s.sel_b1 = res[0];
    s.sel_r1 = res[1];
    s.n_finite = (int32_t)n;
  }
  return true;
}

__global__ __launch_bounds__(1024) void k_sel_find1(PairState* st, uint32_t* __restrict__ hist1) {
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  __shared__ uint32_t h[kHistBins], wsum[16], res[2];
  (void)sel_find1_body(s, hist1 + (size_t)pair * kHistBins, SelLds{h, wsum, res, nullptr, 0});
}

// a pair is done with this iteration; the group's last one builds the next active list
__device__ void pair_done(const IcpIterSync& y) {
  if (!last_arrival(y.pairs, y.al->n)) return;
  active_list_body(y.np, y.pd, y.st, y.al, y.ctr, y.host_n, y.done_sig, y.ticket, y.outT, y.src_pair);
}

// k_sel_hist + (last workgroup of the pair) k_sel_find1; a pair that stops here is done with
// the iteration. kT threads per workgroup over kNNBlock * kSelPerThread readings (two LDS
// sub-histograms, one per half of the workgroup); the tail reads the pair's global histogram.
// 256 threads: with 1024 the sub-histograms' atomic conflicts doubled the kernel (C2 r04,
// rocprofv3: 21.1 against 11.3 us).
template <int kT>
__global__ __launch_bounds__(kT) void k_sel_hist_f(BlockMap m, const PairDesc* __restrict__ pd, PairState* st,
                                                   const float* __restrict__ d2, uint32_t* __restrict__ hist1,
                                                   IcpIterSync y) {
  constexpr int kPer = kNNBlock * kSelPerThread / kT;
  AICP_IP_T0;
  const int pair = m.pair[blockIdx.x];
  if (!st[pair].active) return;
  __shared__ uint32_t h[2][kHistBins];  // one sub-histogram per half workgroup (LDS atomic conflicts)
  __shared__ uint32_t wsum[16], res[2];
  const int t = threadIdx.x;
  for (int i = t; i < 2 * kHistBins; i += kT) (&h[0][0])[i] = 0;
  const PairDesc& d = pd[pair];
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  const uint32_t j0 = m.start[blockIdx.x];
  uint32_t v[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t j = j0 + t + (uint32_t)kT * u;
    v[u] = j < d.n_read ? bits[j] : kInfBits;
  }
  __syncthreads();
  uint32_t* mine = h[t / (kT / 2)];
#pragma unroll
  for (int u = 0; u < kPer; ++u)
    if (v[u] != kInfBits) atomicAdd(&mine[v[u] >> 21], 1u);
  __syncthreads();
  uint32_t* g = hist1 + (size_t)pair * kHistBins;
  for (int b = t; b < kHistBins; b += kT) {
    const uint32_t c = h[0][b] + h[1][b];
    if (c) atomicAdd(&g[b], c);
  }
  const uint32_t nblk = (d.n_read + 256u * kSelPerThread - 1) / (256u * kSelPerThread);
  AICP_IP_BODY(0);
  if (!last_arrival(&y.sel1[pair], nblk)) return;
  AICP_IP_TAIL0;
  __syncthreads();  // (every thread's reads of the sub-histograms precede find1's writes to h[0])
  if (!sel_find1_body(st[pair], g, SelLds{h[0], wsum, res, nullptr, 0})) pair_done(y);
  AICP_IP_TAIL(0);
}
#ifndef AICP_SEL_HIST_THREADS
#define AICP_SEL_HIST_THREADS 256
#endif
constexpr int kSelHistThreads = AICP_SEL_HIST_THREADS;

__global__ __launch_bounds__(256) void k_sel_compact(BlockMap m, const PairDesc* __restrict__ pd,
                                                     const PairState* __restrict__ st, const float* __restrict__ d2,
                                                     uint32_t* __restrict__ cand, uint32_t* __restrict__ cand_cnt) {
  const int pair = m.pair[blockIdx.x];
  const PairState& s = st[pair];
  if (!s.active) return;
  __shared__ uint32_t wcount[4];
  __shared__ uint32_t base;
  const PairDesc& d = pd[pair];
  const uint32_t b1 = s.sel_b1;
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t j0 = m.start[blockIdx.x];
  uint32_t v[kSelPerThread];
#pragma unroll
  for (int u = 0; u < kSelPerThread; ++u) {
    const uint32_t j = j0 + t + 256u * u;
    v[u] = j < d.n_read ? bits[j] : kInfBits;
  }
  uint32_t mine = 0;  // this wave's hits
#pragma unroll
  for (int u = 0; u < kSelPerThread; ++u)
    mine += (uint32_t)__popcll(__ballot(v[u] != kInfBits && (v[u] >> 21) == b1));
  // one atomic per block (the per-pair counter is shared by ~30 blocks)
  if (lane == 0) wcount[w] = mine;
  __syncthreads();
  if (t == 0) {
    const uint32_t tot = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    base = tot ? atomicAdd(&cand_cnt[pair], tot) : 0u;
  }
  __syncthreads();
  if (!wcount[w]) return;
  uint32_t o = base;
  for (int k = 0; k < w; ++k) o += wcount[k];
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int u = 0; u < kSelPerThread; ++u) {
    const bool hit = v[u] != kInfBits && (v[u] >> 21) == b1;
    const uint64_t mk = __ballot(hit);
    if (hit) cand[d.read_off + o + (uint32_t)__popcll(mk & below)] = v[u];
    o += (uint32_t)__popcll(mk);
  }
}

// per pair (one workgroup, any size): digits 2 (bits 20..10) and 3 (bits 9..0) over the candidates.
// The candidates were written by the other workgroups (other XCDs: each load is a fabric round
// trip), so up to kFinalLds of them are read once, eight loads in flight per thread, into LDS and
// both passes run there (the passes over global memory took ~11 us of a C2 iteration, r03).
constexpr uint32_t kFinalLds = 8192;
// b1 / r1: digit 1's bin and the rank in it (s.sel_b1 / sel_r1; passed in, since in k_sel_fused
// they were just written by another thread of the workgroup)
__device__ void sel_final_body(PairState& s, uint32_t b1, uint32_t r1, const uint32_t* __restrict__ cv,
                               uint32_t* cand_cnt, const SelLds& L) {
  uint32_t* h = L.h;
  uint32_t* wsum = L.wsum;
  uint32_t* res = L.res;
  uint32_t* cl = L.cl;
  const int t = threadIdx.x, nt = (int)blockDim.x;
  const uint32_t c = __hip_atomic_load(cand_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool lds = c <= L.cl_cap;
  const uint32_t* src = lds ? cl : cv;
  if (lds) {
    for (uint32_t i0 = 0; i0 < c; i0 += 8u * (uint32_t)nt) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t i = i0 + (uint32_t)(u * nt + t);
        v[u] = i < c ? cv[i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t i = i0 + (uint32_t)(u * nt + t);
        if (i < c) cl[i] = v[u];
      }
    }
  }
  for (int i = t; i < kHistBins; i += nt) h[i] = 0;
  __syncthreads();
  for (uint32_t i = t; i < c; i += nt) atomicAdd(&h[(src[i] >> 10) & 2047u], 1u);
  __syncthreads();
  block_find_rank(h, kHistBins, r1, res, wsum);
  const uint32_t b2 = res[0], r2 = res[1];
  __syncthreads();
  for (int i = t; i < kHistBins; i += nt) h[i] = 0;
  __syncthreads();
  const uint32_t hi21 = (b1 << 11) | b2;
  for (uint32_t i = t; i < c; i += nt) {
    const uint32_t v = src[i];
    if ((v >> 10) == hi21) atomicAdd(&h[v & 1023u], 1u);
  }
  __syncthreads();
  block_find_rank(h, kHist3Bins, r2, res, wsum);
  if (t == 0) {
    s.limit = __uint_as_float((hi21 << 10) | res[0]);
    *cand_cnt = 0;  // ready for the next iteration
  }
}

__global__ __launch_bounds__(1024) void k_sel_final(const PairDesc* __restrict__ pd, PairState* st,
                                                    const uint32_t* __restrict__ cand, uint32_t* __restrict__ cand_cnt) {
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  __shared__ uint32_t h[kHistBins], wsum[16], res[2], cl[kFinalLds];
  sel_final_body(s, s.sel_b1, s.sel_r1, cand + pd[pair].read_off, cand_cnt + pair,
                 SelLds{h, wsum, res, cl, kFinalLds});
}

// k_sel_compact + (last workgroup of the pair) k_sel_final. kT threads per workgroup over the
// same kNNBlock * kSelPerThread readings of a block-map entry: with 1024 the final select's tail
// loads its ~6k candidates (written from every XCD) in one round of loads instead of three.
template <int kT>
__global__ __launch_bounds__(kT) void k_sel_compact_f(BlockMap m, const PairDesc* __restrict__ pd, PairState* st,
                                                      const float* __restrict__ d2, uint32_t* __restrict__ cand,
                                                      uint32_t* __restrict__ cand_cnt, IcpIterSync y) {
  constexpr int kPer = kNNBlock * kSelPerThread / kT, kW = kT / 64;
  AICP_IP_T0;
  const int pair = m.pair[blockIdx.x];
  PairState& s = st[pair];
  if (!s.active) return;
  __shared__ uint32_t wcount[kW];
  __shared__ uint32_t base;
  const PairDesc& d = pd[pair];
  const uint32_t b1 = s.sel_b1;
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t j0 = m.start[blockIdx.x];
  uint32_t v[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t j = j0 + t + (uint32_t)kT * u;
    v[u] = j < d.n_read ? bits[j] : kInfBits;
  }
  uint32_t mine = 0;  // this wave's hits
#pragma unroll
  for (int u = 0; u < kPer; ++u)
    mine += (uint32_t)__popcll(__ballot(v[u] != kInfBits && (v[u] >> 21) == b1));
  if (lane == 0) wcount[w] = mine;
  __syncthreads();
  if (t == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kW; ++k) tot += wcount[k];
    base = tot ? atomicAdd(&cand_cnt[pair], tot) : 0u;
  }
  __syncthreads();
  if (wcount[w]) {
    uint32_t o = base;
    for (int k = 0; k < w; ++k) o += wcount[k];
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const bool hit = v[u] != kInfBits && (v[u] >> 21) == b1;
      const uint64_t mk = __ballot(hit);
      if (hit) cand[d.read_off + o + (uint32_t)__popcll(mk & below)] = v[u];
      o += (uint32_t)__popcll(mk);
    }
  }
  const uint32_t nblk = (d.n_read + 256u * kSelPerThread - 1) / (256u * kSelPerThread);
  AICP_IP_BODY(1);
  if (!last_arrival(&y.sel2[pair], nblk)) return;
  AICP_IP_TAIL0;
  __shared__ uint32_t h[kHistBins], wsum[16], res[2], cl[kFinalLds];
  sel_final_body(s, s.sel_b1, s.sel_r1, cand + d.read_off, cand_cnt + pair, SelLds{h, wsum, res, cl, kFinalLds});
  AICP_IP_TAIL(1);
}
// the values of v[0, kPer) (one block-map entry of the pair, kT threads) whose digit 1 is b into
// the pair's candidate list: per-wave ballot counts, one atomic per workgroup on cand_cnt
template <int kT, int kPer>
__device__ __forceinline__ void sel_compact_bin(const uint32_t (&v)[kPer], uint32_t b, uint32_t* __restrict__ cv,
                                                uint32_t* cnt) {
  constexpr int kW = kT / 64;
  __shared__ uint32_t wcount[kW];
  __shared__ uint32_t base;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t mine = 0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) mine += (uint32_t)__popcll(__ballot(v[u] != kInfBits && (v[u] >> 21) == b));
  if (lane == 0) wcount[w] = mine;
  __syncthreads();
  if (t == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kW; ++k) tot += wcount[k];
    base = tot ? atomicAdd(cnt, tot) : 0u;
  }
  __syncthreads();
  if (wcount[w]) {
    uint32_t o = base;
    for (int k = 0; k < w; ++k) o += wcount[k];
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const bool hit = v[u] != kInfBits && (v[u] >> 21) == b;
      const uint64_t mk = __ballot(hit);
      if (hit) cv[o + (uint32_t)__popcll(mk & below)] = v[u];
      o += (uint32_t)__popcll(mk);
    }
  }
  __syncthreads();  // (wcount / base are rewritten by the next call)
}

// The whole select in one launch from the second ICP iteration on: k_sel_hist_f's histogram, and
// in the same pass the compaction of k_sel_compact_f for a guessed digit-1 bin, the pair's bin of
// the previous iteration (the trimmed limit moves little between iterations). The last workgroup
// of the pair runs find1; when the guess was the bin of the k-th value the candidates are already
// compacted and it runs the final select at once, otherwise it compacts that bin from the pair's
// distances itself first (slower, same candidates: the select is order-independent), so the
// limit is k_sel_hist_f + k_sel_compact_f's bit for bit either way.
// kCl: candidates the final select copies into LDS (beyond them it reads them from global memory).
// Launches of many workgroups (C5: 15k) take kCl = kHistBins: 16 KB of LDS per workgroup, the
// sub-histograms' space reused by both tails, 8 waves per SIMD; a few workgroups (the stream's
// window) take kFinalLds, whose tail then loads all of a pair's ~6k candidates into LDS once.
template <int kT, int kCl>
__global__ __launch_bounds__(kT) void k_sel_fused(BlockMap m, const PairDesc* __restrict__ pd, PairState* st,
                                                  const float* __restrict__ d2, uint32_t* __restrict__ hist1,
                                                  uint32_t* __restrict__ cand, uint32_t* __restrict__ cand_cnt,
                                                  IcpIterSync y) {
  constexpr int kPer = kNNBlock * kSelPerThread / kT;
  static_assert(kCl >= kHistBins, "the final select's histogram and candidates share the LDS");
  const int pair = m.pair[blockIdx.x];
  PairState& s = st[pair];
  if (!s.active) return;
  __shared__ uint32_t lds[kHistBins + kCl];  // sub-histograms (2 x kHistBins), then the tails' scratch
  __shared__ uint32_t wsum[16], res[2];
  uint32_t(*h)[kHistBins] = reinterpret_cast<uint32_t(*)[kHistBins]>(lds);
  const int t = threadIdx.x;
  for (int i = t; i < 2 * kHistBins; i += kT) (&h[0][0])[i] = 0;
  const PairDesc& d = pd[pair];
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  const uint32_t j0 = m.start[blockIdx.x];
  const uint32_t guess = s.sel_b1;  // the previous iteration's bin (find1 rewrites it after every block arrived)
  uint32_t v[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t j = j0 + t + (uint32_t)kT * u;
    v[u] = j < d.n_read ? bits[j] : kInfBits;
  }
  __syncthreads();
  uint32_t* mine = h[t / (kT / 2)];
#pragma unroll
  for (int u = 0; u < kPer; ++u)
    if (v[u] != kInfBits) atomicAdd(&mine[v[u] >> 21], 1u);
  __syncthreads();
  uint32_t* g = hist1 + (size_t)pair * kHistBins;
  for (int b = t; b < kHistBins; b += kT) {
    const uint32_t c = h[0][b] + h[1][b];
    if (c) atomicAdd(&g[b], c);
  }
  uint32_t* cv = cand + d.read_off;
  sel_compact_bin<kT, kPer>(v, guess, cv, cand_cnt + pair);
  const uint32_t nblk = (d.n_read + 256u * kSelPerThread - 1) / (256u * kSelPerThread);
  if (!last_arrival(&y.sel1[pair], nblk)) return;
  __syncthreads();  // (every thread's reads of the sub-histograms precede the tails' writes)
  const SelLds L{lds, wsum, res, lds + kHistBins, (uint32_t)kCl};
  if (!sel_find1_body(s, g, L)) {  // no finite distance: the pair stops (ConvergenceError)
    if (t == 0) cand_cnt[pair] = 0;
    pair_done(y);
    return;
  }
  // find1's bin and rank, written by thread 0: passed on through LDS (a global load of them
  // by another wave could hit a stale L1 line from the guess's load above)
  __shared__ uint32_t s_sel[2];
  if (t == 0) {
    s_sel[0] = s.sel_b1;
    s_sel[1] = s.sel_r1;
  }
  __syncthreads();
  const uint32_t b1 = s_sel[0], r1 = s_sel[1];
  if (b1 != guess) {  // missed: the candidates of bin b1 from all of the pair's distances
    if (t == 0) __hip_atomic_store(cand_cnt + pair, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (uint32_t jb = 0; jb < d.n_read; jb += (uint32_t)kT * kPer) {
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const uint32_t j = jb + t + (uint32_t)kT * u;
        v[u] = j < d.n_read ? bits[j] : kInfBits;
      }
      sel_compact_bin<kT, kPer>(v, b1, cv, cand_cnt + pair);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence();
    __syncthreads();
    if (t == 0) atomicAdd(&s.sel_miss, 1u);
  }
  sel_final_body(s, b1, r1, cv, cand_cnt + pair, L);
}

// The whole select of a pair in one workgroup, for batches of many pairs of at most kSelPairMax
// readings each (C5: 1024 pairs of ~60k): the pair's distances stay in registers, the digit-1
// histogram, find1, the compaction of the k-th value's bin and digits 2 and 3 all run in LDS. No
// global histogram atomics (C5's multi-workgroup select flushed up to 2048 bins per workgroup into
// the pair's global histogram at the memory side: 600-730 us per launch for 245 MB of distances)
// and no hand-off between workgroups. Same limit bit for bit (the k-th smallest value is unique).
constexpr int kSelPairThreads = 1024, kSelPairPer = 64;
constexpr uint32_t kSelPairMax = (uint32_t)kSelPairThreads * kSelPairPer;
constexpr uint32_t kSelPairCand = 12288;  // candidates kept in LDS (beyond: the pair's global slice)
__global__ __launch_bounds__(kSelPairThreads) void k_sel_pair(const PairDesc* __restrict__ pd, PairState* st,
                                                              const float* __restrict__ d2,
                                                              uint32_t* __restrict__ cand, IcpIterSync y) {
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  constexpr int kT = kSelPairThreads;
  __shared__ uint32_t h[2][kHistBins];
  __shared__ uint32_t cl[kSelPairCand];
  __shared__ uint32_t wsum[16], res[2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const PairDesc& d = pd[pair];
  const uint32_t n_read = d.n_read;
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  for (int i = t; i < 2 * kHistBins; i += kT) (&h[0][0])[i] = 0;
  uint32_t v[kSelPairPer];
#pragma unroll
  for (int u = 0; u < kSelPairPer; ++u) {
    const uint32_t j = (uint32_t)t + (uint32_t)kT * u;
    v[u] = j < n_read ? bits[j] : kInfBits;
  }
  __syncthreads();
  uint32_t* mine = h[t / (kT / 2)];
#pragma unroll
  for (int u = 0; u < kSelPairPer; ++u)
    if (v[u] != kInfBits) atomicAdd(&mine[v[u] >> 21], 1u);
  __syncthreads();
  uint32_t cnt = 0;
  for (int b = t; b < kHistBins; b += kT) {
    const uint32_t c = h[0][b] + h[1][b];
    h[0][b] = c;
    cnt += c;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  uint32_t n = 0;
  for (int k = 0; k < kT / 64; ++k) n += wsum[k];
  __syncthreads();  // (wsum is reused by block_find_rank)
  if (n == 0) {  // ConvergenceError("no outlier to filter"), as sel_find1_body
    if (t == 0) {
      s.status = 1;
      s.active = 0;
    }
    pair_done(y);
    return;
  }
  const float ratio = s.ratio;
  uint32_t k;
  if (ratio == 1.0f) {
    k = n - 1;
  } else {
    const float kf = (float)n * ratio;
    k = (uint32_t)kf;
    if (k >= n) k = n - 1;
  }
  block_find_rank(h[0], kHistBins, k, res, wsum);
  const uint32_t b1 = res[0], r1 = res[1];
  if (t == 0) {
    s.sel_b1 = b1;
    s.sel_r1 = r1;
    s.n_finite = (int32_t)n;
  }
  // the values of bin b1: counted per wave, then placed (LDS, or the pair's global slice when
  // more than kSelPairCand)
  uint32_t mine_n = 0;
#pragma unroll
  for (int u = 0; u < kSelPairPer; ++u) mine_n += (uint32_t)__popcll(__ballot(v[u] != kInfBits && (v[u] >> 21) == b1));
  __syncthreads();  // (block_find_rank's last reads of wsum / res precede the writes below)
  if (lane == 0) wsum[w] = mine_n;
  __syncthreads();
  uint32_t c = 0, o = 0;
  for (int q = 0; q < kT / 64; ++q) {
    if (q < w) o += wsum[q];
    c += wsum[q];
  }
  const bool lds = c <= kSelPairCand;
  uint32_t* dst = lds ? cl : cand + d.read_off;
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int u = 0; u < kSelPairPer; ++u) {
    const bool hit = v[u] != kInfBits && (v[u] >> 21) == b1;
    const uint64_t mk = __ballot(hit);
    if (hit) dst[o + (uint32_t)__popcll(mk & below)] = v[u];
    o += (uint32_t)__popcll(mk);
  }
  if (!lds) __threadfence_block();
  __syncthreads();
  // digits 2 (bits 20..10) and 3 (bits 9..0) over the candidates
  for (int i = t; i < kHistBins; i += kT) h[0][i] = 0;
  __syncthreads();
  for (uint32_t i = t; i < c; i += kT) atomicAdd(&h[0][(dst[i] >> 10) & 2047u], 1u);
  __syncthreads();
  block_find_rank(h[0], kHistBins, r1, res, wsum);
  const uint32_t b2 = res[0], r2 = res[1];
  __syncthreads();
  for (int i = t; i < kHistBins; i += kT) h[0][i] = 0;
  __syncthreads();
  const uint32_t hi21 = (b1 << 11) | b2;
  for (uint32_t i = t; i < c; i += kT) {
    const uint32_t x = dst[i];
    if ((x >> 10) == hi21) atomicAdd(&h[0][x & 1023u], 1u);
  }
  __syncthreads();
  block_find_rank(h[0], kHist3Bins, r2, res, wsum);
  if (t == 0) s.limit = __uint_as_float((hi21 << 10) | res[0]);
}

#ifndef AICP_SEL_COMPACT_THREADS
#define AICP_SEL_COMPACT_THREADS 1024
#endif
constexpr int kSelCompactThreads = AICP_SEL_COMPACT_THREADS;

// DPP lane moves of a double (both halves with the same control); lanes outside the
// pattern read 0 (bound_ctrl), which the sums below never use
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// the sum over the lane's row of 16 in a fixed order (quads, then rotations), valid in every
// lane of the row: DPP moves instead of LDS-crossbar shuffles
__device__ __forceinline__ double row_sum_d(double v) {
  v += dpp_d<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);  // quad_perm [2,3,0,1]
  v += dpp_d<0x124>(v); // row_ror:4
  v += dpp_d<0x128>(v); // row_ror:8
  return v;
}

// one reduce workgroup's partial sums (kRedCols) into its slab row
__device__ __forceinline__ void icp_reduce_body(BlockMap m, const PairDesc& d, const PairState& s,
                                                const float4* __restrict__ read_c, const int32_t* __restrict__ match,
                                                const float* __restrict__ d2, const uint32_t* __restrict__ touched,
                                                const float4* __restrict__ bpts, const float4* __restrict__ bnrm,
                                                double* __restrict__ slab) {
  float T[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) T[i] = s.T[i];
  const float limit = s.limit;
  double acc[kRedCols];
#pragma unroll
  for (int i = 0; i < kRedCols; ++i) acc[i] = 0.0;
  uint32_t tpts = 0, tnod = 0;
  // kReduceChunks chunks of kReducePerThread readings per thread (the block's reduction below
  // is paid once per kNNBlock * kReducePerThread * kReduceChunks readings). Per chunk: all
  // loads of the thread's readings first (independent), then the gathers of the kept ones,
  // then the arithmetic: two round trips instead of three per reading.
  for (int ch = 0; ch < kReduceChunks; ++ch) {
    const uint32_t base = m.start[blockIdx.x] + ch * kReducePerThread * kNNBlock;
    bool keep[kReducePerThread];
    int32_t pos[kReducePerThread];
    float4 r[kReducePerThread];
#pragma unroll
    for (int it = 0; it < kReducePerThread; ++it) {
      const uint32_t j = base + it * kNNBlock + threadIdx.x;
      keep[it] = false;
      pos[it] = 0;
      if (j < d.n_read) {
        const uint32_t tc = touched[d.read_off + j];
        tpts += tc & 0xFFFFu;
        tnod += tc >> 16;
        keep[it] = d2[d.read_off + j] <= limit;
        pos[it] = match[d.read_off + j];
        r[it] = read_c[d.read_off + j];
      }
    }
    float4 q[kReducePerThread], nr[kReducePerThread];
#pragma unroll
    for (int it = 0; it < kReducePerThread; ++it)
      if (keep[it]) {
        q[it] = bpts[d.ref_off + pos[it]];
        nr[it] = bnrm[d.ref_off + pos[it]];
      }
#pragma unroll
    for (int it = 0; it < kReducePerThread; ++it) {
      if (!keep[it]) continue;
      float p[3];
      apply4(T, r[it].x, r[it].y, r[it].z, p);
      const float4 n4 = nr[it];
      float F[6];
      F[0] = p[1] * n4.z - p[2] * n4.y;
      F[1] = p[2] * n4.x - p[0] * n4.z;
      F[2] = p[0] * n4.y - p[1] * n4.x;
      F[3] = n4.x;
      F[4] = n4.y;
      F[5] = n4.z;
      const float dl0 = p[0] - q[it].x, dl1 = p[1] - q[it].y, dl2 = p[2] - q[it].z;
      float dot = dl0 * n4.x;
      dot += dl1 * n4.y;
      dot += dl2 * n4.z;
      int c = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = a; b < 6; ++b) acc[c++] += (double)F[a] * (double)F[b];
#pragma unroll
      for (int a = 0; a < 6; ++a) acc[21 + a] += (double)F[a] * (double)dot;
      acc[27] += 1.0;
    }
  }
  acc[28] = (double)tpts;
  acc[29] = (double)tnod;
  // row sums (DPP) -> one partial per row of 16 lanes in LDS -> a fixed-order sum of the
  // block's rows (no cross-row shuffles)
  constexpr int kRows = kNNBlock / 16;
  __shared__ double part[kRows][kRedCols];
  const int lane = threadIdx.x & 63;
  const int row = threadIdx.x >> 4;
#pragma unroll
  for (int i = 0; i < kRedCols; ++i) {
    const double v = row_sum_d(acc[i]);
    if ((lane & 15) == 0) part[row][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < kRedCols) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < kRows; ++w) v += part[w][threadIdx.x];
    // the pair's partial rows start at red_blk_off (m may cover a subset of the pairs)
    const uint32_t row = d.red_blk_off + m.start[blockIdx.x] / (kNNBlock * kReducePerThread * kReduceChunks);
    slab[(size_t)row * kRedCols + threadIdx.x] = v;
  }
}

__global__ __launch_bounds__(kNNBlock) void k_icp_reduce(
    BlockMap m, const PairDesc* __restrict__ pd, const PairState* __restrict__ st,
    const float4* __restrict__ read_c, const int32_t* __restrict__ match,
    const float* __restrict__ d2, const uint32_t* __restrict__ touched, const float4* __restrict__ bpts,
    const float4* __restrict__ bnrm, double* __restrict__ slab) {
  AICP_IP_T0;
  const int pair = m.pair[blockIdx.x];
  const PairState& s = st[pair];
  if (!s.active) return;
  icp_reduce_body(m, pd[pair], s, read_c, match, d2, touched, bpts, bnrm, slab);
  AICP_IP_BODY(2);
}

// a double of lane src (wave-uniform src) on every lane
__device__ __forceinline__ double bcast_d(double v, int src) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// pivqr<6>'s rank (Eigen FullPivHouseholderQR: full pivoting, Householder steps, the rank
// threshold) by one wave, lane c < 6 holding column c. Every element sees the operations of the
// serial loops in their order (the pivot scan column-major with the first strict maximum, the
// reflector sums over rows in order, no contraction), so the rank is pivqr<6>'s. get(r, c):
// element (r, c) of A (a memory read: the column index is the lane's).
template <class Get>
__device__ int wave_pivqr_rank6(Get get) {
  constexpr int N = 6;
  const int lane = threadIdx.x & 63;
  const int c = lane < N ? lane : 0;
  double col[N];
#pragma unroll
  for (int r = 0; r < N; ++r) col[r] = get(r, c);
  const double prec = (double)kFltEps * N;
  int nonzero = N;
  double maxpivot = 0, biggest = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    // this lane's first strict maximum over rows k.., then the lanes k.. in order
    double bl = -1;
    int rl = k;
#pragma unroll
    for (int r = k; r < N; ++r) {
      const double v = fabs(col[r]);
      if (v > bl) {
        bl = v;
        rl = r;
      }
    }
    double bv = -1;
    int br = k, bc = k;
#pragma unroll
    for (int cc = k; cc < N; ++cc) {
      const double v = bcast_d(bl, cc);
      const int rr = __builtin_amdgcn_readlane(rl, cc);
      if (v > bv) {
        bv = v;
        br = rr;
        bc = cc;
      }
    }
    if (k == 0) biggest = bv;
    if (bv <= biggest * prec) {  // (wave-uniform)
      nonzero = k;
      break;
    }
    // rows k <-> br on the columns k.., then columns k <-> bc on all rows
    if (lane >= k && lane < N) {
      double xk = col[k], xb = xk;
#pragma unroll
      for (int r = k + 1; r < N; ++r) xb = r == br ? col[r] : xb;
#pragma unroll
      for (int r = k + 1; r < N; ++r)
        if (r == br) col[r] = xk;
      col[k] = xb;
    }
    if (bc != k) {
#pragma unroll
      for (int r = 0; r < N; ++r) {
        const double xk = bcast_d(col[r], k), xb = bcast_d(col[r], bc);
        col[r] = lane == k ? xb : (lane == bc ? xk : col[r]);
      }
    }
    // the reflector of column k (lane k's values, on every lane)
    double tailSq = 0;
#pragma unroll
    for (int r = k + 1; r < N; ++r) tailSq += col[r] * col[r];
    tailSq = bcast_d(tailSq, k);
    const double c0 = bcast_d(col[k], k);
    double beta, tau;
    const bool flat = tailSq <= kDblMin;
    if (flat) {
      tau = 0;
      beta = c0;
    } else {
      beta = sqrt(c0 * c0 + tailSq);
      if (c0 >= 0) beta = -beta;
      tau = (beta - c0) / beta;
    }
    const double den = c0 - beta;
    if (lane == k) {
#pragma unroll
      for (int r = k + 1; r < N; ++r) col[r] = flat ? 0.0 : col[r] / den;
      col[k] = beta;
    }
    if (fabs(beta) > maxpivot) maxpivot = fabs(beta);
    double v[N];
#pragma unroll
    for (int r = k + 1; r < N; ++r) v[r] = bcast_d(col[r], k);
    if (lane > k && lane < N) {
      double sum = col[k];
#pragma unroll
      for (int r = k + 1; r < N; ++r) sum += v[r] * col[r];
      sum *= tau;
      col[k] -= sum;
#pragma unroll
      for (int r = k + 1; r < N; ++r) col[r] -= sum * v[r];
    }
  }
  const double thr = fabs(maxpivot) * ((double)kFltEps * N);
  int rank = 0;
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (i < nonzero) rank += fabs(bcast_d(col[i], i)) > thr ? 1 : 0;
  return rank;
}

// llt_solve<6>(M, 6, b, x) by one wave, lane i holding row i of L (every element sees the serial
// loops' operations in their order). get(r, c): element (r, c) of M; b on every lane. Returns
// false where llt_solve would (a non-positive pivot); x on every lane.
template <class Get>
__device__ bool wave_llt_solve6(Get get, const double* b, double* x) {
  constexpr int N = 6;
  const int lane = threadIdx.x & 63;
  const int i = lane < N ? lane : 0;
  double L[N];
#pragma unroll
  for (int k = 0; k < N; ++k) L[k] = 0;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double Lj[N];  // row j of L so far (lane j's)
#pragma unroll
    for (int k = 0; k < j; ++k) Lj[k] = bcast_d(L[k], j);
    double d = get(j, j);
#pragma unroll
    for (int k = 0; k < j; ++k) d -= Lj[k] * Lj[k];
    if (!(d > 0)) ok = false;
    const double ljj = sqrt(d);
    if (lane == j) L[j] = ljj;
    if (lane > j && lane < N) {
      double sum = get(i, j);
#pragma unroll
      for (int k = 0; k < j; ++k) sum -= L[k] * Lj[k];
      L[j] = sum / ljj;
    }
  }
  if (!ok) return false;
  double y[N];
#pragma unroll
  for (int r = 0; r < N; ++r) {
    double Lr[N];
#pragma unroll
    for (int k = 0; k <= r; ++k) Lr[k] = bcast_d(L[k], r);
    double sum = b[r];
#pragma unroll
    for (int k = 0; k < r; ++k) sum -= Lr[k] * y[k];
    y[r] = sum / Lr[r];
  }
#pragma unroll
  for (int r = N - 1; r >= 0; --r) {
    double sum = y[r];
#pragma unroll
    for (int k = r + 1; k < N; ++k) sum -= bcast_d(L[r], k) * x[k];
    x[r] = sum / bcast_d(L[r], r);
  }
  return true;
}

// A x = b of the point-to-plane step from the reduced sums (upper triangle, then the rhs)
__device__ __forceinline__ void normal_system(const double* tot, double* A, double* b) {
  int c = 0;
  for (int a = 0; a < 6; ++a)
    for (int bb = a; bb < 6; ++bb) {
      A[a * 6 + bb] = tot[c];
      A[bb * 6 + a] = tot[c];
      ++c;
    }
  for (int a = 0; a < 6; ++a) b[a] = -tot[21 + a];
}

// the serial part of an ICP update (one lane): solve, compose, checkers
// x_full: the LLT solution when the pivoted-QR rank is full (solve6's first path, computed by
// two waves side by side in icp_update_body), or nullptr: solve6 here
__device__ void update_serial(const PairDesc& d, PairState& s, const double* tot, const IcpParams& prm,
                              const double* x_full) {
  s.touched_pts += (uint64_t)tot[28];
  s.touched_nodes += (uint64_t)tot[29];
  const int32_t kept = (int32_t)tot[27];
  s.kept = kept;
  if (kept == 0) {  // ConvergenceError("no point to minimize")
    s.status = 1;
    s.active = 0;
    return;
  }
  double xd[6];
  if (x_full) {
    for (int a = 0; a < 6; ++a) xd[a] = x_full[a];
  } else {
    double A[36], b[6];
    normal_system(tot, A, b);
    solve6(A, b, xd);
  }
  float x[6];
  for (int a = 0; a < 6; ++a) x[a] = (float)xd[a];
  float dT[16];
  delta_transform(x, dT);
  mul4(dT, s.T, s.T);
  s.inlier_ratio = (float)((double)(float)kept / (double)d.n_read);
  // checkers (YAML order): Counter, then Differential. The new T_iter is applied to the reading
  // at the start of the next iteration (or, inside the final T, to the output reading), where
  // RigidTransformation::checkParameters throws TransformationError on |1 - det R| > 0.001.
  if (!rigid_ok(s.T)) {
    s.iters += 1;
    s.status = 5;
    s.active = 0;
    return;
  }
  bool iterate = true;
  s.iters += 1;
  if (s.iters >= prm.max_iter) iterate = false;
  const int h = s.hist_count % kHistRing;
  quat_from_T(s.T, s.qh[h]);
  for (int i = 0; i < 3; ++i) s.th[h][i] = (double)s.T[12 + i];
  if (s.hist_count >= 1) {  // entry i = hist_count against entry i - 1
    const int bprev = (s.hist_count - 1) % kHistRing;
    s.dq[h] = fabs(quat_angdist(s.qh[h], s.qh[bprev]));
    const double dx = s.th[h][0] - s.th[bprev][0];
    const double dy = s.th[h][1] - s.th[bprev][1];
    const double dz = s.th[h][2] - s.th[bprev][2];
    s.dt[h] = sqrt(dx * dx + dy * dy + dz * dz);
  }
  s.hist_count += 1;
  const int sz = s.hist_count;
  if (sz > prm.smooth) {
    double cv0 = 0, cv1 = 0;
    for (int i = sz - 1; i >= sz - prm.smooth; --i) {
      const int a = i % kHistRing;
      cv0 += s.dq[a];
      cv1 += s.dt[a];
    }
    cv0 /= prm.smooth;
    cv1 /= prm.smooth;
    if (cv0 != cv0 || cv1 != cv1) {
      s.status = 1;
      s.active = 0;
      return;
    }
    if (cv0 < (double)prm.min_rot && cv1 < (double)prm.min_trans) {
      if (iterate) s.converged = 1;
      iterate = false;
    }
  }
  s.active = iterate ? 1 : 0;
}

// one pair's update by a 256-thread workgroup: its slab rows summed (thread t sums column
// t % kRedCols over rows t / kRedCols + 8 k -- independent loads, contiguous across the block --
// then a fixed-order sum of the 8 groups), then update_serial on lane 0
__device__ void icp_update_body(const PairDesc& d, PairState& s, const double* __restrict__ slab,
                                const IcpParams& prm) {
  constexpr int kGroups = 256 / kRedCols;
  __shared__ double part[kGroups][kRedCols];
  __shared__ double tot[kRedCols];
  const int t = threadIdx.x;
  if (t < kGroups * kRedCols) {
    const int g = t / kRedCols, c = t - g * kRedCols;
    const double* col = slab + (size_t)d.red_blk_off * kRedCols + c;
    double v = 0.0;
    // rows g, g + kGroups, ... in order; 16 loads in flight (the rows were written by the reduce
    // workgroups on every XCD: each load is a fabric round trip)
    for (uint32_t r0 = g; r0 < d.n_red_blk; r0 += 16u * kGroups) {
      double x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const uint32_t r = r0 + (uint32_t)u * kGroups;
        x[u] = r < d.n_red_blk ? col[(size_t)r * kRedCols] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (r0 + (uint32_t)u * kGroups < d.n_red_blk) v += x[u];
    }
    part[g][c] = v;
  }
  __syncthreads();
  if (t < kRedCols) {
    double v = part[0][t];
#pragma unroll
    for (int g = 1; g < kGroups; ++g) v += part[g][t];
    tot[t] = v;
  }
  __syncthreads();
  // solve6's full-rank path with its two halves side by side: wave 0 the pivoted-QR rank, wave 1
  // the LLT solve (each ~half of the serial solve); a rank below 6 or a failed LLT falls back
  // to solve6 on lane 0
  __shared__ int rank_llt[2];
  __shared__ double xs[6];
  auto tri = [&](int r, int c) {  // A from the upper triangle of the sums
    const int a = r < c ? r : c, bb = r < c ? c : r;
    return tot[a * 6 - a * (a - 1) / 2 + (bb - a)];
  };
  if (t >= 64 && t < 128) {  // wave 1: the LLT solve, a lane per row
    double b[6], x[6];
    for (int a = 0; a < 6; ++a) b[a] = -tot[21 + a];
    const bool ok = wave_llt_solve6(tri, b, x);
    if (t == 64) {
      rank_llt[1] = ok ? 1 : 0;
      for (int a = 0; a < 6; ++a) xs[a] = x[a];
    }
  }
  if (t < 64) {  // wave 0: the pivoted-QR rank, a lane per column (A from the upper triangle)
    const int rk = wave_pivqr_rank6(tri);
    if (t == 0) rank_llt[0] = rk;
  }
  __syncthreads();
  if (t == 0) update_serial(d, s, tot, prm, rank_llt[0] == 6 && rank_llt[1] ? xs : nullptr);
}

__global__ __launch_bounds__(256) void k_icp_update(const PairDesc* __restrict__ pd, PairState* st,
                                                    const double* __restrict__ slab, IcpParams prm) {
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  icp_update_body(pd[pair], s, slab, prm);
}

// k_icp_update + (last pair of the group) the next active list. Kept out of the reduce kernel:
// the update's solve (pivoted QR, LLT / min-norm QR / SVD fallback, fp64) needs 256 VGPRs, and a
// kernel's register allocation is its largest path's, so a fused reduce ran its gathers at one
// wave per SIMD (35-40 us per C2 window iteration against 12.5 + 12.3 us for the two kernels).
__global__ __launch_bounds__(256) void k_icp_update_f(const PairDesc* __restrict__ pd, PairState* st,
                                                      const double* __restrict__ slab, IcpParams prm, IcpIterSync y) {
  AICP_IP_T0;
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  icp_update_body(pd[pair], s, slab, prm);
  AICP_IP_BODY(3);
  AICP_IP_TAIL0;
  pair_done(y);
  AICP_IP_TAIL(3);
}

__global__ void k_finalize(int n_pairs, const PairDesc* __restrict__ pd,
                           PairState* __restrict__ st, float* __restrict__ outT) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  float tmp[16], T[16];
  mul4(pd[p].Tmean, st[p].T, tmp);
  mul4(tmp, pd[p].Tinit, T);
  for (int i = 0; i < 16; ++i) outT[p * 16 + i] = T[i];
  // registerClouds applies T to the output reading (pointmatcher_registration.cpp:128-129)
  if (st[p].status == 0 && !rigid_ok(T)) st[p].status = 5;
}

// ------------------------------------------------------------------------------------------
// kernel-level entry points
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void k_knn_generic(uint32_t nq, const float4* __restrict__ q,
                                                     const uint4* __restrict__ nodes,
                                                     const int32_t* __restrict__ parent,
                                                     const float4* __restrict__ bpts, float maxE2,
                                                     float maxR2, int32_t* __restrict__ ids,
                                                     float* __restrict__ d2, unsigned long long* touched,
                                                     uint32_t* ctr) {
  uint32_t tp = 0, tn = 0;
  persistent_xcd<Trav<K>>(
      nq, ctr, maxE2, maxR2, nodes, bpts, [](uint32_t) {},
      [&](uint32_t s, Trav<K>& t) {
        t.nodes = nodes;
        t.pts = bpts;
        const float4 x = q[s];
        t.reset(x.x, x.y, x.z);
        return true;
      },
      [&](uint32_t s, Trav<K>& t) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          ids[(size_t)s * K + j] = t.best.id[j] < 0 ? -1 : __float_as_int(bpts[t.best.id[j]].w);
          d2[(size_t)s * K + j] = t.best.v[j];
        }
        tp += t.tp;
        tn += t.tn;
      });
  unsigned long long a = tp, b = tn;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&touched[0], a);
    atomicAdd(&touched[1], b);
  }
}

// 1-NN over the node records (Trav<1>)
template <class Eng>
__global__ __launch_bounds__(256) void k_knn1_generic(uint32_t nq, const float4* __restrict__ q,
                                                      const uint4* __restrict__ nodes,
                                                      const float4* __restrict__ bpts, float maxE2, float maxR2,
                                                      int32_t* __restrict__ ids, float* __restrict__ d2,
                                                      unsigned long long* touched, uint32_t* ctr) {
  uint32_t tp = 0, tn = 0;
  persistent_xcd<Eng>(
      nq, ctr, maxE2, maxR2, nodes, bpts, [](uint32_t) {},
      [&](uint32_t s, Eng& t) {
        t.bind(nodes, bpts, 0, 0);
        const float4 x = q[s];
        t.reset(x.x, x.y, x.z);
        return true;
      },
      [&](uint32_t s, Eng& t) {
        const int32_t id = t.res_id();
        ids[s] = id < 0 ? -1 : __float_as_int(bpts[id].w);
        d2[s] = t.res_d2();
        tp += t.tp;
        tn += t.tn;
      });
  unsigned long long a = tp, b = tn;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&touched[0], a);
    atomicAdd(&touched[1], b);
  }
}

__global__ void k_transform(int n, const float* __restrict__ T, const float4* __restrict__ in,
                            float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float Tl[16];
  for (int k = 0; k < 16; ++k) Tl[k] = T[k];
  const float4 p = in[i];
  float o[3];
  apply4(Tl, p.x, p.y, p.z, o);
  out[i] = make_float4(o[0], o[1], o[2], 1.f);
}

// solve6 as the update kernel takes it: the wave-parallel rank and LLT first (a path of 100 + the
// rank if the wave's rank ever disagrees with pivqr<6>'s, 200 if the wave's LLT differs from
// llt_solve<6> in a bit, so the golden test fails loudly)
__global__ __launch_bounds__(64) void k_solve6(const double* A, const double* b, double* x, int32_t* path) {
  const auto get = [&](int r, int c) { return A[r * 6 + c]; };
  const int rk = wave_pivqr_rank6(get);
  double bl[6], xw[6];
  for (int i = 0; i < 6; ++i) bl[i] = b[i];
  const bool okw = wave_llt_solve6(get, bl, xw);
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    PivQR<6> q;
    pivqr<6>(A, q);
    double xl[6];
    const bool okl = llt_solve<6>(A, 6, b, xl);
    bool same = okw == okl;
    for (int i = 0; i < 6 && okl && okw; ++i) same &= __double_as_longlong(xl[i]) == __double_as_longlong(xw[i]);
    const int p = solve6(A, b, x);
    *path = rk != q.rank ? 100 + rk : (!same ? 200 : p);
  }
}

// ------------------------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------------------------
// CU count of the calling thread's current device, cached per device (contexts of
// aicp_hip_multi_* call this from several host threads at once, possibly on different GPU models)
static int device_cus() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  if (dev >= 0 && dev < kMaxDev) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int cus = 0;
  if (dev < 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  if (dev >= 0 && dev < kMaxDev) cache[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

static int persistent_grid(int n_items, int blocks_per_cu = 8) {
  const int cus = device_cus();
  // every work group (blockIdx % kXcdGroups) needs at least one block: a multiple of 8
  int want = (n_items + 255) / 256;
  if (want > cus * blocks_per_cu) want = cus * blocks_per_cu;
  return (want + kXcdGroups - 1) / kXcdGroups * kXcdGroups;
}

void launch_prepare_read(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* raw, float4* out) {
  if (m.n_blocks) k_prepare_read<<<m.n_blocks, 256, 0, s>>>(m, pd, raw, out);
}
void launch_gather_ref(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* raw, const int32_t* perm,
                       float4* bpts) {
  if (m.n_blocks) k_gather_ref<<<m.n_blocks, 256, 0, s>>>(m, pd, raw, perm, bpts);
}
void launch_init_state(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st) {
  k_init_state<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st);
}
bool launch_normals(hipStream_t s, int n_pairs, uint32_t total_ref, const PairDesc* pd, PairState* st,
                    const uint4* nodes, const int32_t* parent, const float4* bpts, float4* bnrm, int knn,
                    int32_t* ids, uint32_t* ctr, int engine) {
  if (!total_ref) return true;
  if (!launch_knn_ids(s, n_pairs, total_ref, pd, nodes, bpts, knn, ids, ctr, nullptr, engine)) return false;
  const int gu = (int)((total_ref + 255) / 256);
  switch (knn) {
    case 10: k_normals_from_ids<10><<<gu, 256, 0, s>>>(n_pairs, total_ref, pd, st, bpts, ids, bnrm); break;
    case 20: k_normals_from_ids<20><<<gu, 256, 0, s>>>(n_pairs, total_ref, pd, st, bpts, ids, bnrm); break;
    case 30: k_normals_from_ids<30><<<gu, 256, 0, s>>>(n_pairs, total_ref, pd, st, bpts, ids, bnrm); break;
    default: return false;
  }
  return true;
}
// k_knn_oct for launches of at most kKnnOctMax queries (engine 2: never, 1: always -- tests
// compare the engines): with eight lanes per query it issues ~2.3x the VALU instructions of
// the per-lane engine, which pays only while the per-lane launch leaves the chip short of waves
// (the C2 stream's single 120k-point reference: 377 -> 245 us); on C5's 61 M queries it ran
// 91.7 ms per launch against the per-lane engine's throughput (C5 3962 -> 3097 clouds/s, r03c).
// (Quads, 4 lanes per query, measured equal to octets on C2, r03.)
constexpr uint32_t kKnnOctMax = 300000;
static bool knn_oct_enabled(uint32_t n_queries, int engine) {
  return engine == 0 ? n_queries <= kKnnOctMax : engine == 1;
}

bool launch_knn_ids(hipStream_t s, int n_pairs, uint32_t total_ref, const PairDesc* pd, const uint4* nodes,
                    const float4* bpts, int knn, int32_t* ids, uint32_t* ctr, unsigned long long* touched,
                    int engine) {
  if (!total_ref) return true;
  if (knn_oct_enabled(total_ref, engine)) {
    const unsigned go = (unsigned)(((uint64_t)total_ref * 8 + 255) / 256);
    switch (knn) {
      case 10: k_knn_oct<10, 8><<<go, 256, 0, s>>>(n_pairs, total_ref, pd, nodes, bpts, ids, touched); break;
      case 20: k_knn_oct<20, 8><<<go, 256, 0, s>>>(n_pairs, total_ref, pd, nodes, bpts, ids, touched); break;
      case 30: k_knn_oct<30, 8><<<go, 256, 0, s>>>(n_pairs, total_ref, pd, nodes, bpts, ids, touched); break;
      default: return false;
    }
    return true;
  }
  // the persistent engine's work counters, zeroed here: the octet engine needs none, and a
  // caller's memset ahead of it put a ~5 us fill kernel on the C2 reference chain for nothing
  if (hipMemsetAsync(ctr, 0, kPersistCtrWords * 4, s) != hipSuccess) return false;
  const int g = persistent_grid((int)total_ref);
  switch (knn) {
    case 10: k_knn_ids<10><<<g, 256, 0, s>>>(n_pairs, total_ref, pd, nodes, nullptr, bpts, ids, ctr, touched); break;
    case 20: k_knn_ids<20><<<g, 256, 0, s>>>(n_pairs, total_ref, pd, nodes, nullptr, bpts, ids, ctr, touched); break;
    case 30: k_knn_ids<30><<<g, 256, 0, s>>>(n_pairs, total_ref, pd, nodes, nullptr, bpts, ids, ctr, touched); break;
    default: return false;
  }
  return true;
}
void launch_active_list(hipStream_t s, int n_pairs, const PairDesc* pd, const PairState* st, ActiveList* al,
                        uint32_t* ctr, uint32_t* host_n, uint64_t* done_sig, const uint64_t* ticket, float* outT,
                        int src_pair) {
  // 256 threads: the first iteration's list is launched while the normals' kNN fills the chip, and
  // a 1024-thread workgroup waited for 16 free wave slots on one CU (C2 trace: 33 us median)
  k_active_list<<<1, 256, 0, s>>>(n_pairs, pd, st, al, ctr, host_n, done_sig, ticket, outT, src_pair);
}
// The ICP matcher's NN engine: Trav2C on the treelet records; Trav<1> on the node records where
// treelets do not fit (bucketSize > 15, references above 4 M points, 2^28 records) or
// AICP_FORCE_TRAV1 (tests). Timed launches (e0, e1 given) carry the events on the kernel's own
// dispatch (hipExtLaunchKernelGGL): the elapsed time is the kernel's execution, as rocprofv3
// reports it, with no marker packets between the NN and its neighbours (separate
// hipEventRecord calls left ~6 us gaps on each side of every timed launch).
template <class E, class Tree>
static void nn_launch(hipStream_t s, int g, hipEvent_t e0, hipEvent_t e1, const PairDesc* pd, const PairState* st,
                      const ActiveList* al, const float4* read_c, const Tree* tree, const int32_t* parent,
                      const float4* bpts, const uint2* ptl, int32_t* match, float* d2, uint32_t* touched,
                      uint32_t* ctr, const IcpParams& prm) {
  if (e0)
    hipExtLaunchKernelGGL(k_icp_nn<E>, dim3(g), dim3(256), 0, s, e0, e1, 0, pd, st, al, read_c, tree, parent, bpts,
                          ptl, match, d2, touched, ctr, prm);
  else
    k_icp_nn<E><<<g, 256, 0, s>>>(pd, st, al, read_c, tree, parent, bpts, ptl, match, d2, touched, ctr, prm);
}

void launch_icp_nn(hipStream_t s, int grid_items, const PairDesc* pd, const PairState* st, const ActiveList* al,
                   const float4* read_c, const uint4* nodes, const uint4* tl, const int32_t* parent,
                   const float4* bpts, const uint2* ptl, int32_t* match, float* d2, uint32_t* touched,
                   uint32_t* ctr, const IcpParams& prm, hipEvent_t e0, hipEvent_t e1) {
  const int g = persistent_grid(grid_items, AICP_NN_WAVES);
  if (g == 0) {  // a pair group without readings (the timing events still complete)
    if (e0) (void)hipEventRecord(e0, s);
    if (e1) (void)hipEventRecord(e1, s);
    return;
  }
  if (tl && ptl)
    nn_launch<Trav2C>(s, g, e0, e1, pd, st, al, read_c, tl, parent, bpts, ptl, match, d2, touched, ctr, prm);
  else
    nn_launch<Trav<1>>(s, g, e0, e1, pd, st, al, read_c, nodes, parent, bpts, (const uint2*)nullptr, match, d2,
                       touched, ctr, prm);
}
void iter_prof_dump() {
#if AICP_ITER_PROF
  unsigned long long h[16];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_iter_prof), sizeof(h)) == hipSuccess) {
    const char* nm[4] = {"hist_f", "compact_f", "reduce", "update_f(body=slab+solve, tail=active list)"};
    for (int k = 0; k < 4; ++k)
      fprintf(stderr, "[iter prof] %s: body %.2f us avg over %llu, tail %.2f us avg over %llu\n", nm[k],
              h[4 * k + 1] ? h[4 * k] / 100.0 / h[4 * k + 1] : 0.0, h[4 * k + 1],
              h[4 * k + 3] ? h[4 * k + 2] / 100.0 / h[4 * k + 3] : 0.0, h[4 * k + 3]);
  }
  unsigned long long z[16] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_iter_prof), z, sizeof(z));
#endif
}

void nn_prof_dump() {
#if AICP_XCD_PROF
  static unsigned long long h[64 * kXcdGroups * 2];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_xcd_prof), sizeof(h)) == hipSuccess) {
    for (int l = 0; l < 64; ++l) {
      unsigned long long t0 = ~0ull, t1 = 0;
      for (int g = 0; g < kXcdGroups; ++g) {
        if (h[(l * kXcdGroups + g) * 2]) t0 = std::min(t0, h[(l * kXcdGroups + g) * 2]);  // (0: not reset yet)
        t1 = std::max(t1, h[(l * kXcdGroups + g) * 2 + 1]);
      }
      if (t1 == 0) continue;
      unsigned long long c[kXcdGroups];
      (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_xcd_cost), sizeof(c), sizeof(c) * l);
      fprintf(stderr, "xcd launch %2d: %6.1f us | per group: start end (us), queries, mean tn+tp:", l,
              (t1 - t0) / 100.0);
      for (int g = 0; g < kXcdGroups; ++g) {
        const unsigned long long q = c[g] >> 40, w = c[g] & ((1ull << 40) - 1);
        const unsigned long long s0 = h[(l * kXcdGroups + g) * 2];
        fprintf(stderr, " [%.1f %.1f %llu %.1f]", s0 ? (s0 - t0) / 100.0 : -1.0,
                (h[(l * kXcdGroups + g) * 2 + 1] - t0) / 100.0, q, q ? (double)w / q : 0.0);
      }
      fprintf(stderr, "\n");
    }
  }
  for (int i = 0; i < 64 * kXcdGroups; ++i) {
    h[2 * i] = ~0ull;
    h[2 * i + 1] = 0;
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_prof), h, sizeof(h));
  static unsigned long long zc[64 * kXcdGroups] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_cost), zc, sizeof(zc));
#endif
#if AICP_NN_PROF
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_nn_prof), sizeof(h)) == hipSuccess) {
    const double tot = (double)(h[0] + h[1] + h[2] + h[3]);
    fprintf(stderr, "nn_prof: fill %.1f%% descent %.1f%% bucket %.1f%% climb %.1f%% | rounds %llu, mean active lanes %.1f | cached starts %llu, full %llu\n",
            100.0 * h[0] / tot, 100.0 * h[1] / tot, 100.0 * h[2] / tot, 100.0 * h[3] / tot, h[4],
            h[4] ? (double)h[5] / h[4] : 0.0, h[6], h[7]);
  }
  unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_nn_prof), z, sizeof(z));
#endif
#if AICP_QLAT_PROF
  static unsigned long long q[512];
  if (hipMemcpyFromSymbol(q, HIP_SYMBOL(g_qlat), sizeof(q)) == hipSuccess) {
    const char* nm[2] = {"query latency", "completion after wave start"};
    for (int k = 0; k < 2; ++k) {
      const unsigned long long* h = q + 256 * k;
      unsigned long long n = 0, acc = 0;
      double mean = 0;
      for (int b = 0; b < 256; ++b) n += h[b], mean += (b + 0.5) * h[b];
      if (!n) continue;
      fprintf(stderr, "qlat %s: n %llu mean %.1f us |", nm[k], n, mean / n);
      const double ps[6] = {0.5, 0.9, 0.99, 0.999, 0.9999, 1.0};
      int p = 0;
      for (int b = 0; b < 256 && p < 6; ++b) {
        acc += h[b];
        while (p < 6 && acc >= (unsigned long long)(ps[p] * n)) {
          fprintf(stderr, " p%g %d", ps[p] * 100, b + 1);
          ++p;
        }
      }
      fprintf(stderr, " us\nqlat %s histogram (2 us bins):", nm[k]);
      for (int b = 0; b < 256; b += 2) {
        const unsigned long long c = h[b] + h[b + 1];
        if (c) fprintf(stderr, " %d:%llu", b, c);
      }
      fprintf(stderr, "\n");
    }
  }
  for (auto& v : q) v = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_qlat), q, sizeof(q));
#endif
}

void launch_icp_select(hipStream_t s, BlockMap m, int n_pairs, const PairDesc* pd, PairState* st, const float* d2,
                       uint32_t* hist1, uint32_t* cand, uint32_t* cand_cnt, int p0) {
  if (!m.n_blocks) return;
  k_sel_hist<<<m.n_blocks, 256, 0, s>>>(m, pd, st, d2, hist1);
  k_sel_find1<<<n_pairs, 1024, 0, s>>>(st + p0, hist1 + (size_t)p0 * kHistBins);
  k_sel_compact<<<m.n_blocks, 256, 0, s>>>(m, pd, st, d2, cand, cand_cnt);
  k_sel_final<<<n_pairs, 1024, 0, s>>>(pd + p0, st + p0, cand, cand_cnt + p0);
}
IcpIterSync icp_sync_layout(uint32_t* words, size_t n_pairs, int group) {
  IcpIterSync y{};
  y.sel1 = words;
  y.sel2 = words + n_pairs;
  y.red = words + 2 * n_pairs;
  y.pairs = words + 3 * n_pairs + group;
  return y;
}
void launch_icp_select_f(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st, const float* d2,
                         uint32_t* hist1, uint32_t* cand, uint32_t* cand_cnt, const IcpIterSync& y) {
  if (!m.n_blocks) return;
  k_sel_hist_f<kSelHistThreads><<<m.n_blocks, kSelHistThreads, 0, s>>>(m, pd, st, d2, hist1, y);
  k_sel_compact_f<kSelCompactThreads><<<m.n_blocks, kSelCompactThreads, 0, s>>>(m, pd, st, d2, cand, cand_cnt, y);
}
void launch_icp_select_fused(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st, const float* d2,
                             uint32_t* hist1, uint32_t* cand, uint32_t* cand_cnt, const IcpIterSync& y) {
  if (!m.n_blocks) return;
  if (m.n_blocks > 2048)  // more workgroups than fit the chip at once: occupancy over the tail's LDS copy
    k_sel_fused<256, kHistBins><<<m.n_blocks, 256, 0, s>>>(m, pd, st, d2, hist1, cand, cand_cnt, y);
  else
    k_sel_fused<256, kFinalLds><<<m.n_blocks, 256, 0, s>>>(m, pd, st, d2, hist1, cand, cand_cnt, y);
}
void launch_icp_select_pair(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const float* d2,
                            uint32_t* cand, const IcpIterSync& y) {
  if (n_pairs > 0) k_sel_pair<<<n_pairs, kSelPairThreads, 0, s>>>(pd, st, d2, cand, y);
}
bool sel_pair_fits(size_t n_pairs, uint64_t max_read, int force) {
  if (max_read > kSelPairMax) return false;
  if (force >= 0) return force == 1;
  return n_pairs >= 256;
}
void launch_icp_reduce_f(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st, const float4* read_c,
                         const int32_t* match, const float* d2, const uint32_t* touched, const float4* bpts,
                         const float4* bnrm, double* slab, const IcpParams& prm, const IcpIterSync& y) {
  if (!m.n_blocks) return;
  k_icp_reduce<<<m.n_blocks, kNNBlock, 0, s>>>(m, pd, st, read_c, match, d2, touched, bpts, bnrm, slab);
  k_icp_update_f<<<y.np, 256, 0, s>>>(y.pd, y.st, slab, prm, y);
}
void launch_icp_reduce(hipStream_t s, BlockMap m, const PairDesc* pd, const PairState* st, const float4* read_c,
                       const int32_t* match, const float* d2, const uint32_t* touched, const float4* bpts,
                       const float4* bnrm, double* slab) {
  if (m.n_blocks)
    k_icp_reduce<<<m.n_blocks, kNNBlock, 0, s>>>(m, pd, st, read_c, match, d2, touched, bpts, bnrm, slab);
}
void launch_icp_update(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const double* slab,
                       const IcpParams& prm) {
  k_icp_update<<<n_pairs, 256, 0, s>>>(pd, st, slab, prm);
}
void launch_finalize(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, float* outT) {
  k_finalize<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st, outT);
}
bool launch_knn_generic(hipStream_t s, uint32_t nq, const float4* q, const uint4* nodes, const int32_t* parent,
                        const float4* bpts, int k, float maxE2, float maxR2, int32_t* ids, float* d2,
                        unsigned long long* touched, uint32_t* ctr) {
  if (!nq) return true;
  const int g = persistent_grid((int)nq);
  switch (k) {
    case 1: k_knn1_generic<Trav<1>><<<g, 256, 0, s>>>(nq, q, nodes, bpts, maxE2, maxR2, ids, d2, touched, ctr); break;
    case 4: k_knn_generic<4><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched, ctr); break;
    case 10: k_knn_generic<10><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched, ctr); break;
    case 20: k_knn_generic<20><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched, ctr); break;
    case 30: k_knn_generic<30><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched, ctr); break;
    default: return false;
  }
  return true;
}
void launch_transform(hipStream_t s, int n, const float* T, const float4* in, float4* out) {
  if (n > 0) k_transform<<<(n + 255) / 256, 256, 0, s>>>(n, T, in, out);
}
void launch_solve6(hipStream_t s, const double* A, const double* b, double* x, int32_t* path) {
  k_solve6<<<1, 64, 0, s>>>(A, b, x, path);
}

}  // namespace aicp
