// kernels_icp.hip — ICP hot path on CDNA4 (gfx950).
//
// Per ICP iteration (libpointmatcher ICP loop), for every pair of a
// batch at once, four launches and no host synchronisation:
//   k_icp_nn      transform (T_iter, fused) + libnabo-order approximate 1-NN + the first radix
//                 digit histogram of d^2 (LDS, flushed with one atomic per non-empty bin)
//   k_icp_select  exact k-th smallest d^2 (Matches::getDistsQuantile) by 3-digit radix select,
//                 one 1024-thread workgroup per pair, candidates of digit 1 kept in LDS
//   k_icp_reduce  TrimmedDist weights + getMatchedPoints gather + point-to-plane F, dot and the
//                 27-entry normal-equation sums in double from exact float products; wave
//                 butterfly + LDS, one deterministic partial row per workgroup (no atomics)
//   k_icp_update  fixed-order sum of the partial rows, 6x6 solve, AngleAxis update of T_iter,
//                 Counter + Differential checkers, per-pair active flag (early exit for the
//                 remaining launches of converged pairs)
#include <hip/hip_runtime.h>

#include "aicp_common.hpp"
#include "icp_math.hpp"
#include "kernels.hpp"

namespace aicp {

// ------------------------------------------------------------------------------------------
// k-NN traversal in libnabo recurseKnn order
// ------------------------------------------------------------------------------------------
// recurseKnn visits the near child first, then the far child if rd' = rd - off[cd]^2 +
// new_off^2 passes (rd' <= maxR2 && rd' * maxE2 < head). Along a run of near children rd and
// off do not change, so the far test of every level of a descent can be evaluated during the
// descent itself; after the leaf the climb (through parent[]) is skipped entirely when the
// smallest such rd' already fails against the current head -- the common case with
// epsilon = 3.16. Far descents push (far child, rd, off[cd], outer min, outer start) on a
// bounded stack (nesting <= tree depth <= kFarStack, checked on the host).
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

template <int K>
__device__ __forceinline__ void best_replace(Best<K>& b, int32_t id, float val) {
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

template <int K>
__device__ __forceinline__ void knn_traverse(const uint2* __restrict__ nodes,
                                             const int32_t* __restrict__ parent,
                                             const float4* __restrict__ pts, float q0, float q1,
                                             float q2, float maxE2, float maxR2, Best<K>& best,
                                             uint32_t& tpts, uint32_t& tnodes) {
  float off0 = 0.f, off1 = 0.f, off2 = 0.f, rd = 0.f;
  int32_t stF[kFarStack];
  float stRd[kFarStack], stOld[kFarStack], stMin[kFarStack];
  int32_t stStart[kFarStack];
  int sp = 0;
  int32_t n = 0, start = 0;
  float minFar;
  for (;;) {
    // ---- descend along near children
    minFar = __builtin_inff();
    uint2 nd = nodes[n];
    while ((nd.y & 3u) != kLeaf) {
      const uint32_t cd = nd.y & 3u;
      const float no = sel3(cd, q0, q1, q2) - __uint_as_float(nd.x);
      const float oc = sel3(cd, off0, off1, off2);
      const float rdf = rd + (-oc * oc + no * no);
      minFar = fminf(minFar, rdf);
      n = (no > 0.f) ? (int32_t)(nd.y >> 2) : n + 1;
      ++tnodes;
      nd = nodes[n];
    }
    // ---- bucket
    {
      const uint32_t b0 = nd.y >> 2, cnt = nd.x;
      for (uint32_t i = 0; i < cnt; ++i) {
        const float4 p = pts[b0 + i];
        const float d0 = q0 - p.x, d1 = q1 - p.y, d2 = q2 - p.z;
        float dist = 0.f;
        dist += d0 * d0;
        dist += d1 * d1;
        dist += d2 * d2;
        if (dist <= maxR2 && dist < best.v[K - 1]) best_replace<K>(best, (int32_t)(b0 + i), dist);
      }
      tpts += cnt;
    }
    // ---- climb
    int32_t c = n;
    if (!(minFar <= maxR2 && minFar * maxE2 < best.v[K - 1])) c = start;
    bool descend = false;
    while (!descend) {
      if (c == start) {
        if (sp == 0) return;
        --sp;
        const uint32_t pcd = (uint32_t)stF[sp] >> 30;
        rd = stRd[sp];
        if (pcd == 0) off0 = stOld[sp];
        else if (pcd == 1) off1 = stOld[sp];
        else off2 = stOld[sp];
        minFar = stMin[sp];
        start = stStart[sp];
        c = parent[c];
        if (!(minFar <= maxR2 && minFar * maxE2 < best.v[K - 1])) c = start;
        continue;
      }
      const int32_t p = parent[c];
      const uint2 pn = nodes[p];
      const uint32_t cd = pn.y & 3u;
      const float no = sel3(cd, q0, q1, q2) - __uint_as_float(pn.x);
      const float oc = sel3(cd, off0, off1, off2);
      const float rdf = rd + (-oc * oc + no * no);
      if (rdf <= maxR2 && rdf * maxE2 < best.v[K - 1]) {
        const int32_t far = (no > 0.f) ? p + 1 : (int32_t)(pn.y >> 2);
        stF[sp] = (int32_t)((uint32_t)far | (cd << 30));
        stRd[sp] = rd;
        stOld[sp] = oc;
        stMin[sp] = minFar;
        stStart[sp] = start;
        ++sp;
        if (cd == 0) off0 = no;
        else if (cd == 1) off1 = no;
        else off2 = no;
        rd = rdf;
        n = far;
        start = far;
        descend = true;
      } else {
        c = p;
      }
    }
  }
}

__device__ __forceinline__ void block_map(const BlockMap& m, int& pair, uint32_t& local) {
  pair = m.pair[blockIdx.x];
  local = m.start[blockIdx.x] + threadIdx.x;
}

// ------------------------------------------------------------------------------------------
// setup kernels
// ------------------------------------------------------------------------------------------
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
  quat_from_T(s.T, s.qh[0]);
  s.th[0][0] = s.th[0][1] = s.th[0][2] = 0.0;
}

__global__ void k_zero_hist(int n_pairs, uint32_t* hist1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_pairs * kHistBins) hist1[i] = 0;
}

// ------------------------------------------------------------------------------------------
// SurfaceNormal on the reference (bucket order queries: spatially coherent waves)
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void k_normals(BlockMap m, const PairDesc* __restrict__ pd,
                                                 PairState* st, const uint2* __restrict__ nodes,
                                                 const int32_t* __restrict__ parent,
                                                 const float4* __restrict__ bpts,
                                                 float4* __restrict__ bnrm) {
  int pair;
  uint32_t j;
  block_map(m, pair, j);
  const PairDesc& d = pd[pair];
  __shared__ uint32_t deg;
  if (threadIdx.x == 0) deg = 0;
  __syncthreads();
  if (j < d.n_ref) {
    const float4* P = bpts + d.ref_off;
    const float4 q = P[j];
    Best<K> best;
    best_init<K>(best);
    uint32_t tp = 0, tn = 0;
    knn_traverse<K>(nodes + d.node_off, parent + d.node_off, P, q.x, q.y, q.z, 1.f,
                    __builtin_inff(), best, tp, tn);
    // d = neighbours with finite distance in heap order; mean; NN = d - mean; C = NN NN^T / k
    float sx = 0.f, sy = 0.f, sz = 0.f;
    int kk = 0;
#pragma unroll
    for (int i = 0; i < K; ++i)
      if (best.v[i] != __builtin_inff()) {
        const float4 p = P[best.id[i]];
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
      if (best.v[i] != __builtin_inff()) {
        const float4 p = P[best.id[i]];
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
    bnrm[d.ref_off + j] = make_float4(nrm[0], nrm[1], nrm[2], 0.f);
    if (dg) atomicAdd(&deg, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0 && deg) atomicAdd(&st[pair].degenerate, (int)deg);
}

// ------------------------------------------------------------------------------------------
// ICP iteration
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kNNBlock) void k_icp_nn(
    BlockMap m, const PairDesc* __restrict__ pd, PairState* st, const float4* __restrict__ read_c,
    const uint2* __restrict__ nodes, const int32_t* __restrict__ parent,
    const float4* __restrict__ bpts, int32_t* __restrict__ match, float* __restrict__ d2out,
    uint32_t* __restrict__ hist1, IcpParams prm) {
  int pair;
  uint32_t j;
  block_map(m, pair, j);
  PairState& s = st[pair];
  if (!s.active) return;
  __shared__ uint32_t lh[kHistBins];
  __shared__ uint32_t ltp, ltn;
  for (int i = threadIdx.x; i < kHistBins; i += kNNBlock) lh[i] = 0;
  if (threadIdx.x == 0) ltp = ltn = 0;
  __syncthreads();
  const PairDesc& d = pd[pair];
  if (j < d.n_read) {
    float T[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) T[i] = s.T[i];
    const float4 r = read_c[d.read_off + j];
    float q[3];
    apply4(T, r.x, r.y, r.z, q);
    Best<1> best;
    best_init<1>(best);
    uint32_t tp = 0, tn = 0;
    knn_traverse<1>(nodes + d.node_off, parent + d.node_off, bpts + d.ref_off, q[0], q[1], q[2],
                    prm.maxE2, prm.maxR2, best, tp, tn);
    match[d.read_off + j] = best.id[0];
    d2out[d.read_off + j] = best.v[0];
    if (best.v[0] != __builtin_inff()) atomicAdd(&lh[__float_as_uint(best.v[0]) >> 21], 1u);
    atomicAdd(&ltp, tp);
    atomicAdd(&ltn, tn);
  }
  __syncthreads();
  uint32_t* gh = hist1 + (size_t)pair * kHistBins;
  for (int i = threadIdx.x; i < kHistBins; i += kNNBlock) {
    const uint32_t v = lh[i];
    if (v) atomicAdd(&gh[i], v);
  }
  if (threadIdx.x == 0) {
    atomicAdd((unsigned long long*)&s.touched_pts, (unsigned long long)ltp);
    atomicAdd((unsigned long long*)&s.touched_nodes, (unsigned long long)ltn);
  }
}

// rank k -> (bin, k - count before bin) over h[nb] with 1024 threads; result in res[0..2]
__device__ void block_find_rank(const uint32_t* h, int nb, uint32_t k, uint32_t* res,
                                uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = nb / 1024;
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

constexpr int kCand = 8192;

__global__ __launch_bounds__(1024) void k_icp_select(const PairDesc* __restrict__ pd, PairState* st,
                                                     const float* __restrict__ d2,
                                                     const uint32_t* __restrict__ hist1) {
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  const PairDesc& d = pd[pair];
  __shared__ uint32_t h[kHistBins];
  __shared__ uint32_t cand[kCand];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t res[2];
  __shared__ uint32_t total, ncand;
  const int t = threadIdx.x;
  for (int i = t; i < kHistBins; i += 1024) h[i] = hist1[(size_t)pair * kHistBins + i];
  if (t == 0) ncand = 0;
  __syncthreads();
  // total finite = sum of digit-1 histogram
  {
    uint32_t v = h[2 * t] + h[2 * t + 1];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((t & 63) == 0) wsum[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
      uint32_t a = 0;
      for (int w = 0; w < 16; ++w) a += wsum[w];
      total = a;
    }
    __syncthreads();
  }
  const uint32_t n = total;
  if (n == 0) {  // ConvergenceError("no outlier to filter")
    if (t == 0) {
      s.status = 1;
      s.active = 0;
    }
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
  block_find_rank(h, kHistBins, k, res, wsum);
  const uint32_t b1 = res[0], r1 = res[1];
  for (int i = t; i < kHistBins; i += 1024) h[i] = 0;
  __syncthreads();
  const uint32_t* bits = (const uint32_t*)(d2 + d.read_off);
  for (uint32_t i = t; i < d.n_read; i += 1024) {
    const uint32_t v = bits[i];
    if ((v >> 21) == b1 && v != 0x7f800000u) {
      atomicAdd(&h[(v >> 10) & 2047u], 1u);
      const uint32_t slot = atomicAdd(&ncand, 1u);
      if (slot < (uint32_t)kCand) cand[slot] = v;
    }
  }
  __syncthreads();
  block_find_rank(h, kHistBins, r1, res, wsum);
  const uint32_t b2 = res[0], r2 = res[1];
  for (int i = t; i < kHistBins; i += 1024) h[i] = 0;
  __syncthreads();
  const uint32_t hi21 = (b1 << 11) | b2;
  if (ncand <= (uint32_t)kCand) {
    for (uint32_t i = t; i < ncand; i += 1024) {
      const uint32_t v = cand[i];
      if ((v >> 10) == hi21) atomicAdd(&h[v & 1023u], 1u);
    }
  } else {
    for (uint32_t i = t; i < d.n_read; i += 1024) {
      const uint32_t v = bits[i];
      if ((v >> 10) == hi21 && v != 0x7f800000u) atomicAdd(&h[v & 1023u], 1u);
    }
  }
  __syncthreads();
  block_find_rank(h, kHist3Bins, r2, res, wsum);
  if (t == 0) {
    s.limit = __uint_as_float((hi21 << 10) | res[0]);
    s.n_finite = (int32_t)n;
  }
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ __launch_bounds__(kNNBlock) void k_icp_reduce(
    BlockMap m, const PairDesc* __restrict__ pd, const PairState* __restrict__ st,
    const float4* __restrict__ read_c, const int32_t* __restrict__ match,
    const float* __restrict__ d2, const float4* __restrict__ bpts,
    const float4* __restrict__ bnrm, double* __restrict__ slab) {
  const int pair = m.pair[blockIdx.x];
  const PairState& s = st[pair];
  if (!s.active) return;
  const PairDesc& d = pd[pair];
  float T[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) T[i] = s.T[i];
  const float limit = s.limit;
  double acc[kRedCols];
#pragma unroll
  for (int i = 0; i < kRedCols; ++i) acc[i] = 0.0;
  const uint32_t base = m.start[blockIdx.x];
#pragma unroll
  for (int it = 0; it < kReducePerThread; ++it) {
    const uint32_t j = base + it * kNNBlock + threadIdx.x;
    if (j >= d.n_read) break;
    const float dd = d2[d.read_off + j];
    if (!(dd <= limit)) continue;
    const int32_t pos = match[d.read_off + j];
    const float4 r = read_c[d.read_off + j];
    float p[3];
    apply4(T, r.x, r.y, r.z, p);
    const float4 q = bpts[d.ref_off + pos];
    const float4 nr = bnrm[d.ref_off + pos];
    float F[6];
    F[0] = p[1] * nr.z - p[2] * nr.y;
    F[1] = p[2] * nr.x - p[0] * nr.z;
    F[2] = p[0] * nr.y - p[1] * nr.x;
    F[3] = nr.x;
    F[4] = nr.y;
    F[5] = nr.z;
    const float dl0 = p[0] - q.x, dl1 = p[1] - q.y, dl2 = p[2] - q.z;
    float dot = dl0 * nr.x;
    dot += dl1 * nr.y;
    dot += dl2 * nr.z;
    int c = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = a; b < 6; ++b) acc[c++] += (double)F[a] * (double)F[b];
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] += (double)F[a] * (double)dot;
    acc[27] += 1.0;
  }
  __shared__ double part[kNNBlock / 64][kRedCols];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kRedCols; ++i) {
    const double v = wave_sum_d(acc[i]);
    if (lane == 0) part[wave][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < kRedCols) {
    double v = 0.0;
    for (int w = 0; w < kNNBlock / 64; ++w) v += part[w][threadIdx.x];
    slab[(size_t)blockIdx.x * kRedCols + threadIdx.x] = v;
  }
}

__global__ __launch_bounds__(256) void k_icp_update(const PairDesc* __restrict__ pd, PairState* st,
                                                    const double* __restrict__ slab,
                                                    uint32_t* __restrict__ hist1, IcpParams prm) {
  const int pair = blockIdx.x;
  PairState& s = st[pair];
  if (!s.active) return;
  const PairDesc& d = pd[pair];
  __shared__ double part[4][kRedCols];
  __shared__ double tot[kRedCols];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int c = 0; c < kRedCols; ++c) {
    double v = 0.0;
    for (uint32_t r = t; r < d.n_red_blk; r += 256) v += slab[(size_t)(d.red_blk_off + r) * kRedCols + c];
    v = wave_sum_d(v);
    if (lane == 0) part[wave][c] = v;
  }
  __syncthreads();
  if (t < kRedCols) tot[t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
  // clear the digit-1 histogram for the next iteration
  for (int i = t; i < kHistBins; i += 256) hist1[(size_t)pair * kHistBins + i] = 0;
  __syncthreads();
  if (t != 0) return;
  const int32_t kept = (int32_t)tot[27];
  s.kept = kept;
  if (kept == 0) {  // ConvergenceError("no point to minimize")
    s.status = 1;
    s.active = 0;
    return;
  }
  double A[36], b[6];
  int c = 0;
  for (int a = 0; a < 6; ++a)
    for (int bb = a; bb < 6; ++bb) {
      A[a * 6 + bb] = tot[c];
      A[bb * 6 + a] = tot[c];
      ++c;
    }
  for (int a = 0; a < 6; ++a) b[a] = -tot[21 + a];
  double xd[6];
  solve6(A, b, xd);
  float x[6];
  for (int a = 0; a < 6; ++a) x[a] = (float)xd[a];
  float dT[16];
  delta_transform(x, dT);
  mul4(dT, s.T, s.T);
  s.inlier_ratio = (float)((double)(float)kept / (double)d.n_read);
  // checkers (YAML order): Counter, then Differential
  bool iterate = true;
  s.iters += 1;
  if (s.iters >= prm.max_iter) iterate = false;
  const int h = s.hist_count % kHistRing;
  quat_from_T(s.T, s.qh[h]);
  for (int i = 0; i < 3; ++i) s.th[h][i] = (double)s.T[12 + i];
  s.hist_count += 1;
  const int sz = s.hist_count;
  if (sz > prm.smooth) {
    double cv0 = 0, cv1 = 0;
    for (int i = sz - 1; i >= sz - prm.smooth; --i) {
      const int a = i % kHistRing, bprev = (i - 1) % kHistRing;
      cv0 += fabs(quat_angdist(s.qh[a], s.qh[bprev]));
      const double dx = s.th[a][0] - s.th[bprev][0];
      const double dy = s.th[a][1] - s.th[bprev][1];
      const double dz = s.th[a][2] - s.th[bprev][2];
      cv1 += sqrt(dx * dx + dy * dy + dz * dz);
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

__global__ void k_finalize(int n_pairs, const PairDesc* __restrict__ pd,
                           const PairState* __restrict__ st, float* __restrict__ outT) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  float tmp[16], T[16];
  mul4(pd[p].Tmean, st[p].T, tmp);
  mul4(tmp, pd[p].Tinit, T);
  for (int i = 0; i < 16; ++i) outT[p * 16 + i] = T[i];
}

// ------------------------------------------------------------------------------------------
// kernel-level entry points
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void k_knn_generic(int nq, const float4* __restrict__ q,
                                                     const uint2* __restrict__ nodes,
                                                     const int32_t* __restrict__ parent,
                                                     const float4* __restrict__ bpts, float maxE2,
                                                     float maxR2, int32_t* __restrict__ ids,
                                                     float* __restrict__ d2,
                                                     unsigned long long* touched) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const float4 x = q[i];
  Best<K> best;
  best_init<K>(best);
  uint32_t tp = 0, tn = 0;
  knn_traverse<K>(nodes, parent, bpts, x.x, x.y, x.z, maxE2, maxR2, best, tp, tn);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    ids[(size_t)i * K + j] = best.id[j] < 0 ? -1 : __float_as_int(bpts[best.id[j]].w);
    d2[(size_t)i * K + j] = best.v[j];
  }
  atomicAdd(&touched[0], (unsigned long long)tp);
  atomicAdd(&touched[1], (unsigned long long)tn);
}

__global__ __launch_bounds__(256) void k_hist_d2(BlockMap m, const PairDesc* __restrict__ pd,
                                                 const float* __restrict__ d2,
                                                 uint32_t* __restrict__ hist1) {
  int pair;
  uint32_t j;
  block_map(m, pair, j);
  const PairDesc& d = pd[pair];
  if (j >= d.n_read) return;
  const float v = d2[d.read_off + j];
  if (v != __builtin_inff()) atomicAdd(&hist1[(size_t)pair * kHistBins + (__float_as_uint(v) >> 21)], 1u);
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

__global__ void k_solve6(const double* A, const double* b, double* x, int32_t* path) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *path = solve6(A, b, x);
}

// ------------------------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------------------------
void launch_prepare_read(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* raw,
                         float4* out) {
  if (m.n_blocks) k_prepare_read<<<m.n_blocks, 256, 0, s>>>(m, pd, raw, out);
}
void launch_gather_ref(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* raw,
                       const int32_t* perm, float4* bpts) {
  if (m.n_blocks) k_gather_ref<<<m.n_blocks, 256, 0, s>>>(m, pd, raw, perm, bpts);
}
void launch_init_state(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       uint32_t* hist1) {
  k_init_state<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st);
  k_zero_hist<<<(n_pairs * kHistBins + 255) / 256, 256, 0, s>>>(n_pairs, hist1);
}
bool launch_normals(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                    const uint2* nodes, const int32_t* parent, const float4* bpts, float4* bnrm,
                    int knn) {
  if (!m.n_blocks) return true;
  switch (knn) {
    case 10: k_normals<10><<<m.n_blocks, 256, 0, s>>>(m, pd, st, nodes, parent, bpts, bnrm); break;
    case 20: k_normals<20><<<m.n_blocks, 256, 0, s>>>(m, pd, st, nodes, parent, bpts, bnrm); break;
    case 30: k_normals<30><<<m.n_blocks, 256, 0, s>>>(m, pd, st, nodes, parent, bpts, bnrm); break;
    default: return false;
  }
  return true;
}
void launch_icp_nn(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                   const float4* read_c, const uint2* nodes, const int32_t* parent,
                   const float4* bpts, int32_t* match, float* d2, uint32_t* hist1,
                   const IcpParams& prm) {
  if (m.n_blocks)
    k_icp_nn<<<m.n_blocks, kNNBlock, 0, s>>>(m, pd, st, read_c, nodes, parent, bpts, match, d2,
                                             hist1, prm);
}
void launch_icp_select(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const float* d2, const uint32_t* hist1) {
  k_icp_select<<<n_pairs, 1024, 0, s>>>(pd, st, d2, hist1);
}
void launch_icp_reduce(hipStream_t s, BlockMap m, const PairDesc* pd, const PairState* st,
                       const float4* read_c, const int32_t* match, const float* d2,
                       const float4* bpts, const float4* bnrm, double* slab) {
  if (m.n_blocks)
    k_icp_reduce<<<m.n_blocks, kNNBlock, 0, s>>>(m, pd, st, read_c, match, d2, bpts, bnrm, slab);
}
void launch_icp_update(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const double* slab, uint32_t* hist1, const IcpParams& prm) {
  k_icp_update<<<n_pairs, 256, 0, s>>>(pd, st, slab, hist1, prm);
}
void launch_finalize(hipStream_t s, int n_pairs, const PairDesc* pd, const PairState* st,
                     float* outT) {
  k_finalize<<<(n_pairs + 63) / 64, 64, 0, s>>>(n_pairs, pd, st, outT);
}
bool launch_knn_generic(hipStream_t s, int nq, const float4* q, const uint2* nodes,
                        const int32_t* parent, const float4* bpts, int k, float maxE2,
                        float maxR2, int32_t* ids, float* d2, unsigned long long* touched) {
  const int g = (nq + 255) / 256;
  if (!g) return true;
  switch (k) {
    case 1: k_knn_generic<1><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched); break;
    case 4: k_knn_generic<4><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched); break;
    case 10: k_knn_generic<10><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched); break;
    case 20: k_knn_generic<20><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched); break;
    case 30: k_knn_generic<30><<<g, 256, 0, s>>>(nq, q, nodes, parent, bpts, maxE2, maxR2, ids, d2, touched); break;
    default: return false;
  }
  return true;
}
void launch_hist_d2(hipStream_t s, BlockMap m, const PairDesc* pd, const float* d2,
                    uint32_t* hist1) {
  if (m.n_blocks) k_hist_d2<<<m.n_blocks, 256, 0, s>>>(m, pd, d2, hist1);
}
void launch_transform(hipStream_t s, int n, const float* T, const float4* in, float4* out) {
  if (n > 0) k_transform<<<(n + 255) / 256, 256, 0, s>>>(n, T, in, out);
}
void launch_solve6(hipStream_t s, const double* A, const double* b, double* x, int32_t* path) {
  k_solve6<<<1, 64, 0, s>>>(A, b, x, path);
}

}  // namespace aicp
