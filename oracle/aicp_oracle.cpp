// aicp_oracle.cpp — TEST INFRASTRUCTURE ONLY (see aicp_oracle.h).
//
// CPU restatement of the reference ICP hot path, written from the algorithm descriptions in
// SURVEY.md Appendix A (libpointmatcher 1.2.x / libnabo / octomap 1.9 are [ext] dependencies
// that are not in /root/reference and not in this image) and from the aicp_core call sites:
//   ICP driver usage          aicp_core/src/registration/pointmatcher_registration.cpp:92-151
//   PCL -> DataPoints layout  aicp_core/src/utils/cloudIO.cpp:81-98 (pad row = 1)
//   ratio auto-tune           aicp_core/src/registration/app.cpp:197-205,
//                             aicp_core/src/utils/fileIO.cpp:179-214
//   chain + parameters        aicp_core/config/icp/icp_autotuned_default.yaml:9-51
//   octree overlap            aicp_core/src/overlap/octrees_overlap.cpp:29-241
//
// Float semantics: compiled with -ffp-contract=off (the reference binaries target generic
// x86-64 without FMA), point arithmetic in float in the reference's operation order. The
// 6x6 normal equations are accumulated in double from exact float products (the reference
// uses a float Eigen GEMM whose blocking order is not reproducible); the 3x3 / 6x6
// decompositions run in double with float-precision rank thresholds. These deviations are
// tolerance-level and documented in DESIGN.md.
#include "aicp_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <unordered_set>
#include <vector>

namespace {

// round(x * 2^40) as int64 (|x| < 2^23), saturating
int64_t fixed40(float x) {
  const double v = std::rint((double)x * 1099511627776.0);
  if (!(v < 9.2233720368547748e18)) return INT64_MAX;
  if (!(v > -9.2233720368547748e18)) return INT64_MIN;
  return (int64_t)v;
}

float mean_fixed40(__int128 acc, uint64_t n) {
  const bool neg = acc < 0;
  const unsigned __int128 mag = neg ? (unsigned __int128)(-acc) : (unsigned __int128)acc;
  const uint64_t hi = (uint64_t)(mag >> 64), lo = (uint64_t)mag;
  const double dm = (double)hi * 18446744073709551616.0 + (double)lo;
  const double mm = dm * (1.0 / 1099511627776.0) / (double)n;
  return (float)(neg ? -mm : mm);
}


constexpr float kInf = std::numeric_limits<float>::infinity();

// ------------------------------------------------------------------------------------------
// libnabo KDTreeUnbalancedPtInLeavesImplicitBoundsStackOpt, dim = 3
// ------------------------------------------------------------------------------------------
constexpr unsigned kDim = 3;
constexpr unsigned kDimBits = 2;  // getStorageBitCount(3)
constexpr uint32_t kDimMask = 3;

struct Node {
  uint32_t dimChildBucketSize;
  union {
    float cutVal;
    uint32_t bucketIndex;
  };
};
struct BucketEntry {
  const float* pt;
  int32_t index;
};
struct BuildPoint {
  float pos[3];
  int32_t index;
};

}  // namespace

struct ao_tree {
  std::vector<float> cloud;  // packed xyz copy
  std::vector<Node> nodes;
  std::vector<BucketEntry> buckets;
  uint32_t bucketSize = 8;
  int32_t depth = 0;
  int32_t leaves = 0;
};

namespace {

inline uint32_t mkDCB(uint32_t dim, uint32_t child) { return dim | (child << kDimBits); }
inline uint32_t getDim(uint32_t v) { return v & kDimMask; }
inline uint32_t getChildBucketSize(uint32_t v) { return v >> kDimBits; }

struct TreeBuilder {
  ao_tree* t;
  std::vector<BuildPoint>& bp;

  unsigned build(int first, int last, const float minV[3], const float maxV[3], int depth) {
    const int count = last - first;
    const unsigned pos = (unsigned)t->nodes.size();
    if (depth > t->depth) t->depth = depth;
    if (count <= (int)t->bucketSize) {
      const uint32_t initBucketsSize = (uint32_t)t->buckets.size();
      for (int i = 0; i < count; ++i) {
        const int32_t index = bp[first + i].index;
        t->buckets.push_back(BucketEntry{&t->cloud[3 * (size_t)index], index});
      }
      Node nd;
      nd.dimChildBucketSize = mkDCB(kDim, (uint32_t)count);
      nd.bucketIndex = initBucketsSize;
      t->nodes.push_back(nd);
      t->leaves++;
      return pos;
    }
    // largest dimension of the box: argMax with strict '>' from maxVal 0
    unsigned cutDim = 0;
    {
      float best = 0;
      for (unsigned i = 0; i < kDim; ++i) {
        const float e = maxV[i] - minV[i];
        if (e > best) {
          best = e;
          cutDim = i;
        }
      }
    }
    const float idealCutVal = (maxV[cutDim] + minV[cutDim]) / 2;
    float lo = std::numeric_limits<float>::max(), hi = std::numeric_limits<float>::lowest();
    for (int i = first; i < last; ++i) {
      const float v = bp[i].pos[cutDim];
      lo = std::min(v, lo);
      hi = std::max(v, hi);
    }
    float cutVal;
    if (idealCutVal < lo)
      cutVal = lo;
    else if (idealCutVal > hi)
      cutVal = hi;
    else
      cutVal = idealCutVal;

    BuildPoint* f = &bp[first];
    int l = 0, r = count - 1;
    for (;;) {
      while (l < count && f[l].pos[cutDim] < cutVal) ++l;
      while (r >= 0 && f[r].pos[cutDim] >= cutVal) --r;
      if (l > r) break;
      std::swap(f[l], f[r]);
      ++l;
      --r;
    }
    const int br1 = l;
    r = count - 1;
    for (;;) {
      while (l < count && f[l].pos[cutDim] <= cutVal) ++l;
      while (r >= br1 && f[r].pos[cutDim] > cutVal) --r;
      if (l > r) break;
      std::swap(f[l], f[r]);
      ++l;
      --r;
    }
    const int br2 = l;
    int leftCount;
    if (idealCutVal < lo)
      leftCount = 1;
    else if (idealCutVal > hi)
      leftCount = count - 1;
    else if (br1 > count / 2)
      leftCount = br1;
    else if (br2 < count / 2)
      leftCount = br2;
    else
      leftCount = count / 2;

    float leftMax[3] = {maxV[0], maxV[1], maxV[2]};
    leftMax[cutDim] = cutVal;
    float rightMin[3] = {minV[0], minV[1], minV[2]};
    rightMin[cutDim] = cutVal;

    Node nd;
    nd.dimChildBucketSize = 0;
    nd.cutVal = cutVal;
    t->nodes.push_back(nd);
    build(first, first + leftCount, minV, leftMax, depth + 1);
    const unsigned rightChild = build(first + leftCount, last, rightMin, maxV, depth + 1);
    t->nodes[pos].dimChildBucketSize = mkDCB(cutDim, rightChild);
    return pos;
  }
};

// IndexHeapBruteForceVector: ascending array, head = last element.
struct Heap {
  std::vector<float> val;
  std::vector<int32_t> idx;
  explicit Heap(int k) : val(k, kInf), idx(k, -1) {}
  void reset() {
    std::fill(val.begin(), val.end(), kInf);
    std::fill(idx.begin(), idx.end(), -1);
  }
  float head() const { return val.back(); }
  void replaceHead(int32_t index, float value) {
    size_t i;
    for (i = val.size() - 1; i > 0; --i) {
      if (val[i - 1] > value) {
        val[i] = val[i - 1];
        idx[i] = idx[i - 1];
      } else {
        break;
      }
    }
    val[i] = value;
    idx[i] = index;
  }
};

struct Searcher {
  const ao_tree* t;
  const float* q;
  Heap* heap;
  float off[3];
  float maxError2, maxRadius2;
  bool allowSelf;
  uint64_t touchedPts = 0, touchedNodes = 0;

  void recurse(unsigned n, float rd) {
    const Node& node = t->nodes[n];
    const uint32_t cd = getDim(node.dimChildBucketSize);
    if (cd == kDim) {
      const BucketEntry* bucket = &t->buckets[node.bucketIndex];
      const uint32_t bucketSize = getChildBucketSize(node.dimChildBucketSize);
      for (uint32_t i = 0; i < bucketSize; ++i) {
        float dist = 0;
        for (unsigned d = 0; d < kDim; ++d) {
          const float diff = q[d] - bucket->pt[d];
          dist += diff * diff;
        }
        if (dist <= maxRadius2 && dist < heap->head() &&
            (allowSelf || dist > std::numeric_limits<float>::epsilon()))
          heap->replaceHead(bucket->index, dist);
        ++bucket;
      }
      touchedPts += bucketSize;
      return;
    }
    touchedNodes++;
    const unsigned rightChild = getChildBucketSize(node.dimChildBucketSize);
    const float old_off = off[cd];
    const float new_off = q[cd] - node.cutVal;
    if (new_off > 0) {
      recurse(rightChild, rd);
      rd += -old_off * old_off + new_off * new_off;
      if (rd <= maxRadius2 && rd * maxError2 < heap->head()) {
        off[cd] = new_off;
        recurse(n + 1, rd);
        off[cd] = old_off;
      }
    } else {
      recurse(n + 1, rd);
      rd += -old_off * old_off + new_off * new_off;
      if (rd <= maxRadius2 && rd * maxError2 < heap->head()) {
        off[cd] = new_off;
        recurse(rightChild, rd);
        off[cd] = old_off;
      }
    }
  }
};

int tree_build_impl(const float* pts, int64_t n, int64_t stride, int bucket, ao_tree* t) {
  t->bucketSize = (uint32_t)bucket;
  t->cloud.resize(3 * (size_t)n);
  for (int64_t i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) t->cloud[3 * i + d] = pts[i * stride + d];
  std::vector<BuildPoint> bp((size_t)n);
  float minV[3], maxV[3];
  for (int d = 0; d < 3; ++d) {
    minV[d] = std::numeric_limits<float>::max();
    maxV[d] = std::numeric_limits<float>::lowest();
  }
  for (int64_t i = 0; i < n; ++i) {
    for (int d = 0; d < 3; ++d) {
      const float v = t->cloud[3 * i + d];
      bp[i].pos[d] = v;
      minV[d] = std::min(minV[d], v);
      maxV[d] = std::max(maxV[d], v);
    }
    bp[i].index = (int32_t)i;
  }
  t->nodes.reserve((size_t)(n / std::max(1, bucket / 2) + 2));
  t->buckets.reserve((size_t)n);
  TreeBuilder b{t, bp};
  b.build(0, (int)n, minV, maxV, 0);
  return 0;
}

void tree_knn_impl(const ao_tree* t, const float* q, int64_t nq, int64_t qstride, int k,
                   float epsilon, bool allowSelf, float maxRadius, int32_t* ids, float* d2,
                   uint64_t* touchedPts, uint64_t* touchedNodes) {
  Heap heap(k);
  Searcher s;
  s.t = t;
  s.heap = &heap;
  s.maxError2 = (1 + epsilon) * (1 + epsilon);
  s.maxRadius2 = maxRadius * maxRadius;
  s.allowSelf = allowSelf;
  for (int64_t i = 0; i < nq; ++i) {
    s.q = q + i * qstride;
    s.off[0] = s.off[1] = s.off[2] = 0;
    heap.reset();
    s.recurse(0, 0);
    for (int j = 0; j < k; ++j) {
      ids[i * k + j] = heap.val[j] == kInf ? -1 : heap.idx[j];
      d2[i * k + j] = heap.val[j];
    }
  }
  if (touchedPts) *touchedPts += s.touchedPts;
  if (touchedNodes) *touchedNodes += s.touchedNodes;
}

// ------------------------------------------------------------------------------------------
// Small dense linear algebra in double
// ------------------------------------------------------------------------------------------

// Full-pivoting Householder QR of an n x n matrix (row-major, in place), following Eigen's
// FullPivHouseholderQR::computeInPlace: pivot = max |a| of the remaining corner, early stop
// when the corner is negligible vs the first pivot (prec = n * eps_float), rank = #|R_ii| >
// n * eps_float * maxpivot. eps is float's because the reference decomposes float matrices.
struct FullPivQR {
  int n;
  double qr[36];
  double hcoeff[6];
  int rowT[6], colT[6];
  int nonzero;
  double maxpivot;
  int rank;

  void compute(const double* A, int n_) {
    n = n_;
    std::memcpy(qr, A, sizeof(double) * n * n);
    const double prec = (double)FLT_EPSILON * n;
    nonzero = n;
    maxpivot = 0;
    double biggest = 0;
    for (int k = 0; k < n; ++k) {
      int br = k, bc = k;
      double bv = -1;
      // Eigen's maxCoeff visits column-major: first max in column order
      for (int c = k; c < n; ++c)
        for (int r = k; r < n; ++r) {
          const double v = std::fabs(qr[r * n + c]);
          if (v > bv) {
            bv = v;
            br = r;
            bc = c;
          }
        }
      if (k == 0) biggest = bv;
      if (bv <= biggest * prec) {
        nonzero = k;
        for (int i = k; i < n; ++i) {
          rowT[i] = i;
          colT[i] = i;
          hcoeff[i] = 0;
        }
        break;
      }
      rowT[k] = br;
      colT[k] = bc;
      if (br != k)
        for (int c = k; c < n; ++c) std::swap(qr[k * n + c], qr[br * n + c]);
      if (bc != k)
        for (int r = 0; r < n; ++r) std::swap(qr[r * n + k], qr[r * n + bc]);
      // makeHouseholderInPlace on column k rows k..n-1
      double tailSq = 0;
      for (int r = k + 1; r < n; ++r) tailSq += qr[r * n + k] * qr[r * n + k];
      const double c0 = qr[k * n + k];
      double beta, tau;
      if (tailSq <= std::numeric_limits<double>::min()) {
        tau = 0;
        beta = c0;
        for (int r = k + 1; r < n; ++r) qr[r * n + k] = 0;
      } else {
        beta = std::sqrt(c0 * c0 + tailSq);
        if (c0 >= 0) beta = -beta;
        for (int r = k + 1; r < n; ++r) qr[r * n + k] /= (c0 - beta);
        tau = (beta - c0) / beta;
      }
      hcoeff[k] = tau;
      qr[k * n + k] = beta;
      if (std::fabs(beta) > maxpivot) maxpivot = std::fabs(beta);
      // apply H = I - tau v v^T (v = [1; qr[k+1..,k]]) to columns k+1..n-1
      for (int c = k + 1; c < n; ++c) {
        double s = qr[k * n + c];
        for (int r = k + 1; r < n; ++r) s += qr[r * n + k] * qr[r * n + c];
        s *= tau;
        qr[k * n + c] -= s;
        for (int r = k + 1; r < n; ++r) qr[r * n + c] -= s * qr[r * n + k];
      }
    }
    const double thr = std::fabs(maxpivot) * ((double)FLT_EPSILON * n);
    rank = 0;
    for (int i = 0; i < nonzero; ++i) rank += (std::fabs(qr[i * n + i]) > thr);
  }
  // Q (n x n, row-major) = P_0 H_0 P_1 H_1 ... P_{n-1} H_{n-1}, built as Eigen's
  // FullPivHouseholderQRMatrixQReturnType::evalTo: from the last step down, apply H_k to
  // rows k.. then swap rows k and rowT[k].
  void matrixQ(double* Q) const {
    for (int i = 0; i < n * n; ++i) Q[i] = 0;
    for (int i = 0; i < n; ++i) Q[i * n + i] = 1;
    for (int k = n - 1; k >= 0; --k) {
      const double tau = (k < nonzero) ? hcoeff[k] : 0.0;
      if (tau != 0) {
        for (int c = k; c < n; ++c) {
          double s = Q[k * n + c];
          for (int r = k + 1; r < n; ++r) s += qr[r * n + k] * Q[r * n + c];
          s *= tau;
          Q[k * n + c] -= s;
          for (int r = k + 1; r < n; ++r) Q[r * n + c] -= s * qr[r * n + k];
        }
      }
      const int r = (k < nonzero) ? rowT[k] : k;
      if (r != k)
        for (int c = 0; c < n; ++c) std::swap(Q[k * n + c], Q[r * n + c]);
    }
  }
  // column permutation as index map: (A P)[:, i] = A[:, perm[i]]
  void colPerm(int* perm) const {
    for (int i = 0; i < n; ++i) perm[i] = i;
    for (int k = 0; k < n; ++k) {
      const int c = (k < nonzero) ? colT[k] : k;
      std::swap(perm[k], perm[c]);
    }
  }
};

// Cholesky of an r x r SPD matrix (row-major) and solve; returns false if not PD.
bool llt_solve(const double* M, int r, const double* b, double* x) {
  double L[36] = {0};
  for (int j = 0; j < r; ++j) {
    double d = M[j * r + j];
    for (int k = 0; k < j; ++k) d -= L[j * r + k] * L[j * r + k];
    if (!(d > 0)) return false;
    const double ljj = std::sqrt(d);
    L[j * r + j] = ljj;
    for (int i = j + 1; i < r; ++i) {
      double s = M[i * r + j];
      for (int k = 0; k < j; ++k) s -= L[i * r + k] * L[j * r + k];
      L[i * r + j] = s / ljj;
    }
  }
  double y[6];
  for (int i = 0; i < r; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i * r + k] * y[k];
    y[i] = s / L[i * r + i];
  }
  for (int i = r - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < r; ++k) s -= L[k * r + i] * x[k];
    x[i] = s / L[i * r + i];
  }
  return true;
}

// Cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (row-major).
// Eigenvalues in w, eigenvectors as columns of V (row-major).
void jacobi_eig(const double* A, int n, double* w, double* V) {
  double a[36];
  std::memcpy(a, A, sizeof(double) * n * n);
  for (int i = 0; i < n * n; ++i) V[i] = 0;
  for (int i = 0; i < n; ++i) V[i * n + i] = 1;
  for (int sweep = 0; sweep < 64; ++sweep) {
    double offn = 0, diag = 0;
    for (int p = 0; p < n; ++p) {
      diag += a[p * n + p] * a[p * n + p];
      for (int q = p + 1; q < n; ++q) offn += a[p * n + q] * a[p * n + q];
    }
    if (offn <= 1e-30 * diag || offn == 0) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = a[p * n + q];
        if (apq == 0) continue;
        const double app = a[p * n + p], aqq = a[q * n + q];
        const double theta = (aqq - app) / (2 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        const double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

int solve6_impl(const double* A, const double* b, double* x, int32_t* path) {
  const int n = 6;
  FullPivQR qr;
  qr.compute(A, n);
  if (qr.rank == n) {
    if (path) *path = 0;
    if (llt_solve(A, n, b, x)) return 0;
    // not numerically PD in double: fall through to the pseudo-inverse
  } else {
    if (path) *path = 1;
    const int r = qr.rank;
    double Q[36];
    qr.matrixQ(Q);
    int perm[6];
    qr.colPerm(perm);
    // Q1t = Q^T[0:r, :]
    double Q1t[36];
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < n; ++j) Q1t[i * n + j] = Q[j * n + i];
    // R1 = (Q1t * A * P)[0:r, :]
    double AP[36];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) AP[i * n + j] = A[i * n + perm[j]];
    double R1[36];
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < n; ++j) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += Q1t[i * n + k] * AP[k * n + j];
        R1[i * n + j] = s;
      }
    double RRt[36];
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < r; ++j) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += R1[i * n + k] * R1[j * n + k];
        RRt[i * r + j] = s;
      }
    double qb[6];
    for (int i = 0; i < r; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += Q1t[i * n + k] * b[k];
      qb[i] = s;
    }
    double y[6];
    bool ok = (r > 0) && llt_solve(RRt, r, qb, y);
    if (ok) {
      double z[6];
      for (int j = 0; j < n; ++j) {  // z = triu(R1)^T y
        double s = 0;
        for (int i = 0; i < r; ++i)
          if (j >= i) s += R1[i * n + j] * y[i];
        z[j] = s;
      }
      for (int i = 0; i < n; ++i) x[perm[i]] = z[i];
      // b.isApprox(A x, 1e-5): ||b - Ax||^2 <= 1e-10 * min(||b||^2, ||Ax||^2)
      double ax[6], nb = 0, nax = 0, nd = 0;
      for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += A[i * n + k] * x[k];
        ax[i] = s;
        nb += b[i] * b[i];
        nax += s * s;
        nd += (b[i] - s) * (b[i] - s);
      }
      if (nd <= 1e-10 * std::min(nb, nax)) return 0;
    }
  }
  // fallback: double JacobiSVD solve == pseudo-inverse for symmetric PSD A
  if (path) *path = 2;
  double w[6], V[36];
  jacobi_eig(A, n, w, V);
  double wmax = 0;
  for (int i = 0; i < n; ++i) wmax = std::max(wmax, std::fabs(w[i]));
  const double thr = std::max(wmax * (n * DBL_EPSILON), std::numeric_limits<double>::min());
  for (int i = 0; i < n; ++i) x[i] = 0;
  for (int e = 0; e < n; ++e) {
    if (std::fabs(w[e]) <= thr) continue;
    double s = 0;
    for (int k = 0; k < n; ++k) s += V[k * n + e] * b[k];
    s /= w[e];
    for (int k = 0; k < n; ++k) x[k] += V[k * n + e] * s;
  }
  return 0;
}

// ------------------------------------------------------------------------------------------
// SurfaceNormalDataPointsFilter
// ------------------------------------------------------------------------------------------
void normal_from_neighbours(const float* pts, int64_t stride, const int32_t* ids, const float* d2,
                            int knn, float* nrm, float* density, int32_t* degenerate) {
  // d = neighbours with finite distance, in heap order
  float d[3][64];
  int realKnn = 0;
  for (int j = 0; j < knn; ++j) {
    if (d2[j] != kInf) {
      const float* p = pts + (int64_t)ids[j] * stride;
      d[0][realKnn] = p[0];
      d[1][realKnn] = p[1];
      d[2][realKnn] = p[2];
      ++realKnn;
    }
  }
  float mean[3];
  for (int r = 0; r < 3; ++r) {
    float s = 0;
    for (int j = 0; j < realKnn; ++j) s += d[r][j];
    mean[r] = s / (float)realKnn;
  }
  float NN[3][64];
  for (int r = 0; r < 3; ++r)
    for (int j = 0; j < realKnn; ++j) NN[r][j] = d[r][j] - mean[r];
  double C[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      double s = 0;
      for (int j = 0; j < realKnn; ++j) s += (double)NN[r][j] * (double)NN[c][j];
      C[r * 3 + c] = s / realKnn;
    }
  FullPivQR qr;
  qr.compute(C, 3);
  if (qr.rank + 1 >= 3) {
    double w[3], V[9];
    jacobi_eig(C, 3, w, V);
    int smallest = 0;
    double sv = std::numeric_limits<double>::max();
    for (int j = 0; j < 3; ++j)
      if (w[j] < sv) {
        sv = w[j];
        smallest = j;
      }
    for (int r = 0; r < 3; ++r) nrm[r] = (float)V[r * 3 + smallest];
  } else {
    // eigenVa = (1,0,0), eigenVe = I  ->  smallest id 1  ->  normal = e_y
    nrm[0] = 0;
    nrm[1] = 1;
    nrm[2] = 0;
    if (degenerate) (*degenerate)++;
  }
  if (density) {
    float mx = 0;
    for (int j = 0; j < realKnn; ++j) {
      const float nn = std::sqrt(NN[0][j] * NN[0][j] + NN[1][j] * NN[1][j] + NN[2][j] * NN[2][j]);
      mx = std::max(mx, nn);
    }
    const float vol = (float)((4. / 3.) * M_PI * std::pow((double)mx, 3));
    *density = (float)realKnn / vol;
  }
}

int normals_impl(const float* pts, int64_t n, int64_t stride, int knn, float* normals,
                 float* densities, int32_t* degenerate) {
  if (knn < 1 || knn > 64) return 2;
  ao_tree t;
  tree_build_impl(pts, n, stride, 8, &t);
  std::vector<int32_t> ids((size_t)knn);
  std::vector<float> d2((size_t)knn);
  int32_t deg = 0;
  Heap heap(knn);
  Searcher s;
  s.t = &t;
  s.heap = &heap;
  s.maxError2 = 1.0f;
  s.maxRadius2 = kInf;
  s.allowSelf = true;
  for (int64_t i = 0; i < n; ++i) {
    s.q = &t.cloud[3 * i];
    s.off[0] = s.off[1] = s.off[2] = 0;
    heap.reset();
    s.recurse(0, 0);
    for (int j = 0; j < knn; ++j) {
      ids[j] = heap.idx[j];
      d2[j] = heap.val[j];
    }
    normal_from_neighbours(t.cloud.data(), 3, ids.data(), d2.data(), knn, normals + 3 * i,
                           densities ? densities + i : nullptr, &deg);
  }
  if (degenerate) *degenerate = deg;
  return 0;
}

// ------------------------------------------------------------------------------------------
// float 4x4 helpers, column-major, sequential k order without FMA (Eigen GEMM/lazy product
// with k-loop accumulation starting from zero)
// ------------------------------------------------------------------------------------------
inline float M4(const float* m, int r, int c) { return m[c * 4 + r]; }
void mul4(const float* A, const float* B, float* C) {
  float t[16];
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) {
      float s = M4(A, r, 0) * M4(B, 0, c);
      s += M4(A, r, 1) * M4(B, 1, c);
      s += M4(A, r, 2) * M4(B, 2, c);
      s += M4(A, r, 3) * M4(B, 3, c);
      t[c * 4 + r] = s;
    }
  std::memcpy(C, t, sizeof(t));
}
inline void apply4(const float* T, const float* p, float* o) {
  for (int r = 0; r < 3; ++r) {
    float s = M4(T, r, 0) * p[0];
    s += M4(T, r, 1) * p[1];
    s += M4(T, r, 2) * p[2];
    s += M4(T, r, 3);
    o[r] = s;
  }
}
void ident4(float* T) {
  for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.f : 0.f;
}

// RigidTransformation::checkParameters: false when |1 - det(R)| > 0.001, R the
// top-left 3x3 block, det by Eigen's first-column cofactor expansion (float). Called by every
// transformations.apply: T_refMean_dataIn, each T_iter applied at the start of an iteration,
// and the final T applied to the output reading (pointmatcher_registration.cpp:128-129).
bool rigid_params_ok(const float* T) {
  const float a = M4(T, 0, 0) * (M4(T, 1, 1) * M4(T, 2, 2) - M4(T, 1, 2) * M4(T, 2, 1));
  const float b = M4(T, 1, 0) * (M4(T, 0, 1) * M4(T, 2, 2) - M4(T, 0, 2) * M4(T, 2, 1));
  const float c = M4(T, 2, 0) * (M4(T, 0, 1) * M4(T, 1, 2) - M4(T, 0, 2) * M4(T, 1, 1));
  const float det = (a - b) + c;
  return !(std::fabs(1.f - det) > 0.001f);
}

// Eigen::AngleAxis<float>(x.head(3).norm(), x.head(3).normalized()).toRotationMatrix()
// with translation x.segment(3,3); sin/cos evaluated in double and rounded to float.
void delta_transform(const float* x, float* T) {
  const float sq = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
  const float angle = std::sqrt(sq);
  float axis[3] = {x[0], x[1], x[2]};
  if (sq > 0) {
    for (int i = 0; i < 3; ++i) axis[i] = x[i] / angle;
  }
  const float sa = (float)std::sin((double)angle), c = (float)std::cos((double)angle);
  const float sin_axis[3] = {sa * axis[0], sa * axis[1], sa * axis[2]};
  const float cos1_axis[3] = {(1.f - c) * axis[0], (1.f - c) * axis[1], (1.f - c) * axis[2]};
  float R[3][3];
  float tmp = cos1_axis[0] * axis[1];
  R[0][1] = tmp - sin_axis[2];
  R[1][0] = tmp + sin_axis[2];
  tmp = cos1_axis[0] * axis[2];
  R[0][2] = tmp + sin_axis[1];
  R[2][0] = tmp - sin_axis[1];
  tmp = cos1_axis[1] * axis[2];
  R[1][2] = tmp - sin_axis[0];
  R[2][1] = tmp + sin_axis[0];
  for (int i = 0; i < 3; ++i) R[i][i] = cos1_axis[i] * axis[i] + c;
  bool nan = false;
  for (int r = 0; r < 3; ++r)
    for (int cc = 0; cc < 3; ++cc) {
      T[cc * 4 + r] = R[r][cc];
      if (R[r][cc] != R[r][cc]) nan = true;
    }
  for (int r = 0; r < 3; ++r) {
    T[12 + r] = x[3 + r];
    if (x[3 + r] != x[3 + r]) nan = true;
  }
  T[3] = T[7] = T[11] = 0;
  T[15] = 1;
  if (nan) {
    for (int r = 0; r < 3; ++r)
      for (int cc = 0; cc < 3; ++cc) T[cc * 4 + r] = (r == cc) ? 1.f : 0.f;
  }
}

// Eigen quaternion from a rotation matrix (Shoemake), in double.
void quat_from_R(const float* T, double* q /* w,x,y,z */) {
  double m[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) m[r][c] = (double)M4(T, r, c);
  double t = (m[0][0] + m[1][1]) + m[2][2];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[0] = 0.5 * t;
    t = 0.5 / t;
    q[1] = (m[2][1] - m[1][2]) * t;
    q[2] = (m[0][2] - m[2][0]) * t;
    q[3] = (m[1][0] - m[0][1]) * t;
  } else {
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
    double v[3];
    v[i] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m[k][j] - m[j][k]) * t;
    v[j] = (m[j][i] + m[i][j]) * t;
    v[k] = (m[k][i] + m[i][k]) * t;
    q[1] = v[0];
    q[2] = v[1];
    q[3] = v[2];
  }
}
double quat_angular_distance(const double* a, const double* b) {
  // d = a * conj(b); 2 * atan2(|d.vec|, |d.w|)
  const double bw = b[0], bx = -b[1], by = -b[2], bz = -b[3];
  const double w = a[0] * bw - a[1] * bx - a[2] * by - a[3] * bz;
  const double x = a[0] * bx + a[1] * bw + a[2] * bz - a[3] * by;
  const double y = a[0] * by + a[2] * bw + a[3] * bx - a[1] * bz;
  const double z = a[0] * bz + a[3] * bw + a[1] * by - a[2] * bx;
  return 2.0 * std::atan2(std::sqrt(x * x + y * y + z * z), std::fabs(w));
}

float quantile_impl(std::vector<float>& values, float quantile, int32_t* err) {
  if (values.empty()) {
    if (err) *err = 1;
    return 0;
  }
  if (err) *err = 0;
  if (quantile == 1.0f) return *std::max_element(values.begin(), values.end());
  size_t k = (size_t)((float)values.size() * quantile);
  if (k >= values.size()) k = values.size() - 1;  // the reference indexes out of range here
  std::nth_element(values.begin(), values.begin() + k, values.end());
  return values[k];
}

// ------------------------------------------------------------------------------------------
// octomap computeRayKeys / coordToKeyChecked
// ------------------------------------------------------------------------------------------
struct OcGeom {
  double resolution, resolution_factor;
  static constexpr int tree_max_val = 32768;
  // ((int)floor(factor * c)) + tree_max_val in [0, 2 * tree_max_val): x86's conversion gives
  // INT_MIN for NaN and out-of-range values, so those are rejected; the test is written on the
  // double to keep that behaviour without relying on the conversion
  bool coordToKeyChecked(double coordinate, uint32_t& key) const {
    const double f = std::floor(resolution_factor * coordinate);
    if (!(f >= -(double)tree_max_val && f < (double)tree_max_val)) return false;
    key = (uint32_t)((int)f + tree_max_val);
    return true;
  }
  bool coordToKeyChecked(const float* c, uint32_t* k) const {
    for (int i = 0; i < 3; ++i)
      if (!coordToKeyChecked((double)c[i], k[i])) return false;
    return true;
  }
  double keyToCoord(uint32_t key) const {
    return (double((int)key - (int)tree_max_val) + 0.5) * resolution;
  }
};
inline uint64_t packKey(const uint32_t* k) {
  return ((uint64_t)k[0] << 32) | ((uint64_t)k[1] << 16) | (uint64_t)k[2];
}

template <class F>
bool computeRayKeys(const OcGeom& g, const float* origin, const float* end, F&& add) {
  uint32_t ko[3], ke[3];
  if (!g.coordToKeyChecked(origin, ko) || !g.coordToKeyChecked(end, ke)) return false;
  if (ko[0] == ke[0] && ko[1] == ke[1] && ko[2] == ke[2]) return true;
  add(packKey(ko));
  float direction[3] = {end[0] - origin[0], end[1] - origin[1], end[2] - origin[2]};
  const float nsq = direction[0] * direction[0] + direction[1] * direction[1] +
                    direction[2] * direction[2];
  const float length = (float)std::sqrt((double)nsq);
  for (int i = 0; i < 3; ++i) direction[i] /= length;
  int step[3];
  double tMax[3], tDelta[3];
  uint32_t cur[3] = {ko[0], ko[1], ko[2]};
  for (int i = 0; i < 3; ++i) {
    if (direction[i] > 0.0)
      step[i] = 1;
    else if (direction[i] < 0.0)
      step[i] = -1;
    else
      step[i] = 0;
    if (step[i] != 0) {
      double voxelBorder = g.keyToCoord(cur[i]);
      voxelBorder += (float)(step[i] * g.resolution * 0.5);
      tMax[i] = (voxelBorder - (double)origin[i]) / (double)direction[i];
      tDelta[i] = g.resolution / (double)std::fabs(direction[i]);
    } else {
      tMax[i] = std::numeric_limits<double>::max();
      tDelta[i] = std::numeric_limits<double>::max();
    }
  }
  for (;;) {
    unsigned dim;
    if (tMax[0] < tMax[1]) {
      dim = (tMax[0] < tMax[2]) ? 0 : 2;
    } else {
      dim = (tMax[1] < tMax[2]) ? 1 : 2;
    }
    cur[dim] = (uint32_t)((int)cur[dim] + step[dim]) & 0xFFFF;
    tMax[dim] += tDelta[dim];
    if (cur[0] == ke[0] && cur[1] == ke[1] && cur[2] == ke[2]) break;
    const double dist_from_origin = std::min(std::min(tMax[0], tMax[1]), tMax[2]);
    if (dist_from_origin > (double)length) break;
    add(packKey(cur));
  }
  return true;
}

void cloud_keys(const OcGeom& g, const float* pts, int64_t n, int64_t stride, const double* org,
                std::unordered_set<uint64_t>& S) {
  const float origin[3] = {(float)org[0], (float)org[1], (float)org[2]};
  for (int64_t i = 0; i < n; ++i) {
    const float* p = pts + i * stride;
    computeRayKeys(g, origin, p, [&](uint64_t k) { S.insert(k); });
    uint32_t k[3];
    if (g.coordToKeyChecked(p, k)) S.insert(packKey(k));
  }
}

}  // namespace

// ==========================================================================================
// C API
// ==========================================================================================
extern "C" {

int ao_tree_build(const float* pts, int64_t n, int64_t stride, int bucket, ao_tree** out) {
  if (!pts || n < 1 || stride < 3 || bucket < 1 || !out) return 2;
  ao_tree* t = new ao_tree();
  tree_build_impl(pts, n, stride, bucket, t);
  *out = t;
  return 0;
}
void ao_tree_free(ao_tree* t) { delete t; }
int ao_tree_info(const ao_tree* t, int32_t* n_nodes, int32_t* depth, int32_t* n_leaves) {
  if (n_nodes) *n_nodes = (int32_t)t->nodes.size();
  if (depth) *depth = t->depth;
  if (n_leaves) *n_leaves = t->leaves;
  return 0;
}
int ao_tree_export(const ao_tree* t, int32_t* cd, float* cut, int32_t* right_or_count,
                   int32_t* bucket_start, int32_t* bucket_ids) {
  for (size_t i = 0; i < t->nodes.size(); ++i) {
    const Node& nd = t->nodes[i];
    const uint32_t d = getDim(nd.dimChildBucketSize);
    cd[i] = (int32_t)d;
    right_or_count[i] = (int32_t)getChildBucketSize(nd.dimChildBucketSize);
    if (d == kDim) {
      cut[i] = 0;
      bucket_start[i] = (int32_t)nd.bucketIndex;
    } else {
      cut[i] = nd.cutVal;
      bucket_start[i] = -1;
    }
  }
  for (size_t i = 0; i < t->buckets.size(); ++i) bucket_ids[i] = t->buckets[i].index;
  return 0;
}
int ao_tree_knn(const ao_tree* t, const float* q, int64_t nq, int64_t qstride, int k,
                float epsilon, int allow_self, float max_radius, int32_t* ids, float* d2,
                uint64_t* touched_points, uint64_t* touched_nodes) {
  if (!t || k < 1) return 2;
  tree_knn_impl(t, q, nq, qstride, k, epsilon, allow_self != 0, max_radius, ids, d2,
                touched_points, touched_nodes);
  return 0;
}

int ao_partition_sequential(float* v, int32_t* idx, int32_t count, float cut, int32_t* pbr1,
                            int32_t* pbr2) {
  int l = 0, r = count - 1;
  for (;;) {
    while (l < count && v[l] < cut) ++l;
    while (r >= 0 && v[r] >= cut) --r;
    if (l > r) break;
    std::swap(v[l], v[r]);
    std::swap(idx[l], idx[r]);
    ++l;
    --r;
  }
  const int br1 = l;
  r = count - 1;
  for (;;) {
    while (l < count && v[l] <= cut) ++l;
    while (r >= br1 && v[r] > cut) --r;
    if (l > r) break;
    std::swap(v[l], v[r]);
    std::swap(idx[l], idx[r]);
    ++l;
    --r;
  }
  *pbr1 = br1;
  *pbr2 = l;
  return 0;
}

// Prefix-count form of the same two passes: in [lo, hi) with left predicate 'good', the
// j-th bad element left of the split swaps with the j-th good element right of it counted
// from the end -- the j of each element is a prefix count, so a parallel build can compute
// every destination independently.
int ao_partition_parallel(float* v, int32_t* idx, int32_t count, float cut, int32_t* pbr1,
                          int32_t* pbr2) {
  // pass 1: good-left = (v < cut) over [0, count)
  auto pass = [&](int lo, int hi, bool le) -> int {
    auto goodL = [&](float x) { return le ? (x <= cut) : (x < cut); };
    int nGood = 0;
    for (int i = lo; i < hi; ++i) nGood += goodL(v[i]);
    const int split = lo + nGood;
    std::vector<int> leftBad, rightBad;  // positions
    for (int i = lo; i < split; ++i)
      if (!goodL(v[i])) leftBad.push_back(i);
    for (int i = hi - 1; i >= split; --i)
      if (goodL(v[i])) rightBad.push_back(i);
    // every pair (leftBad[j], rightBad[j]) swaps; a parallel build computes j by prefix counts
    for (size_t j = 0; j < leftBad.size(); ++j) {
      std::swap(v[leftBad[j]], v[rightBad[j]]);
      std::swap(idx[leftBad[j]], idx[rightBad[j]]);
    }
    return split;
  };
  const int br1 = pass(0, count, false);
  const int br2 = pass(br1, count, true);
  *pbr1 = br1;
  *pbr2 = br2;
  return 0;
}

int ao_surface_normals(const float* pts, int64_t n, int64_t stride, int knn, float* normals,
                       float* densities, int32_t* degenerate) {
  if (!pts || n < 1 || !normals) return 2;
  return normals_impl(pts, n, stride, knn, normals, densities, degenerate);
}

float ao_dists_quantile(const float* d2, int64_t n, float quantile, int32_t* err) {
  std::vector<float> v;
  v.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i)
    if (d2[i] != kInf) v.push_back(d2[i]);
  return quantile_impl(v, quantile, err);
}

int ao_solve6(const double* A, const double* b, double* x, int32_t* path) {
  return solve6_impl(A, b, x, path);
}

int ao_icp(const float* ref, int64_t m, int64_t rs, const float* read, int64_t n, int64_t ds,
           const float* T0, const ao_icp_config* cfg, float* T_out, ao_icp_stats* st) {
  ao_icp_stats dummy;
  if (!st) st = &dummy;
  std::memset(st, 0, sizeof(*st));
  if (!ref || !read || m < 1 || n < 1 || !cfg || !T_out) return st->status = 2;
  const int maxIter = cfg->max_iter;

  // 1. reference filters: SurfaceNormal on the raw reference
  std::vector<float> refn((size_t)m * 3);
  int32_t deg = 0;
  if (!cfg->normals_on_centered) normals_impl(ref, m, rs, cfg->knn_normals, refn.data(), nullptr, &deg);

  // 2. centre of mass and centred reference. The reference's Eigen float row sum depends on
  // the summation order; this restatement fixes an order-independent definition that the
  // device shares: coordinates rounded to multiples of 2^-40, summed exactly
  // (128-bit), then |S| as double * 2^-40 / m rounded to float.
  float mean[3];
  for (int d = 0; d < 3; ++d) {
    __int128 acc = 0;
    for (int64_t i = 0; i < m; ++i) acc += (__int128)fixed40(ref[i * rs + d]);
    mean[d] = mean_fixed40(acc, (uint64_t)m);
  }
  std::vector<float> refc((size_t)m * 3);
  for (int64_t i = 0; i < m; ++i)
    for (int d = 0; d < 3; ++d) refc[3 * i + d] = ref[i * rs + d] - mean[d];

  // 3. matcher->init(reference)
  ao_tree tree;
  tree_build_impl(refc.data(), m, 3, cfg->bucket_size, &tree);
  st->tree_depth = tree.depth;
  st->tree_nodes = (int32_t)tree.nodes.size();
  if (cfg->normals_on_centered) {
    // device design: kNN20 on the centred matcher tree
    Heap heap(cfg->knn_normals);
    Searcher s;
    s.t = &tree;
    s.heap = &heap;
    s.maxError2 = 1.0f;
    s.maxRadius2 = kInf;
    s.allowSelf = true;
    std::vector<int32_t> ids(cfg->knn_normals);
    std::vector<float> dd(cfg->knn_normals);
    for (int64_t i = 0; i < m; ++i) {
      s.q = &refc[3 * i];
      s.off[0] = s.off[1] = s.off[2] = 0;
      heap.reset();
      s.recurse(0, 0);
      for (int j = 0; j < cfg->knn_normals; ++j) {
        ids[j] = heap.idx[j];
        dd[j] = heap.val[j];
      }
      normal_from_neighbours(refc.data(), 3, ids.data(), dd.data(), cfg->knn_normals,
                             &refn[3 * i], nullptr, &deg);
    }
  }
  st->degenerate_normals = deg;
  for (int d = 0; d < 3; ++d) st->mean[d] = mean[d];

  // 4./5. reading in the reference-mean frame: T_refMean_dataIn = T_refIn_refMean^-1 * T0
  float Tmean[16], TmeanInv[16], Tinit[16], TrmDin[16];
  ident4(Tmean);
  ident4(TmeanInv);
  for (int d = 0; d < 3; ++d) {
    Tmean[12 + d] = mean[d];
    TmeanInv[12 + d] = -mean[d];
  }
  if (T0)
    std::memcpy(Tinit, T0, sizeof(Tinit));
  else
    ident4(Tinit);
  mul4(TmeanInv, Tinit, TrmDin);
  if (!rigid_params_ok(TrmDin)) return st->status = 5;  // TransformationError
  std::vector<float> rd((size_t)n * 3);
  for (int64_t i = 0; i < n; ++i) {
    const float p[3] = {read[i * ds + 0], read[i * ds + 1], read[i * ds + 2]};
    apply4(TrmDin, p, &rd[3 * i]);
  }

  // 6. loop
  float Titer[16];
  ident4(Titer);
  std::vector<double> qhist, thist;  // quaternion (4) and translation (3) history
  auto push_hist = [&](const float* T) {
    double q[4];
    quat_from_R(T, q);
    for (int i = 0; i < 4; ++i) qhist.push_back(q[i]);
    for (int i = 0; i < 3; ++i) thist.push_back((double)T[12 + i]);
  };
  push_hist(Titer);
  std::vector<int32_t> ids((size_t)n);
  std::vector<float> d2((size_t)n), step((size_t)n * 3), vals;
  const float maxError2 = (1 + cfg->nn_epsilon) * (1 + cfg->nn_epsilon);
  const float maxRadius2 = cfg->nn_max_dist * cfg->nn_max_dist;
  Heap heap(1);
  Searcher s;
  s.t = &tree;
  s.heap = &heap;
  s.maxError2 = maxError2;
  s.maxRadius2 = maxRadius2;
  s.allowSelf = true;
  int iter = 0;
  bool iterate = true;
  while (iterate) {
    if (!rigid_params_ok(Titer)) return st->status = 5;  // TransformationError
    for (int64_t i = 0; i < n; ++i) apply4(Titer, &rd[3 * i], &step[3 * i]);
    for (int64_t i = 0; i < n; ++i) {
      s.q = &step[3 * i];
      s.off[0] = s.off[1] = s.off[2] = 0;
      heap.reset();
      s.recurse(0, 0);
      ids[i] = heap.val[0] == kInf ? -1 : heap.idx[0];
      d2[i] = heap.val[0];
    }
    vals.clear();
    for (int64_t i = 0; i < n; ++i)
      if (d2[i] != kInf) vals.push_back(d2[i]);
    int32_t qerr = 0;
    const float limit = quantile_impl(vals, cfg->trimmed_ratio, &qerr);
    if (qerr) return st->status = 1;  // "no outlier to filter"
    double A[36] = {0}, b[6] = {0};
    int64_t kept = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (!(d2[i] <= limit)) continue;
      ++kept;
      const float* p = &step[3 * i];
      const float* q = &refc[3 * (size_t)ids[i]];
      const float* nr = &refn[3 * (size_t)ids[i]];
      float F[6];
      F[0] = p[1] * nr[2] - p[2] * nr[1];
      F[1] = p[2] * nr[0] - p[0] * nr[2];
      F[2] = p[0] * nr[1] - p[1] * nr[0];
      F[3] = nr[0];
      F[4] = nr[1];
      F[5] = nr[2];
      const float dl[3] = {p[0] - q[0], p[1] - q[1], p[2] - q[2]};
      float dot = dl[0] * nr[0];
      dot += dl[1] * nr[1];
      dot += dl[2] * nr[2];
      for (int a = 0; a < 6; ++a) {
        for (int c = 0; c < 6; ++c) A[a * 6 + c] += (double)F[a] * (double)F[c];
        b[a] += (double)F[a] * (double)dot;
      }
    }
    if (kept == 0) return st->status = 1;  // "no point to minimize"
    for (int a = 0; a < 6; ++a) b[a] = -b[a];
    if (iter == 0) {
      std::memcpy(st->A0, A, sizeof(A));
      std::memcpy(st->b0, b, sizeof(b));
    }
    double xd[6];
    int32_t path = 0;
    solve6_impl(A, b, xd, &path);
    float x[6];
    for (int a = 0; a < 6; ++a) x[a] = (float)xd[a];
    float dT[16];
    delta_transform(x, dT);
    mul4(dT, Titer, Titer);
    st->inlier_ratio = (float)((double)(float)kept / (double)n);
    if (iter < AO_TRACE_MAX) {
      st->limit[iter] = limit;
      st->kept[iter] = (int32_t)kept;
      st->solve_path[iter] = path;
      std::memcpy(st->T_iter[iter], Titer, sizeof(Titer));
    }
    // checkers in YAML order: Counter, then Differential
    ++iter;
    if (iter >= maxIter) iterate = false;
    push_hist(Titer);
    const size_t sz = qhist.size() / 4;
    if (sz > (size_t)cfg->smooth_length) {
      double cv0 = 0, cv1 = 0;
      for (size_t i = sz - 1; i >= sz - cfg->smooth_length; --i) {
        cv0 += std::fabs(quat_angular_distance(&qhist[4 * i], &qhist[4 * (i - 1)]));
        const double dx = thist[3 * i] - thist[3 * (i - 1)];
        const double dy = thist[3 * i + 1] - thist[3 * (i - 1) + 1];
        const double dz = thist[3 * i + 2] - thist[3 * (i - 1) + 2];
        cv1 += std::sqrt(dx * dx + dy * dy + dz * dz);
      }
      cv0 /= cfg->smooth_length;
      cv1 /= cfg->smooth_length;
      if (cv0 != cv0 || cv1 != cv1) return st->status = 1;
      if (cv0 < (double)cfg->min_diff_rot && cv1 < (double)cfg->min_diff_trans) {
        if (iterate) st->converged = 1;
        iterate = false;
      }
    }
  }
  st->iterations = iter;
  st->nn_points_touched = s.touchedPts;
  st->nn_nodes_touched = s.touchedNodes;
  // T = T_refIn_refMean * T_iter * T_refMean_dataIn
  float tmp[16];
  mul4(Tmean, Titer, tmp);
  mul4(tmp, TrmDin, T_out);
  // registerClouds applies the final T to the reading (pointmatcher_registration.cpp:128-129)
  if (!rigid_params_ok(T_out)) return st->status = 5;
  return st->status = 0;
}

int ao_overlap(const float* ref, int64_t m, int64_t rs, const double* ref_origin,
               const float* read, int64_t n, int64_t ds, const double* read_origin,
               double resolution, float* overlap_percent, uint64_t* counts) {
  if (!ref || !read || !overlap_percent || resolution <= 0) return 2;
  OcGeom g{resolution, 1.0 / resolution};
  std::unordered_set<uint64_t> Sref, Sread;
  Sref.reserve((size_t)m * 8);
  Sread.reserve((size_t)n * 8);
  cloud_keys(g, ref, m, rs, ref_origin, Sref);
  cloud_keys(g, read, n, ds, read_origin, Sread);
  uint64_t ov = 0;
  for (uint64_t k : Sref) ov += Sread.count(k);
  const float a = float(ov) / float(Sref.size());
  const float b = float(ov) / float(Sread.size());
  *overlap_percent = (float)(std::min(a, b) * 100.0);
  if (counts) {
    counts[0] = Sref.size();
    counts[1] = Sread.size();
    counts[2] = ov;
  }
  return 0;
}

int64_t ao_ray_keys(const float origin[3], const float end[3], double resolution, uint64_t* out,
                    int64_t cap) {
  OcGeom g{resolution, 1.0 / resolution};
  int64_t cnt = 0;
  const bool ok = computeRayKeys(g, origin, end, [&](uint64_t k) {
    if (cnt < cap) out[cnt] = k;
    ++cnt;
  });
  return ok ? cnt : -1;
}

float ao_quantize_ratio(float ratio) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%g", (double)ratio);  // ostream << float, precision 6
  return std::strtof(buf, nullptr);                      // lexical_cast<float>
}

float ao_autotune_ratio(float overlap_percent) {
  float current_ratio = (float)(overlap_percent / 100.0);
  if (current_ratio < 0.25)
    current_ratio = 0.25;
  else if (current_ratio > 0.70)
    current_ratio = 0.70;
  return ao_quantize_ratio(current_ratio);
}

}  // extern "C"

/* ---------------------------------------------------------------- box crop --
 * getPointsInOrientedBox, filteringUtils.cpp:619-637, through its [ext] dependencies:
 *  - Eigen 3.3 MatrixBase::eulerAngles(0,1,2) (Geometry/EulerAngles.h): angles (a,b,c) with
 *    R = Rx(a) Ry(b) Rz(c), a in [0, pi];
 *  - pcl::CropBox<PointXYZ>::applyFilter (filters/impl/crop_box.hpp, PCL 1.8): translation
 *    subtracted first, then the inverse of pcl::getTransformation(0,0,0, rx,ry,rz)
 *    (= Rz(rz) Ry(ry) Rx(rx), note the reversed order against eulerAngles) applied with
 *    pcl::transformPoint; kept iff min <= local <= max on every axis; non-finite points dropped.
 * Float throughout, like PointXYZ and Affine3f. Parity unpinned against PCL/Eigen (neither is
 * in the image); the device path is checked against this restatement. */
namespace {
void euler_012(const float R[3][3], float res[3]) {
  const int i = 0, j = 1, k = 2;  // a0 = 0, a1 = 1 -> odd = 0
  res[0] = std::atan2(R[j][k], R[k][k]);
  const float c2 = std::sqrt(R[i][i] * R[i][i] + R[i][j] * R[i][j]);
  if (res[0] > 0.f) {
    res[0] -= float(M_PI);
    res[1] = std::atan2(-R[i][k], -c2);
  } else {
    res[1] = std::atan2(-R[i][k], c2);
  }
  const float s1 = std::sin(res[0]), c1 = std::cos(res[0]);
  res[2] = std::atan2(s1 * R[k][i] - c1 * R[j][i], c1 * R[j][j] - s1 * R[k][j]);
  for (int q = 0; q < 3; ++q) res[q] = -res[q];
}

void crop_inverse(const float rpy[3], float inv[3][3]) {
  // pcl::getTransformation(0,0,0, roll, pitch, yaw)
  const float A = std::cos(rpy[2]), B = std::sin(rpy[2]), C = std::cos(rpy[1]), D = std::sin(rpy[1]),
              E = std::cos(rpy[0]), F = std::sin(rpy[0]);
  const float DE = D * E, DF = D * F;
  const float m[3][3] = {{A * C, A * DF - B * E, B * F + A * DE},
                         {B * C, A * E + B * DF, B * DE - A * F},
                         {-D, C * F, C * E}};
  // Affine3f::inverse(): linear().inverse() by cofactors
  const float c00 = m[1][1] * m[2][2] - m[1][2] * m[2][1];
  const float c10 = m[1][2] * m[2][0] - m[1][0] * m[2][2];
  const float c20 = m[1][0] * m[2][1] - m[1][1] * m[2][0];
  const float det = m[0][0] * c00 + m[0][1] * c10 + m[0][2] * c20;
  const float id = 1.f / det;
  inv[0][0] = c00 * id;
  inv[1][0] = c10 * id;
  inv[2][0] = c20 * id;
  inv[0][1] = (m[0][2] * m[2][1] - m[0][1] * m[2][2]) * id;
  inv[1][1] = (m[0][0] * m[2][2] - m[0][2] * m[2][0]) * id;
  inv[2][1] = (m[0][1] * m[2][0] - m[0][0] * m[2][1]) * id;
  inv[0][2] = (m[0][1] * m[1][2] - m[0][2] * m[1][1]) * id;
  inv[1][2] = (m[0][2] * m[1][0] - m[0][0] * m[1][2]) * id;
  inv[2][2] = (m[0][0] * m[1][1] - m[0][1] * m[1][0]) * id;
}
}  // namespace

extern "C" int ao_crop_box(const float* pts, int64_t n, int64_t stride, float mn, float mx,
                           const float origin[16], float* out, int64_t* out_n, float* rpy_out) {
  if (!pts || !origin || !out || !out_n || stride < 3) return 2;
  float R[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) R[r][c] = origin[c * 4 + r];
  const float t[3] = {origin[12], origin[13], origin[14]};
  float rpy[3];
  euler_012(R, rpy);
  if (rpy_out)
    for (int q = 0; q < 3; ++q) rpy_out[q] = rpy[q];
  float inv[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  const bool rot = rpy[0] != 0.f || rpy[1] != 0.f || rpy[2] != 0.f;
  if (rot) crop_inverse(rpy, inv);
  // `!inverse_transform.matrix().isIdentity()` (Eigen fuzzy test, float precision 1e-5)
  bool ident = true;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      ident = ident && (r == c ? std::fabs(inv[r][c] - 1.f) <= 1e-5f * std::fmin(std::fabs(inv[r][c]), 1.f)
                               : std::fabs(inv[r][c]) <= 1e-5f);
  if (ident)
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) inv[r][c] = r == c ? 1.f : 0.f;
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float* p = pts + i * stride;
    if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
    const float x = p[0] - t[0], y = p[1] - t[1], z = p[2] - t[2];
    float l[3];
    for (int r = 0; r < 3; ++r) l[r] = ((inv[r][0] * x + inv[r][1] * y) + inv[r][2] * z) + 0.f;
    if (l[0] < mn || l[1] < mn || l[2] < mn || l[0] > mx || l[1] > mx || l[2] > mx) continue;
    out[3 * m] = p[0];
    out[3 * m + 1] = p[1];
    out[3 * m + 2] = p[2];
    ++m;
  }
  *out_n = m;
  return 0;
}
