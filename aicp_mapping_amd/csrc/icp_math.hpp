// icp_math.hpp — small fixed-size math of the ICP update, callable on host and device.
//
// Float point arithmetic follows the operation order of the reference (Eigen lazy/GEMM
// products with a sequential k loop, no FMA: the library is compiled -ffp-contract=off).
// Decompositions run in double with float-precision rank thresholds:
//   solvePossiblyUnderdeterminedLinearSystem   (libpointmatcher ErrorMinimizer)
//   Eigen::AngleAxis -> rotation               (PointToPlaneErrorMinimizer::compute)
//   DifferentialTransformationChecker          (quaternion angular distance)
//   SurfaceNormalDataPointsFilter rank test + smallest eigenvector
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define AICP_HD __host__ __device__ inline

namespace aicp {

constexpr float kFltEps = 1.1920928955078125e-07f;
constexpr double kDblEps = 2.220446049250313e-16;
constexpr double kDblMin = 2.2250738585072014e-308;

AICP_HD float m4(const float* m, int r, int c) { return m[c * 4 + r]; }

AICP_HD void mul4(const float* A, const float* B, float* C) {
  float t[16];
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) {
      float s = m4(A, r, 0) * m4(B, 0, c);
      s += m4(A, r, 1) * m4(B, 1, c);
      s += m4(A, r, 2) * m4(B, 2, c);
      s += m4(A, r, 3) * m4(B, 3, c);
      t[c * 4 + r] = s;
    }
  for (int i = 0; i < 16; ++i) C[i] = t[i];
}

// T * (x, y, z, 1), rows 0..2
AICP_HD void apply4(const float* T, float x, float y, float z, float* o) {
  for (int r = 0; r < 3; ++r) {
    float s = m4(T, r, 0) * x;
    s += m4(T, r, 1) * y;
    s += m4(T, r, 2) * z;
    s += m4(T, r, 3);
    o[r] = s;
  }
}

AICP_HD void ident4(float* T) {
  for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.f : 0.f;
}

// RigidTransformation::checkParameters (libpointmatcher 1.2.x): the rotation block
// is accepted when |1 - det R| <= 0.001 (a NaN determinant passes, as the comparison is false).
// Eigen's 3x3 determinant: cofactor expansion along the first column, float.
AICP_HD bool rigid_ok(const float* T) {
  const float d0 = m4(T, 0, 0) * (m4(T, 1, 1) * m4(T, 2, 2) - m4(T, 1, 2) * m4(T, 2, 1));
  const float d1 = m4(T, 1, 0) * (m4(T, 0, 1) * m4(T, 2, 2) - m4(T, 0, 2) * m4(T, 2, 1));
  const float d2 = m4(T, 2, 0) * (m4(T, 0, 1) * m4(T, 1, 2) - m4(T, 0, 2) * m4(T, 1, 1));
  const float det = (d0 - d1) + d2;
  return !(fabsf(1.f - det) > 0.001f);
}

// ΔT from the solution x = (rotation vector, translation), Eigen::AngleAxis semantics.
AICP_HD void delta_transform(const float* x, float* T) {
  const float sq = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
  const float angle = sqrtf(sq);
  float axis[3] = {x[0], x[1], x[2]};
  if (sq > 0.f) {
    for (int i = 0; i < 3; ++i) axis[i] = x[i] / angle;
  }
  const float sa = (float)sin((double)angle);
  const float c = (float)cos((double)angle);
  float sin_axis[3], cos1_axis[3];
  for (int i = 0; i < 3; ++i) {
    sin_axis[i] = sa * axis[i];
    cos1_axis[i] = (1.f - c) * axis[i];
  }
  float R[9];  // row-major
  float tmp = cos1_axis[0] * axis[1];
  R[0 * 3 + 1] = tmp - sin_axis[2];
  R[1 * 3 + 0] = tmp + sin_axis[2];
  tmp = cos1_axis[0] * axis[2];
  R[0 * 3 + 2] = tmp + sin_axis[1];
  R[2 * 3 + 0] = tmp - sin_axis[1];
  tmp = cos1_axis[1] * axis[2];
  R[1 * 3 + 2] = tmp - sin_axis[0];
  R[2 * 3 + 1] = tmp + sin_axis[0];
  for (int i = 0; i < 3; ++i) R[i * 3 + i] = cos1_axis[i] * axis[i] + c;
  bool nan = false;
  for (int r = 0; r < 3; ++r)
    for (int cc = 0; cc < 3; ++cc) {
      T[cc * 4 + r] = R[r * 3 + cc];
      nan |= (R[r * 3 + cc] != R[r * 3 + cc]);
    }
  for (int r = 0; r < 3; ++r) {
    T[12 + r] = x[3 + r];
    nan |= (x[3 + r] != x[3 + r]);
  }
  T[3] = T[7] = T[11] = 0.f;
  T[15] = 1.f;
  if (nan)  // "mOut != mOut": degenerate rotation -> identity block
    for (int r = 0; r < 3; ++r)
      for (int cc = 0; cc < 3; ++cc) T[cc * 4 + r] = (r == cc) ? 1.f : 0.f;
}

// Quaternion (w, x, y, z) of the rotation block, Shoemake's method in double.
AICP_HD void quat_from_T(const float* T, double* q) {
  double m[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) m[r][c] = (double)m4(T, r, c);
  double t = (m[0][0] + m[1][1]) + m[2][2];
  if (t > 0) {
    t = sqrt(t + 1.0);
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
    t = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
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

AICP_HD double quat_angdist(const double* a, const double* b) {
  const double bw = b[0], bx = -b[1], by = -b[2], bz = -b[3];
  const double w = a[0] * bw - a[1] * bx - a[2] * by - a[3] * bz;
  const double x = a[0] * bx + a[1] * bw + a[2] * bz - a[3] * by;
  const double y = a[0] * by + a[2] * bw + a[3] * bx - a[1] * bz;
  const double z = a[0] * bz + a[3] * bw + a[1] * by - a[2] * bx;
  return 2.0 * atan2(sqrt(x * x + y * y + z * z), fabs(w));
}

// ---- full-pivoting Householder QR (Eigen FullPivHouseholderQR semantics), N <= 6 --------
// Register-resident forms: every loop has compile-time bounds and is unrolled, and the
// data-dependent pivots / ranks act through selects and guards, never through a dynamic
// array index (which would put the matrices in scratch memory). Operation order is that of
// the plain loops (and of the oracle).
#define AICP_UNROLL _Pragma("unroll")

template <int N>
struct PivQR {
  int nonzero, rank;
  double a[N * N];
  double tau[N];
  int rowT[N], colT[N];
  double maxpivot;
};

template <int N>
AICP_HD void pivqr(const double* A, PivQR<N>& q) {
  AICP_UNROLL for (int i = 0; i < N * N; ++i) q.a[i] = A[i];
  const double prec = (double)kFltEps * N;
  q.nonzero = N;
  q.maxpivot = 0;
  double biggest = 0;
  bool stop = false;
  AICP_UNROLL for (int k = 0; k < N; ++k) {
    if (stop) {
      q.rowT[k] = k;
      q.colT[k] = k;
      q.tau[k] = 0;
      continue;
    }
    int br = k, bc = k;
    double bv = -1;
    AICP_UNROLL for (int c = k; c < N; ++c)
      AICP_UNROLL for (int r = k; r < N; ++r) {
        const double v = fabs(q.a[r * N + c]);
        if (v > bv) {
          bv = v;
          br = r;
          bc = c;
        }
      }
    if (k == 0) biggest = bv;
    if (bv <= biggest * prec) {
      q.nonzero = k;
      q.rowT[k] = k;
      q.colT[k] = k;
      q.tau[k] = 0;
      stop = true;
      continue;
    }
    q.rowT[k] = br;
    q.colT[k] = bc;
    AICP_UNROLL for (int r = k + 1; r < N; ++r)
      if (r == br)
        AICP_UNROLL for (int c = k; c < N; ++c) {
          const double t = q.a[k * N + c];
          q.a[k * N + c] = q.a[r * N + c];
          q.a[r * N + c] = t;
        }
    AICP_UNROLL for (int c = k + 1; c < N; ++c)
      if (c == bc)
        AICP_UNROLL for (int r = 0; r < N; ++r) {
          const double t = q.a[r * N + k];
          q.a[r * N + k] = q.a[r * N + c];
          q.a[r * N + c] = t;
        }
    double tailSq = 0;
    AICP_UNROLL for (int r = k + 1; r < N; ++r) tailSq += q.a[r * N + k] * q.a[r * N + k];
    const double c0 = q.a[k * N + k];
    double beta, tau;
    if (tailSq <= kDblMin) {
      tau = 0;
      beta = c0;
      AICP_UNROLL for (int r = k + 1; r < N; ++r) q.a[r * N + k] = 0;
    } else {
      beta = sqrt(c0 * c0 + tailSq);
      if (c0 >= 0) beta = -beta;
      const double den = c0 - beta;
      AICP_UNROLL for (int r = k + 1; r < N; ++r) q.a[r * N + k] /= den;
      tau = (beta - c0) / beta;
    }
    q.tau[k] = tau;
    q.a[k * N + k] = beta;
    if (fabs(beta) > q.maxpivot) q.maxpivot = fabs(beta);
    AICP_UNROLL for (int c = k + 1; c < N; ++c) {
      double s = q.a[k * N + c];
      AICP_UNROLL for (int r = k + 1; r < N; ++r) s += q.a[r * N + k] * q.a[r * N + c];
      s *= tau;
      q.a[k * N + c] -= s;
      AICP_UNROLL for (int r = k + 1; r < N; ++r) q.a[r * N + c] -= s * q.a[r * N + k];
    }
  }
  const double thr = fabs(q.maxpivot) * ((double)kFltEps * N);
  q.rank = 0;
  AICP_UNROLL for (int i = 0; i < N; ++i)
    if (i < q.nonzero) q.rank += (fabs(q.a[i * N + i]) > thr) ? 1 : 0;
}

// Q = P0 H0 P1 H1 ... (row-major N x N)
template <int N>
AICP_HD void pivqr_Q(const PivQR<N>& q, double* Q) {
  AICP_UNROLL for (int i = 0; i < N * N; ++i) Q[i] = 0;
  AICP_UNROLL for (int i = 0; i < N; ++i) Q[i * N + i] = 1;
  AICP_UNROLL for (int k = N - 1; k >= 0; --k) {
    const double tau = (k < q.nonzero) ? q.tau[k] : 0.0;
    if (tau != 0) {
      AICP_UNROLL for (int c = k; c < N; ++c) {
        double s = Q[k * N + c];
        AICP_UNROLL for (int r = k + 1; r < N; ++r) s += q.a[r * N + k] * Q[r * N + c];
        s *= tau;
        Q[k * N + c] -= s;
        AICP_UNROLL for (int r = k + 1; r < N; ++r) Q[r * N + c] -= s * q.a[r * N + k];
      }
    }
    const int rr = (k < q.nonzero) ? q.rowT[k] : k;
    AICP_UNROLL for (int r = k + 1; r < N; ++r)
      if (r == rr)
        AICP_UNROLL for (int c = 0; c < N; ++c) {
          const double t = Q[k * N + c];
          Q[k * N + c] = Q[r * N + c];
          Q[r * N + c] = t;
        }
  }
}

// Cholesky solve of the leading r x r block of M (row stride N)
template <int N>
AICP_HD bool llt_solve(const double* M, int r, const double* b, double* x) {
  double L[N * N];
  AICP_UNROLL for (int i = 0; i < N * N; ++i) L[i] = 0;
  bool ok = true;
  AICP_UNROLL for (int j = 0; j < N; ++j) {
    if (j < r) {
      double d = M[j * N + j];
      AICP_UNROLL for (int k = 0; k < j; ++k) d -= L[j * N + k] * L[j * N + k];
      if (!(d > 0)) ok = false;
      const double ljj = sqrt(d);
      L[j * N + j] = ljj;
      AICP_UNROLL for (int i = j + 1; i < N; ++i)
        if (i < r) {
          double s = M[i * N + j];
          AICP_UNROLL for (int k = 0; k < j; ++k) s -= L[i * N + k] * L[j * N + k];
          L[i * N + j] = s / ljj;
        }
    }
  }
  if (!ok) return false;
  double y[N];
  AICP_UNROLL for (int i = 0; i < N; ++i)
    if (i < r) {
      double s = b[i];
      AICP_UNROLL for (int k = 0; k < i; ++k) s -= L[i * N + k] * y[k];
      y[i] = s / L[i * N + i];
    }
  AICP_UNROLL for (int i = N - 1; i >= 0; --i)
    if (i < r) {
      double s = y[i];
      AICP_UNROLL for (int k = i + 1; k < N; ++k)
        if (k < r) s -= L[k * N + i] * x[k];
      x[i] = s / L[i * N + i];
    }
  return true;
}

// Cyclic Jacobi eigen-decomposition (symmetric, row-major), eigenvectors as columns of V.
template <int N>
AICP_HD void jacobi_eig(const double* A, double* w, double* V) {
  double a[N * N];
  AICP_UNROLL for (int i = 0; i < N * N; ++i) a[i] = A[i];
  AICP_UNROLL for (int i = 0; i < N * N; ++i) V[i] = 0;
  AICP_UNROLL for (int i = 0; i < N; ++i) V[i * N + i] = 1;
  for (int sweep = 0; sweep < 64; ++sweep) {
    double offn = 0, diag = 0;
    AICP_UNROLL for (int p = 0; p < N; ++p) {
      diag += a[p * N + p] * a[p * N + p];
      AICP_UNROLL for (int q = p + 1; q < N; ++q) offn += a[p * N + q] * a[p * N + q];
    }
    if (offn <= 1e-30 * diag || offn == 0) break;
    AICP_UNROLL for (int p = 0; p < N; ++p)
      AICP_UNROLL for (int q = p + 1; q < N; ++q) {
        const double apq = a[p * N + q];
        if (apq != 0) {
          const double app = a[p * N + p], aqq = a[q * N + q];
          const double theta = (aqq - app) / (2 * apq);
          const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
          const double c = 1 / sqrt(t * t + 1), s = t * c;
          AICP_UNROLL for (int k = 0; k < N; ++k) {
            const double akp = a[k * N + p], akq = a[k * N + q];
            a[k * N + p] = c * akp - s * akq;
            a[k * N + q] = s * akp + c * akq;
          }
          AICP_UNROLL for (int k = 0; k < N; ++k) {
            const double apk = a[p * N + k], aqk = a[q * N + k];
            a[p * N + k] = c * apk - s * aqk;
            a[q * N + k] = s * apk + c * aqk;
          }
          AICP_UNROLL for (int k = 0; k < N; ++k) {
            const double vkp = V[k * N + p], vkq = V[k * N + q];
            V[k * N + p] = c * vkp - s * vkq;
            V[k * N + q] = s * vkp + c * vkq;
          }
        }
      }
  }
  AICP_UNROLL for (int i = 0; i < N; ++i) w[i] = a[i * N + i];
}

// solvePossiblyUnderdeterminedLinearSystem (A row-major 6x6). Returns the path taken:
// 0 LLT (full rank), 1 rank-r minimal-norm QR, 2 pseudo-inverse (JacobiSVD fallback).
AICP_HD int solve6(const double* A, const double* b, double* x) {
  constexpr int n = 6;
  PivQR<6> qr;
  pivqr<6>(A, qr);
  if (qr.rank == n) {
    if (llt_solve<6>(A, n, b, x)) return 0;
  } else if (qr.rank > 0) {
    const int r = qr.rank;
    double Q[36];
    pivqr_Q<6>(qr, Q);
    int perm[6];
    AICP_UNROLL for (int i = 0; i < n; ++i) perm[i] = i;
    AICP_UNROLL for (int k = 0; k < n; ++k) {
      const int c = (k < qr.nonzero) ? qr.colT[k] : k;
      AICP_UNROLL for (int j = k + 1; j < n; ++j)
        if (j == c) {
          const int t = perm[k];
          perm[k] = perm[j];
          perm[j] = t;
        }
    }
    // AP[k][j] = A[k][perm[j]] (column gather by selects)
    double AP[36];
    AICP_UNROLL for (int j = 0; j < n; ++j)
      AICP_UNROLL for (int k = 0; k < n; ++k) {
        double v = A[k * n + 0];
        AICP_UNROLL for (int c = 1; c < n; ++c) v = (perm[j] == c) ? A[k * n + c] : v;
        AP[k * n + j] = v;
      }
    double R1[36], RRt[36], qb[6], y[6];
    AICP_UNROLL for (int i = 0; i < n; ++i)
      if (i < r)
        AICP_UNROLL for (int j = 0; j < n; ++j) {
          double s = 0;
          AICP_UNROLL for (int k = 0; k < n; ++k) s += Q[k * n + i] * AP[k * n + j];
          R1[i * n + j] = s;
        }
    AICP_UNROLL for (int i = 0; i < n; ++i)
      AICP_UNROLL for (int j = 0; j < n; ++j)
        if (i < r && j < r) {
          double s = 0;
          AICP_UNROLL for (int k = 0; k < n; ++k) s += R1[i * n + k] * R1[j * n + k];
          RRt[i * n + j] = s;
        }
    AICP_UNROLL for (int i = 0; i < n; ++i)
      if (i < r) {
        double s = 0;
        AICP_UNROLL for (int k = 0; k < n; ++k) s += Q[k * n + i] * b[k];
        qb[i] = s;
      }
    if (llt_solve<6>(RRt, r, qb, y)) {
      double z[6];
      AICP_UNROLL for (int j = 0; j < n; ++j) {
        double s = 0;
        AICP_UNROLL for (int i = 0; i < n; ++i)
          if (i < r && j >= i) s += R1[i * n + j] * y[i];
        z[j] = s;
      }
      // x[perm[i]] = z[i] (scatter by selects)
      AICP_UNROLL for (int c = 0; c < n; ++c) {
        double v = 0;
        AICP_UNROLL for (int i = 0; i < n; ++i) v = (perm[i] == c) ? z[i] : v;
        x[c] = v;
      }
      double nb = 0, nax = 0, nd = 0;
      AICP_UNROLL for (int i = 0; i < n; ++i) {
        double s = 0;
        AICP_UNROLL for (int k = 0; k < n; ++k) s += A[i * n + k] * x[k];
        nb += b[i] * b[i];
        nax += s * s;
        nd += (b[i] - s) * (b[i] - s);
      }
      if (nd <= 1e-10 * (nb < nax ? nb : nax)) return 1;
    }
  }
  double w[6], V[36];
  jacobi_eig<6>(A, w, V);
  double wmax = 0;
  AICP_UNROLL for (int i = 0; i < n; ++i) wmax = fmax(wmax, fabs(w[i]));
  double thr = wmax * (n * kDblEps);
  if (thr < kDblMin) thr = kDblMin;
  AICP_UNROLL for (int i = 0; i < n; ++i) x[i] = 0;
  AICP_UNROLL for (int e = 0; e < n; ++e) {
    if (fabs(w[e]) <= thr) continue;
    double s = 0;
    AICP_UNROLL for (int k = 0; k < n; ++k) s += V[k * n + e] * b[k];
    s /= w[e];
    AICP_UNROLL for (int k = 0; k < n; ++k) x[k] += V[k * n + e] * s;
  }
  return 2;
}

// SurfaceNormal: rank(fullPivQR(C)) + 1 >= 3 -> smallest eigenvector, else e_y.
AICP_HD bool normal_from_cov(const double* C, float* nrm) {
  PivQR<3> qr;
  pivqr<3>(C, qr);
  if (qr.rank + 1 >= 3) {
    double w[3], V[9];
    jacobi_eig<3>(C, w, V);
    int s = 0;
    double sv = 1.79769313486231570e308;
    AICP_UNROLL for (int j = 0; j < 3; ++j)
      if (w[j] < sv) {
        sv = w[j];
        s = j;
      }
    AICP_UNROLL for (int r = 0; r < 3; ++r) nrm[r] = (float)(s == 0 ? V[r * 3] : (s == 1 ? V[r * 3 + 1] : V[r * 3 + 2]));
    return false;
  }
  nrm[0] = 0.f;
  nrm[1] = 1.f;
  nrm[2] = 0.f;
  return true;
}

// Translation of the corrected pose of an accepted reading: correction_iso * prior_pose
// (AlignedCloud::updateCloud, aligned_cloud.cpp:61-70; removePitchRollCorrection keeps the
// translation), with correction_iso = fromMatrix4fToIsometry3d(T) (common.cpp:4-23):
// Eigen::Quaternionf of T's rotation block (float, Eigen's trace / largest-diagonal branches),
// cast to double, Quaterniond::toRotationMatrix, translation = float T(0..2, 3) as double.
// Only the prior pose's translation o enters: R_q * o + t, row sums left to right, no FMA.
// The float square root is the correctly rounded one ((float)sqrt(double), exact for floats).
AICP_HD void corrected_origin(const float* T, const double* o, double* out) {
  float m[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) m[r][c] = T[c * 4 + r];
  float q[4];  // x, y, z, w
  float t = (m[0][0] + m[1][1]) + m[2][2];
  if (t > 0.f) {
    t = (float)sqrt((double)(t + 1.f));
    q[3] = 0.5f * t;
    t = 0.5f / t;
    q[0] = (m[2][1] - m[1][2]) * t;
    q[1] = (m[0][2] - m[2][0]) * t;
    q[2] = (m[1][0] - m[0][1]) * t;
  } else {
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = (float)sqrt((double)(((m[i][i] - m[j][j]) - m[k][k]) + 1.f));
    q[i] = 0.5f * t;
    t = 0.5f / t;
    q[3] = (m[k][j] - m[j][k]) * t;
    q[j] = (m[j][i] + m[i][j]) * t;
    q[k] = (m[k][i] + m[i][k]) * t;
  }
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  const double R[3][3] = {{1.0 - (tyy + tzz), txy - twz, txz + twy},
                          {txy + twz, 1.0 - (txx + tzz), tyz - twx},
                          {txz - twy, tyz + twx, 1.0 - (txx + tyy)}};
  for (int r = 0; r < 3; ++r) out[r] = ((R[r][0] * o[0] + R[r][1] * o[1]) + R[r][2] * o[2]) + (double)T[12 + r];
}

// App::processCloud's drop test (app.cpp:366-373): any |T(i,3)| > max_correction_magnitude
AICP_HD bool correction_rejected(const float* T, float max_corr) {
  return fabsf(T[12]) > max_corr || fabsf(T[13]) > max_corr || fabsf(T[14]) > max_corr;
}

// replaceRatioConfigFile text round trip for r in [0.1, 1): "%g" keeps 6 significant digits
// = 1e-6 resolution; m = rint(r * 1e6) is exact in double and float(m / 1e6) is the
// correctly rounded parse (no double-rounding hazard: m/1e6 is never within 2^-54 of a
// float midpoint). tests/test_library_cpu.py checks it against snprintf + strtof.
AICP_HD float quantize_ratio_fast(float r) {
  const double m = rint((double)r * 1e6);
  return (float)(m / 1e6);
}

AICP_HD float autotune_ratio_fast(float overlap_percent) {
  float cur = (float)(overlap_percent / 100.0);
  if (cur < 0.25)
    cur = 0.25f;
  else if (cur > 0.70)
    cur = 0.70f;
  if (cur != cur) return cur;
  return quantize_ratio_fast(cur);
}

}  // namespace aicp

namespace aicp {

// ---- reference centroid (ICP::compute step 2) ----------------------------------
// Order-independent definition shared with the oracle: every coordinate is rounded to a
// multiple of 2^-40 (exact for |x| >= 2^-16; |x| < 2^23 m), summed exactly in 128-bit
// two's complement, and mean = float((|S| as double) * 2^-40 / n) with the sign applied.
AICP_HD int64_t fixed40(float x) {
  const double v = rint((double)x * 1099511627776.0);
  const double lim = 9.2233720368547748e18;  // 2^63
  if (!(v < lim)) return INT64_MAX;
  if (!(v > -lim)) return INT64_MIN;
  return (int64_t)v;
}

AICP_HD float mean_from_fixed40(uint64_t lo, uint64_t hi, uint32_t n) {
  const bool neg = (int64_t)hi < 0;
  if (neg) {
    lo = ~lo + 1;
    hi = ~hi + (lo == 0 ? 1 : 0);
  }
  const double mag = (double)hi * 18446744073709551616.0 + (double)lo;
  const double m = mag * (1.0 / 1099511627776.0) / (double)n;
  return (float)(neg ? -m : m);
}

}  // namespace aicp
