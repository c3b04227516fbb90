// Cycle cost of the ICP update's serial pieces on one lane (icp_math.hpp), to see where
// k_icp_update_f's ~11.6 us serial tail goes. hipcc --offload-arch=gfx950 -O3 -I../../aicp_mapping_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include "icp_math.hpp"
using namespace aicp;

__global__ void k_bench(const double* Ain, const double* bin, double* out, long long* cyc, int reps) {
  if (threadIdx.x != 0) return;
  double A[36], b[6];
  for (int i = 0; i < 36; ++i) A[i] = Ain[i];
  for (int i = 0; i < 6; ++i) b[i] = bin[i];
  double acc = 0;
  long long t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < reps; ++r) {
    A[0] += 1e-12 * acc;  // a dependency between repetitions
    long long c0 = clock64();
    PivQR<6> q;
    pivqr<6>(A, q);
    acc += q.a[0] + q.rank;
    long long c1 = clock64();
    double x[6];
    llt_solve<6>(A, 6, b, x);
    acc += x[0];
    long long c2 = clock64();
    solve6(A, b, x);
    acc += x[1];
    long long c3 = clock64();
    float xf[6], dT[16], T[16];
    for (int i = 0; i < 6; ++i) xf[i] = (float)(x[i] + 1e-3 * acc);
    delta_transform(xf, dT);
    mul4(dT, dT, T);
    acc += T[5];
    long long c4 = clock64();
    double qa[4], qb[4];
    quat_from_T(T, qa);
    quat_from_T(dT, qb);
    acc += qa[0] + qb[1];
    long long c5 = clock64();
    double s = 0;
    for (int k = 0; k < 3; ++k) s += fabs(quat_angdist(qa, qb)) + 1e-3 * k * acc;
    acc += s;
    long long c6 = clock64();
    t[0] += c1 - c0; t[1] += c2 - c1; t[2] += c3 - c2; t[3] += c4 - c3; t[4] += c5 - c4; t[5] += c6 - c5;
  }
  for (int i = 0; i < 6; ++i) cyc[i] = t[i] / reps;
  out[0] = acc;
}

int main() {
  double A[36], b[6];
  // an SPD 6x6 like the point-to-plane normal equations
  double M[36];
  for (int i = 0; i < 36; ++i) M[i] = 0.3 * ((i * 7919) % 13) - 1.7;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) {
      double s = 0;
      for (int k = 0; k < 6; ++k) s += M[i * 6 + k] * M[j * 6 + k];
      A[i * 6 + j] = s + (i == j ? 3.0 : 0.0);
    }
  for (int i = 0; i < 6; ++i) b[i] = 0.1 * i - 0.2;
  double *dA, *db, *dout;
  long long* dc;
  hipMalloc(&dA, 288); hipMalloc(&db, 48); hipMalloc(&dout, 8); hipMalloc(&dc, 64);
  hipMemcpy(dA, A, 288, hipMemcpyHostToDevice);
  hipMemcpy(db, b, 48, hipMemcpyHostToDevice);
  k_bench<<<1, 64>>>(dA, db, dout, dc, 10);
  hipDeviceSynchronize();
  k_bench<<<1, 64>>>(dA, db, dout, dc, 200);
  long long c[8];
  hipMemcpy(c, dc, 64, hipMemcpyDeviceToHost);
  const char* nm[6] = {"pivqr<6>", "llt_solve<6>", "solve6", "delta_transform+mul4", "quat_from_T x2", "quat_angdist x3"};
  // clock64 = s_memtime (shader clock)
  for (int i = 0; i < 6; ++i) std::printf("%-22s %8lld cycles\n", nm[i], c[i]);
  return 0;
}
