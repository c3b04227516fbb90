// pf_eig_check.hip — prints the device's PCL eigen33 intermediates for covariance matrices given
// on stdin (9 floats per line, hex bits), to compare with the oracle. Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math
//        -I aicp_mapping_amd/csrc tools/experiments/pf_eig_check.hip -o tools/experiments/pf_eig_check
#include "../aicp_mapping_amd/csrc/kernels_prefilter.hip"
#include <cstdio>
#include <vector>

__global__ void k_check(int n, const float* cov, float* out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const float* m = cov + 9 * i;
  float scale = 0.f;
  for (int k = 0; k < 9; ++k) scale = fmaxf(scale, fabsf(m[k]));
  float s[9];
  for (int k = 0; k < 9; ++k) s[k] = __fdiv_rn(m[k], scale);
  const float m00 = s[0], m01 = s[1], m02 = s[2], m11 = s[4], m12 = s[5], m22 = s[8];
  const float c0 = m00 * m11 * m22 + 2.f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 - m22 * m01 * m01;
  const float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
  const float c2 = m00 + m11 + m22;
  const float s_inv3 = (float)(1.0 / 3.0);
  const float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.f) a_over_3 = 0.f;
  const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.f) q = 0.f;
  const float rho = aicp::sqrt_rn(-a_over_3);
  const float theta = (float)atan2((double)aicp::sqrt_rn(-q), (double)half_b) * s_inv3;
  const float cos_t = (float)cos((double)theta);
  const float sin_t = (float)sin((double)theta);
  float lambda, nx, ny, nz;
  aicp::eigen33(m, lambda, nx, ny, nz);
  float* o = out + 16 * i;
  o[0] = c0; o[1] = c1; o[2] = c2; o[3] = half_b; o[4] = q; o[5] = rho; o[6] = theta; o[7] = cos_t; o[8] = sin_t;
  o[9] = lambda; o[10] = nx; o[11] = ny; o[12] = nz; o[13] = scale;
}

int main() {
  std::vector<float> c;
  unsigned u[9];
  while (scanf("%x %x %x %x %x %x %x %x %x", u, u + 1, u + 2, u + 3, u + 4, u + 5, u + 6, u + 7, u + 8) == 9)
    for (int k = 0; k < 9; ++k) { float f; memcpy(&f, &u[k], 4); c.push_back(f); }
  const int n = (int)c.size() / 9;
  float *dc, *dout;
  (void)hipMalloc(&dc, c.size() * 4);
  (void)hipMalloc(&dout, (size_t)n * 64);
  (void)hipMemcpy(dc, c.data(), c.size() * 4, hipMemcpyHostToDevice);
  k_check<<<(n + 63) / 64, 64>>>(n, dc, dout);
  std::vector<float> o((size_t)n * 16);
  (void)hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 14; ++k) { unsigned b; memcpy(&b, &o[16 * i + k], 4); printf("%08x ", b); }
    printf("\n");
  }
  return 0;
}
