// microbench.hip — variant timing for the NN traversal and the overlap ray marking.
// Not part of the product; used to choose designs (results in profiles/).
// Usage: microbench ref.bin read.bin   (float32 xyz, little endian; ref and read of one pair)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <string>
#include <algorithm>
#include "kdtree_host.hpp"
#include "../aicp_mapping_amd/csrc/kernels.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ float sel3(uint32_t cd, float a, float b, float c) { return cd == 0 ? a : (cd == 1 ? b : c); }

// V: 0 = scratch stack (48), 1 = no far descents (lower bound), 2 = 4-entry register stack
template <int V>
__global__ __launch_bounds__(256) void k_mark(int n, const float4* __restrict__ pts, float ox, float oy, float oz,
    double res, int mn0, int mn1, int mn2, int dm0, int dm1, int dm2, unsigned* bm, unsigned char* bytes, unsigned* sink) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const double rf = 1.0 / res;
  const float o[3] = {ox, oy, oz};
  const float4 p4 = pts[j];
  const float e[3] = {p4.x, p4.y, p4.z};
  int ko[3], ke[3];
  for (int i = 0; i < 3; ++i) { ko[i] = (int)floor(rf * (double)o[i]) + 32768; ke[i] = (int)floor(rf * (double)e[i]) + 32768; }
  unsigned acc = 0;
  auto mark = [&](int k0, int k1, int k2) {
    const unsigned long long idx = ((unsigned long long)(k0 - mn0) * dm1 + (k1 - mn1)) * dm2 + (k2 - mn2);
    if (V == 0) { const unsigned bit = 1u << (idx & 31); unsigned* w = bm + (idx >> 5); if (!(*(volatile unsigned*)w & bit)) atomicOr(w, bit); }
    else if (V == 1) { bytes[idx] = 1; }
    else { acc += (unsigned)idx; }
  };
  if (!(ko[0] == ke[0] && ko[1] == ke[1] && ko[2] == ke[2])) {
    mark(ko[0], ko[1], ko[2]);
    float dir[3] = {e[0] - o[0], e[1] - o[1], e[2] - o[2]};
    const float nsq = dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2];
    const float length = (float)sqrt((double)nsq);
    for (int i = 0; i < 3; ++i) dir[i] /= length;
    int step[3]; double tMax[3], tDelta[3]; int cur[3] = {ko[0], ko[1], ko[2]};
    for (int i = 0; i < 3; ++i) {
      step[i] = dir[i] > 0.0f ? 1 : (dir[i] < 0.0f ? -1 : 0);
      if (step[i]) { double vb = (double(cur[i] - 32768) + 0.5) * res; vb += (float)(step[i] * res * 0.5);
        tMax[i] = (vb - (double)o[i]) / (double)dir[i]; tDelta[i] = res / (double)fabsf(dir[i]); }
      else { tMax[i] = 1.7976931348623157e308; tDelta[i] = 1.7976931348623157e308; }
    }
    const double len = (double)length;
    for (;;) {
      int dim; if (tMax[0] < tMax[1]) dim = (tMax[0] < tMax[2]) ? 0 : 2; else dim = (tMax[1] < tMax[2]) ? 1 : 2;
      cur[dim] += step[dim]; tMax[dim] += tDelta[dim];
      if (cur[0] == ke[0] && cur[1] == ke[1] && cur[2] == ke[2]) break;
      if (fmin(fmin(tMax[0], tMax[1]), tMax[2]) > len) break;
      mark(cur[0], cur[1], cur[2]);
    }
  }
  mark(ke[0], ke[1], ke[2]);
  if (V == 2 && acc == 0x12345678u) sink[0] = acc;
}

static std::vector<float> load(const char* f) {
  FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); long sz = ftell(fp); fseek(fp, 0, SEEK_SET);
  std::vector<float> v(sz / 4); fread(v.data(), 4, v.size(), fp); fclose(fp); return v;
}

int main(int argc, char** argv) {
  std::vector<float> ref = load(argv[1]), rd = load(argv[2]);
  const int M = ref.size() / 3, N = rd.size() / 3, REP = 16;  // 16 copies of the reading as queries (a 16-pair batch)
  double mu[3] = {0, 0, 0};
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) mu[d] += ref[3 * i + d];
  float m[3]; for (int d = 0; d < 3; ++d) m[d] = (float)(mu[d] / M);
  std::vector<float> c(3 * M); for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) c[3 * i + d] = ref[3 * i + d] - m[d];
  aicp::HostTree t; aicp::build_kdtree_host(c.data(), M, 8, t);
  printf("M=%d N=%d nodes=%zu depth=%d\n", M, N, t.parent.size(), t.depth);
  std::vector<float> bp(4 * M); for (int j = 0; j < M; ++j) { int id = t.perm[j]; for (int d = 0; d < 3; ++d) bp[4 * j + d] = c[3 * id + d]; memcpy(&bp[4 * j + 3], &id, 4); }
  // optional Morton order of the queries (argv[3] == "morton")
  std::vector<int> qord(N);
  for (int i = 0; i < N; ++i) qord[i] = i;
  if (argc > 3 && std::string(argv[3]) == "morton") {
    float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
    for (int i = 0; i < N; ++i) for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], rd[3 * i + d]); hi[d] = std::max(hi[d], rd[3 * i + d]); }
    auto spread = [](uint64_t v) { uint64_t x = v & 0x1fffff; x = (x | x << 32) & 0x1f00000000ffffull; x = (x | x << 16) & 0x1f0000ff0000ffull; x = (x | x << 8) & 0x100f00f00f00f00full; x = (x | x << 4) & 0x10c30c30c30c30c3ull; x = (x | x << 2) & 0x1249249249249249ull; return x; };
    std::vector<uint64_t> key(N);
    for (int i = 0; i < N; ++i) { uint64_t c[3]; for (int d = 0; d < 3; ++d) c[d] = (uint64_t)((rd[3 * i + d] - lo[d]) / (hi[d] - lo[d] + 1e-6f) * 2097151.0f); key[i] = spread(c[0]) | spread(c[1]) << 1 | spread(c[2]) << 2; }
    std::sort(qord.begin(), qord.end(), [&](int a, int b) { return key[a] < key[b]; });
    printf("queries in Morton order\n");
  }
  std::vector<float> qq(4 * (size_t)N * REP);
  for (int r = 0; r < REP; ++r) for (int i = 0; i < N; ++i) { for (int d = 0; d < 3; ++d) qq[4 * ((size_t)r * N + i) + d] = rd[3 * qord[i] + d] - m[d]; qq[4 * ((size_t)r * N + i) + 3] = 1; }
  float4 *dq, *dp; uint4* dn; int *dpar, *dids; float* dd2; unsigned* dcnt;
  const size_t NQ = (size_t)N * REP;
  CK(hipMalloc(&dq, NQ * 16)); CK(hipMalloc(&dp, M * 16)); CK(hipMalloc(&dn, t.parent.size() * 16)); CK(hipMalloc(&dpar, t.parent.size() * 4));
  CK(hipMalloc(&dids, NQ * 4)); CK(hipMalloc(&dd2, NQ * 4)); CK(hipMalloc(&dcnt, 64));
  CK(hipMemcpy(dq, qq.data(), NQ * 16, hipMemcpyHostToDevice)); CK(hipMemcpy(dp, bp.data(), M * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dn, t.nodes.data(), t.parent.size() * 16, hipMemcpyHostToDevice)); CK(hipMemcpy(dpar, t.parent.data(), t.parent.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const float maxE2 = (1 + 3.16f) * (1 + 3.16f);
  auto timeit = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipMemset(dcnt, 0, 64));
    CK(hipEventRecord(a)); for (int r = 0; r < 5; ++r) launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); unsigned cnt[2]; CK(hipMemcpy(cnt, dcnt, 8, hipMemcpyDeviceToHost));
    printf("%-32s %9.1f us   far=%u  sum(wave max far)=%u\n", name, 1e3 * ms / 5, cnt[0] / 5, cnt[1] / 5);
  };
  const int g = (NQ + 255) / 256;
  unsigned long long* dtouch; unsigned* dctr2;
  CK(hipMalloc(&dtouch, 64)); CK(hipMalloc(&dctr2, 1024));
  timeit("nn persistent (library)", [&] { CK(hipMemsetAsync(dctr2, 0, 1024)); aicp::launch_knn_generic(0, NQ, dq, dn, dpar, dp, 1, maxE2, __builtin_inff(), dids, dd2, dtouch, dctr2); });
  timeit("nn persistent eps0 (library)", [&] { CK(hipMemsetAsync(dctr2, 0, 1024)); aicp::launch_knn_generic(0, NQ, dq, dn, dpar, dp, 1, 1.0f, __builtin_inff(), dids, dd2, dtouch, dctr2); });
  // overlap: reading cloud rays from origin (1.5, 0, 0.7) approx; box from data
  int lo[3] = {1 << 30, 1 << 30, 1 << 30}, hi[3] = {-(1 << 30), -(1 << 30), -(1 << 30)};
  const double res = (double)0.2f;
  float org[3] = {0.f, 0.f, 0.7f};
  for (int i = 0; i <= M; ++i) for (int d = 0; d < 3; ++d) { float v = i < M ? ref[3 * i + d] : org[d]; int k = (int)floor(v / res) + 32768; lo[d] = std::min(lo[d], k); hi[d] = std::max(hi[d], k); }
  int mn[3], dm[3]; size_t vox = 1; for (int d = 0; d < 3; ++d) { mn[d] = lo[d] - 2; dm[d] = hi[d] - lo[d] + 5; vox *= dm[d]; }
  printf("voxels %zu\n", vox);
  std::vector<float> rr(4 * (size_t)M * REP);
  for (int r = 0; r < REP; ++r) for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) rr[4 * ((size_t)r * M + i) + d] = ref[3 * i + d];
  float4* dr; unsigned* bm; unsigned char* by;
  CK(hipMalloc(&dr, rr.size() * 4)); CK(hipMemcpy(dr, rr.data(), rr.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&bm, vox / 8 + 64)); CK(hipMalloc(&by, vox + 64));
  const int gm = (M * REP + 255) / 256;
  timeit("mark atomicOr bitmap", [&] { k_mark<0><<<gm, 256>>>(M * REP, dr, org[0], org[1], org[2], res, mn[0], mn[1], mn[2], dm[0], dm[1], dm[2], bm, by, dcnt); });
  timeit("mark byte store", [&] { k_mark<1><<<gm, 256>>>(M * REP, dr, org[0], org[1], org[2], res, mn[0], mn[1], mn[2], dm[0], dm[1], dm[2], bm, by, dcnt); });
  timeit("mark DDA only", [&] { k_mark<2><<<gm, 256>>>(M * REP, dr, org[0], org[1], org[2], res, mn[0], mn[1], mn[2], dm[0], dm[1], dm[2], bm, by, dcnt); });
  return 0;
}
