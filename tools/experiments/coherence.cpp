// coherence.cpp — design experiment (not product), see tools/coherence.py.
// Build: g++ -O2 -std=c++17 coherence.cpp kdtree_host.cpp -o coherence
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "kdtree_host.hpp"

static std::vector<float> load(const char* f) {
  FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
  std::vector<float> v(n / 4); if (fread(v.data(), 4, v.size(), fp) != v.size()) abort(); fclose(fp); return v;
}

int main() {
  auto ref = load("/tmp/coh_ref.bin"), rd = load("/tmp/coh_read.bin"), Tv = load("/tmp/coh_T.bin");
  const int M = ref.size() / 3, N = rd.size() / 3, K = (Tv.size() - 3) / 16;
  const float mu[3] = {Tv[0], Tv[1], Tv[2]};
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) ref[3 * i + d] -= mu[d];
  aicp::HostTree t;
  aicp::build_kdtree_host(ref.data(), M, 8, t);
  auto node = [&](int n) { return &t.nodes[4 * n]; };
  std::vector<float> prevq(3 * N), margin(N), mar3(3 * N);
  std::vector<int> leaf(N);
  for (int k = 0; k < K; ++k) {
    const float* T = &Tv[3 + 16 * k];  // column-major
    size_t same = 0, skip = 0, skip3 = 0;
    double sumd = 0, summ = 0;
    for (int i = 0; i < N; ++i) {
      const float r[3] = {rd[3 * i] - mu[0], rd[3 * i + 1] - mu[1], rd[3 * i + 2] - mu[2]};
      float q[3];
      for (int a = 0; a < 3; ++a) q[a] = T[a] * r[0] + T[4 + a] * r[1] + T[8 + a] * r[2] + T[12 + a];
      int n = 0;
      float m = INFINITY, m3[3] = {INFINITY, INFINITY, INFINITY};
      while ((node(n)[1] & 3u) != 3u) {
        const uint32_t* nd = node(n);
        const int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
        const float no = q[cd] - cut;
        m = fminf(m, fabsf(no));
        m3[cd] = fminf(m3[cd], fabsf(no));
        n = no > 0 ? (int)(nd[1] >> 2) : n + 1;
      }
      if (k > 0) {
        float dl = 0;
        for (int a = 0; a < 3; ++a) dl = fmaxf(dl, fabsf(q[a] - prevq[3 * i + a]));
        sumd += dl; summ += margin[i];
        if (dl < margin[i]) ++skip;
        bool ok3 = true;
        for (int a = 0; a < 3; ++a) ok3 = ok3 && fabsf(q[a] - prevq[3 * i + a]) < mar3[3 * i + a];
        skip3 += ok3;
        if (leaf[i] == n) ++same;
      }
      for (int a = 0; a < 3; ++a) prevq[3 * i + a] = q[a];
      margin[i] = m;
      for (int a = 0; a < 3; ++a) mar3[3 * i + a] = m3[a];
      leaf[i] = n;
    }
    if (k > 0)
      printf("iteration %2d: same leaf %.1f%%, provable skip (displacement < path margin) %.1f%%, per axis %.1f%%, mean displacement %.2e m, mean margin %.2e m\n",
             k, 100.0 * same / N, 100.0 * skip / N, 100.0 * skip3 / N, sumd / N, summ / N);
  }
}
