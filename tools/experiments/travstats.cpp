// travstats.cpp — CPU replay of the libnabo-order 1-NN traversal (Trav<1>) with per-phase load
// counters, to see where the dependent loads of k_icp_nn go. Not part of the product.
// Build: g++ -O2 -std=c++17 travstats.cpp kdtree_host.cpp -o travstats
// Usage: travstats ref.bin read.bin [eps]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "kdtree_host.hpp"

struct Stats { double desc = 0, leafv = 0, leaves = 0, climb_pre = 0, climb_post = 0, far = 0, pops = 0, q = 0, maxfar = 0; };

static std::vector<float> load(const char* f) {
  FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
  std::vector<float> v(n / 4); fread(v.data(), 4, v.size(), fp); fclose(fp); return v;
}

int main(int argc, char** argv) {
  auto ref = load(argv[1]), rd = load(argv[2]);
  const float eps = argc > 3 ? atof(argv[3]) : 3.16f;
  const int M = ref.size() / 3, N = rd.size() / 3;
  double m[3] = {0, 0, 0};
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) m[d] += ref[3 * i + d];
  for (int d = 0; d < 3; ++d) m[d] /= M;
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) ref[3 * i + d] -= (float)m[d];
  aicp::HostTree t;
  aicp::build_kdtree_host(ref.data(), M, 8, t);
  std::vector<float> bp(3 * M);
  for (int j = 0; j < M; ++j) for (int d = 0; d < 3; ++d) bp[3 * j + d] = ref[3 * t.perm[j] + d];
  auto node = [&](int n) { return &t.nodes[4 * n]; };
  const float E = (1 + eps) * (1 + eps), R = INFINITY;
  Stats S;
  std::vector<int> hist_far(64, 0);
  for (int qi = 0; qi < N; ++qi) {
    const float q[3] = {rd[3 * qi] - (float)m[0], rd[3 * qi + 1] - (float)m[1], rd[3 * qi + 2] - (float)m[2]};
    float off[3] = {0, 0, 0}, rd_ = 0, best = INFINITY;
    struct Fr { int far, start, P, PP; float rd, old, mn; int cd; };
    std::vector<Fr> st;
    int n = 0, start = 0;
    bool after_pop = false;
    int nfar = 0;
    for (;;) {
      float minFar = INFINITY;
      const uint32_t* nd = node(n);
      S.desc++;
      while ((nd[1] & 3u) != 3u) {
        const int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
        const float no = q[cd] - cut, oc = off[cd];
        const float rdf = rd_ + (-oc * oc + no * no);
        minFar = fminf(minFar, rdf);
        n = no > 0 ? (int)(nd[1] >> 2) : n + 1;
        nd = node(n); S.desc++;
      }
      S.leaves++; S.leafv += nd[0];
      for (uint32_t i = 0; i < nd[0]; ++i) {
        const float* p = &bp[3 * ((nd[1] >> 2) + i)];
        const float d0 = q[0] - p[0], d1 = q[1] - p[1], d2 = q[2] - p[2];
        float dist = 0; dist += d0 * d0; dist += d1 * d1; dist += d2 * d2;
        if (dist <= R && dist < best) best = dist;
      }
      int c = n, pc = (int)nd[2];
      after_pop = false;
      if (!(minFar <= R && minFar * E < best)) c = start;
      bool descend = false;
      while (!descend) {
        if (c == start) {
          if (st.empty()) goto done;
          Fr f = st.back(); st.pop_back(); S.pops++;
          rd_ = f.rd; off[f.cd] = f.old; minFar = f.mn; start = f.start; c = f.P; pc = f.PP;
          after_pop = true;
          if (!(minFar <= R && minFar * E < best)) c = start;
          continue;
        }
        const int p = pc; const uint32_t* pn = node(p);
        if (after_pop) S.climb_post++; else S.climb_pre++;
        const int cd = pn[1] & 3; float cut; memcpy(&cut, &pn[0], 4);
        const float no = q[cd] - cut, oc = off[cd];
        const float rdf = rd_ + (-oc * oc + no * no);
        if (rdf <= R && rdf * E < best) {
          const int far = no > 0 ? p + 1 : (int)(pn[1] >> 2);
          st.push_back({far, start, p, (int)pn[2], rd_, oc, minFar, cd});
          off[cd] = no; rd_ = rdf; n = far; start = far; descend = true; S.far++; nfar++;
        } else { c = p; pc = (int)pn[2]; }
      }
    }
  done:
    S.q++;
    hist_far[std::min(nfar, 63)]++;
  }
  printf("queries %d depth %d nodes %zu\n", (int)S.q, t.depth, t.parent.size());
  printf("per query: descent loads %.2f, leaves %.2f (points %.2f), climb loads before first pop %.2f, after pops %.2f, far descents %.2f, pops %.2f\n",
         S.desc / S.q, S.leaves / S.q, S.leafv / S.q, S.climb_pre / S.q, S.climb_post / S.q, S.far / S.q, S.pops / S.q);
  printf("far-descent histogram:");
  for (int i = 0; i < 12; ++i) printf(" %d:%d", i, hist_far[i]);
  printf("\n");
}
