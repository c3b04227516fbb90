// gridstats.cpp — design experiment (not product): how deep does a uniform-grid point location
// put each ICP query into the libnabo-order kd-tree? For every cell of a grid of side h over the
// reference's bounding box, D(cell) = the deepest node whose region holds the whole cell; the
// libnabo descent of a query in that cell passes through D, so it can start there.
// Build: g++ -O2 -std=c++17 gridstats.cpp kdtree_host.cpp -o gridstats
// Usage: gridstats ref.bin read.bin cells_per_point
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>
#include "kdtree_host.hpp"

static std::vector<float> load(const char* f) {
  FILE* fp = fopen(f, "rb"); fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
  std::vector<float> v(n / 4); if (fread(v.data(), 4, v.size(), fp) != v.size()) abort(); fclose(fp); return v;
}

int main(int argc, char** argv) {
  auto ref = load(argv[1]), rd = load(argv[2]);
  const int M = ref.size() / 3, N = rd.size() / 3;
  double m[3] = {0, 0, 0};
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) m[d] += ref[3 * i + d];
  for (int d = 0; d < 3; ++d) m[d] /= M;
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) ref[3 * i + d] -= (float)m[d];
  aicp::HostTree t;
  aicp::build_kdtree_host(ref.data(), M, 8, t);
  auto node = [&](int n) { return &t.nodes[4 * n]; };
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], ref[3 * i + d]); hi[d] = fmaxf(hi[d], ref[3 * i + d]); }

  const double budget = argc > 3 ? atof(argv[3]) * M : 2.0 * M;
  double e[3], vol = 1;
  for (int d = 0; d < 3; ++d) { e[d] = std::max(1e-3, (double)hi[d] - lo[d]); vol *= e[d]; }
  double hh = cbrt(vol / budget);
  int dims[3];
  for (;;) { size_t c = 1; for (int d = 0; d < 3; ++d) { dims[d] = std::max(1, (int)ceil(e[d] / hh)); c *= dims[d]; } if (c <= budget) break; hh *= 1.02; }
  const float h = (float)hh, invh = (float)(1.0 / hh);
  const size_t cells = (size_t)dims[0] * dims[1] * dims[2];
  std::vector<int32_t> D(cells);
  std::vector<int> Ddepth(cells);
  std::vector<float> box(cells * 6);
  size_t leafcells = 0;
  for (int z = 0; z < dims[2]; ++z) for (int y = 0; y < dims[1]; ++y) for (int x = 0; x < dims[0]; ++x) {
    const float bl[3] = {lo[0] + x * h, lo[1] + y * h, lo[2] + z * h};
    const float bh[3] = {bl[0] + h, bl[1] + h, bl[2] + h};
    float rl[3] = {-INFINITY, -INFINITY, -INFINITY}, rh[3] = {INFINITY, INFINITY, INFINITY};
    int n = 0, dep = 0;
    for (;;) {
      const uint32_t* nd = node(n);
      if ((nd[1] & 3u) == 3u) break;
      const int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
      if (bl[cd] - cut > 0) { n = nd[1] >> 2; ++dep; rl[cd] = cut; }
      else if (bh[cd] - cut <= 0) { n = n + 1; ++dep; rh[cd] = cut; }
      else break;
    }
    const size_t c = ((size_t)z * dims[1] + y) * dims[0] + x;
    D[c] = n; Ddepth[c] = dep;
    for (int d = 0; d < 3; ++d) { box[6 * c + d] = rl[d]; box[6 * c + 3 + d] = rh[d]; }
    if ((node(n)[1] & 3u) == 3u) ++leafcells;
  }
  double full = 0, rest = 0, hitleaf = 0, outside = 0, fails = 0;
  std::vector<int> hist(40, 0);
  for (int qi = 0; qi < N; ++qi) {
    const float q[3] = {rd[3 * qi] - (float)m[0], rd[3 * qi + 1] - (float)m[1], rd[3 * qi + 2] - (float)m[2]};
    int n = 0, dep = 0;
    std::vector<int> path;
    for (;;) {
      path.push_back(n);
      const uint32_t* nd = node(n);
      if ((nd[1] & 3u) == 3u) break;
      const int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
      n = (q[cd] - cut > 0) ? (int)(nd[1] >> 2) : n + 1; ++dep;
    }
    full += dep;
    int c3[3]; bool in = true;
    for (int d = 0; d < 3; ++d) {
      int c = (int)floorf((q[d] - lo[d]) * invh);
      if (c < 0 || c >= dims[d]) in = false;
      c3[d] = std::min(std::max(c, 0), dims[d] - 1);
    }
    if (!in) outside++;
    const size_t c = ((size_t)c3[2] * dims[1] + c3[1]) * dims[0] + c3[0];
    bool ok = true;
    for (int d = 0; d < 3; ++d) ok = ok && !(q[d] - box[6 * c + d] <= 0) && (q[d] - box[6 * c + 3 + d] <= 0);
    int r = dep;
    if (ok) {
      if (Ddepth[c] >= (int)path.size() || path[Ddepth[c]] != D[c]) { printf("MISMATCH q %d\n", qi); return 1; }
      r = dep - Ddepth[c];
      if (r == 0) hitleaf++;
    } else fails++;
    rest += r;
    hist[std::min(r, 39)]++;
  }
  printf("M %d N %d h %.3f grid %dx%dx%d = %zu cells (%.1f MB), leaf cells %.1f%%\n", M, N, h, dims[0], dims[1], dims[2],
         cells, cells * 4 / 1e6, 100.0 * leafcells / cells);
  printf("descent levels per query: full %.2f, from grid %.2f; ends at D itself %.1f%%, outside grid %.2f%%, membership fails %.2f%%\n", full / N, rest / N, 100 * hitleaf / N, 100 * outside / N, 100 * fails / N);
  printf("remaining-levels histogram:");
  for (int i = 0; i < 20; ++i) printf(" %d:%.1f%%", i, 100.0 * hist[i] / N);
  printf("\n");
}
