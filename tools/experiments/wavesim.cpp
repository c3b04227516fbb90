// wavesim.cpp — design experiment (not product): dependent-load "ticks" per query of the ICP
// NN kernel's persistent waves, from the exact libnabo-order traversal of every query (Trav2
// two-level records) replayed in 64-lane waves. A wave round = refill (read_c load, plus the
// grid cell and node-region loads with a grid start), a descent phase of at most K record
// loads (lanes that reach their leaf wait for the others), one cooperative bucket load, and
// the climb (parent loads) of the lanes that did their bucket. Lanes whose descent is cut off
// by K continue it in the next round.
// Build: g++ -O2 -std=c++17 wavesim.cpp kdtree_host.cpp -o wavesim
// Usage: wavesim ref.bin read.bin cells_per_point
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

struct Round { int desc, climb; std::vector<int> dn, cn; int b0; };  // record loads of the descent (ids dn), bucket start, parent loads (ids cn)

int main(int argc, char** argv) {
  auto ref = load(argv[1]), rd = load(argv[2]);
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
  auto isleaf = [&](int n) { return (node(n)[1] & 3u) == 3u; };
  // grid
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < M; ++i) for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], ref[3 * i + d]); hi[d] = fmaxf(hi[d], ref[3 * i + d]); }
  const double budget = (argc > 3 ? atof(argv[3]) : 2.0) * M;
  double e[3], vol = 1;
  for (int d = 0; d < 3; ++d) { e[d] = std::max(1e-3, (double)hi[d] - lo[d]); vol *= e[d]; }
  double hh = cbrt(vol / budget);
  int dims[3];
  for (;;) { size_t c = 1; for (int d = 0; d < 3; ++d) { dims[d] = std::max(1, (int)ceil(e[d] / hh)); c *= dims[d]; } if (c <= budget) break; hh *= 1.02; }
  const float h = (float)hh, invh = (float)(1.0 / hh);
  const size_t cells = (size_t)dims[0] * dims[1] * dims[2];
  std::vector<int32_t> D(cells);
  std::vector<float> box(cells * 6);
  for (int z = 0; z < dims[2]; ++z) for (int y = 0; y < dims[1]; ++y) for (int x = 0; x < dims[0]; ++x) {
    const float bl[3] = {lo[0] + x * h, lo[1] + y * h, lo[2] + z * h};
    const float bh[3] = {bl[0] + h, bl[1] + h, bl[2] + h};
    float rl[3] = {-INFINITY, -INFINITY, -INFINITY}, rh[3] = {INFINITY, INFINITY, INFINITY};
    int n = 0;
    while (!isleaf(n)) {
      const uint32_t* nd = node(n);
      const int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
      if (bl[cd] - cut > 0) { n = nd[1] >> 2; rl[cd] = std::max(rl[cd], cut); }
      else if (bh[cd] - cut <= 0) { n = n + 1; rh[cd] = std::min(rh[cd], cut); }
      else break;
    }
    const size_t c = ((size_t)z * dims[1] + y) * dims[0] + x;
    D[c] = n;
    for (int d = 0; d < 3; ++d) { box[6 * c + d] = rl[d]; box[6 * c + 3 + d] = rh[d]; }
  }
  const float E = (1 + 3.16f) * (1 + 3.16f), R = INFINITY;
  // Morton order of the reading (kernels_order.hip sorts each reading on 0.25 m cells)
  {
    std::vector<std::pair<uint64_t, int>> key(N);
    for (int i = 0; i < N; ++i) {
      uint64_t k = 0;
      uint32_t c[3];
      for (int d = 0; d < 3; ++d) c[d] = (uint32_t)std::min(std::max((int)floorf((rd[3 * i + d] + 512.f) / 0.25f), 0), 1 << 20);
      for (int b = 20; b >= 0; --b) for (int d = 2; d >= 0; --d) k = (k << 1) | ((c[d] >> b) & 1);
      key[i] = {k, i};
    }
    std::stable_sort(key.begin(), key.end(), [](auto& a, auto& b) { return a.first < b.first; });
    std::vector<float> r2(rd.size());
    for (int i = 0; i < N; ++i) for (int d = 0; d < 3; ++d) r2[3 * i + d] = rd[3 * key[i].second + d];
    rd.swap(r2);
  }
  // per query, per grid mode: rounds
  std::vector<std::vector<Round>> Q[2];
  for (int g = 0; g < 2; ++g) Q[g].resize(N);
  for (int qi = 0; qi < N; ++qi) {
    const float q[3] = {rd[3 * qi] - (float)m[0], rd[3 * qi + 1] - (float)m[1], rd[3 * qi + 2] - (float)m[2]};
    int gstart = 0;
    {
      int c3[3];
      for (int d = 0; d < 3; ++d) c3[d] = std::min(std::max((int)floorf((q[d] - lo[d]) * invh), 0), dims[d] - 1);
      const size_t c = ((size_t)c3[2] * dims[1] + c3[1]) * dims[0] + c3[0];
      bool ok = true;
      for (int d = 0; d < 3; ++d) ok = ok && (q[d] - box[6 * c + d] > 0) && (q[d] - box[6 * c + 3 + d] <= 0);
      if (ok) gstart = D[c];
    }
    for (int g = 0; g < 2; ++g) {
      // Trav<1>-semantics traversal, counting Trav2 record loads for descents
      float off[3] = {0, 0, 0}, rd_ = 0, best = INFINITY;
      struct Fr { int P, PP, start; float rd, old, mn; int cd; };
      std::vector<Fr> st;
      int start = 0;
      int n = g ? gstart : 0;
      bool first = true;
      for (;;) {
        // descent (levels above a grid start are folded into minFar exactly; recompute from root)
        float minFar = INFINITY;
        if (first && g) {
          int a = 0;
          while (a != n) {
            const uint32_t* nd = node(a);
            const int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
            const float no = q[cd] - cut; minFar = fminf(minFar, no * no);
            a = no > 0 ? (int)(nd[1] >> 2) : a + 1;
          }
        }
        first = false;
        int loads = 0;
        // Trav2: one record load decides the node and (if inner) its chosen child
        std::vector<int> dn, cn;
        for (;;) {
          ++loads; dn.push_back(n);
          if (isleaf(n)) break;
          const uint32_t* nd = node(n);
          int cd = nd[1] & 3; float cut; memcpy(&cut, &nd[0], 4);
          float no = q[cd] - cut, oc = off[cd];
          minFar = fminf(minFar, rd_ + (-oc * oc + no * no));
          n = no > 0 ? (int)(nd[1] >> 2) : n + 1;
          if (isleaf(n)) break;
          nd = node(n);
          cd = nd[1] & 3; memcpy(&cut, &nd[0], 4);
          no = q[cd] - cut; oc = off[cd];
          minFar = fminf(minFar, rd_ + (-oc * oc + no * no));
          n = no > 0 ? (int)(nd[1] >> 2) : n + 1;
        }
        const uint32_t* lf = node(n);
        for (uint32_t i = 0; i < lf[0]; ++i) {
          const float* p = &bp[3 * ((lf[1] >> 2) + i)];
          const float d0 = q[0] - p[0], d1 = q[1] - p[1], d2 = q[2] - p[2];
          float dist = 0; dist += d0 * d0; dist += d1 * d1; dist += d2 * d2;
          if (dist <= R && dist < best) best = dist;
        }
        int climb = 0;
        int c = n, pc = (int)lf[2];
        if (!(minFar <= R && minFar * E < best)) c = start;
        bool descend = false, done = false;
        while (!descend) {
          if (c == start) {
            if (st.empty()) { done = true; break; }
            Fr f = st.back(); st.pop_back();
            rd_ = f.rd; off[f.cd] = f.old; minFar = f.mn; start = f.start; c = f.P; pc = f.PP;
            if (!(minFar <= R && minFar * E < best)) c = start;
            continue;
          }
          const int p = pc; const uint32_t* pn = node(p); ++climb; cn.push_back(p);
          const int cd = pn[1] & 3; float cut; memcpy(&cut, &pn[0], 4);
          const float no = q[cd] - cut, oc = off[cd];
          const float rdf = rd_ + (-oc * oc + no * no);
          if (rdf <= R && rdf * E < best) {
            const int far = no > 0 ? p + 1 : (int)(pn[1] >> 2);
            st.push_back({p, (int)pn[2], start, rd_, oc, minFar, cd});
            off[cd] = no; rd_ = rdf; n = far; start = far; descend = true;
          } else { c = p; pc = (int)pn[2]; }
        }
        Q[g][qi].push_back({loads, climb, dn, cn, (int)(lf[1] >> 2)});
        if (done) break;
      }
    }
  }
  for (int g = 0; g < 2; ++g) {
    double ld = 0, rounds = 0;
    for (auto& v : Q[g]) for (auto& r : v) { ld += r.desc; rounds++; }
    printf("grid %d: record loads per query %.2f, rounds per query %.3f\n", g, ld / N, rounds / N);
    if (g == 0) {
      double cl = 0, withclimb = 0, withfar = 0, firstclimb = 0;
      std::vector<int> hr(10, 0);
      for (auto& v : Q[g]) {
        int c = 0; for (auto& r : v) c += r.climb;
        cl += c; withclimb += c > 0; withfar += v.size() > 1; firstclimb += v[0].climb;
        hr[std::min<size_t>(v.size(), 9)]++;
      }
      printf("  climb loads per query %.2f (first round %.2f); queries with a climb %.1f%%, with a far descent %.1f%%\n", cl / N, firstclimb / N, 100 * withclimb / N, 100 * withfar / N);
      printf("  rounds histogram:"); for (int i = 1; i < 10; ++i) printf(" %d:%.1f%%", i, 100.0 * hr[i] / N); printf("\n");
    }
  }
  // "if-if" replay: every iteration each lane takes one step of its own phase (a descent record,
  // a climb load); lanes at a leaf wait until at least B lanes are at leaves (or no lane can step),
  // then one cooperative bucket pass (1 tick, 8 instructions) serves all of them.
  for (int g = 0; g < 1; ++g)
    for (int B : {1, 8, 16, 32, 64}) {
      size_t next = 0;
      struct Lane { int q = -1; size_t r = 0; int ph = 0; int k = 0; };  // ph 0 descent, 1 at leaf, 2 climb
      std::vector<Lane> L(64);
      double ticks = 0, ins = 0, lanesteps = 0;
      for (;;) {
        bool any = false, refill = false;
        for (auto& l : L) {
          if (l.q < 0 && next < (size_t)N) { l.q = (int)next++; l.r = 0; l.ph = 0; l.k = 0; refill = true; }
          if (l.q >= 0) any = true;
        }
        if (!any) break;
        if (refill) ins += 1;
        int atleaf = 0, stepping = 0;
        for (auto& l : L) if (l.q >= 0) { if (l.ph == 1) ++atleaf; else ++stepping; }
        if (atleaf > 0 && (atleaf >= B || stepping == 0)) {
          ticks += 1; ins += 8;
          for (auto& l : L) if (l.q >= 0 && l.ph == 1) { l.ph = 2; l.k = 0; }
        }
        // one step for every lane in descent or climb
        bool d = false, c = false;
        for (auto& l : L) {
          if (l.q < 0) continue;
          const Round& R = Q[g][l.q][l.r];
          if (l.ph == 0) { d = true; lanesteps++; if (++l.k >= R.desc) { l.ph = 1; } }
          else if (l.ph == 2) {
            if (l.k < R.climb) { c = true; lanesteps++; ++l.k; }
            if (l.k >= R.climb) {
              l.r++; l.k = 0;
              if (l.r >= Q[g][l.q].size()) l.q = -1; else l.ph = 0;
            }
          }
        }
        if (d || c) ticks += 1;
        ins += (d ? 1 : 0) + (c ? 1 : 0);
      }
      const double W = N / 64.0;
      printf("if-if B %2d: ticks per 64 queries %.1f, instructions %.1f, lane utilisation %.2f\n", B, ticks / W, ins / W, lanesteps / (64.0 * ticks));
    }
  // wave replay of the current kernel (descent to the leaf, cooperative bucket, climb), counting
  // wave-instructions and distinct 128-B lines (TA tag work) per phase
  for (int g = 0; g < 2; ++g) {
    size_t next = 0;
    struct Lane { int q = -1; size_t r = 0; };
    std::vector<Lane> L(64);
    double ins[4] = {0, 0, 0, 0}, tags[4] = {0, 0, 0, 0}, ticks = 0;  // refill, descent, bucket, climb
    std::vector<long> lines;
    auto distinct = [&](std::vector<long>& v) { std::sort(v.begin(), v.end()); return (double)(std::unique(v.begin(), v.end()) - v.begin()); };
    for (;;) {
      bool any = false;
      lines.clear();
      for (auto& l : L) {
        if (l.q < 0 && next < (size_t)N) { l.q = (int)next++; l.r = 0; lines.push_back(l.q / 8); }
        if (l.q >= 0) any = true;
      }
      if (!any) break;
      if (!lines.empty()) { ins[0] += 1 + 2 * g; tags[0] += distinct(lines) * (1 + 2 * g); ticks += 1 + g; }
      int maxd = 0, maxc = 0;
      for (auto& l : L) if (l.q >= 0) { maxd = std::max(maxd, Q[g][l.q][l.r].desc); maxc = std::max(maxc, Q[g][l.q][l.r].climb); }
      for (int k = 0; k < maxd; ++k) {
        lines.clear();
        for (auto& l : L) if (l.q >= 0 && k < Q[g][l.q][l.r].desc) lines.push_back(Q[g][l.q][l.r].dn[k] / 4);
        ins[1] += 2; tags[1] += 2 * distinct(lines); ticks += 1;
      }
      for (int j = 0; j < 8; ++j) {
        lines.clear();
        for (int o = 0; o < 8; ++o) {
          const Lane& l = L[8 * o + j];
          if (l.q < 0) continue;
          const int b0 = Q[g][l.q][l.r].b0, cnt = node(0) ? 8 : 8;
          for (int i = 0; i < cnt; ++i) lines.push_back((b0 + i) / 8);
        }
        ins[2] += 1; tags[2] += distinct(lines);
      }
      ticks += 1;
      for (int k = 0; k < maxc; ++k) {
        lines.clear();
        for (auto& l : L) if (l.q >= 0 && k < Q[g][l.q][l.r].climb) lines.push_back(Q[g][l.q][l.r].cn[k] / 4);
        ins[3] += 1; tags[3] += distinct(lines); ticks += 1;
      }
      for (auto& l : L) if (l.q >= 0) { l.r++; if (l.r >= Q[g][l.q].size()) l.q = -1; }
    }
    const double W = N / 64.0;
    printf("grid %d per 64 queries: ticks %.1f | instr refill %.1f descent %.1f bucket %.1f climb %.1f | tags refill %.0f descent %.0f bucket %.0f climb %.0f (total %.0f, %.1f per instr)\n",
           g, ticks / W, ins[0] / W, ins[1] / W, ins[2] / W, ins[3] / W, tags[0] / W, tags[1] / W, tags[2] / W, tags[3] / W,
           (tags[0] + tags[1] + tags[2] + tags[3]) / W, (tags[0] + tags[1] + tags[2] + tags[3]) / (ins[0] + ins[1] + ins[2] + ins[3]));
  }
}
