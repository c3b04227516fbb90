// kdtree_host.cpp — see kdtree_host.hpp.
#include "kdtree_host.hpp"

#include <algorithm>
#include <cstring>
#include <limits>

namespace aicp {
namespace {

struct BP {
  float p[3];
  int32_t id;
};

struct Builder {
  std::vector<BP>& pts;
  HostTree& t;
  int bucket;

  int32_t emit(uint32_t x, uint32_t y, int32_t par) {
    const int32_t pos = (int32_t)t.parent.size();
    t.nodes.push_back(x);
    t.nodes.push_back(y);
    t.nodes.push_back((uint32_t)par);
    t.nodes.push_back(0u);
    t.parent.push_back(par);
    return pos;
  }

  int32_t build(int first, int last, const float* mn, const float* mx, int32_t par, int depth) {
    const int count = last - first;
    if (depth > t.depth) t.depth = depth;
    if (count <= bucket) {
      for (int i = first; i < last; ++i) t.perm.push_back(pts[i].id);
      return emit((uint32_t)count, 3u | ((uint32_t)first << 2), par);
    }
    int cd = 0;
    float widest = 0;
    for (int d = 0; d < 3; ++d) {
      const float e = mx[d] - mn[d];
      if (e > widest) {
        widest = e;
        cd = d;
      }
    }
    const float ideal = (mx[cd] + mn[cd]) / 2;
    float lo = std::numeric_limits<float>::max(), hi = std::numeric_limits<float>::lowest();
    for (int i = first; i < last; ++i) {
      lo = std::min(pts[i].p[cd], lo);
      hi = std::max(pts[i].p[cd], hi);
    }
    const float cut = ideal < lo ? lo : (ideal > hi ? hi : ideal);
    BP* f = pts.data() + first;
    int l = 0, r = count - 1;
    while (true) {
      while (l < count && f[l].p[cd] < cut) ++l;
      while (r >= 0 && f[r].p[cd] >= cut) --r;
      if (l > r) break;
      std::swap(f[l++], f[r--]);
    }
    const int br1 = l;
    r = count - 1;
    while (true) {
      while (l < count && f[l].p[cd] <= cut) ++l;
      while (r >= br1 && f[r].p[cd] > cut) --r;
      if (l > r) break;
      std::swap(f[l++], f[r--]);
    }
    const int br2 = l;
    int left;
    if (ideal < lo)
      left = 1;
    else if (ideal > hi)
      left = count - 1;
    else if (br1 > count / 2)
      left = br1;
    else if (br2 < count / 2)
      left = br2;
    else
      left = count / 2;
    uint32_t cutBits;
    std::memcpy(&cutBits, &cut, 4);
    const int32_t me = emit(cutBits, 0, par);
    float lmx[3] = {mx[0], mx[1], mx[2]};
    lmx[cd] = cut;
    float rmn[3] = {mn[0], mn[1], mn[2]};
    rmn[cd] = cut;
    build(first, first + left, mn, lmx, me, depth + 1);
    const int32_t right = build(first + left, last, rmn, mx, me, depth + 1);
    t.nodes[4 * me + 1] = (uint32_t)cd | ((uint32_t)right << 2);
    return me;
  }
};

}  // namespace

void build_kdtree_host(const float* xyz, int64_t n, int bucket, HostTree& out) {
  std::vector<BP> pts((size_t)n);
  float mn[3], mx[3];
  for (int d = 0; d < 3; ++d) {
    mn[d] = std::numeric_limits<float>::max();
    mx[d] = std::numeric_limits<float>::lowest();
  }
  for (int64_t i = 0; i < n; ++i) {
    for (int d = 0; d < 3; ++d) {
      const float v = xyz[3 * i + d];
      pts[i].p[d] = v;
      mn[d] = std::min(mn[d], v);
      mx[d] = std::max(mx[d], v);
    }
    pts[i].id = (int32_t)i;
  }
  out.nodes.clear();
  out.parent.clear();
  out.perm.clear();
  out.depth = 0;
  out.nodes.reserve((size_t)(n / std::max(1, bucket / 2) + 4) * 4);
  out.parent.reserve((size_t)(n / std::max(1, bucket / 2) + 4));
  out.perm.reserve((size_t)n);
  Builder b{pts, out, bucket};
  b.build(0, (int)n, mn, mx, -1, 0);
}

}  // namespace aicp
