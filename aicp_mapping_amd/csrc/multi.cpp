// multi.cpp — one host process driving several GPUs with independent registration pairs
// ("independent reading/reference cloud pairs shard embarrassingly across the
// 8 GPUs of one node ... used only to gather per-pair transforms").
//
// A C++ host (the ROS node's worker, app.cpp:528-550) has no torch.distributed; this is its
// multi-GPU path. One context per device, one host thread per device, no data-path exchange:
// each device runs aicp_hip_align_batch on its shard, and the "gather" of the 72-byte results
// is the threads writing them into the caller's arrays at the pairs' own indices. Shards are the
// longest-processing-time greedy over a per-pair cost of n_read * log2(n_ref) (ties by index),
// the weighted form of sharding.py's shard_pairs. A pair's result does not depend on the batch
// it runs in (test_batch_deterministic_and_order_independent), so the output equals one
// device's aicp_hip_align_batch over all pairs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/aicp_hip.h"

struct aicp_hip_multi {
  std::vector<aicp_hip_ctx*> ctx;
  std::vector<int> device;
  std::string err;
};

namespace {

// owner[i] = the shard of pair i
std::vector<int> lpt_owners(const aicp_pair* pairs, size_t n, int shards) {
  std::vector<double> w(n);
  for (size_t i = 0; i < n; ++i)
    w[i] = (double)pairs[i].n_read * std::log2((double)std::max<uint64_t>(2, pairs[i].n_ref));
  std::vector<size_t> idx(n);
  std::iota(idx.begin(), idx.end(), size_t(0));
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return w[a] > w[b]; });
  std::vector<double> load((size_t)shards, 0.0);
  std::vector<int> owner(n, 0);
  for (size_t i : idx) {
    const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    owner[i] = g;
    load[(size_t)g] += w[i];
  }
  return owner;
}

}  // namespace

extern "C" {

int aicp_hip_multi_create(const int* devices, int n_devices, aicp_hip_multi** out) {
  if (!out) return AICP_ERR_INVALID;
  *out = nullptr;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail <= 0) return AICP_ERR_HIP;
  std::vector<int> dev;
  if (devices) {
    if (n_devices <= 0) return AICP_ERR_INVALID;
    dev.assign(devices, devices + n_devices);
  } else {
    const int n = n_devices > 0 ? n_devices : avail;
    for (int g = 0; g < n; ++g) dev.push_back(g);
  }
  for (int g : dev)
    if (g < 0 || g >= avail) return AICP_ERR_INVALID;
  aicp_hip_multi* m = new aicp_hip_multi();
  for (int g : dev) {
    aicp_hip_ctx* c = nullptr;
    const int rc = aicp_hip_create(g, &c);
    if (rc) {
      aicp_hip_multi_destroy(m);
      return rc;
    }
    m->ctx.push_back(c);
    m->device.push_back(g);
  }
  *out = m;
  return AICP_OK;
}

void aicp_hip_multi_destroy(aicp_hip_multi* m) {
  if (!m) return;
  for (aicp_hip_ctx* c : m->ctx) aicp_hip_destroy(c);
  delete m;
}

int aicp_hip_multi_size(const aicp_hip_multi* m) { return m ? (int)m->ctx.size() : 0; }

aicp_hip_ctx* aicp_hip_multi_context(aicp_hip_multi* m, int i) {
  return (m && i >= 0 && i < (int)m->ctx.size()) ? m->ctx[(size_t)i] : nullptr;
}

const char* aicp_hip_multi_last_error(const aicp_hip_multi* m) { return m ? m->err.c_str() : "null handle"; }

int aicp_hip_multi_align_batch(aicp_hip_multi* m, const aicp_icp_config* cfg, const aicp_pair* pairs, size_t n_pairs,
                               double resolution, int flags, float* out_T, aicp_icp_stats* stats, int* out_device) {
  if (!m || m->ctx.empty() || !cfg || (n_pairs && (!pairs || !out_T))) return AICP_ERR_INVALID;
  m->err.clear();
  if (n_pairs == 0) return AICP_OK;
  const int G = (int)m->ctx.size();
  const std::vector<int> owner = lpt_owners(pairs, n_pairs, G);
  std::vector<std::vector<size_t>> mine((size_t)G);
  for (size_t i = 0; i < n_pairs; ++i) mine[(size_t)owner[i]].push_back(i);
  std::vector<int> rc((size_t)G, AICP_OK);
  std::vector<std::string> msg((size_t)G);
  auto run = [&](int g) {
    const std::vector<size_t>& ids = mine[(size_t)g];
    if (ids.empty()) return;
    std::vector<aicp_pair> sub(ids.size());
    for (size_t k = 0; k < ids.size(); ++k) sub[k] = pairs[ids[k]];
    std::vector<float> T(16 * ids.size());
    std::vector<aicp_icp_stats> st(stats ? ids.size() : 0);
    aicp_hip_ctx* c = m->ctx[(size_t)g];
    rc[(size_t)g] = aicp_hip_align_batch(c, cfg, sub.data(), sub.size(), resolution, flags, T.data(),
                                         stats ? st.data() : nullptr);
    if (rc[(size_t)g]) msg[(size_t)g] = aicp_hip_last_error(c);
    // the gather: every pair's record at its own index (per-pair statuses stay meaningful when
    // the call reports an error, as on one device)
    for (size_t k = 0; k < ids.size(); ++k) {
      std::copy(T.begin() + 16 * k, T.begin() + 16 * (k + 1), out_T + 16 * ids[k]);
      if (stats) stats[ids[k]] = st[k];
      if (out_device) out_device[ids[k]] = m->device[(size_t)g];
    }
  };
  int cur = 0;
  const bool had = hipGetDevice(&cur) == hipSuccess;
  std::vector<std::thread> th;
  for (int g = 1; g < G; ++g) th.emplace_back(run, g);
  run(0);
  for (std::thread& t : th) t.join();
  if (had) (void)hipSetDevice(cur);  // (shard 0 ran on the calling thread)
  for (int g = 0; g < G; ++g)
    if (rc[(size_t)g]) {
      m->err = "device " + std::to_string(m->device[(size_t)g]) + ": " + msg[(size_t)g];
      return rc[(size_t)g];
    }
  return AICP_OK;
}

}  // extern "C"
