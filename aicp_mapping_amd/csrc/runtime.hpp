// runtime.hpp — host-side runtime shared by the C-ABI translation units (aicp_hip.cpp, sequence.cpp):
// device / pinned buffers, kd-tree work space, the context and batch objects, error macros.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/aicp_hip.h"
#include "aicp_common.hpp"
#include "kernels.hpp"

namespace aicp {
namespace rt {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

inline hipError_t ensure(DevBuf& b, size_t bytes) {
  if (bytes <= b.cap && b.p) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  const size_t nb = std::max<size_t>(256, bytes + bytes / 4);
  const hipError_t e = hipMalloc(&b.p, nb);
  if (e == hipSuccess) b.cap = nb;
  return e;
}
inline hipError_t ensure(PinBuf& b, size_t bytes) {
  if (bytes <= b.cap && b.p) return hipSuccess;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  const size_t nb = std::max<size_t>(256, bytes + bytes / 4);
  const hipError_t e = hipHostMalloc(&b.p, nb, hipHostMallocDefault);
  if (e == hipSuccess) b.cap = nb;
  return e;
}
inline void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}
inline void release(PinBuf& b) {
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

// A fixed pool of host threads for packing (spawning 16 threads per call costs more than the
// packing of a C2 cloud: the stream's windows and the one-shot calls of a context share one).
class WorkerPool {
 public:
  explicit WorkerPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // fn(task) for task in [0, n), on the pool and the calling thread; returns when all are done
  // and no worker is inside the task loop any more (so the next run() may reset the counter)
  void run(size_t n, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    {
      std::lock_guard<std::mutex> l(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [&] { return done_ == n_ && active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= n_) return;
      (*fn_)(i);
      std::lock_guard<std::mutex> l(mu_);
      if (++done_ == n_) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || (gen_ != seen && fn_ != nullptr); });
        if (stop_) return;
        seen = gen_;
        ++active_;
      }
      work();
      std::lock_guard<std::mutex> l(mu_);
      if (--active_ == 0 && done_ == n_) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0, done_ = 0;
  int active_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Work space of one kd-tree construction (kernels_tree.hip). Two sets: the raw-coordinate
// tree (SurfaceNormal) and the centred matcher tree are built concurrently on two streams.
struct TreeBufs {
  DevBuf W0, W1, segof0, segof1, seg0, seg1, flag, X1, X2, posL, posR, ev, valid, subs, mids, ecnt, sums, pdepth,
      ctl, scan, lb;
  PinBuf pin_ctl;
  TreeWork tw{};    // device_trees_begin -> device_trees_end
  int planned = 0;  // global levels enqueued without host polling (0: polled build)
  int needed = 0;   // global levels the last planned build actually used
  uint32_t lvl_min = 1u << 22;  // aicp_hip_options::tree_lvl_min of the owning context
  bool prof = false;            // aicp_hip_options::profile
  void release_all() {
    for (DevBuf* b : {&W0, &W1, &segof0, &segof1, &seg0, &seg1, &flag, &X1, &X2, &posL, &posR, &ev, &valid, &subs,
                      &mids, &ecnt, &lb, &sums, &pdepth, &ctl, &scan})
      release(*b);
    release(pin_ctl);
  }
};

struct Maps {  // block maps of one flat grid
  std::vector<int32_t> pair;
  std::vector<uint32_t> start;
  void add(int p, uint32_t n, uint32_t per_block) {
    for (uint32_t s = 0; s < n; s += per_block) {
      pair.push_back(p);
      start.push_back(s);
    }
  }
};

// ICP pair groups (1 or 2; AICP_ICP_GROUPS=2 selects two). Two groups measured slower on C2
// (3480 -> 3390 clouds/s): an NN launch over half the pairs takes 62 % of a full one.

// SurfaceNormalDataPointsFilter builds its own libnabo tree with the default bucket size (8),
// whatever bucketSize the chain gives the KDTreeMatcher
constexpr int kNormalsBucket = 8;

struct PackSeg {
  const float* src;
  uint64_t n, stride;
  float* dst4;
};
// Strided xyz -> float4 (w = 1) for many clouds at once, split into equal point ranges over
// up to 16 host threads
void pack_many(const std::vector<PackSeg>& segs, WorkerPool* pool = nullptr);
void pack_xyz4(const float* src, uint64_t n, uint64_t stride_bytes, float* dst4);
bool valid_pair(const aicp_pair& p);
double ev_ms(hipEvent_t a, hipEvent_t b);
// the context options a tree buffer set follows (tree_lvl_min, profile)
void tree_opts(TreeBufs& T, const aicp_hip_options& o);

// Centroid (center = 1) + libnabo-order kd-trees of P clouds on the device (kernels_tree.hip).
// launch = false: allocate the work space only (nothing enqueued; before a stream capture);
// part: launch_tree_prepare's (1: the kernels that do not read the points, 2: the rest, 0: all)
int device_trees_begin(TreeBufs& T, std::string& err, hipStream_t s, size_t P, uint64_t total, PairDesc* dDesc,
                       const float4* raw, int center, int bucket, DevBuf& bpts_out, DevBuf& nodes_out,
                       bool launch = true, int part = 0);
// plan > 0: `plan` global levels with no host read-back; the control block is copied to
// ctl_dst (default T.pin_ctl) at the end of the build unless copy_ctl is false
int device_trees_end(TreeBufs& T, std::string& err, hipStream_t s, size_t P, uint64_t total, PairDesc* dDesc,
                     int bucket, DevBuf& bpts_out, DevBuf& nodes_out, int plan, TreeCtl* ctl_dst = nullptr,
                     bool copy_ctl = true, hipEvent_t levels_done = nullptr);
// errors of a planned build whose control block is in hctl (after its stream completed)
int device_trees_check_ctl(TreeBufs& T, const TreeCtl* hctl, std::string& err);
int device_trees_check(TreeBufs& T, std::string& err);
// force: aicp_hip_options::tree_plan
int plan_levels(uint64_t n_max, const TreeBufs& T, int force, bool lean = false);
int check_cfg(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, int flags);

// The drop-in path's reference cache. App registers reading after reading against one reference
// (app.cpp:72-73, a new one every reference_update_frequency readings, app.cpp:383-391) and calls
// computeOverlap + registerClouds per reading (app.cpp:132-135, 205-210): the reference side of a
// one-shot call (aicp_hip_register / _overlap / _align_batch with one reference array) stays
// resident in the context and is reused while the next call passes the same reference.
struct RefCache {
  // identity: the caller's array (pointer, count, stride), and its points, packed, compared byte
  // for byte on every call (the caller may rewrite the array in place)
  const float* ptr = nullptr;
  uint64_t n = 0, stride = 0;
  std::vector<float> pts;
  // ctx->bpts, bnrm, nodes, tl, ptl, rdesc, rstate hold its matcher tree, treelets and normals
  bool trees = false;
  int bucket = 0, knn = 0;
  uint64_t tl_total = 0;
  // ctx->bitmap[0, od.bytes) holds its voxel map for (origin, res); gst its group state (|A|, key box)
  bool ovl = false;
  double origin[3] = {0, 0, 0};
  double res = 0;
  OvlDesc od{};
  DevBuf gst;
  // this call
  bool use = false;  // the call may reuse / record (one reference array, a one-shot call)
  bool hit_trees = false, hit_ovl = false;
  uint64_t tree_hits = 0, tree_builds = 0, ovl_hits = 0, ovl_builds = 0;
  void invalidate() {
    trees = ovl = false;
    hit_trees = hit_ovl = use = false;
  }
};

// The reading of the last one-shot call (one pair): App passes the same reading to
// computeOverlap and then to registerClouds (app.cpp:132-135, 205-210), so the second call reuses
// its upload and Morton order (the one-shot batch's read_raw, ctx->read_s) when the array is the
// same and its points are byte-identical.
struct ReadCache {
  const float* ptr = nullptr;
  uint64_t n = 0, stride = 0;
  std::vector<float> pts;
  bool valid = false;
  bool sorted = false;  // its Morton order is in read_s (else the one-shot batch's read_raw serves)
  bool hit = false;  // this call
  uint64_t hits = 0;
};

struct SeqState;  // sequence.cpp
void seq_state_free(SeqState* s);

}  // namespace rt
}  // namespace aicp

struct aicp_hip_batch {
  size_t P = 0;
  std::vector<aicp::PairDesc> desc;
  std::vector<aicp::PairDesc> rdesc;  // one per distinct reference cloud (tree + normals built once)
  std::vector<aicp::PairDesc> gdesc;  // one per overlap group: distinct (reference cloud, origin)
  uint64_t total_ref = 0, total_read = 0;
  uint32_t n_red_total = 0;
  aicp::rt::DevBuf ref_raw, read_raw, maps;
  aicp::BlockMap m_read{}, m_gref{}, m_red{}, m_sel{};
  bool refs_event = false;  // upload_pairs recorded ctx->ev[14] after the references' copy
};

struct aicp_hip_map {  // a device-resident point cloud (float4, w = 1)
  aicp::rt::DevBuf pts;
  size_t n = 0;
};

struct aicp_hip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // raw kd-tree + normals, concurrent with the overlap on `stream`
  hipStream_t stream3 = nullptr;  // centroid + matcher kd-tree, concurrent with both
  std::string err;
  aicp::rt::DevBuf read_c, bpts, bnrm, nodes, match, d2, desc, state, touch, slab, bitmap, outT, scratch, active,
      ctrs, nbids, ref1, sel_hist, sel_cand, sel_cnt, qmap, ovl, rdesc, rstate, rdesc_raw, bpts_raw, nodes_raw,
      nrm_raw, inv, gdesc, gstate, read_s, ord_k0, ord_k1, ord_v0, ord_v1, ord_tmp, tl, ptl,
      tl_rank, pf_a, pf_b, pf_bpts, pf_nodes;  // pf_*: the pre-filter's own (the reference cache keeps bpts / nodes)
  uint64_t tl_total = 0;  // matcher treelet records allotted for this batch (0: no treelets, Trav<1>)
  aicp::rt::TreeBufs tb[2];  // [0] raw-coordinate tree (stream2), [1] centred matcher tree (stream3)
  aicp::rt::PinBuf pin_desc, pin_state, pin_out, pin_io, pin_ovl, pin_rdesc, pin_gdesc, pin_gstate;
  aicp::rt::PinBuf pin_pf;  // pre-filter read-backs (PfHost): outlive any early return of pf_core
  std::vector<hipEvent_t> nn_ev;
  hipEvent_t ev[16] = {};
  int last_nn_launches = 0;
  double last_nn_ms = 0, last_nn_bytes = 0;
  uint64_t last_queries = 0;
  double last_phase[5] = {0, 0, 0, 0, 0};
  aicp_prefilter_stats last_pf{};  // timing and kNN counts of the last pre-filter
  aicp_hip_batch* oneshot = nullptr;  // buffers of aicp_hip_align_batch, kept across calls
  hipEvent_t pf_ev[8] = {};
  aicp::rt::SeqState* seq = nullptr;  // aicp_hip_sequence_run's buffers (sequence.cpp), kept across calls
  aicp_hip_batch* mapbatch = nullptr;  // aicp_hip_map_register_batch's batch buffers
  aicp::rt::DevBuf crop_ws;            // its crop work space
  aicp::rt::DevBuf ovl_sp, ovl_keys;   // sparse overlap: clouds, counts, offsets / key words
  aicp::rt::DevBuf isync;              // fused ICP iteration: arrival counters (icp_sync_words)
  aicp::rt::PinBuf pin_crop;
  aicp::rt::PinBuf pin_maps;  // upload_pairs' block maps
  aicp::rt::RefCache refc;  // the drop-in path's resident reference (runtime.hpp)
  aicp::rt::ReadCache rdc;  // and its last reading
  aicp::rt::WorkerPool* pool = nullptr;  // host threads of the one-shot calls (packing, the reference compare)
  uint32_t* poll_host = nullptr;  // the batch loop's active counts (hipHostMalloc, mapped), kBatchPolls words
  uint32_t* poll_dev = nullptr;
  aicp_hip_options opt{};  // aicp_hip_set_options (read by the calls; nothing reads the environment)
};
constexpr int kBatchPolls = 64;

#define HIPC(x)                                                                   \
  do {                                                                            \
    const hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                       \
      ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                  \
      return AICP_ERR_HIP;                                                        \
    }                                                                             \
  } while (0)

#define FAIL(code, msg)   \
  do {                    \
    ctx->err = (msg);     \
    return (code);        \
  } while (0)

// Tree builders report errors into `err` (they also run on a worker thread, see run_batch).
#define TCHK(x)                                                                   \
  do {                                                                            \
    const hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                       \
      err = std::string(#x) + ": " + hipGetErrorString(e_);                       \
      return AICP_ERR_HIP;                                                        \
    }                                                                             \
  } while (0)
#define TFAIL(code, msg) \
  do {                   \
    err = (msg);         \
    return (code);       \
  } while (0)
