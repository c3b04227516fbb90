// sequence.cpp — App's frame-to-reference stream on the device (aicp_hip_sequence_run).
//
// Reference behaviour (aicp_core/src/registration/app.cpp:282-414, robot working mode):
//   - the first cloud is the reference (app.cpp:285-312);
//   - every reading: overlap with the reference -> auto-tuned ratio -> ICP (runAicpPipeline,
//     app.cpp:218-247);
//   - |t_i| > max_correction_magnitude drops the reading (app.cpp:366-373);
//   - an accepted reading is transformed by its correction (pcl::transformPointCloud) and added
//     to the graph; the reference_update_frequency-th accepted reading since the last update
//     becomes the reference, its corrected pose (correction * prior pose) the new sensor origin
//     (app.cpp:375-391, aligned_cloud.cpp:61-70);
//   - an exception from registerClouds ends the worker (app.cpp:210).
//
// Device design. Readings go in windows of F = reference_update_frequency: the readings of a
// window are independent given its reference, so they run as one batch. Window w+1's reference
// is the last reading of window w corrected by its own T: k_seq_ref_points builds it
// on the device right after window w's ICP, and the whole sequence is enqueued at once with no
// host synchronisation between windows (the host packs and uploads window w+1 while the device
// runs window w). That schedule predicts that every reading is accepted; the host checks the
// prediction once at the end and, at the first window with a dropped reading, keeps the results
// up to there and enqueues the rest again from the true state (same reference, fewer readings
// still to collect). Results therefore equal App's order of events in every case.
//
// Per window, four streams (HIP shares GPU_MAX_HW_QUEUES hardware queues per priority level;
// streams beyond that run in submission order, so the sequence keeps to few):
//   rd   H2D of the readings and descriptors (pinned staging, ring of K slots), then the
//        reading side: state init, Morton order, reading voxel maps (independent of the reference)
//   r3   next reference points (k_seq_ref_points), centroid + matcher kd-tree
//   r2   raw kd-tree + SurfaceNormal, normals into the matcher tree's order
//   icp  reference voxel map, overlap counts, ratio, ICP loop, corrections
// Window w's ICP loop is enqueued iteration by iteration; k_active_list (fused into the previous
// iteration's reduce) writes the active count into mapped host memory, and the host, one
// iteration ahead, stops enqueueing once it reads 0. Window w+1's reference (r3) then waits for
// w's ICP with an event. (r03: all maxIterationCount launches as one graph with r3 waiting for a
// ticket in signal memory, hipStreamWaitValue64, measured 2.79 against 2.25 ms per window: the
// trailing no-op launches held stream icp.)
// The matcher kd-tree build -- ~100 short kernels -- is replayed from a hipGraph captured per
// slot. Device buffers live in K window slots (reused with event waits);
// states and corrections of all readings are committed to sequence-wide arrays for the read-back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/aicp_hip.h"
#include "aicp_common.hpp"
#include "icp_math.hpp"
#include "kernels.hpp"
#include "runtime.hpp"

using namespace aicp;
using namespace aicp::rt;

namespace aicp {
namespace rt {

// A captured launch sequence (hipGraph) replayed while its key -- every argument and buffer
// address it was captured with -- stays the same: one graph launch instead of ~100 kernel
// launches per kd-tree build, ~160 per ICP loop (the host cost of those launches, ~5 us each,
// was the stream's bottleneck).
struct GraphCache {
  std::vector<uint64_t> key;
  hipGraphExec_t exec = nullptr;
  bool broken = false;  // a capture failed: direct launches from then on
  void reset() {
    if (exec) (void)hipGraphExecDestroy(exec);
    exec = nullptr;
    key.clear();
  }
};


struct Key {
  std::vector<uint64_t> v;
  template <class T>
  Key& operator<<(const T& x) {
    static_assert(std::is_trivially_copyable<T>::value, "plain values");
    uint64_t w[(sizeof(T) + 7) / 8] = {};
    std::memcpy(w, &x, sizeof(T));
    v.insert(v.end(), w, w + (sizeof(T) + 7) / 8);
    return *this;
  }
};

constexpr int kSlots = 3;  // window slots in flight (>= 2: a window reads the previous slot's reading)
constexpr int kMaxPolls = 64;  // ICP iterations that can end a window's loop early


struct SeqSlot {
  // reading side (window-local offsets)
  DevBuf read_raw, read_s, read_c, match, d2, touch, cand, slab, ord_k0, ord_k1, ord_v0, ord_v1, ord_tmp, maps, bitmap,
      ovl, caps, sel_hist, sel_cnt, ctrs, active;
  // reference side
  DevBuf ref_src, ref_raw, bpts, bnrm, nodes, tl, ptl, tl_rank, bpts_raw, nodes_raw, nrm_raw, nbids,
      inv, rd, tsrc,  // rd: rdesc, rdesc_raw, gdesc (PairDesc) + rstate, gstate (PairState); tsrc: source T
      wdesc, wstate, woutT, isync,  // the window's readings (committed to the sequence's arrays at its end)
      sp_par, sp_cnt, sp_off, sp_keys_r, sp_keys_g, sp_tmp_r, sp_tmp_g, sp_pc;  // sorted-key overlap (sparse windows)
  TreeBufs tb[2];
  PinBuf pin_read, pin_par, pin_src;
  hipEvent_t ev_up = nullptr, ev_rd = nullptr, ev_ref = nullptr, ev_s3 = nullptr, ev_s2 = nullptr, ev_done = nullptr;
  hipEvent_t ev_src = nullptr;  // recorded on stream icp once the window's last reading has stopped (early_reference)
  // early exit of the ICP loops: active counts written by the update kernels into mapped host
  // memory, one word per iteration, in two areas (debug mode's consecutive per-reading loops
  // alternate, so a loop's trailing write never lands in its successor's words)
  uint32_t* poll_host = nullptr;  // hipHostMalloc(mapped), 2 * kMaxPolls words
  uint32_t* poll_dev = nullptr;   // its device address
  GraphCache g_match;
  bool used = false;
};

struct SeqState {
  hipStream_t s_up = nullptr, s_rd = nullptr, s_r2 = nullptr, s_r3 = nullptr, s_icp = nullptr;
  hipStream_t s_probe = nullptr;  // opt.profile: an idle stream whose markers time the host's enqueue
  SeqSlot slot[kSlots];
  DevBuf desc, state, outT;
  DevBuf initT;  // debug working mode: initialT_ (16 floats), then its value before each reading
  PinBuf pin_state, pin_out, pin_ctl, pin_desc;
  std::vector<hipEvent_t> nn_ev;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;
  std::vector<hipEvent_t> tev;  // opt.profile: 10 timing events per window
  aicp_hip_options opt{};        // the context's options at the start of the running call
  WorkerPool pool{std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1};
  aicp_sequence_timing last{};
  int device = 0;
};

void seq_state_free(SeqState* S) {
  if (!S) return;
  for (hipStream_t q : {S->s_up, S->s_rd, S->s_r2, S->s_r3, S->s_icp})
    if (q) (void)hipStreamSynchronize(q);
  for (SeqSlot& sl : S->slot) {
    for (DevBuf* b : {&sl.read_raw, &sl.read_s, &sl.read_c, &sl.match, &sl.d2, &sl.touch, &sl.cand, &sl.slab,
                      &sl.ord_k0, &sl.ord_k1, &sl.ord_v0, &sl.ord_v1, &sl.ord_tmp, &sl.maps, &sl.bitmap, &sl.ovl,
                      &sl.caps, &sl.sel_hist, &sl.sel_cnt, &sl.ctrs, &sl.active, &sl.ref_src, &sl.ref_raw, &sl.bpts,
                      &sl.bnrm, &sl.nodes, &sl.tl, &sl.ptl, &sl.tl_rank, &sl.bpts_raw,
                      &sl.nodes_raw, &sl.nrm_raw, &sl.nbids, &sl.inv, &sl.rd, &sl.tsrc, &sl.wdesc, &sl.wstate,
                      &sl.woutT, &sl.isync, &sl.sp_par, &sl.sp_cnt, &sl.sp_off, &sl.sp_keys_r,
                      &sl.sp_keys_g, &sl.sp_tmp_r, &sl.sp_tmp_g, &sl.sp_pc})
      release(*b);
    for (auto& t : sl.tb) t.release_all();
    sl.g_match.reset();
    for (PinBuf* b : {&sl.pin_read, &sl.pin_par, &sl.pin_src}) release(*b);
    for (hipEvent_t e : {sl.ev_up, sl.ev_rd, sl.ev_ref, sl.ev_s3, sl.ev_s2, sl.ev_done, sl.ev_src})
      if (e) (void)hipEventDestroy(e);
    if (sl.poll_host) (void)hipHostFree(sl.poll_host);
  }
  for (DevBuf* b : {&S->desc, &S->state, &S->outT, &S->initT}) release(*b);
  for (PinBuf* b : {&S->pin_state, &S->pin_out, &S->pin_ctl, &S->pin_desc}) release(*b);
  for (hipEvent_t e : S->nn_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : S->tev) (void)hipEventDestroy(e);
  for (hipEvent_t e : {S->ev_begin, S->ev_end})
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t q : {S->s_rd, S->s_icp, S->s_probe})  // (s_up = s_rd; s_r2, s_r3: the context's)
    if (q) (void)hipStreamDestroy(q);
  delete S;
}

}  // namespace rt
}  // namespace aicp

namespace {

// float AABB of a cloud's points and its sensor origin (the extent bounds its voxel maps)
struct Box {
  float lo[3], hi[3];
  void reset() {
    for (int k = 0; k < 3; ++k) {
      lo[k] = INFINITY;
      hi[k] = -INFINITY;
    }
  }
  void add(float x, float y, float z) {
    const float v[3] = {x, y, z};
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], v[k]);
      hi[k] = std::max(hi[k], v[k]);
    }
  }
  void merge(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
};

// xyz at a byte stride -> float4 (w = 1) and the AABB of the finite points, in chunks over the pool
void pack_clouds(WorkerPool& pool, const std::vector<PackSeg>& segs, std::vector<Box>& boxes) {
  constexpr uint64_t kChunk = 1 << 15;
  struct Task {
    size_t seg;
    uint64_t a, b;
  };
  std::vector<Task> tasks;
  for (size_t s = 0; s < segs.size(); ++s)
    for (uint64_t a = 0; a < segs[s].n; a += kChunk) tasks.push_back({s, a, std::min(segs[s].n, a + kChunk)});
  std::vector<Box> part(tasks.size());
  pool.run(tasks.size(), [&](size_t t) {
    const Task& k = tasks[t];
    const PackSeg& g = segs[k.seg];
    Box bx;
    bx.reset();
    const char* src = reinterpret_cast<const char*>(g.src);
    for (uint64_t i = k.a; i < k.b; ++i) {
      const float* p = reinterpret_cast<const float*>(src + i * g.stride);
      float* d = g.dst4 + 4 * i;
      d[0] = p[0];
      d[1] = p[1];
      d[2] = p[2];
      d[3] = 1.f;
      if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2])) bx.add(p[0], p[1], p[2]);
    }
    part[t] = bx;
  });
  boxes.assign(segs.size(), Box{});
  for (Box& b : boxes) b.reset();
  for (size_t t = 0; t < tasks.size(); ++t) boxes[tasks[t].seg].merge(part[t]);
}

// voxel-map capacity (bytes) of a cloud with AABB b plus origin o at resolution res: `rigid`
// allows any rotation (a rigid motion keeps the diameter; the device sizes the box after the
// transform), otherwise the axis extents. Both include the 2 + 2 voxels of padding, one more
// for the floor of each end, the rounding of the corrected origin, and the brick alignment of
// both box ends (ovl_axis: up to 2 x 7 voxels).
uint64_t map_cap(const Box& b0, const double* o, double res, bool rigid) {
  Box b = b0;
  b.add((float)o[0], (float)o[1], (float)o[2]);
  double ext[3], d2 = 0;
  for (int k = 0; k < 3; ++k) {
    ext[k] = std::max(0.0, (double)b.hi[k] - (double)b.lo[k]);
    d2 += ext[k] * ext[k];
  }
  uint64_t vox = 1;
  for (int k = 0; k < 3; ++k) {
    const double e = rigid ? std::sqrt(d2) : ext[k];
    vox *= (uint64_t)std::ceil(e / res) + 8 + 2 * (kOvlBrick0 - 1);
  }
  return (vox + kOvlBrickBytes - 1) / kOvlBrickBytes * kOvlBrickBytes;
}

// A window's voxel maps beyond this many bytes (all of them together) take the sorted-key path
// instead: a far return (a key box of 10^9+ voxels) or a very wide scan. The C2/C3 scenes need
// ~3 MB per reading map and ~80 MB for a reference (sized for any rotation of its source).
constexpr uint64_t kSeqMapBudget = uint64_t(1) << 30;
constexpr uint64_t kMaxRayKeys = 3 * 65536 + 8;  // keys are 16-bit per axis: a ray's walk is bounded

// Upper bound of the keys computeRayKeys(o, p) + p's own key visit, summed over a cloud: one
// step per key crossed on an axis, plus the origin, the endpoint and a margin for the walk's
// float overshoot. rigid: for any rigid motion of both cloud and origin (the corrected reference
// of the next window), from the distance: sum_i |dk_i| <= sqrt(3) |p - o| / res + 3.
// A point without a key (non-finite or beyond the key range) visits nothing.
uint64_t key_bound(WorkerPool& pool, const aicp_cloud& c, const double* org, double res, bool rigid) {
  constexpr uint64_t kChunk = 1 << 15;
  const size_t tasks = (size_t)((c.n + kChunk - 1) / kChunk);
  std::vector<uint64_t> part(tasks, 0);
  const double rf = 1.0 / res;
  const float of[3] = {(float)org[0], (float)org[1], (float)org[2]};
  double ko[3];
  for (int k = 0; k < 3; ++k) ko[k] = std::floor(rf * (double)of[k]);
  pool.run(tasks, [&](size_t t) {
    const char* src = reinterpret_cast<const char*>(c.pts);
    uint64_t sum = 0;
    const uint64_t a = t * kChunk, b = std::min<uint64_t>(c.n, a + kChunk);
    for (uint64_t i = a; i < b; ++i) {
      const float* p = reinterpret_cast<const float*>(src + i * c.stride);
      if (!(std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]))) continue;
      double v;
      if (rigid) {
        double d2 = 0;
        for (int k = 0; k < 3; ++k) d2 += ((double)p[k] - org[k]) * ((double)p[k] - org[k]);
        v = std::ceil(1.7320508075688772 * (std::sqrt(d2) * (1 + 1e-5) + 1e-3) * rf) + 8;
      } else {
        v = 8;
        for (int k = 0; k < 3; ++k) v += std::fabs(std::floor(rf * (double)p[k]) - ko[k]);
      }
      sum += v < (double)kMaxRayKeys ? (uint64_t)v : kMaxRayKeys;
    }
    part[t] = sum;
  });
  uint64_t s = 0;
  for (uint64_t v : part) s += v;
  return s;
}

// the error message of work run on a host thread of its own (copied into ctx->err after the join,
// so two threads never write that string at once)
struct ErrSink {
  std::string err;
};

struct Win {
  size_t p0, np;
  int src;  // -1: the first cloud; else the reading whose corrected cloud is the reference
  int slot;
  int index;  // window number in this pass
};

}  // namespace

// One window's device work in three parts, enqueued in this order across windows:
//   upload(w+1)  H2D + reading side of the next window (independent of the reference)
//   icp(w)       the ICP loop, with early exit: the host polls the active count
//   reference(w+1) next reference (it waits for icp(w)'s corrections) + trees + normals + overlap
// so the reading side of w+1 overlaps window w, and window w's loop stops once its readings have
// all converged instead of running maxIterationCount launches.
struct WinRun {
  Win w;
  size_t np = 0;
  uint64_t nread = 0;
  uint32_t n_ref = 0;
  size_t tl_cap = 0;
  bool use_tl = false;
  BlockMap m_read{}, m_gref{}, m_red{}, m_sel{};
  std::vector<uint64_t> cap;
  uint64_t cap_max = 0;
  const float4* src_pts = nullptr;
  const float4* readS = nullptr;
  TreeCtl* ctl_w = nullptr;
  const PairDesc* src_desc = nullptr;   // the reference source's descriptor and correction
  const float* src_T = nullptr;
  const PairState* src_state = nullptr;  // (a source in the previous window: its state, k_seq_ref_points)
  hipEvent_t src_ev = nullptr;           // the reference waits for it instead of the previous ev_done
  int next_src = -1;  // early_reference: the pair of this window that is the next window's source
  // S->opt.profile: ref start, matcher done, normals done, ICP start, ICP done, commit done, host at the
  // next reference's enqueue (a marker on an idle stream), its upload ready on r3, reading side
  // start and end
  hipEvent_t* tev = nullptr;
  std::vector<uint32_t> n_read;         // the readings' point counts
  bool sparse = false;                  // overlap on sorted key lists (a map over kSeqMapBudget)
  OvlKeySide kr{}, kg{};                // its readings' and reference's sides
  unsigned long long* per_pair = nullptr;
  // debug working mode: the readings one after the other (per-reading loops and overlaps)
  bool debug = false;
  std::vector<uint32_t> loff;               // each reading's first point in the window
  std::vector<uint32_t> b_read, b_sel, b_red;  // each reading's first block in m_read / m_sel / m_red (+ end)
  std::vector<OvlKeySide> kr1;              // sparse: each reading's own key side
};

// Run `enqueue` on stream s through the cache: replay the graph if the key matches, otherwise
// capture it (the enqueue must not allocate or synchronise) and replay; direct launches when
// graphs are off or a capture failed.
static int graph_run(aicp_hip_ctx* ctx, GraphCache& gc, hipStream_t s, const Key& key,
                     const std::function<int()>& enqueue) {
  if (gc.broken) return enqueue();
  if (!gc.exec || gc.key != key.v) {
    gc.reset();
    if (hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) != hipSuccess) {
      (void)hipGetLastError();
      gc.broken = true;
      return enqueue();
    }
    const int rc = enqueue();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s, &g);
    hipGraphExec_t ex = nullptr;
    const bool ok = rc == AICP_OK && e == hipSuccess && g && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
    if (g) (void)hipGraphDestroy(g);
    if (!ok) {
      (void)hipGetLastError();
      gc.broken = true;
      if (rc) return rc;
      return enqueue();
    }
    gc.exec = ex;
    gc.key = key.v;
  }
  HIPC(hipGraphLaunch(gc.exec, s));
  return AICP_OK;
}

// The host parts: pack + upload the readings (and the reference source when it is not
// resident), descriptors, block maps, map capacities; then the reading side (stream rd).
// (C: aicp_hip_ctx, or ErrSink on the upload thread: only ctx->err is used)
template <class C>
static int win_upload(C* ctx, SeqState* S, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                      const aicp_cloud* first, const aicp_cloud* rd, const float4* src_resident,
                      std::vector<Box>& rbox, WinRun& R) {
  const Win& w = R.w;
  SeqSlot& sl = S->slot[w.slot];
  const bool doOvl = prm->flags & AICP_RUN_OVERLAP;
  const bool debug = prm->flags & AICP_SEQ_DEBUG;
  const double res = prm->resolution;
  const size_t np = w.np;
  const aicp_cloud& src = w.src < 0 ? *first : rd[w.src];
  const uint32_t n_ref = (uint32_t)src.n;
  uint64_t nread = 0;
  for (size_t i = 0; i < np; ++i) nread += rd[w.p0 + i].n;
  // slot buffers (sizes grow to the largest window seen)
  const size_t tl_cap = 4 * (size_t)n_ref + 4;
  const bool use_tl = cfg->bucket_size <= 15 && n_ref <= 4000000u && tl_cap < (1ull << 28) && S->opt.nn_engine != 1;
  constexpr uint32_t kRedBlk = kNNBlock * kReducePerThread * kReduceChunks;
  if (sl.used) {
    // the slot's previous window (w - K) must be done before its buffers are rewritten, and so
    // must window w - K + 1, whose reference was built from a reading in this slot: its ICP
    // (the event of the next slot, ordered after its k_transform) covers both
    const SeqSlot& nx = S->slot[(w.slot + 1) % kSlots];
    hipEvent_t e = nx.used ? nx.ev_done : sl.ev_done;
    for (hipStream_t q : {S->s_up, S->s_rd, S->s_r2, S->s_r3, S->s_icp}) HIPC(hipStreamWaitEvent(q, e, 0));
    HIPC(hipEventSynchronize(sl.ev_up));  // pinned staging free again
  }
  sl.used = true;
  HIPC(ensure(sl.read_raw, nread * 16));
  HIPC(ensure(sl.read_s, nread * 16));
  HIPC(ensure(sl.read_c, nread * 16));
  HIPC(ensure(sl.match, nread * 4));
  HIPC(ensure(sl.d2, nread * 4));
  HIPC(ensure(sl.touch, nread * 4));
  HIPC(ensure(sl.cand, nread * 4));
  HIPC(ensure(sl.sel_hist, np * kHistBins * 4));
  HIPC(ensure(sl.sel_cnt, np * 4));
  HIPC(ensure(sl.ctrs, kCtrWords * 4));
  HIPC(ensure(sl.active, active_list_bytes(nread, np)));
  HIPC(ensure(sl.ref_raw, (size_t)n_ref * 16));
  HIPC(ensure(sl.bpts, (size_t)n_ref * 16));
  HIPC(ensure(sl.bnrm, (size_t)n_ref * 16));
  HIPC(ensure(sl.nrm_raw, (size_t)n_ref * 16));
  HIPC(ensure(sl.nbids, (size_t)n_ref * 4 * cfg->knn_normals));
  HIPC(ensure(sl.inv, (size_t)n_ref * 4));
  HIPC(ensure(sl.rd, 3 * sizeof(PairDesc) + 2 * sizeof(PairState)));
  HIPC(ensure(sl.tsrc, 64));
  HIPC(ensure(sl.wdesc, np * sizeof(PairDesc)));
  HIPC(ensure(sl.wstate, np * sizeof(PairState)));
  HIPC(ensure(sl.woutT, np * 64));
  HIPC(ensure(sl.isync, icp_sync_words(np) * 4));
  PairDesc* dRdesc = sl.rd.as<PairDesc>();
  PairDesc* dDesc = sl.wdesc.as<PairDesc>();

  // ---- host: pack the readings (+ AABBs), descriptors, block maps
  HIPC(ensure(sl.pin_read, nread * 16));
  std::vector<PackSeg> segs;
  std::vector<uint32_t> loff(np);
  {
    uint64_t o = 0;
    for (size_t i = 0; i < np; ++i) {
      const aicp_cloud& c = rd[w.p0 + i];
      loff[i] = (uint32_t)o;
      segs.push_back(PackSeg{c.pts, c.n, c.stride, sl.pin_read.as<float>() + 4 * o});
      o += c.n;
    }
  }
  const bool upload_src = src_resident == nullptr;
  if (upload_src) {
    HIPC(ensure(sl.pin_src, (size_t)n_ref * 16));
    segs.push_back(PackSeg{src.pts, src.n, src.stride, sl.pin_src.as<float>()});
  }
  std::vector<Box> boxes;
  pack_clouds(S->pool, segs, boxes);
  for (size_t i = 0; i < np; ++i) rbox[w.p0 + i] = boxes[i];
  // AABB of the reference source: packed now, or by its own window (resident)
  const Box src_box = upload_src ? boxes.back() : rbox[w.src];
  Maps mr, mg, md, ms;
  std::vector<PairDesc> hd(np);
  uint32_t red = 0;
  for (size_t i = 0; i < np; ++i) {
    const aicp_cloud& c = rd[w.p0 + i];
    PairDesc& d = hd[i];
    d = PairDesc{};
    d.ref_off = 0;
    d.n_ref = n_ref;
    d.read_off = loff[i];
    d.n_read = (uint32_t)c.n;
    d.red_blk_off = red;
    d.n_red_blk = (uint32_t)((c.n + kRedBlk - 1) / kRedBlk);
    red += d.n_red_blk;
    ident4(d.Tin);
    d.ratio = cfg->trimmed_ratio;
    d.ref_id = 0;
    d.ogroup = 0;
    for (int k = 0; k < 3; ++k) {
      d.read_origin[k] = c.origin[k];
      d.ref_origin[k] = w.src < 0 ? first->origin[k] : 0.0;  // device-written for corrected references
    }
    mr.add((int)i, d.n_read, kNNBlock);
    md.add((int)i, d.n_read, kRedBlk);
    ms.add((int)i, d.n_read, kNNBlock * kSelPerThread);
  }
  mg.add(0, n_ref, kNNBlock);
  PairDesc r{};
  r.n_ref = n_ref;
  r.ratio = cfg->trimmed_ratio;
  ident4(r.Tin);
  r.tl_off = 0;
  r.tl_cap = (uint32_t)tl_cap;
  PairDesc g = r;
  for (int k = 0; k < 3; ++k) g.ref_origin[k] = w.src < 0 ? first->origin[k] : 0.0;
  // voxel maps: [0] the reference (capacity for any rigid motion of its source), [1 + i] readings
  std::vector<OvlDesc> od(np + 1);
  std::vector<uint64_t> cap(np + 1);
  uint64_t bm = 0, cap_max = 0;
  for (size_t i = 0; i <= np; ++i) {
    cap[i] = i == 0 ? map_cap(src_box, src.origin, res, w.src >= 0)
                    : map_cap(boxes[i - 1], rd[w.p0 + i - 1].origin, res, debug);  // debug: moved by initialT_
    od[i] = OvlDesc{};
    od[i].off = bm;
    bm += cap[i];
    cap_max = std::max(cap_max, cap[i]);
  }
  // a window whose maps do not fit the budget runs its overlap on sorted key lists: sized by host
  // bounds of the rays' keys (readings from their own points; the reference for any rigid
  // motion of its source), so the stream needs no read-back
  const bool sparse = doOvl && (S->opt.overlap_path == 1 || bm > kSeqMapBudget);
  std::vector<OvlCloud> scl;
  std::vector<uint32_t> sbc, sbs;
  uint64_t cap_r = 0, cap_g = 0;
  size_t tmp_r = 0, tmp_g = 0;
  std::vector<uint64_t> kb_read;  // each reading's key bound
  if (sparse) {
    uint64_t slot = 0;
    for (size_t i = 0; i <= np; ++i) {  // readings 0..np-1, then the reference
      const bool ref = i == np;
      const aicp_cloud& c = ref ? src : rd[w.p0 + i];
      OvlCloud o{};
      o.pts_off = ref ? 0u : loff[i];
      o.n = (uint32_t)c.n;
      o.side = ref ? 0u : 1u;
      for (int k = 0; k < 3; ++k) o.origin[k] = ref ? (w.src < 0 ? first->origin[k] : 0.0) : c.origin[k];
      o.slot = ref ? 0 : slot;
      slot += ref ? 0 : c.n;
      scl.push_back(o);
      const uint32_t ci = ref ? 0u : (uint32_t)i;
      for (uint32_t j = 0; j < o.n; j += 256) {
        sbc.push_back(ci);
        sbs.push_back(j);
      }
      const uint64_t kb = key_bound(S->pool, c, c.origin, res, (ref && w.src >= 0) || (!ref && debug));
      if (!ref) kb_read.push_back(kb);
      (ref ? cap_g : cap_r) += kb;
    }
    tmp_r = ovl_keys_temp_bytes(nread, cap_r, (int)np);
    if (debug)  // the readings one at a time: each side's own scan / sort
      for (size_t i = 0; i < np; ++i) tmp_r = std::max(tmp_r, ovl_keys_temp_bytes(rd[w.p0 + i].n, kb_read[i], 1));
    tmp_g = ovl_keys_temp_bytes(n_ref, cap_g, 1);
    size_t free_b = 0, total_b = 0;
    HIPC(hipMemGetInfo(&free_b, &total_b));
    const uint64_t need = 16 * (cap_r + cap_g) + tmp_r + tmp_g;
    if (need > sl.sp_keys_r.cap + sl.sp_keys_g.cap + sl.sp_tmp_r.cap + sl.sp_tmp_g.cap + free_b / 2)
      FAIL(AICP_ERR_UNSUPPORTED, "sparse overlap: " + std::to_string(cap_r + cap_g) + " ray keys do not fit");
    HIPC(ensure(sl.sp_cnt, (nread + n_ref) * 4));
    HIPC(ensure(sl.sp_off, (nread + n_ref) * 8));
    HIPC(ensure(sl.sp_keys_r, cap_r * 16 + 16));
    HIPC(ensure(sl.sp_keys_g, cap_g * 16 + 16));
    HIPC(ensure(sl.sp_tmp_r, tmp_r));
    HIPC(ensure(sl.sp_tmp_g, tmp_g));
    HIPC(ensure(sl.sp_pc, (2 * np + 1) * 8));
  } else if (doOvl) {
    HIPC(ensure(sl.bitmap, bm));
    HIPC(ensure(sl.ovl, (np + 1) * sizeof(OvlDesc)));
    HIPC(ensure(sl.caps, (np + 1) * 8));
  }
  // pinned parameter block: pair descs | rdesc, rdesc_raw, gdesc | ovl descs | caps | block maps
  const size_t nr = mr.pair.size(), nf = mg.pair.size(), nd = md.pair.size(), ns = ms.pair.size();
  const size_t words = 2 * (nr + nf + nd + ns);
  const size_t o_desc = 0, o_r = o_desc + np * sizeof(PairDesc), o_ovl = o_r + 3 * sizeof(PairDesc),
               o_cap = o_ovl + (np + 1) * sizeof(OvlDesc), o_maps = o_cap + (np + 1) * 8,
               o_sp = (o_maps + words * 4 + 15) & ~size_t(15),
               // clouds | block clouds | block starts [debug: | clouds with count slot 0 | zero tags]
               sp_bytes = (scl.size() * sizeof(OvlCloud) + 8 * sbc.size()) * (debug ? 2 : 1),
               total = o_sp + sp_bytes;
  HIPC(ensure(sl.pin_par, total));
  HIPC(ensure(sl.maps, words * 4));
  char* P = sl.pin_par.as<char>();
  std::memcpy(P + o_desc, hd.data(), np * sizeof(PairDesc));
  std::memcpy(P + o_r, &r, sizeof(PairDesc));
  std::memcpy(P + o_r + sizeof(PairDesc), &r, sizeof(PairDesc));
  std::memcpy(P + o_r + 2 * sizeof(PairDesc), &g, sizeof(PairDesc));
  std::memcpy(P + o_ovl, od.data(), (np + 1) * sizeof(OvlDesc));
  std::memcpy(P + o_cap, cap.data(), (np + 1) * 8);
  BlockMap m_read{}, m_gref{}, m_red{}, m_sel{};
  {
    uint32_t* mp = reinterpret_cast<uint32_t*>(P + o_maps);
    size_t o = 0;
    auto put = [&](const Maps& m, BlockMap& b) {
      const size_t cnt = m.pair.size();
      std::memcpy(mp + o, m.pair.data(), cnt * 4);
      std::memcpy(mp + o + cnt, m.start.data(), cnt * 4);
      b.pair = sl.maps.as<int32_t>() + o;
      b.start = sl.maps.as<uint32_t>() + o + cnt;
      b.n_blocks = (uint32_t)cnt;
      o += 2 * cnt;
    };
    put(mr, m_read);
    put(mg, m_gref);
    put(md, m_red);
    put(ms, m_sel);
  }
  HIPC(ensure(sl.slab, (size_t)red * kRedCols * 8));
  if (sparse) {  // clouds (readings, reference) | block clouds | block starts
    const size_t nb = sbc.size(), ncl = scl.size();
    std::memcpy(P + o_sp, scl.data(), ncl * sizeof(OvlCloud));
    std::memcpy(P + o_sp + ncl * sizeof(OvlCloud), sbc.data(), nb * 4);
    std::memcpy(P + o_sp + ncl * sizeof(OvlCloud) + nb * 4, sbs.data(), nb * 4);
    if (debug) {  // each reading alone: its counts start at its own first point, its words tagged 0
      OvlCloud* c1 = reinterpret_cast<OvlCloud*>(P + o_sp + ncl * sizeof(OvlCloud) + 8 * nb);
      std::memcpy(c1, scl.data(), ncl * sizeof(OvlCloud));
      for (size_t c = 0; c < ncl; ++c) c1[c].slot = 0;
      std::memset(P + o_sp + 2 * ncl * sizeof(OvlCloud) + 8 * nb, 0, 4 * nb);
    }
    HIPC(ensure(sl.sp_par, sp_bytes));
    char* D = sl.sp_par.as<char>();
    OvlCloud* dcl = reinterpret_cast<OvlCloud*>(D);
    const uint32_t* dbc = reinterpret_cast<const uint32_t*>(D + ncl * sizeof(OvlCloud));
    const uint32_t* dbs = dbc + nb;
    const uint32_t nbr = (uint32_t)(nb - (n_ref + 255) / 256);  // the readings' blocks come first
    unsigned long long* pc = sl.sp_pc.as<unsigned long long>();
    R.kr = OvlKeySide{dcl, (int)np, dbc, dbs, nbr, (uint32_t)nread, sl.sp_cnt.as<uint32_t>(),
                      sl.sp_off.as<uint64_t>(), cap_r, sl.sp_keys_r.as<uint64_t>(),
                      sl.sp_keys_r.as<uint64_t>() + cap_r, sl.sp_tmp_r.p, tmp_r, pc};
    R.kg = OvlKeySide{dcl + np, 1, dbc + nbr, dbs + nbr, (uint32_t)(nb - nbr), n_ref,
                      sl.sp_cnt.as<uint32_t>() + nread, sl.sp_off.as<uint64_t>() + nread, cap_g,
                      sl.sp_keys_g.as<uint64_t>(), sl.sp_keys_g.as<uint64_t>() + cap_g, sl.sp_tmp_g.p, tmp_g, pc + np};
    R.per_pair = pc + np + 1;
    if (debug) {  // reading i alone: cloud i (its key words tagged 0), keys at its own offset
      R.kr1.assign(np, OvlKeySide{});
      OvlCloud* c1 = reinterpret_cast<OvlCloud*>(D + ncl * sizeof(OvlCloud) + 8 * nb);
      const uint32_t* bc0 = reinterpret_cast<const uint32_t*>(D + 2 * ncl * sizeof(OvlCloud) + 8 * nb);
      uint32_t b0 = 0;
      uint64_t k0 = 0;
      for (size_t i = 0; i < np; ++i) {
        const uint32_t nbi = (uint32_t)((rd[w.p0 + i].n + 255) / 256);
        OvlKeySide& k = R.kr1[i];
        k = R.kr;
        k.clouds = c1 + i;
        k.n_clouds = 1;
        k.blk_cloud = bc0 + b0;
        k.blk_start = dbs + b0;
        k.n_blocks = nbi;
        k.n_points = (uint32_t)rd[w.p0 + i].n;
        k.cnt = R.kr.cnt + loff[i];
        k.off = R.kr.off + loff[i];
        k.cap = kb_read[i];
        k.keys0 = R.kr.keys0 + 2 * k0;  // (the readings' key area holds 2 * cap_r words: per reading keys0 | keys1)
        k.keys1 = R.kr.keys0 + 2 * k0 + kb_read[i];
        k.per_cloud = pc + i;
        b0 += nbi;
        k0 += kb_read[i];
      }
    }
  }

  // ---- up: readings, descriptors, maps (and a non-resident reference source)
  hipStream_t su = S->s_up;
  HIPC(hipMemcpyAsync(sl.read_raw.p, sl.pin_read.p, nread * 16, hipMemcpyHostToDevice, su));
  HIPC(hipMemcpyAsync(dDesc, P + o_desc, np * sizeof(PairDesc), hipMemcpyHostToDevice, su));
  HIPC(hipMemcpyAsync(dRdesc, P + o_r, 3 * sizeof(PairDesc), hipMemcpyHostToDevice, su));
  if (doOvl) {
    HIPC(hipMemcpyAsync(sl.ovl.p, P + o_ovl, (np + 1) * sizeof(OvlDesc), hipMemcpyHostToDevice, su));
    HIPC(hipMemcpyAsync(sl.caps.p, P + o_cap, (np + 1) * 8, hipMemcpyHostToDevice, su));
  }
  HIPC(hipMemcpyAsync(sl.maps.p, P + o_maps, words * 4, hipMemcpyHostToDevice, su));
  if (sparse) HIPC(hipMemcpyAsync(sl.sp_par.p, P + o_sp, sp_bytes, hipMemcpyHostToDevice, su));
  const float4* src_pts = src_resident;
  if (upload_src) {
    HIPC(ensure(sl.ref_src, (size_t)n_ref * 16));
    HIPC(hipMemcpyAsync(sl.ref_src.p, sl.pin_src.p, (size_t)n_ref * 16, hipMemcpyHostToDevice, su));
    src_pts = sl.ref_src.as<float4>();
  }
  HIPC(hipEventRecord(sl.ev_up, su));

  R.np = np;
  R.nread = nread;
  R.n_read.resize(np);
  for (size_t i = 0; i < np; ++i) R.n_read[i] = (uint32_t)rd[w.p0 + i].n;
  R.n_ref = n_ref;
  R.tl_cap = tl_cap;
  R.use_tl = use_tl;
  R.m_read = m_read;
  R.m_gref = m_gref;
  R.m_red = m_red;
  R.m_sel = m_sel;
  R.cap = cap;
  R.cap_max = cap_max;
  R.src_pts = src_pts;
  R.readS = sl.read_raw.as<float4>();
  R.sparse = sparse;
  R.debug = debug;
  R.loff = loff;
  {  // each reading's first block in the three block maps (pair-major), and the end
    R.b_read.assign(np + 1, 0);
    R.b_sel.assign(np + 1, 0);
    R.b_red.assign(np + 1, 0);
    for (size_t i = 0; i < np; ++i) {
      const uint64_t n = rd[w.p0 + i].n;
      R.b_read[i + 1] = R.b_read[i] + (uint32_t)((n + kNNBlock - 1) / kNNBlock);
      R.b_sel[i + 1] = R.b_sel[i] + (uint32_t)((n + kNNBlock * kSelPerThread - 1) / (kNNBlock * kSelPerThread));
      R.b_red[i + 1] = R.b_red[i] + (uint32_t)((n + kRedBlk - 1) / kRedBlk);
    }
  }
  return AICP_OK;
}


#define WIN_REFS                                                   \
  const Win& w = R.w;                                              \
  SeqSlot& sl = S->slot[w.slot];                                   \
  const bool doOvl = prm->flags & AICP_RUN_OVERLAP;                \
  const double res = prm->resolution;                              \
  const size_t np = R.np;                                          \
  const uint32_t n_ref = R.n_ref;                                  \
  PairDesc* dRdesc = sl.rd.as<PairDesc>();                         \
  PairDesc* dRraw = dRdesc + 1;                                    \
  PairDesc* dG = dRdesc + 2;                                       \
  PairState* dRst = reinterpret_cast<PairState*>(dRdesc + 3);      \
  PairState* dGst = dRst + 1;                                      \
  PairDesc* dDesc = sl.wdesc.as<PairDesc>();                       \
  PairState* dState = sl.wstate.as<PairState>();                   \
  float* dOutT = sl.woutT.as<float>();                             \
  OvlDesc* dOvl = doOvl ? sl.ovl.as<OvlDesc>() : nullptr;          \
  const uint64_t* dCap = doOvl ? sl.caps.as<uint64_t>() : nullptr; \
  uint8_t* bmp = doOvl ? sl.bitmap.as<uint8_t>() : nullptr;        \
  (void)dRraw;                                                     \
  (void)dG;                                                        \
  (void)dOvl;                                                      \
  (void)n_ref;                                                     \
  (void)dRst;                                                      \
  (void)dGst;                                                      \
  (void)dOutT;                                                     \
  (void)np;                                                        \
  (void)dDesc;                                                     \
  (void)dState;                                                    \
  (void)dCap;                                                      \
  (void)bmp;                                                       \
  (void)res

// The reading side of the window on stream rd (independent of the reference): state init, Morton
// order, the readings' voxel maps. Enqueued after the window's reference, so that it fills the
// CUs the kd-tree builds leave idle instead of competing with the previous window's ICP loop.
template <class C>
static int win_read_side(C* ctx, SeqState* S, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                         WinRun& R) {
  WIN_REFS;
  (void)ctx;
  (void)cfg;
  const uint64_t nread = R.nread;
  const BlockMap m_read = R.m_read;
  const uint64_t cap_max = R.cap_max;
  hipStream_t sr = S->s_rd;
  HIPC(hipStreamWaitEvent(sr, sl.ev_up, 0));
  if (R.tev) HIPC(hipEventRecord(R.tev[8], sr));
  launch_init_state(sr, (int)np, dDesc, dState);
  const float4* readS = sl.read_raw.as<float4>();
  if (R.debug) {  // the points move with initialT_ right before each reading's loop (in place)
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(sl.ev_rd, sr));
    R.readS = readS;
    return AICP_OK;
  }
  {
    const size_t tb = read_order_temp_bytes(nread, (int)np);
    HIPC(ensure(sl.ord_k0, nread * 8));
    HIPC(ensure(sl.ord_k1, nread * 8));
    HIPC(ensure(sl.ord_v0, nread * 4));
    HIPC(ensure(sl.ord_v1, nread * 4));
    HIPC(ensure(sl.ord_tmp, tb));
    HIPC(launch_read_order(sr, m_read, (int)np, dDesc, sl.read_raw.as<float4>(), (uint32_t)nread,
                           sl.ord_k0.as<uint64_t>(), sl.ord_k1.as<uint64_t>(), sl.ord_v0.as<uint32_t>(),
                           sl.ord_v1.as<uint32_t>(), sl.ord_tmp.p, tb, sl.read_s.as<float4>()));
    readS = sl.read_s.as<float4>();
  }
  if (doOvl && R.sparse) {
    launch_ovl_init(sr, (int)np, dDesc, dState, res, 2);
    HIPC(launch_ovl_keys(sr, R.kr, nullptr, readS, res, dState, 1));
  } else if (doOvl) {
    launch_ovl_init(sr, (int)np, dDesc, dState, res, 2);
    launch_ovl_bbox(sr, m_read, dDesc, dState, readS, 1, res);
    launch_ovl_size(sr, (int)np, dState, dOvl + 1, dCap + 1);
    launch_ovl_clear(sr, (int)np, dOvl + 1, bmp, cap_max);
    launch_ovl_mark(sr, m_read, dDesc, dOvl + 1, dState, readS, 1, res, bmp, false);
    launch_ovl_popcount(sr, (int)np, dOvl + 1, dState, 1, bmp);
  }
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(sl.ev_rd, sr));
  if (R.tev) HIPC(hipEventRecord(R.tev[9], sr));
  R.readS = readS;
  return AICP_OK;
}

// The reference of the window on streams r3 and r2: its points (the previous window's last
// reading corrected on the device, once that window's ticket is out), centroid, matcher kd-tree
// and treelets (r3), raw kd-tree + SurfaceNormal scattered into the matcher's order (r2). The two
// builds are replayed from graphs (graph_run). Nothing here runs on stream icp, so it can be
// enqueued before the previous window's ICP loop.
static int win_ref_trees(aicp_hip_ctx* ctx, SeqState* S, const aicp_icp_config* cfg,
                         const aicp_sequence_params* prm, WinRun& R) {
  WIN_REFS;
  const float4* src_pts = R.src_pts;
  const bool use_tl = R.use_tl;
  const size_t tl_cap = R.tl_cap;
  TreeCtl* ctl_w = R.ctl_w;
  // ---- r3: the reference points
  hipStream_t s3 = S->s_r3;
  if (R.tev) HIPC(hipEventRecord(R.tev[6], S->s_probe));
  HIPC(hipStreamWaitEvent(s3, sl.ev_up, 0));
  if (R.tev) HIPC(hipEventRecord(R.tev[7], s3));
  if (w.src >= 0) {
    // the source's correction must be final: from the previous window of this pass (its loop's
    // end, ev_done), or from an earlier pass (synchronised)
    const SeqSlot& ps = S->slot[(w.slot + kSlots - 1) % kSlots];
    // (early_reference: the previous window's loop is still running, its source pair stopped)
    if (w.index > 0) HIPC(hipStreamWaitEvent(s3, R.src_ev ? R.src_ev : ps.ev_done, 0));
    if (R.tev) HIPC(hipEventRecord(R.tev[0], s3));
    // debug mode, a source from an earlier pass (uploaded as given): it was registered as
    // initialT_ * its points (initialT_ as before it, kept by k_debug_prep)
    if (R.debug && w.index == 0)
      launch_transform(s3, (int)n_ref, S->initT.as<float>() + 16 * (1 + (size_t)w.src), src_pts,
                       const_cast<float4*>(src_pts));
    launch_seq_ref_points(s3, (int)n_ref, dG, R.src_desc, R.src_state, R.src_T, sl.tsrc.as<float>(), src_pts,
                          sl.ref_raw.as<float4>());
  } else {
    if (R.tev) HIPC(hipEventRecord(R.tev[0], s3));
    HIPC(hipMemcpyAsync(sl.ref_raw.p, src_pts, (size_t)n_ref * 16, hipMemcpyDeviceToDevice, s3));
  }
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(sl.ev_ref, s3));
  // work spaces first: nothing may be allocated inside a capture
  const int bucket = cfg->bucket_size;
  int rc = device_trees_begin(sl.tb[0], ctx->err, S->s_r2, 1, n_ref, dRraw, sl.ref_raw.as<float4>(), 0,
                              kNormalsBucket, sl.bpts_raw, sl.nodes_raw, false);
  if (rc) return rc;
  rc = device_trees_begin(sl.tb[1], ctx->err, s3, 1, n_ref, dRdesc, sl.ref_raw.as<float4>(), 1, bucket, sl.bpts,
                          sl.nodes, false);
  if (rc) return rc;
  const uint32_t ncap = 2 * n_ref + 2;
  if (use_tl) {
    HIPC(ensure(sl.tl, tl_cap * 16));
    HIPC(ensure(sl.ptl, tl_cap * 8));
    HIPC(ensure(sl.tl_rank, ((size_t)ncap + 1) * 4));
  }
  const int plan0 = plan_levels(n_ref, sl.tb[0], S->opt.tree_plan), plan1 = plan_levels(n_ref, sl.tb[1], S->opt.tree_plan);
  const bool capturable = plan0 > 0 && plan1 > 0;  // (a host-polled build cannot be captured)
  // ---- r2: raw-coordinate tree + SurfaceNormal (reference as given)
  hipStream_t s2 = S->s_r2;
  uint32_t* nCtr = sl.ctrs.as<uint32_t>() + kKnnCtrOff;
  // the raw build's kernels that do not read the reference points (state, zeroed work space,
  // frames: no centring here) run while s2 waits for them; they need only the window's
  // descriptors (ev_up)
  auto raw_begin = [&]() -> int {
    HIPC(hipStreamWaitEvent(s2, sl.ev_up, 0));
    launch_init_state(s2, 1, dRraw, dRst);
    int r = device_trees_begin(sl.tb[0], ctx->err, s2, 1, n_ref, dRraw, sl.ref_raw.as<float4>(), 0, kNormalsBucket,
                               sl.bpts_raw, sl.nodes_raw, true, 1);
    if (r) return r;
    HIPC(hipStreamWaitEvent(s2, sl.ev_ref, 0));
    return device_trees_begin(sl.tb[0], ctx->err, s2, 1, n_ref, dRraw, sl.ref_raw.as<float4>(), 0, kNormalsBucket,
                              sl.bpts_raw, sl.nodes_raw, true, 2);
  };
  auto raw_build = [&]() -> int {
    int r = device_trees_end(sl.tb[0], ctx->err, s2, 1, n_ref, dRraw, kNormalsBucket, sl.bpts_raw, sl.nodes_raw, plan0,
                         ctl_w, !capturable);
    if (r) return r;
    if (!launch_normals(s2, 1, n_ref, dRraw, dRst, sl.nodes_raw.as<uint4>(), nullptr, sl.bpts_raw.as<float4>(),
                        sl.nrm_raw.as<float4>(), cfg->knn_normals, sl.nbids.as<int32_t>(), nCtr,
                        S->opt.normals_knn_engine))
      FAIL(AICP_ERR_UNSUPPORTED, "normals knn");
    HIPC(hipGetLastError());
    return AICP_OK;
  };
  // the raw tree + SurfaceNormal as direct launches (replayed from a graph they finished 0.08 ms
  // later on the device, r03)
  auto raw_enqueue = [&]() -> int { return raw_build(); };
  // ---- r3: centroid + matcher tree + treelets
  auto match_build = [&]() -> int {
    int r = device_trees_begin(sl.tb[1], ctx->err, s3, 1, n_ref, dRdesc, sl.ref_raw.as<float4>(), 1, bucket, sl.bpts,
                               sl.nodes);
    if (r) return r;
    r = device_trees_end(sl.tb[1], ctx->err, s3, 1, n_ref, dRdesc, bucket, sl.bpts, sl.nodes, plan1, ctl_w + 1,
                         !capturable);
    if (r) return r;
    if (use_tl)
      HIPC(launch_treelets(s3, 1, ncap, dRdesc, sl.nodes.as<uint4>(), bucket, sl.tl_rank.as<uint32_t>(),
                           sl.tl.as<uint4>(), sl.ptl.as<uint2>(), sl.tb[1].tw));
    HIPC(hipGetLastError());
    return AICP_OK;
  };
  auto match_enqueue = [&]() -> int {
    int r;
    if (capturable) {
      Key k;
      k << n_ref << plan1 << bucket << use_tl << tl_cap << dRdesc << sl.ref_raw.p << sl.bpts.p << sl.nodes.p
        << sl.tb[1].tw;
      if (use_tl) k << sl.tl.p << sl.ptl.p << sl.tl_rank.p;
      r = graph_run(ctx, sl.g_match, s3, k, match_build);
    } else {
      r = match_build();
    }
    if (r) return r;
    HIPC(hipEventRecord(sl.ev_s3, s3));
    if (R.tev) HIPC(hipEventRecord(R.tev[1], s3));
    // the build's control block for the host's check after the run, behind the event the loop
    // waits for (in front of it, the D2H copy held the loop start ~15 us per window, r04 trace)
    if (capturable || use_tl)
      HIPC(hipMemcpyAsync(ctl_w + 1, sl.tb[1].tw.ctl, sizeof(TreeCtl), hipMemcpyDeviceToHost, s3));
    return AICP_OK;
  };
  // The raw tree's first kernels (state, zero, frames, centre, roots) go first, then the matcher
  // tree's graph, then the raw tree's levels and SurfaceNormal: the raw tree -> kNN -> normals
  // chain gates the loop's first reduce, the matcher tree (~0.3 ms shorter) only its first NN.
  // Enqueued after the graph, the raw chain's first kernels waited on the host (C2 trace, r06).
  // (The whole raw chain ahead of the graph delayed the matcher tree past the normals: C2 2529-2666
  // against 2784-2816 clouds/s, r06.)
  rc = raw_begin();
  if (!rc) rc = match_enqueue();
  if (!rc) rc = raw_enqueue();
  if (rc) return rc;

  HIPC(hipStreamWaitEvent(s2, sl.ev_s3, 0));
  launch_normals_to_matcher(s2, 1, n_ref, dRdesc, sl.bpts.as<float4>(), sl.bpts_raw.as<float4>(),
                            sl.nrm_raw.as<float4>(), sl.inv.as<uint32_t>(), sl.bnrm.as<float4>());
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(sl.ev_s2, s2));
  if (R.tev) HIPC(hipEventRecord(R.tev[2], s2));
  if (capturable) HIPC(hipMemcpyAsync(ctl_w, sl.tb[0].tw.ctl, sizeof(TreeCtl), hipMemcpyDeviceToHost, s2));
  return AICP_OK;
}

// The window's set-up on stream icp: the reference voxel map (from the next reference's points,
// ev_ref), the overlap counts and ratio (with the reading side, ev_rd), the pairs' frames (matcher
// tree, ev_s3), the normals (ev_s2) and the centred readings. Enqueued after the previous window's
// ICP loop, which runs on the same stream.
static int win_ref_icp(aicp_hip_ctx* ctx, SeqState* S, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                       WinRun& R) {
  WIN_REFS;
  (void)ctx;
  (void)cfg;
  const float4* readS = R.readS;
  hipStream_t si = S->s_icp;
  // the reference's voxel map (or key list)
  if (doOvl && R.sparse) {
    HIPC(hipStreamWaitEvent(si, sl.ev_ref, 0));
    launch_ovl_init(si, 1, dG, dGst, res, 1);
    HIPC(launch_ovl_keys(si, R.kg, w.src >= 0 ? dG->ref_origin : nullptr, sl.ref_raw.as<float4>(), res, dGst, 0));
  } else if (doOvl) {
    HIPC(hipStreamWaitEvent(si, sl.ev_ref, 0));
    launch_ovl_init(si, 1, dG, dGst, res, 1);
    launch_ovl_bbox(si, R.m_gref, dG, dGst, sl.ref_raw.as<float4>(), 0, res);
    launch_ovl_size(si, 1, dGst, dOvl, dCap);
    launch_ovl_clear(si, 1, dOvl, bmp, R.cap[0]);
    launch_ovl_mark(si, R.m_gref, dG, dOvl, dGst, sl.ref_raw.as<float4>(), 0, res, bmp, false);
    launch_ovl_popcount(si, 1, dOvl, dGst, 0, bmp);
  }
  HIPC(hipStreamWaitEvent(si, sl.ev_rd, 0));  // (the slot's previous window is done: its upload waited)
  // the loop's selection histogram, counts and hand-off words: before the wait on the trees
  launch_zero_words3(si, sl.sel_hist.as<uint32_t>(), np * kHistBins, sl.sel_cnt.as<uint32_t>(), np,
                     sl.isync.as<uint32_t>(), icp_sync_words(np));
  if (doOvl && !R.debug) {
    if (R.sparse)
      HIPC(launch_ovl_keys_intersect(si, R.kr, R.kg, R.per_pair, dState));
    else
      launch_ovl_intersect(si, (int)np, dDesc, dOvl + 1, dOvl, dState, bmp);
    launch_ovl_finish(si, (int)np, dDesc, dState, dGst, 1);
  }
  HIPC(hipStreamWaitEvent(si, sl.ev_s3, 0));
  launch_pairs_from_refs(si, (int)np, dDesc, dRdesc);
  launch_pairs_degenerate_part(si, (int)np, dDesc, dState, dRst, 2);
  // the normals (ev_s2) are waited for by the first iteration's reduce (loop_part): the
  // first NN and select need only the matcher tree, which is ready ~0.2 ms earlier on C2
  if (!R.debug) launch_prepare_read(si, R.m_read, dDesc, readS, sl.read_c.as<float4>());
  HIPC(hipGetLastError());
  return AICP_OK;
}

// The ICP loop of a window, polled: from iteration smoothLength on (no pair can stop earlier
// except on an error) the update kernel of the last pair to finish an iteration writes the next
// active count into mapped host memory (a system-scope store), and the host reads the word
// itself. An iteration is enqueued in two parts: its NN launch as soon as the previous iteration
// is enqueued (so the device never waits for the host), the rest (select, reduce, update) once
// the iteration's active count is known to be non-zero; when it reads 0 only the NN launch, a
// no-op, was enqueued for nothing. (r05 enqueued whole iterations one ahead: the trailing no-op
// iteration was four launches. r03 recorded an event per poll and queried it: each marker left a
// 5-10 us gap before the next NN launch, C2 2512 against 2620 clouds/s in r04.) The window's
// states and corrections are then committed to the sequence's arrays (ev_done), which the next
// reference waits for.
// (r03, measured and removed: the window's last reading -- the next reference's source -- in a
// loop of its own with the others on a second stream: the one-reading loop took 0.99 against
// 1.06 ms, but the others' NN launches beside the next reference's kd-trees slowed those from 0.88
// to 1.63 ms; the next reference started on the stop poll instead of the loop's end: 1 % slower.)
struct IcpLoop {
  WinRun* R = nullptr;
  int sub = -1;   // debug mode: the one reading of the window this loop registers
  int area = 0;   // poll words / events used: [area * kMaxPolls, + kMaxPolls)
  int it = 0;      // iterations enqueued whole
  int nn = 0;      // iterations whose NN launch is enqueued (it or it + 1)
  bool stop = false;
  int wait_it = -1;  // the poll word being waited for since wait_t0 (the drained-stream check)
  std::chrono::steady_clock::time_point wait_t0;
  bool src_done = false;  // the next window's source pair has stopped: ev_src recorded
};

// the blocks [off, off + cnt) of a block map
static BlockMap map_sub(const BlockMap& m, uint32_t off, uint32_t cnt) {
  BlockMap r = m;
  r.pair += off;
  r.start += off;
  r.n_blocks = cnt;
  return r;
}

static IcpParams icp_params(const aicp_icp_config* cfg) {
  IcpParams ip;
  std::memset(&ip, 0, sizeof(ip));
  ip.maxE2 = (1 + cfg->nn_epsilon) * (1 + cfg->nn_epsilon);
  ip.maxR2 = cfg->nn_max_dist * cfg->nn_max_dist;
  ip.max_iter = cfg->max_iter;
  ip.smooth = cfg->smooth_length;
  ip.min_rot = cfg->min_diff_rot;
  ip.min_trans = cfg->min_diff_trans;
  ip.knn_normals = cfg->knn_normals;
  return ip;
}

// whether the host waits for poll word k, the active count at the start of iteration k, before
// it enqueues the rest of that iteration (from smoothLength on: no pair can stop earlier except on
// an error)
static bool loop_polled(const SeqState* S, const aicp_icp_config* cfg, int k) {
  return !S->opt.no_early_exit && k >= cfg->smooth_length && k < kMaxPolls && k < cfg->max_iter;
}
// whether poll word k is written at all: every iteration's, so that the words written so far are a
// prefix and the last of them tells whether more will come (loop_poll)
static bool loop_written(const SeqState* S, int k) { return !S->opt.no_early_exit && k < kMaxPolls; }

// The pairs one loop iterates: the window's, or (debug mode) reading q.sub alone.
struct LoopPairs {
  int np_l;
  PairDesc* gd;
  PairState* gs;
  uint64_t reads;
};

// one part of iteration q.it: part 0 its NN launch (with the first active list at iteration 0),
// part 1 the rest (select, reduce, update)
static int loop_part(aicp_hip_ctx* ctx, SeqState* S, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                     IcpLoop& q, int part, bool timeNN, int& nn_launches) {
  WinRun& R = *q.R;
  WIN_REFS;
  const int it = q.it;
  ActiveList* al = sl.active.as<ActiveList>();
  uint32_t* ctr = sl.ctrs.as<uint32_t>();
  const int r = q.sub;
  const LoopPairs lp{r >= 0 ? 1 : (int)np, r >= 0 ? dDesc + r : dDesc, r >= 0 ? dState + r : dState,
                     r >= 0 ? R.n_read[r] : R.nread};
  uint32_t* poll_host = sl.poll_host + q.area * kMaxPolls;
  uint32_t* poll_dev = sl.poll_dev + q.area * kMaxPolls;
  IcpParams ip = icp_params(cfg);
  ip.prof_slot = nn_launches;
  hipStream_t st = S->s_icp;
  // poll word k holds the active count at the start of iteration k, written by the launch that
  // builds that iteration's active list (k_active_list at it = 0, else the previous update); it
  // is marked unwritten before that launch is enqueued
  if (part == 0) {
    uint32_t* hn_this = nullptr;
    if (it == 0 && loop_written(S, it)) {
      poll_host[it] = 0xffffffffu;
      hn_this = poll_dev + it;
    }
    if (timeNN)
      while ((int)S->nn_ev.size() < 2 * (nn_launches + 1)) {
        hipEvent_t e;
        // timing only (the NN launch's own start / end): no system-scope fence, whose cache
        // write-back and invalidation the elapsed time would otherwise include
        HIPC(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        S->nn_ev.push_back(e);
      }
    if (it == 0) launch_active_list(st, lp.np_l, lp.gd, lp.gs, al, ctr, hn_this, nullptr, nullptr, nullptr, R.next_src);
    launch_icp_nn(st, (int)lp.reads, lp.gd, lp.gs, al, sl.read_c.as<float4>(), sl.nodes.as<uint4>(),
                  R.use_tl ? sl.tl.as<uint4>() : nullptr, nullptr, sl.bpts.as<float4>(),
                  R.use_tl ? sl.ptl.as<uint2>() : nullptr, sl.match.as<int32_t>(), sl.d2.as<float>(),
                  sl.touch.as<uint32_t>(), ctr, ip, timeNN ? S->nn_ev[2 * nn_launches] : nullptr,
                  timeNN ? S->nn_ev[2 * nn_launches + 1] : nullptr);
    HIPC(hipGetLastError());
    ++nn_launches;
    q.nn = it + 1;
    return AICP_OK;
  }
  const BlockMap msel = r >= 0 ? map_sub(R.m_sel, R.b_sel[r], R.b_sel[r + 1] - R.b_sel[r]) : R.m_sel;
  const BlockMap mred = r >= 0 ? map_sub(R.m_red, R.b_red[r], R.b_red[r + 1] - R.b_red[r]) : R.m_red;
  uint32_t* hn_next = nullptr;
  if (loop_written(S, it + 1)) {
    poll_host[it + 1] = 0xffffffffu;
    hn_next = poll_dev + it + 1;
  }
  IcpIterSync y = icp_sync_layout(sl.isync.as<uint32_t>(), np, 0);
  y.np = lp.np_l;
  y.pd = lp.gd;
  y.st = lp.gs;
  y.al = al;
  y.ctr = ctr;
  y.host_n = hn_next;
  y.src_pair = R.next_src;
  const int ff = S->opt.select_fused_from;
  if (ff > 0 && it >= ff)  // (iteration 0 has no previous bin to guess)
    launch_icp_select_fused(st, msel, dDesc, dState, sl.d2.as<float>(), sl.sel_hist.as<uint32_t>(),
                            sl.cand.as<uint32_t>(), sl.sel_cnt.as<uint32_t>(), y);
  else
    launch_icp_select_f(st, msel, dDesc, dState, sl.d2.as<float>(), sl.sel_hist.as<uint32_t>(), sl.cand.as<uint32_t>(),
                        sl.sel_cnt.as<uint32_t>(), y);
  if (it == 0) {  // the reduce gathers the reference normals (stream r2, scattered into matcher order)
    HIPC(hipStreamWaitEvent(st, sl.ev_s2, 0));
    launch_pairs_degenerate_part(st, lp.np_l, lp.gd, lp.gs, dRst, 1);
  }
  launch_icp_reduce_f(st, mred, dDesc, dState, sl.read_c.as<float4>(), sl.match.as<int32_t>(), sl.d2.as<float>(),
                      sl.touch.as<uint32_t>(), sl.bpts.as<float4>(), sl.bnrm.as<float4>(), sl.slab.as<double>(), ip, y);
  HIPC(hipGetLastError());
  ++q.it;
  if (q.it >= cfg->max_iter) q.stop = true;
  return AICP_OK;
}

// the window's corrections, its commit to the sequence's arrays and ev_done
static int loop_finish(aicp_hip_ctx* ctx, SeqState* S, const aicp_sequence_params* prm, IcpLoop& q) {
  WinRun& R = *q.R;
  WIN_REFS;
  hipStream_t st = S->s_icp;
  if (!R.debug) launch_finalize(st, (int)np, dDesc, dState, dOutT);  // (debug: k_debug_post per reading)
  if (R.tev) HIPC(hipEventRecord(R.tev[4], st));
  launch_seq_commit(st, (int)np, dDesc, dState, dOutT, S->desc.as<PairDesc>() + w.p0, S->state.as<PairState>() + w.p0,
                    S->outT.as<float>() + 16 * w.p0);
  HIPC(hipGetLastError());
  if (R.tev) HIPC(hipEventRecord(R.tev[5], st));
  HIPC(hipEventRecord(sl.ev_done, st));
  return AICP_OK;
}

// poll word q.it of the loop (got: known; q.stop set when it reads 0)
static int loop_poll(aicp_hip_ctx* ctx, SeqState* S, IcpLoop& q, bool& got) {
  got = false;
  SeqSlot& sl = S->slot[q.R->w.slot];
  volatile uint32_t* w = sl.poll_host + q.area * kMaxPolls;
  if (w[q.it] == 0xffffffffu) {
    // Not written yet. Every iteration's word is written by the launch that builds its active
    // list (loop_written; reset before that launch is enqueued), so the words written so far are a
    // prefix: when the last of them is 0, no launch after it had an active pair and this one stays
    // unwritten -- the loop is over. (r06: the drained-stream test by hipStreamQuery that this
    // replaces enqueued a marker behind the NN launch, and the next iteration's select waited
    // ~7.5 us behind it, C2 kernel trace.)
    int m = q.it - 1;
    while (m >= 0 && w[m] == 0xffffffffu) --m;
    if (m >= 0 && w[m] == 0u) {
      got = true;
      q.stop = true;
      return AICP_OK;
    }
    // a stream that drained without writing it (not expected: a kernel that returned early on an
    // error): checked only after a long wait
    const auto now = std::chrono::steady_clock::now();
    if (q.wait_it != q.it) {
      q.wait_it = q.it;
      q.wait_t0 = now;
      return AICP_OK;
    }
    if (now - q.wait_t0 < std::chrono::milliseconds(20)) return AICP_OK;
    const hipError_t r = hipStreamQuery(S->s_icp);
    if (r == hipErrorNotReady) return AICP_OK;
    HIPC(r);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (w[q.it] == 0xffffffffu) {
      got = true;
      q.stop = true;
      return AICP_OK;
    }
  }
  got = true;
  const uint32_t v = w[q.it];
  if (v == 0) {
    q.stop = true;
  } else if (q.R->next_src >= 0 && !q.src_done && !(v >> 31)) {
    // the next window's source pair has stopped: its final state was written by the update
    // before this iteration's NN launch, the last launch on the stream so far (bit 31 of the
    // word, active_list_body)
    HIPC(hipEventRecord(sl.ev_src, S->s_icp));
    q.src_done = true;
  }
  return AICP_OK;
}

// Debug working mode, before reading q.sub's loop (app.cpp:87-96): initialT_ into its history
// slot, the prior origin moved by it, its points moved in place (pcl::transformPointCloud), then
// its overlap with the window's reference (the key box / bound allows any rigid motion) and
// its centred copy
static int sub_prep(aicp_hip_ctx* ctx, SeqState* S, const aicp_sequence_params* prm, IcpLoop& q) {
  WinRun& R = *q.R;
  WIN_REFS;
  const int r = q.sub;
  hipStream_t si = S->s_icp;
  float* initT = S->initT.as<float>();
  float4* pts = sl.read_raw.as<float4>() + R.loff[r];
  launch_debug_prep(si, dDesc + r, initT, initT + 16 * (1 + w.p0 + (size_t)r));
  launch_transform(si, (int)R.n_read[r], initT, pts, pts);
  const BlockMap mrd = map_sub(R.m_read, R.b_read[r], R.b_read[r + 1] - R.b_read[r]);
  if (doOvl) {
    launch_ovl_init(si, 1, dDesc + r, dState + r, res, 2);
    if (R.sparse) {
      HIPC(launch_ovl_keys(si, R.kr1[r], dDesc[r].read_origin, sl.read_raw.as<float4>(), res, dState + r, 1));
      HIPC(launch_ovl_keys_intersect(si, R.kr1[r], R.kg, R.per_pair + r, dState + r));
    } else {
      launch_ovl_bbox(si, mrd, dDesc, dState, sl.read_raw.as<float4>(), 1, res);
      launch_ovl_size(si, 1, dState + r, dOvl + 1 + r, dCap + 1 + r);
      launch_ovl_clear(si, 1, dOvl + 1 + r, bmp, R.cap[1 + r]);
      launch_ovl_mark(si, mrd, dDesc, dOvl + 1, dState, sl.read_raw.as<float4>(), 1, res, bmp, false);
      launch_ovl_popcount(si, 1, dOvl + 1 + r, dState + r, 1, bmp);
      launch_ovl_intersect(si, 1, dDesc + r, dOvl + 1 + r, dOvl, dState + r, bmp);
    }
    launch_ovl_finish(si, 1, dDesc + r, dState + r, dGst, 1);
  }
  launch_prepare_read(si, mrd, dDesc, sl.read_raw.as<float4>(), sl.read_c.as<float4>());
  HIPC(hipGetLastError());
  return AICP_OK;
}

// after reading q.sub's loop: its correction, and initialT_ = correction * initialT_ when it is
// accepted (app.cpp:366-373, 414)
static int sub_post(aicp_hip_ctx* ctx, SeqState* S, const aicp_sequence_params* prm, IcpLoop& q) {
  WinRun& R = *q.R;
  WIN_REFS;
  const int r = q.sub;
  launch_debug_post(S->s_icp, dDesc + r, dState + r, dOutT + 16 * r, S->initT.as<float>(), prm->max_correction_magnitude);
  HIPC(hipGetLastError());
  return AICP_OK;
}

static int seq_init(aicp_hip_ctx* ctx, size_t n) {
  if (!ctx->seq) {
    SeqState* S = new SeqState();
    ctx->seq = S;
    S->device = ctx->device;
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
    // Few streams: HIP gives each priority level a pool of GPU_MAX_HW_QUEUES (4) hardware
    // queues and shares them beyond that, and streams sharing a queue run in submission order.
    // The tree streams are the context's (stream2, stream3: high priority); the ICP stream is
    // the third high-priority one; uploads and the reading side share one low-priority stream.
    HIPC(hipStreamCreateWithPriority(&S->s_rd, hipStreamNonBlocking, lo));
    HIPC(hipStreamCreateWithPriority(&S->s_icp, hipStreamNonBlocking, hi));
    S->s_up = S->s_rd;
    S->s_r2 = ctx->stream2;
    S->s_r3 = ctx->stream3;
    for (SeqSlot& sl : S->slot) {
      // the events that only order streams of this device release at device scope (no system-scope
      // fence when they are recorded); ev_up, which the host waits on before it reuses the pinned
      // staging, keeps the default
      HIPC(hipEventCreateWithFlags(&sl.ev_up, hipEventDisableTiming));
      for (hipEvent_t* e : {&sl.ev_rd, &sl.ev_ref, &sl.ev_s3, &sl.ev_s2, &sl.ev_done, &sl.ev_src})
        HIPC(hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice));
      HIPC(hipHostMalloc((void**)&sl.poll_host, 2 * kMaxPolls * 4, hipHostMallocMapped));
      HIPC(hipHostGetDevicePointer((void**)&sl.poll_dev, sl.poll_host, 0));
    }
    HIPC(hipEventCreate(&S->ev_begin));
    HIPC(hipEventCreate(&S->ev_end));
    (void)hipGetLastError();
  }
  SeqState* S = ctx->seq;
  S->opt = ctx->opt;
  for (SeqSlot& sl : S->slot) {
    sl.used = false;
    for (auto& t : sl.tb) tree_opts(t, S->opt);
  }
  HIPC(ensure(S->desc, n * sizeof(PairDesc)));
  HIPC(ensure(S->state, n * sizeof(PairState)));
  HIPC(ensure(S->outT, n * 64));
  HIPC(ensure(S->pin_state, n * sizeof(PairState)));
  HIPC(ensure(S->pin_out, n * 64));
  return AICP_OK;
}

static int seq_sync(aicp_hip_ctx* ctx, SeqState* S) {
  for (hipStream_t q : {S->s_up, S->s_rd, S->s_r2, S->s_r3, S->s_icp}) HIPC(hipStreamSynchronize(q));
  return AICP_OK;
}

extern "C" {

void aicp_hip_default_sequence_params(aicp_sequence_params* p) {
  if (!p) return;
  *p = aicp_sequence_params{};
  p->reference_update_frequency = 5;  // aicp.launch:61
  p->max_correction_magnitude = 1.0f;  // aicp.launch:63
  p->resolution = (double)0.2f;        // octomapResolution read as float (yaml_configurator.cpp:81)
  p->flags = AICP_RUN_OVERLAP;
}

int aicp_hip_sequence_run(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                          const aicp_cloud* first, const aicp_cloud* readings, size_t n, float* out_T,
                          aicp_sequence_result* out, size_t* n_done) {
  if (!ctx || !cfg || !prm || !first || (n && (!readings || !out_T || !out)) || !n_done) return AICP_ERR_INVALID;
  const auto t0 = std::chrono::steady_clock::now();
  *n_done = 0;
  const int F = prm->reference_update_frequency;
  if (F < 1) FAIL(AICP_ERR_INVALID, "reference_update_frequency must be >= 1");
  const bool doOvl = prm->flags & AICP_RUN_OVERLAP;
  const bool debug = prm->flags & AICP_SEQ_DEBUG;
  if (doOvl && !(prm->resolution > 0)) FAIL(AICP_ERR_INVALID, "resolution");
  int rc = check_cfg(ctx, cfg, AICP_RUN_ICP | (doOvl ? AICP_RUN_OVERLAP : 0));
  if (rc) return rc;
  auto valid = [](const aicp_cloud& c) {
    return c.pts && c.n >= 1 && c.n < (1ull << 28) && c.stride >= 12 && c.stride % 4 == 0;
  };
  if (!valid(*first)) FAIL(AICP_ERR_INVALID, "invalid first cloud");
  for (size_t i = 0; i < n; ++i)
    if (!valid(readings[i])) FAIL(AICP_ERR_INVALID, "invalid reading " + std::to_string(i));
  if ((size_t)F > (size_t)kMaxPairs) FAIL(AICP_ERR_UNSUPPORTED, "reference_update_frequency above 4096");
  {  // a window holds at most F consecutive readings: their points index 32-bit offsets
    uint64_t run = 0;
    for (size_t i = 0; i < n; ++i) {
      run += readings[i].n;
      if (i >= (size_t)F) run -= readings[i - F].n;
      if (run >= (1ull << 31)) FAIL(AICP_ERR_UNSUPPORTED, "a window's readings exceed 2^31 points");
    }
  }
  if (n == 0) return AICP_OK;
  HIPC(hipSetDevice(ctx->device));
  rc = seq_init(ctx, n);
  if (rc) return rc;
  SeqState* S = ctx->seq;
  S->last = aicp_sequence_timing{};  // (an error return leaves no stale timing behind)
  if (debug) {
    HIPC(ensure(S->initT, 64 * (n + 1)));
    HIPC(ensure(S->pin_desc, n * sizeof(PairDesc)));
  }
  const bool timeNN = prm->flags & AICP_RUN_TIME_NN;
  int nn_launches = 0, windows = 0, replans = 0;
  HIPC(hipEventRecord(S->ev_begin, S->s_up));
  // state at the start of a pass: next reading, reference source, accepted since its update
  size_t p = 0;
  int src = -1, acc = 0;
  std::vector<uint8_t> accepted(n, 0);
  std::vector<Box> rbox(n);
  int status = AICP_OK;
  while (p < n) {
    // plan: every reading accepted
    std::vector<Win> plan;
    {
      size_t q = p;
      int s = src, a = acc, k = 0;
      while (q < n) {
        const size_t np = std::min<size_t>((size_t)(F - a), n - q);
        plan.push_back(Win{q, np, s, k % kSlots, k});
        q += np;
        s = (int)(q - 1);
        a = 0;
        ++k;
      }
    }
    HIPC(ensure(S->pin_ctl, plan.size() * 2 * sizeof(TreeCtl)));
    TreeCtl* ctl = S->pin_ctl.as<TreeCtl>();
    std::memset(ctl, 0, plan.size() * 2 * sizeof(TreeCtl));
    std::vector<WinRun> runs(plan.size());
    if (S->opt.profile) {
      if (!S->s_probe) HIPC(hipStreamCreateWithFlags(&S->s_probe, hipStreamNonBlocking));
      while (S->tev.size() < 10 * plan.size()) {
        hipEvent_t e;
        HIPC(hipEventCreate(&e));
        S->tev.push_back(e);
      }
      for (size_t k = 0; k < plan.size(); ++k) runs[k].tev = S->tev.data() + 10 * k;
    }
    auto upload = [&](auto* ec, size_t k) {
      const Win& w = plan[k];
      runs[k].w = w;
      runs[k].ctl_w = ctl + 2 * k;
      if (k > 0) {  // the source is the previous window's last reading, still in its slot
        const Win& pw = plan[k - 1];
        const size_t off = (size_t)w.src - pw.p0;
        runs[k].src_desc = S->slot[pw.slot].wdesc.as<PairDesc>() + off;
        runs[k].src_T = S->slot[pw.slot].woutT.as<float>() + 16 * off;
        // its correction from its state (k_finalize's product): final before that window's loop
        // ends once the pair has stopped (early_reference)
        if (!debug) runs[k].src_state = S->slot[pw.slot].wstate.as<PairState>() + off;
      } else if (w.src >= 0) {  // a reading of an earlier pass: committed
        runs[k].src_desc = S->desc.as<PairDesc>() + w.src;
        runs[k].src_T = S->outT.as<float>() + 16 * (size_t)w.src;
      }
      // the reference source is resident in the previous window's slot, except for the first
      // window of a pass (the first cloud, or a reading of an earlier pass): uploaded again
      const float4* resident = nullptr;
      if (k > 0) {
        const Win& pw = plan[k - 1];
        uint64_t off = 0;
        for (size_t i = pw.p0; i < (size_t)w.src; ++i) off += readings[i].n;
        resident = S->slot[pw.slot].read_raw.as<float4>() + off;
      }
      return win_upload(ec, S, cfg, prm, first, readings, resident, rbox, runs[k]);
    };
    const bool prof = S->opt.profile;
    double hp[5] = {0, 0, 0, 0, 0};  // upload (its thread), reference trees, icp loop, join, reference icp
    auto timed = [&](int slot, const std::function<int()>& f) {
      const auto a = std::chrono::steady_clock::now();
      const int r = f();
      hp[slot] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
      return r;
    };
    // The reading side of window k + 1 (Morton order, voxel maps) is enqueued with its upload,
    // during window k's loop. (Enqueued with the next reference instead, to keep it off the loop's
    // CUs, it slowed the kd-tree builds on the critical path: 2.29 against 2.20 ms per window.)
    auto read_side = [&](auto* ec, size_t k) { return win_read_side(ec, S, cfg, prm, runs[k]); };
    std::vector<IcpLoop> loops(plan.size());
    std::vector<uint8_t> done_enq(plan.size(), 0);  // the window's ev_done recorded
    // enqueue iterations while the host is less than one iteration ahead of the oldest poll, read
    // the polls that have completed, finish the loop once one reads 0
    auto advance = [&](IcpLoop& q, bool& progress) -> int {
      while (!q.stop) {
        if (q.nn == q.it) {  // the next NN launch: enqueued before its active count is known
          const int r = loop_part(ctx, S, cfg, prm, q, 0, timeNN, nn_launches);
          if (r) return r;
          progress = true;
          continue;
        }
        // the rest of iteration q.it, once some pair is known to be active in it
        if (loop_polled(S, cfg, q.it)) {
          bool got = false;
          const int r = loop_poll(ctx, S, q, got);
          if (r) return r;
          if (!got) break;
          progress = true;
          if (q.stop) break;
        }
        const int r = loop_part(ctx, S, cfg, prm, q, 1, timeNN, nn_launches);
        if (r) return r;
        progress = true;
      }
      if (q.stop && q.it >= 0) {
        // debug mode: this reading's correction / initialT_, and the window's commit after its
        // last reading; otherwise the window's corrections and commit
        int r = q.sub >= 0 ? sub_post(ctx, S, prm, q) : AICP_OK;
        if (!r && (q.sub < 0 || q.sub + 1 == (int)q.R->np)) {
          r = loop_finish(ctx, S, prm, q);
          if (!r) done_enq[q.R->w.index] = 1;
        }
        if (r) return r;
        q.it = -1;  // finished
        progress = true;
      }
      return AICP_OK;
    };
    // upload(k + 1) reuses the slot of window k - 2 and waits (on the device) for ev_done of
    // window k - 1, which exists once that window's loop has been finished here
    auto can_upload = [&](size_t k) { return k + 1 < plan.size() && (k < 1 || done_enq[k - 1]); };
    if (debug) {  // initialT_ at the pass's first reading: identity, or its value before reading p
      static const float kI[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
      if (p == 0)
        HIPC(hipMemcpyAsync(S->initT.p, kI, 64, hipMemcpyHostToDevice, S->s_icp));
      else
        HIPC(hipMemcpyAsync(S->initT.p, S->initT.as<float>() + 16 * (1 + p), 64, hipMemcpyDeviceToDevice, S->s_icp));
    }
    rc = timed(0, [&] { return upload(ctx, 0); });
    if (!rc) rc = timed(0, [&] { return read_side(ctx, 0); });
    if (!rc) rc = timed(1, [&] { return win_ref_trees(ctx, S, cfg, prm, runs[0]); });
    if (!rc) rc = timed(4, [&] { return win_ref_icp(ctx, S, cfg, prm, runs[0]); });
    for (size_t k = 0; k < plan.size() && !rc; ++k) {
      const bool next = k + 1 < plan.size();
      bool uploaded = !next;
      // The next window's upload (host packing of its readings, ~0.35 ms per C2 window, then its
      // H2D and reading side) runs on a host thread of its own, started once this window's first
      // iterations are enqueued: on the polling thread it held the poll that enqueues iteration
      // smoothLength + 1, and the device waited ~0.25 ms per window for it (r04 trace).
      std::thread up_thr;
      std::atomic<bool> up_fin{false};
      int up_rc = AICP_OK;
      ErrSink up_err;  // the upload thread's error message (ctx->err belongs to this thread)
      auto try_upload = [&]() -> int {
        if (uploaded || !can_upload(k)) return AICP_OK;
        uploaded = true;
        up_thr = std::thread([&, k] {
          if (hipSetDevice(S->device) != hipSuccess) {
            up_err.err = "hipSetDevice on the upload thread";
            up_rc = AICP_ERR_HIP;
            return;
          }
          int r = timed(0, [&] { return upload(&up_err, k + 1); });
          if (!r) r = timed(0, [&] { return read_side(&up_err, k + 1); });
          up_rc = r;
          up_fin = true;
        });
        return AICP_OK;
      };
      auto join_upload = [&]() -> int {
        if (up_thr.joinable()) up_thr.join();
        return up_rc;
      };
      if (runs[k].tev) {
        rc = hipEventRecord(runs[k].tev[3], S->s_icp) == hipSuccess ? AICP_OK : AICP_ERR_HIP;
        if (rc) break;
      }
      // one loop per window; debug mode: one per reading, in order (reading i + 1 is moved by
      // the initialT_ that reading i's correction updates)
      const int n_sub = debug ? (int)runs[k].np : 1;
      // early_reference: the next window's reference starts once its source -- this window's last
      // reading -- has stopped iterating, beside this window's other readings (their loop runs on)
      runs[k].next_src = -1;
      if (!debug && next && S->opt.early_reference && plan[k + 1].index > 0 &&
          plan[k + 1].src == (int)(plan[k].p0 + plan[k].np - 1))
        runs[k].next_src = (int)plan[k].np - 1;
      bool ref_early = false;
      // the next window's reference trees, enqueued once the source pair has stopped and the next
      // window's upload is done (its thread joined), after this iteration's launches
      auto try_ref_early = [&]() -> int {
        if (ref_early || runs[k].next_src < 0 || !loops[k].src_done || !uploaded || !up_fin) return AICP_OK;
        if (up_thr.joinable()) up_thr.join();
        if (up_rc) {
          ctx->err = up_err.err;
          return up_rc;
        }
        ref_early = true;
        runs[k + 1].src_ev = S->slot[plan[k].slot].ev_src;
        return timed(1, [&] { return win_ref_trees(ctx, S, cfg, prm, runs[k + 1]); });
      };
      for (int sub = 0; sub < n_sub && !rc; ++sub) {
        IcpLoop& q = loops[k];
        q = IcpLoop{};
        q.R = &runs[k];
        q.sub = debug ? sub : -1;
        q.area = sub & 1;
        if (debug) rc = sub_prep(ctx, S, prm, q);
        if (rc) break;
        rc = timed(2, [&]() -> int {
          while (q.it >= 0) {
            bool progress = false;
            int r = advance(q, progress);
            if (!r) r = try_upload();
            if (!r) r = try_ref_early();
            if (r) return r;
            if (!progress) std::this_thread::yield();
          }
          return try_upload();
        });
      }
      {
        const int ur = timed(3, join_upload);  // (before any return: the thread uses this scope)
        if (!rc && ur) {  // the first error wins: the upload's message only if this thread had none
          rc = ur;
          ctx->err = up_err.err;
        }
      }
      if (!rc && next && !ref_early) rc = timed(1, [&] { return win_ref_trees(ctx, S, cfg, prm, runs[k + 1]); });
      if (!rc && next) rc = timed(4, [&] { return win_ref_icp(ctx, S, cfg, prm, runs[k + 1]); });
      ++windows;
    }
    if (prof)
      std::fprintf(stderr,
                   "[aicp seq] host ms: upload %.2f reference trees %.2f reference icp %.2f icp(incl. polls) %.2f "
                   "upload join %.2f over %zu windows\n",
                   hp[0], hp[1], hp[4], hp[2], hp[3], plan.size());
    if (rc) {
      (void)seq_sync(ctx, S);
      return rc;
    }
    // read back every reading of this pass
    const size_t pe = n;
    HIPC(hipMemcpyAsync(S->pin_state.as<PairState>() + p, S->state.as<PairState>() + p, (pe - p) * sizeof(PairState),
                        hipMemcpyDeviceToHost, S->s_icp));
    HIPC(hipMemcpyAsync(S->pin_out.as<float>() + 16 * p, S->outT.as<float>() + 16 * p, (pe - p) * 64,
                        hipMemcpyDeviceToHost, S->s_icp));
    if (debug)  // the prior origins moved by initialT_ (k_debug_prep), for the corrected poses
      HIPC(hipMemcpyAsync(S->pin_desc.as<PairDesc>() + p, S->desc.as<PairDesc>() + p, (pe - p) * sizeof(PairDesc),
                          hipMemcpyDeviceToHost, S->s_icp));
    HIPC(hipEventRecord(S->ev_end, S->s_icp));
    rc = seq_sync(ctx, S);
    if (rc) return rc;
    if (prof) {  // diagnostic builds' counters (-DAICP_ITER_PROF)
      iter_prof_dump();
      tree_prof_dump();
    }
    if (prof && plan.size() > 2) {  // device phase times, averaged over the windows after the first
      double a[5] = {0, 0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, c[3] = {0, 0, 0};
      const size_t m = plan.size() - 1;
      for (size_t k = 1; k < plan.size(); ++k) {
        const hipEvent_t* t = runs[k].tev;
        a[0] += ev_ms(t[0], t[1]);
        a[1] += ev_ms(t[0], t[2]);
        a[2] += ev_ms(t[0], t[3]);
        a[3] += ev_ms(t[3], t[4]);
        // the period from window 1 on: window 0's reference side starts the call with nothing
        // prepared ahead of it, and counting its period made the average ~0.09 ms longer than the
        // sum of the steady windows' phases (C2, r05)
        if (k >= 2) a[4] += ev_ms(runs[k - 1].tev[0], t[0]);
        const hipEvent_t* u = runs[k - 1].tev;  // the hand-off from window k - 1's commit
        b[0] += ev_ms(u[4], u[5]);
        b[1] += ev_ms(u[5], t[6]);
        b[2] += ev_ms(u[5], t[7]);
        b[3] += ev_ms(u[5], t[0]);
        // window k's reading side (enqueued during window k - 1's loop) against that loop
        c[0] += ev_ms(u[3], t[8]);
        c[1] += ev_ms(t[8], t[9]);
        c[2] += ev_ms(u[4], t[9]);
      }
      std::fprintf(stderr,
                   "[aicp seq] reading side ms/window: start after the previous loop's start %.3f, duration %.3f, "
                   "end after that loop's end %.3f\n",
                   c[0] / m, c[1] / m, c[2] / m);
      std::fprintf(stderr,
                   "[aicp seq] hand-off ms/window: commit %.3f, from its end: host enqueue %.3f upload ready %.3f "
                   "reference start %.3f\n",
                   b[0] / m, b[1] / m, b[2] / m, b[3] / m);
      std::fprintf(stderr,
                   "[aicp seq] device ms/window: ref->matcher %.3f ref->normals %.3f ref->icp start %.3f icp %.3f "
                   "period %.3f\n",
                   a[0] / m, a[1] / m, a[2] / m, a[3] / m, a[4] / (m - 1));
      // the pass's ends: from its first device work to window 0's reference start (window 0's
      // upload, which nothing runs beside), and from the last window's commit to the read-back
      std::fprintf(stderr,
                   "[aicp seq] pass ms: begin->window 0 reference %.3f, window 0 ref->next ref %.3f (ref->matcher %.3f "
                   "ref->normals %.3f ref->icp start %.3f icp %.3f), last commit->end %.3f, total %.3f over %zu windows\n",
                   ev_ms(S->ev_begin, runs[0].tev[0]), ev_ms(runs[0].tev[0], runs[1].tev[0]),
                   ev_ms(runs[0].tev[0], runs[0].tev[1]), ev_ms(runs[0].tev[0], runs[0].tev[2]),
                   ev_ms(runs[0].tev[0], runs[0].tev[3]), ev_ms(runs[0].tev[3], runs[0].tev[4]),
                   ev_ms(runs[plan.size() - 1].tev[5], S->ev_end), ev_ms(S->ev_begin, S->ev_end), plan.size());
    }
    for (size_t k = 0; k < plan.size(); ++k) {
      for (int t = 0; t < 2; ++t) {
        rc = device_trees_check_ctl(S->slot[plan[k].slot].tb[t], ctl + 2 * k + t, ctx->err);
        if (rc) return rc;
      }
      if ((ctl[2 * k + 1].error & 4)) FAIL(AICP_ERR_HIP, "matcher treelets exceed their allotment");
    }
    // check the prediction window by window
    const PairState* hs = S->pin_state.as<PairState>();
    const float* hT = S->pin_out.as<float>();
    bool replan = false;
    for (const Win& w : plan) {
      int a = (w.p0 == p) ? acc : 0;
      for (size_t i = w.p0; i < w.p0 + w.np; ++i) {
        int st = hs[i].status;
        if (doOvl && hs[i].ovl_err && !st) st = AICP_ERR_HIP;
        out[i].status = st;
        out[i].reference = w.src;
        out[i].is_reference = 0;
        if (st) {  // the worker ends here (app.cpp:210): nothing after this reading happened
          status = st;
          *n_done = i + 1;
          accepted[i] = 0;
          break;
        }
        accepted[i] = !correction_rejected(hT + 16 * i, prm->max_correction_magnitude);
        a += accepted[i];
      }
      if (status) break;
      if (a == F) {
        out[w.p0 + w.np - 1].is_reference = 1;
        continue;
      }
      if (w.p0 + w.np < n) {  // a reading was dropped: the reference stays, the window goes on
        p = w.p0 + w.np;
        src = w.src;
        acc = a;
        replan = true;
        ++replans;
        break;
      }
    }
    if (status || !replan) {
      if (!status) *n_done = n;
      break;
    }
  }
  // results
  const PairState* hs = S->pin_state.as<PairState>();
  const float* hT = S->pin_out.as<float>();
  for (size_t i = 0; i < *n_done; ++i) {
    std::memcpy(out_T + 16 * i, hT + 16 * i, 64);
    aicp_sequence_result& r = out[i];
    r.accepted = accepted[i];
    for (int k = 0; k < 3; ++k) r.corrected_origin[k] = 0.0;
    if (r.accepted)
      corrected_origin(hT + 16 * i, debug ? S->pin_desc.as<PairDesc>()[i].read_origin : readings[i].origin,
                       r.corrected_origin);
    const PairState& st = hs[i];
    aicp_icp_stats& o = r.icp;
    std::memset(&o, 0, sizeof(o));
    o.status = r.status;
    o.iterations = st.iters;
    o.converged = st.converged;
    o.degenerate_normals = st.degenerate;
    o.inlier_ratio = st.inlier_ratio;
    o.trimmed_ratio = st.ratio;
    o.overlap_percent = st.overlap;
    o.nn_points_touched = st.touched_pts;
    o.nn_nodes_touched = st.touched_nodes;
    for (int k = 0; k < 3; ++k) o.overlap_keys[k] = st.ovl_counts[k];
  }
  if (S->opt.profile) {  // guessed bins of the fused select that missed, against its launches
    uint64_t miss = 0, fused = 0;
    for (size_t i = 0; i < *n_done; ++i) {
      miss += hs[i].sel_miss;
      fused += hs[i].iters > 1 ? (uint64_t)(hs[i].iters - 1) : 0;
    }
    std::fprintf(stderr, "[aicp seq] fused select: %llu of %llu guessed bins missed\n", (unsigned long long)miss,
                 (unsigned long long)fused);
    nn_prof_dump();  // diagnostic builds' counters (AICP_QLAT_PROF / AICP_XCD_PROF / AICP_NN_PROF)
  }
  // timing
  ctx->last_nn_launches = timeNN ? nn_launches : 0;
  ctx->last_nn_ms = 0;
  if (timeNN)
    for (int i = 0; i < nn_launches; ++i) ctx->last_nn_ms += ev_ms(S->nn_ev[2 * i], S->nn_ev[2 * i + 1]);
  uint64_t queries = 0, tp = 0, tn = 0;
  for (size_t i = 0; i < *n_done; ++i) {
    queries += (uint64_t)hs[i].iters * readings[i].n;
    tp += hs[i].touched_pts;
    tn += hs[i].touched_nodes;
  }
  ctx->last_nn_bytes = timeNN ? (double)queries * 20.0 + (double)tp * 16.0 + (double)tn * 8.0 : 0.0;
  ctx->last_queries = queries;
  S->last.windows = windows;
  S->last.replans = replans;
  S->last.device_ms = ev_ms(S->ev_begin, S->ev_end);
  S->last.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (status) ctx->err = "reading " + std::to_string(*n_done - 1) + ": status " + std::to_string(status);
  return status;
}

int aicp_hip_last_sequence_timing(const aicp_hip_ctx* ctx, aicp_sequence_timing* out) {
  if (!ctx || !out) return AICP_ERR_INVALID;
  *out = ctx->seq ? ctx->seq->last : aicp_sequence_timing{};
  return AICP_OK;
}

}  // extern "C"
