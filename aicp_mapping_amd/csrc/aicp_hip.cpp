// aicp_hip.cpp — C-ABI of libaicp_hip.so: context, device arena, batch pipeline.
//
// One batch run (aicp_hip_batch_run) for P pairs, one HIP stream, no per-iteration host sync:
//   1. [device] overlap: origin/endpoint key boxes (k_ovl_init, k_ovl_bbox) -> D2H (the only
//      host sync before the loop: it sizes the voxel maps)
//   2. [device] voxel maps; DDA ray marking, sums, overlap% and the auto-tuned ratio per pair
//      (App::computeRegistration, app.cpp:197-205)
//   3. [device] centroid, centred reference and the libnabo-order kd-tree of every pair
//      (ICP::compute "matcher->init(reference)", kernels_tree.hip), level by level; the host
//      polls the segment count every few levels
//   4. [device] reading into the ref-mean frame, SurfaceNormal on the reference
//   5. [device] max_iter x {NN, select, reduce, update}; converged pairs exit early
//   6. [device] T = T_refIn_refMean * T_iter * T_refMean_dataIn; D2H of T and pair states
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
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

void tree_opts(TreeBufs& T, const aicp_hip_options& o) {
  T.lvl_min = o.tree_lvl_min;
  T.prof = o.profile != 0;
}

bool valid_pair(const aicp_pair& p) {
  if (!p.ref || !p.read || p.n_ref < 1 || p.n_read < 1) return false;
  if (p.ref_stride < 12 || p.read_stride < 12 || (p.ref_stride % 4) || (p.read_stride % 4)) return false;
  if (p.n_ref >= (1ull << 30) || p.n_read >= (1ull << 30)) return false;
  return true;
}

void pack_xyz(const float* src, uint64_t n, uint64_t stride_bytes, float* dst3) {
  const char* b = reinterpret_cast<const char*>(src);
  for (uint64_t i = 0; i < n; ++i) {
    const float* p = reinterpret_cast<const float*>(b + i * stride_bytes);
    dst3[3 * i] = p[0];
    dst3[3 * i + 1] = p[1];
    dst3[3 * i + 2] = p[2];
  }
}
// Strided xyz -> float4 for many clouds at once, split into equal point ranges over host
// threads (the packing, not the DMA, bounded the host-buffer path: one thread moves ~5 GB/s)
void pack_many(const std::vector<PackSeg>& segs, WorkerPool* pool) {
  uint64_t total = 0;
  for (const PackSeg& g : segs) total += g.n;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned nt = total < (1u << 16) ? 1u : hw;
  if (nt == 1) {
    for (const PackSeg& g : segs) pack_xyz4(g.src, g.n, g.stride, g.dst4);
    return;
  }
  auto work = [&](uint64_t lo, uint64_t hi) {  // global point range [lo, hi)
    uint64_t base = 0;
    for (const PackSeg& g : segs) {
      const uint64_t a = std::max(lo, base), b = std::min(hi, base + g.n);
      if (a < b) {
        const char* src = reinterpret_cast<const char*>(g.src) + (a - base) * g.stride;
        pack_xyz4(reinterpret_cast<const float*>(src), b - a, g.stride, g.dst4 + 4 * (a - base));
      }
      base += g.n;
      if (base >= hi) break;
    }
  };
  if (pool) {  // the context's threads
    pool->run(nt, [&](size_t t) { work(total * t / nt, total * (t + 1) / nt); });
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, total * t / nt, total * (t + 1) / nt);
  work(0, total / nt);
  for (auto& x : th) x.join();
}

WorkerPool* ctx_pool(aicp_hip_ctx* ctx) {
  if (!ctx->pool) ctx->pool = new WorkerPool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
  return ctx->pool;
}

void pack_xyz4(const float* src, uint64_t n, uint64_t stride_bytes, float* dst4) {
  const char* b = reinterpret_cast<const char*>(src);
  for (uint64_t i = 0; i < n; ++i) {
    const float* p = reinterpret_cast<const float*>(b + i * stride_bytes);
    dst4[4 * i] = p[0];
    dst4[4 * i + 1] = p[1];
    dst4[4 * i + 2] = p[2];
    dst4[4 * i + 3] = 1.f;
  }
}

int check_cfg(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, int flags) {
  if (!cfg) FAIL(AICP_ERR_INVALID, "null config");
  if (cfg->knn_match != 1) FAIL(AICP_ERR_UNSUPPORTED, "KDTreeMatcher.knn != 1");
  if (flags & AICP_RUN_ICP) {
    if (cfg->knn_normals != 10 && cfg->knn_normals != 20 && cfg->knn_normals != 30)
      FAIL(AICP_ERR_UNSUPPORTED, "SurfaceNormal knn must be 10, 20 or 30");
    if (cfg->max_iter < 1 || cfg->max_iter > 1000) FAIL(AICP_ERR_INVALID, "maxIterationCount");
    if (cfg->smooth_length < 1 || cfg->smooth_length >= kHistRing) FAIL(AICP_ERR_UNSUPPORTED, "smoothLength");
    if (cfg->bucket_size < 1) FAIL(AICP_ERR_INVALID, "bucketSize");
    if (!(flags & AICP_RUN_OVERLAP) && !(cfg->trimmed_ratio > 0.f && cfg->trimmed_ratio <= 1.f))
      FAIL(AICP_ERR_INVALID, "TrimmedDistOutlierFilter.ratio");
    if (!(cfg->nn_epsilon >= 0.f)) FAIL(AICP_ERR_INVALID, "epsilon");
  }
  return AICP_OK;
}

// refs_on_device: every pair has a reference of its own (n_ref points) that the caller writes
// into B->ref_raw at rdesc[i].ref_off afterwards (the localization batch's map crops); the
// pairs' ref pointers are then not read.
// skip_refs: the reference points are not needed on the device (the context's cached reference
// serves every reading of the call): not packed, not uploaded.
// nosync: the caller synchronises the stream before the pinned staging is written again (a one-shot
// call does, at its end); otherwise this returns once the copies are done
int upload_pairs(aicp_hip_ctx* ctx, const aicp_pair* pairs, size_t n, aicp_hip_batch* B, bool refs_on_device,
                 bool skip_refs = false, bool skip_reads = false, bool nosync = false) {
  if (!pairs || n == 0) FAIL(AICP_ERR_INVALID, "no pairs");
  B->P = n;
  B->desc.assign(n, PairDesc{});
  B->rdesc.clear();
  B->gdesc.clear();
  uint64_t ro = 0, wo = 0;
  uint32_t red = 0;
  Maps mr, mf, md, ms;
  // pairs whose reference is the same caller array (pointer, count, stride) share one copy,
  // one kd-tree and one set of normals (a reference window serves several readings)
  std::vector<size_t> rep;  // representative pair of each distinct reference
  for (size_t i = 0; i < n; ++i) {
    const aicp_pair& p = pairs[i];
    if (!valid_pair(p)) FAIL(AICP_ERR_INVALID, "invalid pair " + std::to_string(i));
    PairDesc& d = B->desc[i];
    int32_t rid = -1;
    for (size_t r = 0; r < rep.size() && !refs_on_device; ++r) {
      const aicp_pair& q = pairs[rep[r]];
      if (q.ref == p.ref && q.n_ref == p.n_ref && q.ref_stride == p.ref_stride) {
        rid = (int32_t)r;
        break;
      }
    }
    if (rid < 0) {
      rid = (int32_t)rep.size();
      rep.push_back(i);
      PairDesc r{};
      r.ref_off = (uint32_t)ro;
      r.n_ref = (uint32_t)p.n_ref;
      r.ref_id = rid;
      r.ratio = 0.5f;
      ident4(r.Tin);
      B->rdesc.push_back(r);
      ro += p.n_ref;
    }
    d.ref_id = rid;
    d.ref_off = B->rdesc[rid].ref_off;
    int32_t gid = -1;
    for (size_t g = 0; g < B->gdesc.size(); ++g) {
      const PairDesc& gd = B->gdesc[g];
      if (gd.ref_id == rid && gd.ref_origin[0] == p.ref_origin[0] && gd.ref_origin[1] == p.ref_origin[1] &&
          gd.ref_origin[2] == p.ref_origin[2]) {
        gid = (int32_t)g;
        break;
      }
    }
    if (gid < 0) {
      gid = (int32_t)B->gdesc.size();
      PairDesc g{};
      g.ref_id = rid;
      g.ref_off = d.ref_off;
      g.n_ref = (uint32_t)p.n_ref;
      for (int k = 0; k < 3; ++k) g.ref_origin[k] = p.ref_origin[k];
      B->gdesc.push_back(g);
      mf.add(gid, g.n_ref, kNNBlock);
    }
    d.ogroup = gid;
    d.n_ref = (uint32_t)p.n_ref;
    d.read_off = (uint32_t)wo;
    d.n_read = (uint32_t)p.n_read;
    d.red_blk_off = red;
    constexpr uint32_t kRedBlk = kNNBlock * kReducePerThread * kReduceChunks;
    d.n_red_blk = (uint32_t)((p.n_read + kRedBlk - 1) / kRedBlk);
    for (int k = 0; k < 3; ++k) {
      d.ref_origin[k] = p.ref_origin[k];
      d.read_origin[k] = p.read_origin[k];
    }
    red += d.n_red_blk;
    wo += p.n_read;
    // reference positions travel as 28-bit fields in the NN kernel's bucket exchange (Trav2C)
    if (ro >= (1ull << 28) || wo >= (1ull << 31)) FAIL(AICP_ERR_UNSUPPORTED, "batch too large");
    if (p.init_T)
      std::memcpy(d.Tin, p.init_T, 64);
    else
      ident4(d.Tin);
    mr.add((int)i, d.n_read, kNNBlock);
    md.add((int)i, d.n_read, kNNBlock * kReducePerThread * kReduceChunks);
    ms.add((int)i, d.n_read, kNNBlock * kSelPerThread);
  }
  B->total_ref = ro;
  B->total_read = wo;
  B->n_red_total = red;
  // raw clouds as float4
  HIPC(ensure(B->ref_raw, ro * 16));
  HIPC(ensure(B->read_raw, wo * 16));
  const bool pack_refs = !refs_on_device && !skip_refs;
  HIPC(ensure(ctx->pin_io, ((pack_refs ? ro : 0) + wo) * 16));  // references, then readings: the readings are
  float* st = ctx->pin_io.as<float>();          // packed while the references' DMA runs
  std::vector<PackSeg> segs;
  // pack and copy in chunks of >= kPackChunk points, so each chunk's DMA runs while the next one
  // is packed (C5: 983 MB of references per side took ~15 ms to pack before the first byte moved)
  constexpr uint64_t kPackChunk = 4u << 20;
  auto pack_copy = [&](const std::vector<PackSeg>& all, const float* host0, void* dev0) -> int {
    size_t a = 0;
    while (a < all.size()) {
      size_t b = a;
      uint64_t pts = 0;
      while (b < all.size() && (pts < kPackChunk || b == a)) pts += all[b++].n;
      std::vector<PackSeg> part(all.begin() + a, all.begin() + b);
      pack_many(part, ctx_pool(ctx));
      const uint64_t off = (uint64_t)(all[a].dst4 - host0) / 4;  // first point of the chunk
      HIPC(hipMemcpyAsync(static_cast<char*>(dev0) + off * 16, all[a].dst4, pts * 16, hipMemcpyHostToDevice,
                          ctx->stream));
      a = b;
    }
    return AICP_OK;
  };
  if (pack_refs) {
    for (size_t r = 0; r < rep.size(); ++r) {
      const PairDesc& d = B->rdesc[r];
      segs.push_back(PackSeg{pairs[rep[r]].ref, d.n_ref, pairs[rep[r]].ref_stride, st + 4ull * d.ref_off});
    }
    if (int rc = pack_copy(segs, st, B->ref_raw.p)) return rc;
  }
  // the reference side (trees, normals) waits for this event only, so its kernels run while the
  // readings are packed and copied (references written on the device later record it in run_batch)
  B->refs_event = pack_refs;
  if (pack_refs) {
    if (!ctx->ev[14]) HIPC(hipEventCreateWithFlags(&ctx->ev[14], hipEventReleaseToDevice));
    HIPC(hipEventRecord(ctx->ev[14], ctx->stream));
  }
  float* sw = pack_refs ? st + 4ull * ro : st;
  segs.clear();
  for (size_t i = 0; i < n; ++i) {
    const PairDesc& d = B->desc[i];
    segs.push_back(PackSeg{pairs[i].read, d.n_read, pairs[i].read_stride, sw + 4ull * d.read_off});
  }
  if (!skip_reads) {  // (skip_reads: the previous call's reading, still on the device)
    if (int rc = pack_copy(segs, sw, B->read_raw.p)) return rc;
  }
  // block maps: [read pair][read start][ref pair][ref start][red pair][red start]
  const size_t nr = mr.pair.size(), nf = mf.pair.size(), nd = md.pair.size(), ns = ms.pair.size();
  const size_t words = 2 * (nr + nf + nd + ns);
  HIPC(ensure(B->maps, words * 4));
  HIPC(ensure(ctx->pin_maps, words * 4));  // (staged apart from pin_io, whose copy may still run)
  uint32_t* mp = ctx->pin_maps.as<uint32_t>();
  size_t o = 0;
  auto put = [&](const Maps& m, BlockMap& bm) {
    const size_t cnt = m.pair.size();
    std::memcpy(mp + o, m.pair.data(), cnt * 4);
    std::memcpy(mp + o + cnt, m.start.data(), cnt * 4);
    bm.pair = B->maps.as<int32_t>() + o;
    bm.start = B->maps.as<uint32_t>() + o + cnt;
    bm.n_blocks = (uint32_t)cnt;
    o += 2 * cnt;
  };
  put(mr, B->m_read);
  put(mf, B->m_gref);
  put(md, B->m_red);
  put(ms, B->m_sel);
  HIPC(hipMemcpyAsync(B->maps.p, mp, words * 4, hipMemcpyHostToDevice, ctx->stream));
  if (!nosync) HIPC(hipStreamSynchronize(ctx->stream));
  return AICP_OK;
}

// Centroid (center = 1) + libnabo-order kd-trees of P clouds on the device: raw[ΣM] float4,
// dDesc with ref_off / n_ref / Tin. Writes bpts_out (bucket order, w = local id), nodes_out
// and the desc fields mean, Tmean, Tinit, node_off, n_nodes, tree_depth.
int device_trees_begin(TreeBufs& T, std::string& err, hipStream_t s, size_t P, uint64_t total, PairDesc* dDesc,
                       const float4* raw, int center, int bucket, DevBuf& bpts_out, DevBuf& nodes_out, bool launch,
                       int part) {
  const size_t n = (size_t)total;
  const size_t max_seg = n / 2 + P + 1;
  TCHK(ensure(bpts_out, n * 16));
  TCHK(ensure(nodes_out, (2 * n + 2) * 16));
  TCHK(ensure(T.W0, n * 16));
  TCHK(ensure(T.W1, n * 16));
  TCHK(ensure(T.segof0, n * 4));
  TCHK(ensure(T.segof1, n * 4));
  TCHK(ensure(T.seg0, max_seg * sizeof(TreeSeg)));
  TCHK(ensure(T.seg1, max_seg * sizeof(TreeSeg)));
  TCHK(ensure(T.flag, (n + 2) * 4));
  TCHK(ensure(T.X1, (n + 2) * 4));
  TCHK(ensure(T.X2, (n + 2) * 4));
  TCHK(ensure(T.posL, n * 4));
  TCHK(ensure(T.posR, n * 4));
  TCHK(ensure(T.ev, (2 * n + 2) * sizeof(NodeEvent)));
  TCHK(ensure(T.valid, 2 * n + 2));
  TCHK(ensure(T.subs, max_seg * sizeof(SubSeg)));
  TCHK(ensure(T.mids, max_seg * sizeof(SubSeg)));
  TCHK(ensure(T.lb, lb_bytes((uint32_t)n)));
  TCHK(ensure(T.ecnt, (n + 2) * 4));
  TCHK(ensure(T.sums, (P + tree_sum_tiles(n)) * 6 * 8));  // per pair, then per tile (k_tr_sum)
  TCHK(ensure(T.pdepth, P * 4));
  TCHK(ensure(T.ctl, sizeof(TreeCtl)));
  const size_t tb = tree_scan_temp_bytes(n + 2);
  TCHK(ensure(T.scan, tb));
  TCHK(ensure(T.pin_ctl, sizeof(TreeCtl)));
  TreeWork w;
  std::memset(&w, 0, sizeof(w));  // (a graph key in sequence.cpp compares its bytes)
  w.W[0] = T.W0.as<float4>();
  w.W[1] = T.W1.as<float4>();
  w.segof[0] = T.segof0.as<int32_t>();
  w.segof[1] = T.segof1.as<int32_t>();
  w.seg[0] = T.seg0.as<TreeSeg>();
  w.seg[1] = T.seg1.as<TreeSeg>();
  w.flag = T.flag.as<uint32_t>();
  w.X1 = T.X1.as<uint32_t>();
  w.X2 = T.X2.as<uint32_t>();
  w.posL = T.posL.as<uint32_t>();
  w.posR = T.posR.as<uint32_t>();
  w.ev = T.ev.as<NodeEvent>();
  w.valid = T.valid.as<uint8_t>();
  w.subs = T.subs.as<SubSeg>();
  w.mids = T.mids.as<SubSeg>();
  w.lb = T.lb.as<uint64_t>();
  w.lb_stride = lb_stride_words((uint32_t)n);
  w.mid_max = tree_mid_max();
  w.lvl_min = T.lvl_min;
  w.n_pairs = (int)P;
  w.ecnt = T.ecnt.as<uint32_t>();
  w.sums = T.sums.as<uint64_t>();
  w.pair_depth = T.pdepth.as<int32_t>();
  w.ctl = T.ctl.as<TreeCtl>();
  w.scan_temp = T.scan.p;
  w.scan_temp_bytes = T.scan.cap;
  w.max_seg = max_seg;
  T.tw = w;
  if (!launch) return AICP_OK;  // work space only (before a stream capture)
  TCHK(launch_tree_prepare(s, (int)P, (uint32_t)n, dDesc, raw, center, w, bpts_out.as<float4>(), bucket, part));
  return AICP_OK;
}

// Global levels, wave subtrees, node records; see device_trees_begin. plan > 0: enqueue
// `plan` global levels without any host read-back (the whole build is asynchronous) plus an
// async copy of the control block, checked after the batch by device_trees_check; plan = 0:
// the host polls the next level's segment count from level 4 on (fallback when a planned
// build turned out too shallow). levels_done (optional) is recorded after the global levels and
// the mid-size segments, before the subtree kernels.
int device_trees_end(TreeBufs& T, std::string& err, hipStream_t s, size_t P, uint64_t total, PairDesc* dDesc,
                     int bucket, DevBuf& bpts_out, DevBuf& nodes_out, int plan, TreeCtl* ctl_dst, bool copy_ctl,
                     hipEvent_t levels_done) {
  const size_t n = (size_t)total;
  const TreeWork& w = T.tw;
  float4* bpts = bpts_out.as<float4>();
  TreeCtl* hctl = ctl_dst ? ctl_dst : T.pin_ctl.as<TreeCtl>();
  T.planned = 0;
  if (plan > 0) {
    plan = std::min(plan, kFarStack - 2);
    for (int level = 0; level < plan; ++level)
      TCHK(launch_tree_level(s, level, (uint32_t)n, w, bpts, bucket, level == plan - 1));
    TCHK(launch_tree_mid(s, (uint32_t)n, w, bpts, bucket));
    if (levels_done) TCHK(hipEventRecord(levels_done, s));
    TCHK(launch_tree_subtrees(s, (uint32_t)n, w, bpts, bucket));
    TCHK(launch_tree_finish(s, (int)P, (uint32_t)n, dDesc, w, nodes_out.as<uint4>()));
    if (copy_ctl) TCHK(hipMemcpyAsync(hctl, w.ctl, sizeof(TreeCtl), hipMemcpyDeviceToHost, s));
    T.planned = plan;
    return AICP_OK;
  }
  bool done = false;
  for (int level = 0; level < kFarStack - 1 && !done; ++level) {
    TCHK(launch_tree_level(s, level, (uint32_t)n, w, bpts, bucket, false));
    if (level >= 4 || level == kFarStack - 2) {
      TCHK(hipMemcpyAsync(hctl, w.ctl, sizeof(TreeCtl), hipMemcpyDeviceToHost, s));
      TCHK(hipStreamSynchronize(s));
      if (hctl->nseg[level + 1] == 0) done = true;
    }
  }
  if (!done) TFAIL(AICP_ERR_UNSUPPORTED, "kd-tree deeper than the device stack (48 levels)");
  TCHK(launch_tree_mid(s, (uint32_t)n, w, bpts, bucket));
  if (levels_done) TCHK(hipEventRecord(levels_done, s));
  TCHK(launch_tree_subtrees(s, (uint32_t)n, w, bpts, bucket));
  TCHK(launch_tree_finish(s, (int)P, (uint32_t)n, dDesc, w, nodes_out.as<uint4>()));
  TCHK(hipMemcpyAsync(&hctl->error, &w.ctl->error, 4, hipMemcpyDeviceToHost, s));
  TCHK(hipStreamSynchronize(s));
  if (hctl->error & 1) TFAIL(AICP_ERR_UNSUPPORTED, "kd-tree deeper than the device stack (48 levels)");
  if (hctl->error) TFAIL(AICP_ERR_HIP, "kd-tree construction overflow " + std::to_string(hctl->error));
  return AICP_OK;
}

// After the stream of a planned build has completed: its errors (the control block was copied
// back asynchronously at the end of the build). Segments left above kMidMax points at the last
// planned level were finished by the subtree kernel's global path, so the tree is complete.
int device_trees_check(TreeBufs& T, std::string& err) {
  return device_trees_check_ctl(T, T.pin_ctl.as<TreeCtl>(), err);
}
int device_trees_check_ctl(TreeBufs& T, const TreeCtl* hctl, std::string& err) {
  if (!T.planned) return AICP_OK;
  int used = 0;
  while (used < kFarStack + 1 && hctl->nseg[used]) ++used;
  // oversized segments at the last planned level: plan deeper next time
  T.needed = hctl->n_big ? std::min(kFarStack - 3, T.planned + 2) : used;
  if (T.prof) {
    std::fprintf(stderr, "[aicp tree] planned %d used %d next %d: n_big %u n_mid %u n_small %u segments/level", T.planned,
                 used, T.needed, hctl->n_big, hctl->n_mid, hctl->n_small);
    for (int l = 0; l < used; ++l) std::fprintf(stderr, " %u", hctl->nseg[l]);
    std::fprintf(stderr, "\n");
  }
  if (hctl->error & 1) TFAIL(AICP_ERR_UNSUPPORTED, "kd-tree deeper than the device stack (48 levels)");
  if (hctl->error & ~4) TFAIL(AICP_ERR_HIP, "kd-tree construction overflow " + std::to_string(hctl->error));
  return AICP_OK;
}

// Global levels to enqueue for clouds of at most n_max points: segments above kSubMax points
// halve per level on balanced data; sliding-midpoint splits can peel off small slices, so the
// first plan keeps a margin, and later plans follow what the previous build of this tree used
// (every planned level costs its launches and two full-length scans even when no segment is
// left: C2 with 8 instead of 11 levels, +2 %).
// force (aicp_hip_options::tree_plan): k > 0 forces k levels (tests: a too-shallow plan), -1 the
// host-polled build (A/B measurements).
int plan_levels(uint64_t n_max, const TreeBufs& T, int force, bool lean) {
  if (force > 0) return std::min(kFarStack - 2, force);
  if (force < 0) return 0;
  int l = 0;
  while (((uint64_t)tree_mid_max() << l) < n_max) ++l;
  // lean: the balanced estimate + 1, whatever the previous build used; the few segments still
  // above kSubMax go to the subtree kernel's global path (used for the raw-coordinate tree on
  // the critical stream: C2 +2 %, the leftovers cost less than the full-length levels)
  if (lean) return std::min(kFarStack - 2, l + 1);
  // with a previous build of this tree: the levels it used (a cloud that needs more leaves a few
  // segments above kSubMax to the subtree kernel's global path once, and the next plan grows);
  // without one: a margin of 4 levels over the balanced estimate
  return std::min(kFarStack - 2, T.needed > 0 ? std::max(l + 1, T.needed) : l + 4);
}

// The overlap's second half on stream s (the first, the key boxes, is queued before the trees):
// wait for the boxes, size one byte map per reading and per reference group, mark, count,
// ratio. Runs on its own host thread while the main thread queues the trees, so the marking
// starts as soon as the boxes are known instead of after the raw tree's host polls.
// The overlap from sorted key words (kernels_overlap_sparse.hip) when the dense voxel maps of a
// batch do not fit: counts per point -> offsets (one host read of the total) -> words -> sort ->
// distinct counts and intersections. Same sets, same counts as the maps.
int overlap_sparse(aicp_hip_ctx* ctx, aicp_hip_batch* B, size_t P, size_t G, PairDesc* dDesc, PairState* dState,
                   PairState* dGst, const float4* readS, double res, bool set_ratio, std::string& err) {
  hipStream_t s = ctx->stream;
  std::vector<OvlCloud> cl(G + P);
  std::vector<uint32_t> bc, bs;
  uint64_t slots = 0;
  for (size_t c = 0; c < G + P; ++c) {
    OvlCloud& o = cl[c];
    o = OvlCloud{};
    const PairDesc& d = c < G ? B->gdesc[c] : B->desc[c - G];
    o.side = c < G ? 0 : 1;
    o.pts_off = c < G ? d.ref_off : d.read_off;
    o.n = c < G ? d.n_ref : d.n_read;
    for (int k = 0; k < 3; ++k) o.origin[k] = c < G ? d.ref_origin[k] : d.read_origin[k];
    o.slot = slots;
    slots += o.n;
    for (uint32_t j = 0; j < o.n; j += 256) {
      bc.push_back((uint32_t)c);
      bs.push_back(j);
    }
  }
  if (slots >= (1ull << 32)) TFAIL(AICP_ERR_UNSUPPORTED, "sparse overlap: more than 2^32 points");
  const size_t nb = bc.size();
  const size_t scan_b = ovl_sparse_scan_bytes(slots);
  const size_t o_cl = 0, o_bc = o_cl + (G + P) * sizeof(OvlCloud), o_bs = o_bc + nb * 4,
               o_cnt = (o_bs + nb * 4 + 255) & ~size_t(255), o_off = (o_cnt + slots * 4 + 255) & ~size_t(255),
               o_pc = o_off + slots * 8, o_pp = o_pc + (G + P) * 8, o_tmp = (o_pp + P * 8 + 255) & ~size_t(255);
  TCHK(ensure(ctx->ovl_sp, o_tmp + scan_b));
  const size_t o_tail = (o_bs + nb * 4 + 7) & ~size_t(7);  // read-back of the key total
  TCHK(ensure(ctx->pin_ovl, o_tail + 16));
  char* h = ctx->pin_ovl.as<char>();
  std::memcpy(h + o_cl, cl.data(), (G + P) * sizeof(OvlCloud));
  std::memcpy(h + o_bc, bc.data(), nb * 4);
  std::memcpy(h + o_bs, bs.data(), nb * 4);
  char* d = ctx->ovl_sp.as<char>();
  TCHK(hipMemcpyAsync(d, h, o_bs + nb * 4, hipMemcpyHostToDevice, s));
  TCHK(hipEventRecord(ctx->ev[6], s));
  const OvlCloud* dcl = (const OvlCloud*)(d + o_cl);
  const uint32_t* dbc = (const uint32_t*)(d + o_bc);
  const uint32_t* dbs = (const uint32_t*)(d + o_bs);
  uint32_t* cnt = (uint32_t*)(d + o_cnt);
  uint64_t* off = (uint64_t*)(d + o_off);
  TCHK(launch_ovl_sparse_count(s, (uint32_t)nb, dbc, dbs, dcl, B->ref_raw.as<float4>(), readS, res, (uint32_t)slots,
                               cnt, off, d + o_tmp, scan_b));
  uint64_t* tail = (uint64_t*)(h + o_tail);
  TCHK(hipMemcpyAsync(tail, off + (slots - 1), 8, hipMemcpyDeviceToHost, s));
  uint32_t* tailc = (uint32_t*)(tail + 1);
  TCHK(hipMemcpyAsync(tailc, cnt + (slots - 1), 4, hipMemcpyDeviceToHost, s));
  TCHK(hipStreamSynchronize(s));
  const uint64_t n_keys = slots ? tail[0] + tailc[0] : 0;
  const size_t sort_b = ovl_sparse_sort_bytes(n_keys);
  size_t free_b = 0, total_b = 0;
  TCHK(hipMemGetInfo(&free_b, &total_b));
  if (n_keys * 16 + sort_b > ctx->ovl_keys.cap + free_b / 2)
    TFAIL(AICP_ERR_UNSUPPORTED, "sparse overlap: " + std::to_string(n_keys) + " ray keys do not fit");
  TCHK(ensure(ctx->ovl_keys, n_keys * 16 + sort_b + 256));
  uint64_t* k0 = ctx->ovl_keys.as<uint64_t>();
  uint64_t* k1 = k0 + n_keys;
  void* tmp = (void*)(((uintptr_t)(k1 + n_keys) + 255) & ~uintptr_t(255));
  TCHK(launch_ovl_sparse_sets(s, (uint32_t)nb, dbc, dbs, dcl, B->ref_raw.as<float4>(), readS, res, off, n_keys, k0, k1,
                              tmp, sort_b, (int)G, (int)P, dDesc, (unsigned long long*)(d + o_pc),
                              (unsigned long long*)(d + o_pp), dGst, dState));
  launch_ovl_finish(s, (int)P, dDesc, dState, dGst, set_ratio ? 1 : 0);
  TCHK(hipGetLastError());
  return AICP_OK;
}

// dense voxel maps of one batch beyond this size take the sorted-key path instead (a 60 x 60 x 6 m
// scene at 0.2 m is ~2.7 MB per map; 8 GiB covers thousands of such clouds)
constexpr uint64_t kDenseMapBudget = uint64_t(8) << 30;
constexpr unsigned long long kReadOrderMin = 200000;


int overlap_maps(aicp_hip_ctx* ctx, aicp_hip_batch* B, size_t P, size_t G, PairDesc* dDesc, PairState* dState,
                 PairDesc* dG, PairState* dGst, const float4* readS, double res, bool set_ratio, std::string& err) {
  hipStream_t s = ctx->stream;
  TCHK(hipSetDevice(ctx->device));
  TCHK(hipEventSynchronize(ctx->ev[1]));
  RefCache& rc = ctx->refc;
  const bool hit = rc.hit_ovl;  // the one group's map is the cached reference's (ctx->bitmap[0, rc.od.bytes))
  if (ctx->opt.overlap_path == 1) {  // the sorted-key path for every batch (tests)
    rc.ovl = false;
    return overlap_sparse(ctx, B, P, G, dDesc, dState, dGst, readS, res, set_ratio, err);
  }
  // one map per overlap group (reference side) and one per pair (reading side), each over
  // the padded key box of that cloud's keys and origin; the groups' maps first, so a cached
  // reference's map keeps its place at offset 0
  uint64_t bm_bytes = 0;
  TCHK(ensure(ctx->pin_ovl, (P + G) * sizeof(OvlDesc)));
  TCHK(ensure(ctx->ovl, (P + G) * sizeof(OvlDesc)));
  OvlDesc* ho = ctx->pin_ovl.as<OvlDesc>();
  auto size_map = [&](const PairState& hs, OvlDesc& o) -> bool {
    const int br[3] = {kOvlBrick0, kOvlBrick1, kOvlBrick2};
    for (int k = 0; k < 3; ++k) ovl_axis(hs.ovl_bbox[k], hs.ovl_bbox[3 + k], br[k], o.min[k], o.dim[k]);
    const uint64_t vox = ovl_bytes(o.dim);
    o.bytes = vox;
    o.off = bm_bytes;
    bm_bytes += o.bytes;
    return vox <= (1ull << 34);
  };
  bool fits = true;
  if (hit) {
    ho[P] = rc.od;
    bm_bytes = rc.od.bytes;
  } else {
    for (size_t g = 0; g < G; ++g) fits &= size_map(ctx->pin_gstate.as<PairState>()[g], ho[P + g]);
  }
  const uint64_t ref_bytes = bm_bytes;
  for (size_t i = 0; i < P; ++i) fits &= size_map(ctx->pin_state.as<PairState>()[i], ho[i]);
  // all maps of the batch at once within half the free device memory (beyond what the arena
  // already holds); otherwise (far outlier points: key boxes of 10^9+ voxels) the sorted-key path
  size_t free_b = 0, total_b = 0;
  TCHK(hipMemGetInfo(&free_b, &total_b));
  const uint64_t limit = std::min<uint64_t>(ctx->bitmap.cap + free_b / 2, kDenseMapBudget);
  if (!fits || bm_bytes > limit) {  // (a cached group state is in dGst; the sparse path recounts |A|)
    rc.ovl = false;
    return overlap_sparse(ctx, B, P, G, dDesc, dState, dGst, readS, res, set_ratio, err);
  }
  if (hit && bm_bytes > ctx->bitmap.cap) {  // grow, keeping the cached map
    DevBuf nb;
    hipError_t e = ensure(nb, bm_bytes);
    if (e == hipSuccess) e = hipMemcpyAsync(nb.p, ctx->bitmap.p, ref_bytes, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) release(nb);  // (a DevBuf is not released by its destructor)
    TCHK(e);
    release(ctx->bitmap);
    ctx->bitmap = nb;
  }
  TCHK(ensure(ctx->bitmap, bm_bytes));
  TCHK(hipMemcpyAsync(ctx->ovl.p, ho, (P + G) * sizeof(OvlDesc), hipMemcpyHostToDevice, s));
  TCHK(hipEventRecord(ctx->ev[6], s));
  uint8_t* bm = ctx->bitmap.as<uint8_t>();
  const OvlDesc* dOvl = ctx->ovl.as<OvlDesc>();
  // the marks' LDS cache of stored voxels pays off where many rays share the maps (C5: 66 against
  // 111 GB written per dispatch); a few clouds mark faster with plain stores (the
  // stream's measurement)
  const bool filter = P + G > 8;
  if (hit) {  // the readings' maps only: the reference's map and |A| are the cached ones
    TCHK(hipMemsetAsync(bm + ref_bytes, 0, bm_bytes - ref_bytes, s));
    launch_ovl_mark(s, B->m_read, dDesc, dOvl, dState, readS, 1, res, bm, filter);
    launch_ovl_popcount(s, (int)P, dOvl, dState, 1, bm, P == 1);
    launch_ovl_intersect(s, (int)P, dDesc, dOvl, dOvl + P, dState, bm, P == 1);
    ++rc.ovl_hits;
  } else {
    TCHK(hipMemsetAsync(bm, 0, bm_bytes, s));
    launch_ovl_mark(s, B->m_gref, dG, dOvl + P, dGst, B->ref_raw.as<float4>(), 0, res, bm, filter);
    launch_ovl_mark(s, B->m_read, dDesc, dOvl, dState, readS, 1, res, bm, filter);
    launch_ovl_count(s, (int)P, (int)G, dDesc, dOvl, dOvl + P, dState, dGst, bm);
    rc.ovl = false;
    if (rc.use && G == 1) {  // keep the reference's map (offset 0) and its group state for the next call
      TCHK(ensure(rc.gst, sizeof(PairState)));
      TCHK(hipMemcpyAsync(rc.gst.p, dGst, sizeof(PairState), hipMemcpyDeviceToDevice, s));
      rc.ovl = true;
      rc.od = ho[P];
      rc.res = res;
      for (int k = 0; k < 3; ++k) rc.origin[k] = B->gdesc[0].ref_origin[k];
      ++rc.ovl_builds;
    }
  }
  launch_ovl_finish(s, (int)P, dDesc, dState, dGst, set_ratio ? 1 : 0);
  TCHK(hipGetLastError());
  return AICP_OK;
}

// the centred reference's matcher tree and the pairs' frames, on stream3 (worker thread)
int matcher_trees(aicp_hip_ctx* ctx, aicp_hip_batch* B, int bucket, PairDesc* dDesc, PairDesc* dRdesc,
                  int plan, std::string& err, hipEvent_t after = nullptr) {
  hipStream_t s3 = ctx->stream3;
  const size_t R = B->rdesc.size();
  TCHK(hipSetDevice(ctx->device));  // the current device is per host thread
  TCHK(hipStreamWaitEvent(s3, ctx->ev[14], 0));  // the reference points are on the device
  TCHK(hipEventRecord(ctx->ev[12], s3));
  TCHK(hipMemcpyAsync(dRdesc, ctx->pin_rdesc.p, R * sizeof(PairDesc), hipMemcpyHostToDevice, s3));
  if (after) TCHK(hipStreamWaitEvent(s3, after, 0));  // the raw tree first (raw_tree_first())
  int rc = device_trees_begin(ctx->tb[1], err, s3, R, B->total_ref, dRdesc, B->ref_raw.as<float4>(), 1, bucket,
                              ctx->bpts, ctx->nodes);
  if (rc) return rc;
  rc = device_trees_end(ctx->tb[1], err, s3, R, B->total_ref, dRdesc, bucket, ctx->bpts, ctx->nodes, plan);
  if (rc) return rc;
  // treelet records of the matcher trees (Trav2C), then the control block again: the treelet check
  // reports into its error word, checked after the batch
  if (ctx->tl_total) {
    const uint32_t cap = (uint32_t)(2 * B->total_ref + 2);  // node records allotted
    TCHK(ensure(ctx->tl, ctx->tl_total * 16));
    TCHK(ensure(ctx->ptl, ctx->tl_total * 8));  // treelet links {parent, grandparent}
    TCHK(ensure(ctx->tl_rank, ((size_t)cap + 1) * 4));
    TreeBufs& T = ctx->tb[1];
    TCHK(launch_treelets(s3, (int)R, cap, dRdesc, ctx->nodes.as<uint4>(), bucket, ctx->tl_rank.as<uint32_t>(),
                         ctx->tl.as<uint4>(), ctx->ptl.as<uint2>(), T.tw));
    TCHK(hipMemcpyAsync(T.pin_ctl.p, T.tw.ctl, sizeof(TreeCtl), hipMemcpyDeviceToHost, s3));
  }
  TCHK(hipStreamWaitEvent(s3, ctx->ev[7], 0));  // the pairs' descriptors are on the device
  launch_pairs_from_refs(s3, (int)B->P, dDesc, dRdesc);
  TCHK(hipEventRecord(ctx->ev[3], s3));
  return AICP_OK;
}

// aicp_hip_options::raw_tree_first 0/1 forces the order; by default batches of >= 4 M reference
// points build the raw tree first
bool raw_tree_first(uint64_t total_ref, const aicp_hip_options& o) {
  return o.raw_tree_first >= 0 ? o.raw_tree_first > 0 : total_ref >= (4ull << 20);
}

// With the raw tree first, the matcher tree starts when the raw tree's global levels and mid-size
// segments are done (2, default: its bandwidth-bound levels beside the raw tree's latency-bound
// subtree kernel) or when the whole raw tree is (raw_first_at = 1: the normals' kNN, launched
// at the same time, then holds every wave slot and the matcher kernels wait behind it). C5, same
// box, alternating: 3578 / 3494 (2) against 3409 / 3265 (1) and 3244 / 3352 clouds/s (both trees
// together). Also measured: the normals' kNN waiting for the matcher tree's mid-size segments
// (k_tr_mid needs most of a CU's LDS per workgroup and starves behind the persistent kNN):
// 3420 / 3368 against 3495 / 3433.

double ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0;
  return ms;
}

int run_batch(aicp_hip_ctx* ctx, aicp_hip_batch* B, const aicp_icp_config* cfg, double res,
              int flags, float* outT, aicp_icp_stats* stats, float* out_overlap) {
  const auto t_start = std::chrono::steady_clock::now();
  int rc = check_cfg(ctx, cfg, flags);
  if (rc) return rc;
  const bool doOvl = flags & AICP_RUN_OVERLAP, doIcp = flags & AICP_RUN_ICP;
  if (doOvl && !(res > 0)) FAIL(AICP_ERR_INVALID, "resolution");
  const size_t P = B->P;
  RefCache& rcache = ctx->refc;
  if (!rcache.use) rcache.invalidate();  // (this run rewrites the buffers a cached reference lives in)
  const bool read_hit = ctx->rdc.hit;
  if (!read_hit) ctx->rdc.valid = false;  // (read_s is rewritten below; oneshot() re-validates)
  const bool hit_trees = rcache.use && rcache.hit_trees && doIcp;
  const bool hit_ovl = rcache.use && rcache.hit_ovl && doOvl;
  hipStream_t s = ctx->stream;
  // the events that order this context's streams release at device scope; ev[1], which the host
  // waits on before it reads the key boxes copied to pinned memory, keeps the system-scope fence
  for (size_t k = 0; k < sizeof(ctx->ev) / sizeof(ctx->ev[0]); ++k)
    if (!ctx->ev[k]) HIPC(hipEventCreateWithFlags(&ctx->ev[k], k == 1 ? hipEventDefault : hipEventReleaseToDevice));
  const bool timeNN = (flags & AICP_RUN_TIME_NN) && doIcp;
  if (timeNN)
    while ((int)ctx->nn_ev.size() < 2 * cfg->max_iter) {
      hipEvent_t e;
      // timing only (the NN launch's own start / end): no system-scope fence, whose cache
      // write-back and invalidation the elapsed time would otherwise include
      HIPC(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
      ctx->nn_ev.push_back(e);
    }
  std::vector<PairDesc> desc = B->desc;
  for (auto& d : desc) d.ratio = cfg->trimmed_ratio;
  HIPC(ensure(ctx->desc, P * sizeof(PairDesc)));
  HIPC(ensure(ctx->state, P * sizeof(PairState)));
  if (P > (size_t)kMaxPairs) FAIL(AICP_ERR_UNSUPPORTED, "more than 4096 pairs in one batch");
  {
    uint64_t nr = 0;
    for (const PairDesc& d : desc) nr += d.n_read;
    HIPC(ensure(ctx->active, active_list_bytes(nr, P)));
  }
  HIPC(ensure(ctx->ctrs, kCtrWords * 4));
  HIPC(ensure(ctx->pin_desc, 3 * P * sizeof(PairDesc)));
  HIPC(ensure(ctx->pin_state, P * sizeof(PairState)));
  HIPC(ensure(ctx->outT, P * 64));
  HIPC(ensure(ctx->pin_out, P * 64));
  PairDesc* pdA = ctx->pin_desc.as<PairDesc>();
  PairDesc* pdB = pdA + P;
  PairDesc* pdC = pdB + P;  // device descriptors read back at the end
  PairDesc* dDesc = ctx->desc.as<PairDesc>();
  PairState* dState = ctx->state.as<PairState>();
  uint32_t* dCtr = ctx->ctrs.as<uint32_t>();
  // Two streams: s runs the overlap (bbox -> host sizes the voxel maps -> marking -> counts ->
  // ratio), s2 the centroid, kd-trees, reading frame and normals; s joins s2 before the loop.
  hipStream_t s2 = ctx->stream2;
  std::memcpy(pdA, desc.data(), P * sizeof(PairDesc));
  HIPC(hipEventRecord(ctx->ev[0], s));
  HIPC(hipMemcpyAsync(dDesc, pdA, P * sizeof(PairDesc), hipMemcpyHostToDevice, s));
  launch_init_state(s, (int)P, dDesc, dState);
  HIPC(hipEventRecord(ctx->ev[7], s));
  if (!B->refs_event) HIPC(hipEventRecord(ctx->ev[14], s));
  B->refs_event = false;  // (a later run of the same batch records it here)
  // readings in Morton order inside each pair's range (kernels_order.hip): the overlap and
  // the ICP loop both visit the sorted copy
  const float4* readS = B->read_raw.as<float4>();
  // Morton order from read_order_min (200000) reading points on: a single C2 reading's NN launches
  // gain less than its sort costs (the app bench, r05: 1.18-1.25 ms per overlap + registerClouds
  // without, 1.29-1.37 with)
  const bool order = B->total_read >= ctx->opt.read_order_min;
  if (read_hit) {  // the previous one-shot call's reading: its Morton-ordered copy is in read_s
    if (ctx->rdc.sorted) readS = ctx->read_s.as<float4>();
  } else if (!order) {
    ctx->rdc.sorted = false;
  } else {
    ctx->rdc.sorted = true;
    const size_t n = B->total_read;
    const size_t tb = read_order_temp_bytes(n, (int)P);
    HIPC(ensure(ctx->read_s, n * 16));
    HIPC(ensure(ctx->ord_k0, n * 8));
    HIPC(ensure(ctx->ord_k1, n * 8));
    HIPC(ensure(ctx->ord_v0, n * 4));
    HIPC(ensure(ctx->ord_v1, n * 4));
    HIPC(ensure(ctx->ord_tmp, tb));
    HIPC(launch_read_order(s, B->m_read, (int)P, dDesc, B->read_raw.as<float4>(), (uint32_t)n,
                           ctx->ord_k0.as<uint64_t>(), ctx->ord_k1.as<uint64_t>(), ctx->ord_v0.as<uint32_t>(),
                           ctx->ord_v1.as<uint32_t>(), ctx->ord_tmp.p, tb, ctx->read_s.as<float4>()));
    readS = ctx->read_s.as<float4>();
  }
  HIPC(hipEventRecord(ctx->ev[11], s));
  const size_t G = B->gdesc.size();
  PairDesc* dG = nullptr;
  PairState* dGst = nullptr;
  if (doOvl) {
    HIPC(ensure(ctx->gdesc, G * sizeof(PairDesc)));
    HIPC(ensure(ctx->gstate, G * sizeof(PairState)));
    HIPC(ensure(ctx->pin_gdesc, G * sizeof(PairDesc)));
    HIPC(ensure(ctx->pin_gstate, G * sizeof(PairState)));
    dG = ctx->gdesc.as<PairDesc>();
    dGst = ctx->gstate.as<PairState>();
    std::memcpy(ctx->pin_gdesc.p, B->gdesc.data(), G * sizeof(PairDesc));
    HIPC(hipMemcpyAsync(dG, ctx->pin_gdesc.p, G * sizeof(PairDesc), hipMemcpyHostToDevice, s));
    launch_ovl_init(s, (int)P, dDesc, dState, res, 2);
    if (hit_ovl) {  // the cached reference's group state (|A|, key box): its map is kept too
      HIPC(hipMemcpyAsync(dGst, rcache.gst.p, sizeof(PairState), hipMemcpyDeviceToDevice, s));
    } else {
      launch_ovl_init(s, (int)G, dG, dGst, res, 1);
      launch_ovl_bbox(s, B->m_gref, dG, dGst, B->ref_raw.as<float4>(), 0, res);
    }
    launch_ovl_bbox(s, B->m_read, dDesc, dState, readS, 1, res);
    HIPC(hipMemcpyAsync(ctx->pin_state.p, dState, P * sizeof(PairState), hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(ctx->pin_gstate.p, dGst, G * sizeof(PairState), hipMemcpyDeviceToHost, s));
  }
  HIPC(hipEventRecord(ctx->ev[1], s));
  // s2: per distinct reference: centroid, centred cloud, root segments (the levels follow
  // once the overlap is queued)
  const size_t R = B->rdesc.size();
  PairDesc* dRdesc = nullptr;
  PairState* dRstate = nullptr;
  std::thread worker;
  int wrc = AICP_OK;
  std::string werr;
  struct Joiner {  // every return after the worker started joins it (std::thread must not leak)
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } joiner{worker};
  auto join_worker = [&](int r) {
    if (worker.joinable()) worker.join();
    if (!r && wrc) {
      ctx->err = werr;
      r = wrc;
    }
    return r;
  };
  // the overlap's map sizing and marking (stream s), on its own host thread when the trees are
  // queued too
  std::thread ovl_thread;
  int orc = AICP_OK;
  std::string oerr;
  Joiner ojoiner{ovl_thread};
  auto join_ovl = [&](int r) {
    if (ovl_thread.joinable()) ovl_thread.join();
    if (!r && orc) {
      ctx->err = oerr;
      r = orc;
    }
    return r;
  };
  if (doOvl && doIcp)
    ovl_thread = std::thread([&] { orc = overlap_maps(ctx, B, P, G, dDesc, dState, dG, dGst, readS, res, true, oerr); });
  if (doIcp && hit_trees) {
    // the cached reference's centroid, trees, treelets and normals (ctx->rdesc / rstate / bpts /
    // bnrm / nodes / tl / ptl) serve this call: only the pairs' frames are new (below)
    ctx->tl_total = rcache.tl_total;
    dRdesc = ctx->rdesc.as<PairDesc>();
    dRstate = ctx->rstate.as<PairState>();
    for (int e : {8, 10, 12, 3}) HIPC(hipEventRecord(ctx->ev[e], s2));
    ++rcache.tree_hits;
  } else if (doIcp) {
    HIPC(ensure(ctx->rdesc, R * sizeof(PairDesc)));
    HIPC(ensure(ctx->rstate, R * sizeof(PairState)));
    HIPC(ensure(ctx->pin_rdesc, R * sizeof(PairDesc)));
    dRdesc = ctx->rdesc.as<PairDesc>();
    dRstate = ctx->rstate.as<PairState>();
    std::memcpy(ctx->pin_rdesc.p, B->rdesc.data(), R * sizeof(PairDesc));
    // matcher treelet records allotted per reference (kernels_tree.hip: at most 1 + 4 per inner
    // node at even depth); leaf slots hold a 4-bit count, so larger buckets use Trav<1>
    ctx->tl_total = 0;
    if (cfg->bucket_size <= 15) {
      for (size_t r = 0; r < R; ++r) {
        PairDesc& rd = ctx->pin_rdesc.as<PairDesc>()[r];
        rd.tl_off = (uint32_t)ctx->tl_total;
        rd.tl_cap = (uint32_t)(4 * (uint64_t)rd.n_ref + 4);
        ctx->tl_total += rd.tl_cap;
      }
      if (ctx->tl_total >= (1ull << 28)) ctx->tl_total = 0;  // 32-bit byte offsets do not fit: Trav<1>
      // the NN kernel's LDS frames keep a node id (< 16 * (n_ref + 1)) in 26 bits
      for (size_t r = 0; r < R; ++r)
        if (ctx->pin_rdesc.as<PairDesc>()[r].n_ref > 4000000u) ctx->tl_total = 0;
      if (ctx->opt.nn_engine == 1) ctx->tl_total = 0;
    }
    HIPC(ensure(ctx->rdesc_raw, R * sizeof(PairDesc)));
    HIPC(hipStreamWaitEvent(s2, ctx->ev[14], 0));  // the reference points (not the readings) are on the device
    HIPC(hipEventRecord(ctx->ev[8], s2));
    HIPC(hipMemcpyAsync(ctx->rdesc_raw.p, ctx->pin_rdesc.p, R * sizeof(PairDesc), hipMemcpyHostToDevice, s2));
    launch_init_state(s2, (int)R, ctx->rdesc_raw.as<PairDesc>(), dRstate);
    uint64_t n_ref_max = 0;
    for (const PairDesc& r : B->rdesc) n_ref_max = std::max<uint64_t>(n_ref_max, r.n_ref);
    // s3 (worker thread; it still polls its levels in a polled redo): centroid, centred
    // reference, matcher tree, pair frames
    const int plan1 = plan_levels(n_ref_max, ctx->tb[1], ctx->opt.tree_plan);
    // Large batches build the raw tree first and the matcher tree beside the normals' kNN
    // (raw_tree_first()): the raw tree gates the kNN, which gates the loop, while the matcher
    // tree is needed only by the loop; built together, the two trees' latency-bound subtree
    // kernels share the CUs' wave slots and both finish late.
    const bool raw_first = raw_tree_first(B->total_ref, ctx->opt);
    if (!raw_first)
      worker = std::thread([&, plan1] { wrc = matcher_trees(ctx, B, cfg->bucket_size, dDesc, dRdesc, plan1, werr); });
    // SurfaceNormal runs on the reference as given, before the centring (ICP::compute,
    // SURVEY A.1 steps 1-2): its own libnabo tree over the raw coordinates first
    rc = device_trees_begin(ctx->tb[0], ctx->err, s2, R, B->total_ref, ctx->rdesc_raw.as<PairDesc>(),
                            B->ref_raw.as<float4>(), 0, kNormalsBucket, ctx->bpts_raw, ctx->nodes_raw);
    if (rc) return join_worker(rc);
    // s2: raw tree levels + subtrees, SurfaceNormal, all enqueued before the host waits for
    // the overlap's key boxes
    const int rf = ctx->opt.raw_first_at;
    rc = device_trees_end(ctx->tb[0], ctx->err, s2, R, B->total_ref, ctx->rdesc_raw.as<PairDesc>(), kNormalsBucket,
                          ctx->bpts_raw, ctx->nodes_raw, plan_levels(n_ref_max, ctx->tb[0], ctx->opt.tree_plan, true), nullptr, true,
                          raw_first && rf == 2 ? ctx->ev[13] : nullptr);
    if (rc) return join_worker(rc);
    if (raw_first) {
      if (rf != 2) HIPC(hipEventRecord(ctx->ev[13], s2));
      worker = std::thread(
          [&, plan1] { wrc = matcher_trees(ctx, B, cfg->bucket_size, dDesc, dRdesc, plan1, werr, ctx->ev[13]); });
    }
    // normals on the raw tree (bucket order of that tree)
    HIPC(ensure(ctx->nrm_raw, B->total_ref * 16));
    HIPC(ensure(ctx->nbids, B->total_ref * 4 * (size_t)cfg->knn_normals));
    uint32_t* nCtr = dCtr + kKnnCtrOff;
    if (!launch_normals(s2, (int)R, (uint32_t)B->total_ref, ctx->rdesc_raw.as<PairDesc>(), dRstate,
                        ctx->nodes_raw.as<uint4>(), nullptr, ctx->bpts_raw.as<float4>(), ctx->nrm_raw.as<float4>(),
                        cfg->knn_normals, ctx->nbids.as<int32_t>(), nCtr, ctx->opt.normals_knn_engine))
      FAIL(AICP_ERR_UNSUPPORTED, "normals knn");
    HIPC(hipEventRecord(ctx->ev[10], s2));
  }
  if (doOvl) {
    rc = join_ovl(doIcp ? AICP_OK : overlap_maps(ctx, B, P, G, dDesc, dState, dG, dGst, readS, res, false, oerr));
    if (!doIcp && rc) ctx->err = oerr;
    if (rc) return join_worker(rc);
  }
  HIPC(hipEventRecord(ctx->ev[2], s));
  IcpParams prm{};
  int nn_launches = 0;
  if (doIcp) {
    // the matcher tree (s3) must be complete, and the worker done with ctx->bpts / nodes
    rc = join_worker(AICP_OK);
    if (rc) return rc;
    HIPC(hipStreamWaitEvent(s2, ctx->ev[3], 0));
    HIPC(ensure(ctx->read_c, B->total_read * 16));
    HIPC(ensure(ctx->bpts, B->total_ref * 16));
    HIPC(ensure(ctx->bnrm, B->total_ref * 16));
    HIPC(ensure(ctx->match, B->total_read * 4));
    HIPC(ensure(ctx->d2, B->total_read * 4));
    HIPC(ensure(ctx->touch, B->total_read * 4));
    HIPC(ensure(ctx->slab, (size_t)B->n_red_total * kRedCols * 8));
    HIPC(ensure(ctx->sel_hist, P * kHistBins * 4));
    HIPC(ensure(ctx->sel_cand, B->total_read * 4));
    HIPC(ensure(ctx->sel_cnt, P * 4));
    HIPC(hipMemsetAsync(ctx->sel_hist.p, 0, P * kHistBins * 4, s));
    HIPC(hipMemsetAsync(ctx->sel_cnt.p, 0, P * 4, s));
    HIPC(ensure(ctx->isync, icp_sync_words(P) * 4));
    HIPC(hipMemsetAsync(ctx->isync.p, 0, icp_sync_words(P) * 4, s));
    float4* bpts = ctx->bpts.as<float4>();
    float4* bnrm = ctx->bnrm.as<float4>();
    float4* readc = ctx->read_c.as<float4>();
    const uint4* nodes = ctx->nodes.as<uint4>();
    HIPC(hipStreamWaitEvent(s2, ctx->ev[11], 0));
    if (hit_trees) launch_pairs_from_refs(s2, (int)P, dDesc, dRdesc);  // (the matcher worker's step)
    launch_prepare_read(s2, B->m_read, dDesc, readS, readc);
    // normals from the raw tree's bucket order into the matcher tree's bucket order (a cached
    // reference's are there already)
    HIPC(ensure(ctx->inv, B->total_ref * 4));
    if (!hit_trees)
      launch_normals_to_matcher(s2, (int)R, (uint32_t)B->total_ref, dRdesc, bpts, ctx->bpts_raw.as<float4>(),
                                ctx->nrm_raw.as<float4>(), ctx->inv.as<uint32_t>(), bnrm);
    launch_pairs_degenerate(s2, (int)P, dDesc, dState, dRstate);
    HIPC(hipEventRecord(ctx->ev[4], s2));
    HIPC(hipStreamWaitEvent(s, ctx->ev[4], 0));
    HIPC(hipEventRecord(ctx->ev[9], s));
    prm.maxE2 = (1 + cfg->nn_epsilon) * (1 + cfg->nn_epsilon);
    prm.maxR2 = cfg->nn_max_dist * cfg->nn_max_dist;
    prm.max_iter = cfg->max_iter;
    prm.smooth = cfg->smooth_length;
    prm.min_rot = cfg->min_diff_rot;
    prm.min_trans = cfg->min_diff_trans;
    prm.knn_normals = cfg->knn_normals;
    // The ICP loop on s: per iteration the NN, then select + reduce with the per-pair steps and
    // the next active list inside (launch_icp_select_f / _reduce_f)
    uint32_t reads = 0, max_read = 0;
    for (size_t i = 0; i < P; ++i) {
      reads += B->desc[i].n_read;
      max_read = std::max(max_read, B->desc[i].n_read);
    }
    ActiveList* al = ctx->active.as<ActiveList>();
    const int sel_ff = ctx->opt.select_fused_from;
    const bool sel_pair = sel_pair_fits(P, max_read, ctx->opt.select_pair);
    // Polled loop (the sequence's, sequence.cpp): from iteration smoothLength on the update of
    // the last pair writes the next active count into mapped host memory; the host stays one
    // iteration ahead and stops enqueueing once it reads 0, instead of maxIterationCount launches
    // of which the ones after convergence are no-ops (~25 us each).
    if (!ctx->poll_host) {
      HIPC(hipHostMalloc((void**)&ctx->poll_host, kBatchPolls * 4, hipHostMallocMapped));
      HIPC(hipHostGetDevicePointer((void**)&ctx->poll_dev, ctx->poll_host, 0));
    }
    const bool early = !ctx->opt.no_early_exit;
    auto polled = [&](int k) { return early && k >= cfg->smooth_length && k < kBatchPolls && k < cfg->max_iter; };
    // every iteration's active count is written (not only the polled ones'), so the words written
    // so far are a prefix and its last word tells whether more will come (see sequence.cpp, loop_poll)
    auto written = [&](int k) { return early && k < kBatchPolls; };
    std::deque<int> pending;
    bool stop = false;
    for (int it = 0; it < cfg->max_iter && !stop; ++it) {
      // every poll slot before this iteration read: its active count was not 0
      while (!pending.empty() && pending.front() < it && !stop) {
        const int k = pending.front();
        volatile uint32_t* w = ctx->poll_host;
        const auto t0 = std::chrono::steady_clock::now();
        while (w[k] == 0xffffffffu) {
          // the last word written so far is 0: no launch after it had an active pair, so this one
          // stays unwritten (no hipStreamQuery on the way: it enqueues a marker the next kernel
          // waits behind)
          int m = k - 1;
          while (m >= 0 && w[m] == 0xffffffffu) --m;
          if (m >= 0 && w[m] == 0u) break;
          if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) {
            const hipError_t q = hipStreamQuery(s);  // (a stream that drained without writing it)
            if (q != hipErrorNotReady) {
              HIPC(q);
              std::atomic_thread_fence(std::memory_order_seq_cst);
              break;
            }
          }
          std::this_thread::yield();
        }
        stop = w[k] == 0u || w[k] == 0xffffffffu;
        pending.pop_front();
      }
      if (stop) break;
      if (it == 0) {
        uint32_t* hn0 = nullptr;
        if (written(0)) {
          ctx->poll_host[0] = 0xffffffffu;
          hn0 = ctx->poll_dev;
        }
        launch_active_list(s, (int)P, dDesc, dState, al, dCtr, hn0);
      }
      prm.prof_slot = nn_launches;
      launch_icp_nn(s, (int)reads, dDesc, dState, al, readc, nodes, ctx->tl_total ? ctx->tl.as<uint4>() : nullptr,
                    nullptr, bpts, ctx->tl_total ? ctx->ptl.as<uint2>() : nullptr, ctx->match.as<int32_t>(),
                    ctx->d2.as<float>(), ctx->touch.as<uint32_t>(), dCtr, prm,
                    timeNN ? ctx->nn_ev[2 * nn_launches] : nullptr, timeNN ? ctx->nn_ev[2 * nn_launches + 1] : nullptr);
      HIPC(hipGetLastError());
      ++nn_launches;
      IcpIterSync y = icp_sync_layout(ctx->isync.as<uint32_t>(), P, 0);
      y.np = (int)P;
      y.pd = dDesc;
      y.st = dState;
      y.al = al;
      y.ctr = dCtr;
      if (written(it + 1)) {
        ctx->poll_host[it + 1] = 0xffffffffu;  // (before the launch that writes it)
        y.host_n = ctx->poll_dev + it + 1;
        if (polled(it + 1)) pending.push_back(it + 1);
      }
      if (sel_pair)
        launch_icp_select_pair(s, (int)P, dDesc, dState, ctx->d2.as<float>(), ctx->sel_cand.as<uint32_t>(), y);
      else if (sel_ff > 0 && it >= sel_ff)
        launch_icp_select_fused(s, B->m_sel, dDesc, dState, ctx->d2.as<float>(), ctx->sel_hist.as<uint32_t>(),
                                ctx->sel_cand.as<uint32_t>(), ctx->sel_cnt.as<uint32_t>(), y);
      else
        launch_icp_select_f(s, B->m_sel, dDesc, dState, ctx->d2.as<float>(), ctx->sel_hist.as<uint32_t>(),
                            ctx->sel_cand.as<uint32_t>(), ctx->sel_cnt.as<uint32_t>(), y);
      launch_icp_reduce_f(s, B->m_red, dDesc, dState, readc, ctx->match.as<int32_t>(), ctx->d2.as<float>(),
                          ctx->touch.as<uint32_t>(), bpts, bnrm, ctx->slab.as<double>(), prm, y);
    }
    launch_finalize(s, (int)P, dDesc, dState, ctx->outT.as<float>());
    if (ctx->opt.profile) {  // the diagnostic build's counters (-DAICP_DIAG=1)
      HIPC(hipStreamSynchronize(s));
      nn_prof_dump();
      tree_prof_dump();
    }
  } else {
    HIPC(hipEventRecord(ctx->ev[8], s));
    HIPC(hipEventRecord(ctx->ev[10], s));
    HIPC(hipEventRecord(ctx->ev[12], s));
    HIPC(hipEventRecord(ctx->ev[3], s));
    HIPC(hipEventRecord(ctx->ev[4], s));
    HIPC(hipEventRecord(ctx->ev[9], s));
  }
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(ctx->ev[5], s));
  HIPC(hipMemcpyAsync(ctx->pin_state.p, dState, P * sizeof(PairState), hipMemcpyDeviceToHost, s));
  if (doIcp) HIPC(hipMemcpyAsync(ctx->pin_out.p, ctx->outT.p, P * 64, hipMemcpyDeviceToHost, s));
  HIPC(hipMemcpyAsync(pdC, dDesc, P * sizeof(PairDesc), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (doIcp && !hit_trees) {  // planned tree builds: errors recorded on the device
    rcache.trees = false;
    rc = device_trees_check(ctx->tb[0], ctx->err);
    if (!rc) rc = device_trees_check(ctx->tb[1], ctx->err);
    if (rc) return rc;
    if (ctx->tl_total && (ctx->tb[1].pin_ctl.as<TreeCtl>()->error & 4))
      FAIL(AICP_ERR_HIP, "matcher treelets exceed their allotment");
    if (rcache.use && R == 1) {  // kept for the next call against the same reference
      rcache.trees = true;
      rcache.bucket = cfg->bucket_size;
      rcache.knn = cfg->knn_normals;
      rcache.tl_total = ctx->tl_total;
      ++rcache.tree_builds;
    }
  }
  // results
  const PairState* hs = ctx->pin_state.as<PairState>();
  int first_err = AICP_OK;
  uint64_t queries = 0, tp = 0, tn = 0;
  for (size_t i = 0; i < P; ++i) {
    const PairState& st = hs[i];
    int status = st.status;
    if (doOvl && st.ovl_err && !status) status = AICP_ERR_HIP;
    if (status && !first_err) first_err = status;
    if (outT && doIcp) std::memcpy(outT + 16 * i, ctx->pin_out.as<float>() + 16 * i, 64);
    if (out_overlap) out_overlap[i] = st.overlap;
    queries += (uint64_t)st.iters * desc[i].n_read;
    const uint64_t ptp = st.touched_pts, ptn = st.touched_nodes;
    tp += ptp;
    tn += ptn;
    if (stats) {
      aicp_icp_stats& o = stats[i];
      std::memset(&o, 0, sizeof(o));
      o.status = status;
      o.iterations = st.iters;
      o.converged = st.converged;
      o.degenerate_normals = st.degenerate;
      o.inlier_ratio = st.inlier_ratio;
      o.trimmed_ratio = st.ratio;
      o.overlap_percent = st.overlap;
      o.tree_depth = pdC[i].tree_depth;
      o.nn_points_touched = ptp;
      o.nn_nodes_touched = ptn;
      for (int k = 0; k < 3; ++k) o.overlap_keys[k] = st.ovl_counts[k];
    }
  }
  ctx->last_nn_launches = timeNN ? nn_launches : 0;
  ctx->last_nn_ms = 0;
  if (timeNN)
    for (int it = 0; it < nn_launches; ++it) ctx->last_nn_ms += ev_ms(ctx->nn_ev[2 * it], ctx->nn_ev[2 * it + 1]);
  // N*(12 B query + 8 B id/d2) + V*16 B + W*8 B
  ctx->last_nn_bytes = timeNN ? (double)queries * 20.0 + (double)tp * 16.0 + (double)tn * 8.0 : 0.0;
  ctx->last_queries = queries;
  ctx->last_phase[0] = doOvl ? ev_ms(ctx->ev[0], ctx->ev[1]) + ev_ms(ctx->ev[6], ctx->ev[2]) : 0;
  // tree and normals run on the second stream, concurrently with the overlap
  // [1] raw-coordinate tree + SurfaceNormal (s2), [2] centroid + matcher tree (s3)
  ctx->last_phase[1] = doIcp ? ev_ms(ctx->ev[8], ctx->ev[10]) : 0;
  ctx->last_phase[2] = doIcp ? ev_ms(ctx->ev[12], ctx->ev[3]) : 0;
  ctx->last_phase[3] = doIcp ? ev_ms(ctx->ev[9], ctx->ev[5]) : 0;
  ctx->last_phase[4] =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  if (first_err) ctx->err = "pair status " + std::to_string(first_err);
  return first_err;
}

void free_batch(aicp_hip_batch* B) {
  if (!B) return;
  release(B->ref_raw);
  release(B->read_raw);
  release(B->maps);
  delete B;
}

// single-cloud kd-tree on the points as given (no centring) for the kernel-level entry points
int upload_tree(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, PairDesc& d) {
  hipStream_t s = ctx->stream;
  ctx->refc.invalidate();  // (ctx->bpts / nodes / bnrm are rewritten)
  HIPC(ensure(ctx->ref1, n * 16));
  HIPC(ensure(ctx->pin_io, n * 16));
  pack_xyz4(pts, n, stride, ctx->pin_io.as<float>());
  HIPC(hipMemcpyAsync(ctx->ref1.p, ctx->pin_io.p, n * 16, hipMemcpyHostToDevice, s));
  d = PairDesc{};
  d.n_ref = (uint32_t)n;
  d.ratio = 0.5f;
  ident4(d.Tin);
  HIPC(ensure(ctx->desc, sizeof(PairDesc)));
  HIPC(hipMemcpyAsync(ctx->desc.p, &d, sizeof(d), hipMemcpyHostToDevice, s));
  int rc = device_trees_begin(ctx->tb[0], ctx->err, s, 1, n, ctx->desc.as<PairDesc>(), ctx->ref1.as<float4>(), 0, 8,
                              ctx->bpts, ctx->nodes);
  if (rc) return rc;
  rc = device_trees_end(ctx->tb[0], ctx->err, s, 1, n, ctx->desc.as<PairDesc>(), 8, ctx->bpts, ctx->nodes, 0);
  if (rc) return rc;
  HIPC(hipMemcpyAsync(&d, ctx->desc.p, sizeof(d), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  return AICP_OK;
}

}  // namespace rt
}  // namespace aicp

extern "C" {

const char* aicp_hip_version(void) { return "aicp_hip 0.1 (gfx950)"; }

void aicp_hip_default_options(aicp_hip_options* o) {
  if (!o) return;
  *o = aicp_hip_options{};
  o->select_pair = -1;
  o->select_fused_from = 3;  // (iterations 1-2 missed the guessed bin on C2 2 times in 3, 3+ never: r05)
  o->raw_tree_first = -1;
  o->raw_first_at = 2;
  o->tree_lvl_min = 1u << 22;
  o->reference_cache = 1;
  o->oneshot_keep_mib = 4096;
  o->early_reference = 1;
  o->read_order_min = kReadOrderMin;
}

int aicp_hip_set_options(aicp_hip_ctx* ctx, const aicp_hip_options* o) {
  if (!ctx || !o) return AICP_ERR_INVALID;
  if (o->nn_engine < 0 || o->nn_engine > 1 || o->overlap_path < 0 || o->overlap_path > 1 ||
      o->normals_knn_engine < 0 || o->normals_knn_engine > 2 || o->select_pair < -1 || o->select_pair > 1 ||
      o->select_fused_from < 0 || o->raw_tree_first < -1 || o->raw_tree_first > 1 || o->raw_first_at < 1 ||
      o->raw_first_at > 2 || o->tree_plan < -1 || o->reference_cache < 0 || o->reference_cache > 1 ||
      o->early_reference < 0 || o->early_reference > 1)
    FAIL(AICP_ERR_INVALID, "aicp_hip_set_options: value out of range");
  // the reference cache was built under the previous options (engine, tree plan): drop it
  ctx->refc.invalidate();
  ctx->rdc.valid = false;
  ctx->opt = *o;
  for (auto& t : ctx->tb) tree_opts(t, ctx->opt);
  return AICP_OK;
}

int aicp_hip_get_options(const aicp_hip_ctx* ctx, aicp_hip_options* out) {
  if (!ctx || !out) return AICP_ERR_INVALID;
  *out = ctx->opt;
  return AICP_OK;
}

int aicp_hip_test_force_scan_stall(int on) { return set_lb_force_stall(on) == hipSuccess ? AICP_OK : AICP_ERR_HIP; }

int aicp_hip_create(int device, aicp_hip_ctx** out) {
  if (!out) return AICP_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return AICP_ERR_HIP;
  if (device < 0 || device >= n) return AICP_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return AICP_ERR_HIP;
  aicp_hip_ctx* c = new aicp_hip_ctx();
  c->device = device;
  aicp_hip_default_options(&c->opt);
  for (auto& t : c->tb) tree_opts(t, c->opt);
  // the overlap (stream) yields the CUs to the kd-tree streams, whose chains of short
  // level kernels are the critical path before the ICP loop
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  const int prio3 = prio_hi;  // (measured: stream 3 at the low priority is no faster)
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_lo) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, prio3) != hipSuccess) {
    for (hipStream_t q : {c->stream, c->stream2, c->stream3})
      if (q) (void)hipStreamDestroy(q);
    delete c;
    return AICP_ERR_HIP;
  }
  *out = c;
  return AICP_OK;
}

void aicp_hip_destroy(aicp_hip_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  for (DevBuf* b : {&ctx->read_s, &ctx->ord_k0, &ctx->ord_k1, &ctx->ord_v0, &ctx->ord_v1, &ctx->ord_tmp, &ctx->read_c, &ctx->bpts, &ctx->bnrm, &ctx->nodes, &ctx->match, &ctx->d2, &ctx->desc,
                    &ctx->state, &ctx->touch, &ctx->slab, &ctx->bitmap, &ctx->outT, &ctx->scratch, &ctx->active,
                    &ctx->ctrs, &ctx->nbids, &ctx->ref1, &ctx->sel_hist, &ctx->sel_cand, &ctx->sel_cnt,
                    &ctx->qmap, &ctx->ovl, &ctx->rdesc, &ctx->rstate, &ctx->rdesc_raw, &ctx->bpts_raw,
                    &ctx->nodes_raw, &ctx->nrm_raw, &ctx->inv, &ctx->gdesc, &ctx->gstate, &ctx->tl, &ctx->ptl,
                    &ctx->tl_rank, &ctx->pf_a, &ctx->pf_b, &ctx->pf_bpts, &ctx->pf_nodes})
    release(*b);
  for (auto& t : ctx->tb) t.release_all();
  free_batch(ctx->oneshot);
  free_batch(ctx->mapbatch);
  release(ctx->crop_ws);
  release(ctx->ovl_sp);
  release(ctx->ovl_keys);
  release(ctx->isync);
  release(ctx->refc.gst);
  release(ctx->pin_crop);
  release(ctx->pin_maps);
  if (ctx->poll_host) (void)hipHostFree(ctx->poll_host);
  delete ctx->pool;
  seq_state_free(ctx->seq);
  for (PinBuf* b : {&ctx->pin_desc, &ctx->pin_state, &ctx->pin_out, &ctx->pin_io, &ctx->pin_ovl,
                    &ctx->pin_rdesc, &ctx->pin_gdesc, &ctx->pin_gstate, &ctx->pin_pf})
    release(*b);
  for (auto e : ctx->nn_ev) (void)hipEventDestroy(e);
  for (auto e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : ctx->pf_ev)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(ctx->stream);
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->stream3) (void)hipStreamDestroy(ctx->stream3);
  delete ctx;
}

const char* aicp_hip_last_error(const aicp_hip_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int aicp_hip_batch_upload(aicp_hip_ctx* ctx, const aicp_pair* pairs, size_t n_pairs, aicp_hip_batch** out) {
  if (!ctx || !out) return AICP_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  aicp_hip_batch* B = new aicp_hip_batch();
  const int rc = upload_pairs(ctx, pairs, n_pairs, B, false);
  if (rc) {
    free_batch(B);
    *out = nullptr;
    return rc;
  }
  *out = B;
  return AICP_OK;
}

void aicp_hip_batch_free(aicp_hip_ctx* ctx, aicp_hip_batch* batch) {
  if (ctx) (void)hipStreamSynchronize(ctx->stream);
  free_batch(batch);
}

int aicp_hip_batch_run(aicp_hip_ctx* ctx, aicp_hip_batch* batch, const aicp_icp_config* cfg, double resolution,
                       int flags, float* out_T, aicp_icp_stats* stats) {
  if (!ctx || !batch) return AICP_ERR_INVALID;
  if (!(flags & (AICP_RUN_ICP | AICP_RUN_OVERLAP))) FAIL(AICP_ERR_INVALID, "nothing to run");
  HIPC(hipSetDevice(ctx->device));
  return run_batch(ctx, batch, cfg, resolution, flags, out_T, stats, nullptr);
}


namespace {

// x, y, z of n points at a byte stride == packed[3 n], byte for byte; split over host threads for
// large clouds (a C2 reference is ~2 MB to read on every call)
bool same_points(WorkerPool* pool, const float* pts, uint64_t n, uint64_t stride, const float* packed) {
  // bitwise equality (NaN payloads included): one memcmp of the range for packed xyz rows, else the
  // XOR of the three words of every row OR-ed together (no branch per point: vectorised)
  auto cmp = [&](uint64_t a, uint64_t b) {
    const char* src = reinterpret_cast<const char*>(pts);
    if (stride == 12) return std::memcmp(src + a * 12, packed + 3 * a, (b - a) * 12) == 0;
    uint32_t diff = 0;
    for (uint64_t i = a; i < b; ++i) {
      uint32_t x[3], y[3];
      std::memcpy(x, src + i * stride, 12);
      std::memcpy(y, packed + 3 * i, 12);
      diff |= (x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2]);
    }
    return diff == 0;
  };
  const unsigned nt = n < (1u << 16) ? 1u : std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  if (nt == 1) return cmp(0, n);
  std::vector<char> ok(nt, 1);
  pool->run(nt, [&](size_t t) { ok[t] = cmp(n * t / nt, n * (t + 1) / nt); });
  for (char v : ok)
    if (!v) return false;
  return true;
}

// packed[3 n] = x, y, z of n points at a byte stride (the caches' host copies), over the pool
void copy_points(WorkerPool* pool, const float* pts, uint64_t n, uint64_t stride, float* packed) {
  auto cp = [&](uint64_t a, uint64_t b) {
    const char* src = reinterpret_cast<const char*>(pts);
    if (stride == 12) {
      std::memcpy(packed + 3 * a, src + a * 12, (b - a) * 12);
      return;
    }
    for (uint64_t i = a; i < b; ++i) std::memcpy(packed + 3 * i, src + i * stride, 12);
  };
  const unsigned nt = n < (1u << 16) ? 1u : std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  if (nt == 1) return cp(0, n);
  pool->run(nt, [&](size_t t) { cp(n * t / nt, n * (t + 1) / nt); });
}

// The reference cache's check at the start of a one-shot call (runtime.hpp: RefCache): every pair
// must pass the same reference array; it is the cached one when (pointer, count, stride) match
// and its points are byte-identical to the cached copy. Sets what the call reuses; returns
// whether the reference points need no upload (everything reference-side is cached; the
// one-shot batch's ref_raw still holds them for a sparse-overlap fallback).
bool refcache_begin(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_pair* pairs, size_t n, double res,
                    int flags) {
  RefCache& c = ctx->refc;
  c.use = c.hit_trees = c.hit_ovl = false;
  if (!ctx->opt.reference_cache) {  // (aicp_hip_options: nothing kept, copied or compared)
    c.invalidate();
    return false;
  }
  if (!pairs || n == 0 || !valid_pair(pairs[0])) return false;
  const aicp_pair& p = pairs[0];
  bool one_origin = true;
  for (size_t i = 1; i < n; ++i) {
    const aicp_pair& q = pairs[i];
    if (q.ref != p.ref || q.n_ref != p.n_ref || q.ref_stride != p.ref_stride) {
      c.invalidate();
      return false;
    }
    for (int k = 0; k < 3; ++k) one_origin &= q.ref_origin[k] == p.ref_origin[k];
  }
  const bool same = (c.trees || c.ovl) && c.ptr == p.ref && c.n == p.n_ref && c.stride == p.ref_stride &&
                    c.pts.size() == 3 * (size_t)p.n_ref && same_points(ctx_pool(ctx), p.ref, p.n_ref, p.ref_stride, c.pts.data());
  if (!same) {  // a new reference (or the cached one changed in place): rebuilt and kept by this call
    c.invalidate();
    c.ptr = p.ref;
    c.n = p.n_ref;
    c.stride = p.ref_stride;
    c.pts.resize(3 * (size_t)p.n_ref);
    copy_points(ctx_pool(ctx), p.ref, p.n_ref, p.ref_stride, c.pts.data());
  }
  c.use = true;
  const bool icp = flags & AICP_RUN_ICP, ovl = flags & AICP_RUN_OVERLAP;
  if (same) {
    c.hit_trees = icp && c.trees && cfg && c.bucket == cfg->bucket_size && c.knn == cfg->knn_normals;
    c.hit_ovl = ovl && c.ovl && one_origin && c.res == res && c.origin[0] == p.ref_origin[0] &&
                c.origin[1] == p.ref_origin[1] && c.origin[2] == p.ref_origin[2];
  }
  return (!icp || c.hit_trees) && (!ovl || c.hit_ovl);
}

// register / overlap / align_batch: one-shot batches reuse the context's batch buffers (no device
// allocation per call) and its reference cache
int oneshot(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_pair* pairs, size_t n_pairs, double resolution,
            int flags, float* out_T, aicp_icp_stats* stats, float* out_overlap) {
  if (!ctx) return AICP_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  if (!(flags & (AICP_RUN_ICP | AICP_RUN_OVERLAP))) FAIL(AICP_ERR_INVALID, "nothing to run");
  if (!ctx->oneshot) ctx->oneshot = new aicp_hip_batch();
  aicp_hip_batch* B = ctx->oneshot;
  using clk = std::chrono::steady_clock;
  const auto h0 = clk::now();
  const bool skip_refs = refcache_begin(ctx, cfg, pairs, n_pairs, resolution, flags);
  const auto h1 = clk::now();
  // the reading of the previous call again (computeOverlap, then registerClouds)?
  ReadCache& rd = ctx->rdc;
  const aicp_pair* p0 = n_pairs == 1 && pairs && valid_pair(pairs[0]) ? pairs : nullptr;
  rd.hit = p0 && rd.valid && rd.ptr == p0->read && rd.n == p0->n_read && rd.stride == p0->read_stride &&
           rd.pts.size() == 3 * (size_t)p0->n_read &&
           same_points(ctx_pool(ctx), p0->read, p0->n_read, p0->read_stride, rd.pts.data());
  const auto h2 = clk::now();
  int rc = upload_pairs(ctx, pairs, n_pairs, B, false, skip_refs, rd.hit, true);
  const auto h3 = clk::now();
  if (!rc) rc = run_batch(ctx, B, cfg, resolution, flags, out_T, stats, out_overlap);
  if (ctx->opt.profile) {  // host time per part of a one-shot call (us)
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    const auto h4 = clk::now();
    std::fprintf(stderr, "[aicp oneshot] flags %d pairs %zu: reference compare %.0f, reading compare %.0f, upload %.0f, run %.0f us%s%s\n",
                 flags, n_pairs, us(h0, h1), us(h1, h2), us(h2, h3), us(h3, h4), skip_refs ? " (reference resident)" : "",
                 rd.hit ? " (reading resident)" : "");
  }
  ctx->refc.use = false;
  const bool was_hit = rd.hit;
  rd.hit = false;
  if (was_hit) ++rd.hits;
  if (rc) {
    ctx->refc.invalidate();  // (an error may leave the reference side half written)
    (void)hipStreamSynchronize(ctx->stream);  // (the staging copies of upload_pairs are not awaited there)
  }
  rd.valid = !rc && p0 && ctx->opt.reference_cache;
  if (rd.valid && !was_hit) {  // the reading this call uploaded: its copy for the next call's compare
    rd.ptr = p0->read;
    rd.n = p0->n_read;
    rd.stride = p0->read_stride;
    rd.pts.resize(3 * (size_t)p0->n_read);
    copy_points(ctx_pool(ctx), p0->read, p0->n_read, p0->read_stride, rd.pts.data());
  }
  // the input copies of a very large one-shot batch are not kept for the next call
  if (B->ref_raw.cap + B->read_raw.cap > ((size_t)ctx->opt.oneshot_keep_mib << 20)) {
    (void)hipStreamSynchronize(ctx->stream);
    release(B->ref_raw);
    release(B->read_raw);
    ctx->refc.invalidate();
    rd.valid = false;
  }
  return rc;
}

}  // namespace

int aicp_hip_align_batch(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_pair* pairs, size_t n_pairs,
                         double resolution, int flags, float* out_T, aicp_icp_stats* stats) {
  return oneshot(ctx, cfg, pairs, n_pairs, resolution, flags, out_T, stats, nullptr);
}

int aicp_hip_register_batch(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_pair* pairs, size_t n_pairs,
                            float* out_T, aicp_icp_stats* stats) {
  return aicp_hip_align_batch(ctx, cfg, pairs, n_pairs, 0.0, AICP_RUN_ICP, out_T, stats);
}

int aicp_hip_register(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_pair* pair, float out_T[16],
                      aicp_icp_stats* stats) {
  return aicp_hip_register_batch(ctx, cfg, pair, 1, out_T, stats);
}

int aicp_hip_overlap_batch(aicp_hip_ctx* ctx, const aicp_pair* pairs, size_t n_pairs, double resolution,
                           float* out_overlap_percent, aicp_icp_stats* stats) {
  aicp_icp_config cfg;
  aicp_hip_default_config(&cfg);
  return oneshot(ctx, &cfg, pairs, n_pairs, resolution, AICP_RUN_OVERLAP, nullptr, stats, out_overlap_percent);
}

int aicp_hip_reference_cache_stats(const aicp_hip_ctx* ctx, uint64_t out[4]) {
  if (!ctx || !out) return AICP_ERR_INVALID;
  out[0] = ctx->refc.tree_hits;
  out[1] = ctx->refc.tree_builds;
  out[2] = ctx->refc.ovl_hits;
  out[3] = ctx->refc.ovl_builds;
  return AICP_OK;
}

int aicp_hip_overlap(aicp_hip_ctx* ctx, const aicp_pair* pair, double resolution, float* out) {
  return aicp_hip_overlap_batch(ctx, pair, 1, resolution, out, nullptr);
}

int aicp_hip_transform(aicp_hip_ctx* ctx, const float T[16], const float* in, size_t n, size_t stride,
                       float* out) {
  if (!ctx || !T || !in || !out || stride < 12) return AICP_ERR_INVALID;
  if (n == 0) return AICP_OK;
  HIPC(hipSetDevice(ctx->device));
  HIPC(ensure(ctx->scratch, 64 + 2 * n * 16));
  HIPC(ensure(ctx->pin_io, n * 16));
  float* h = ctx->pin_io.as<float>();
  pack_xyz4(in, n, stride, h);
  char* d = ctx->scratch.as<char>();
  HIPC(hipMemcpy(d, T, 64, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(d + 64, h, n * 16, hipMemcpyHostToDevice));
  launch_transform(ctx->stream, (int)n, (const float*)d, (const float4*)(d + 64), (float4*)(d + 64 + n * 16));
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  HIPC(hipMemcpy(h, d + 64 + n * 16, n * 16, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) out[3 * i + k] = h[4 * i + k];
  return AICP_OK;
}

// Box frame of getPointsInOrientedBox (filteringUtils.cpp:619-637): Eigen eulerAngles(0,1,2)
// of origin.R, pcl::getTransformation(0,0,0,rx,ry,rz) = Rz Ry Rx, Affine3f::inverse() by
// cofactors, and CropBox's fuzzy isIdentity() skip. Scalar float setup on the host; the
// per-point test runs in k_crop_count / k_crop_scatter.
static void crop_box_frame(const float origin[16], float inv[9], float t[3], float rpy[3]) {
  auto R = [&](int r, int c) { return origin[c * 4 + r]; };
  float a0 = std::atan2(R(1, 2), R(2, 2)), a1;
  const float c2 = std::sqrt(R(0, 0) * R(0, 0) + R(0, 1) * R(0, 1));
  if (a0 > 0.f) {
    a0 -= float(M_PI);
    a1 = std::atan2(-R(0, 2), -c2);
  } else {
    a1 = std::atan2(-R(0, 2), c2);
  }
  const float s1 = std::sin(a0), c1 = std::cos(a0);
  const float a2 = std::atan2(s1 * R(2, 0) - c1 * R(1, 0), c1 * R(1, 1) - s1 * R(2, 1));
  rpy[0] = -a0;
  rpy[1] = -a1;
  rpy[2] = -a2;
  for (int q = 0; q < 3; ++q) t[q] = origin[12 + q];
  for (int q = 0; q < 9; ++q) inv[q] = (q % 4 == 0) ? 1.f : 0.f;
  if (rpy[0] == 0.f && rpy[1] == 0.f && rpy[2] == 0.f) return;
  const float A = std::cos(rpy[2]), B = std::sin(rpy[2]), C = std::cos(rpy[1]), D = std::sin(rpy[1]),
              E = std::cos(rpy[0]), F = std::sin(rpy[0]);
  const float DE = D * E, DF = D * F;
  const float m[3][3] = {{A * C, A * DF - B * E, B * F + A * DE}, {B * C, A * E + B * DF, B * DE - A * F},
                         {-D, C * F, C * E}};
  const float k00 = m[1][1] * m[2][2] - m[1][2] * m[2][1], k10 = m[1][2] * m[2][0] - m[1][0] * m[2][2],
              k20 = m[1][0] * m[2][1] - m[1][1] * m[2][0];
  const float id = 1.f / (m[0][0] * k00 + m[0][1] * k10 + m[0][2] * k20);
  const float w[9] = {k00 * id,
                      (m[0][2] * m[2][1] - m[0][1] * m[2][2]) * id,
                      (m[0][1] * m[1][2] - m[0][2] * m[1][1]) * id,
                      k10 * id,
                      (m[0][0] * m[2][2] - m[0][2] * m[2][0]) * id,
                      (m[0][2] * m[1][0] - m[0][0] * m[1][2]) * id,
                      k20 * id,
                      (m[0][1] * m[2][0] - m[0][0] * m[2][1]) * id,
                      (m[0][0] * m[1][1] - m[0][1] * m[1][0]) * id};
  bool ident = true;
  for (int q = 0; q < 9; ++q)
    ident = ident && (q % 4 == 0 ? std::fabs(w[q] - 1.f) <= 1e-5f * std::fmin(std::fabs(w[q]), 1.f)
                                 : std::fabs(w[q]) <= 1e-5f);
  if (!ident)
    for (int q = 0; q < 9; ++q) inv[q] = w[q];
}

// the crop kernels on n device points; kept points (input order) to host out, capacity cap
static int crop_device(aicp_hip_ctx* ctx, const float4* din, size_t n, const float inv[9], const float t[3], float mn,
                       float mx, float* out, size_t cap, size_t* out_n) {
  const size_t tiles = aicp::crop_tiles(n);
  const size_t tile_bytes = (2 * tiles * 4 + 255) & ~size_t(255);
  HIPC(ensure(ctx->scratch, 256 + tile_bytes + n * 16));
  HIPC(ensure(ctx->pin_io, n * 16 + 16));
  char* d = ctx->scratch.as<char>();
  uint32_t* total = (uint32_t*)d;
  uint32_t* tcnt = (uint32_t*)(d + 256);
  uint32_t* toff = tcnt + tiles;
  float4* dout = (float4*)(d + 256 + tile_bytes);
  aicp::launch_crop_box(ctx->stream, (int)n, inv, t, mn, mx, din, tcnt, toff, total, dout);
  HIPC(hipGetLastError());
  uint32_t m = 0;
  HIPC(hipMemcpyAsync(&m, total, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  if (m > n) FAIL(AICP_ERR_HIP, "crop: kept count exceeds the input");
  if (m > cap) FAIL(AICP_ERR_INVALID, "crop: output capacity too small");
  float* h = ctx->pin_io.as<float>();
  if (m) HIPC(hipMemcpy(h, dout, (size_t)m * 16, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < m; ++i)
    for (int k = 0; k < 3; ++k) out[3 * i + k] = h[4 * i + k];
  *out_n = m;
  return AICP_OK;
}

int aicp_hip_crop_box(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, float mn, float mx,
                      const float origin[16], float* out, size_t* out_n, float* rpy_out) {
  if (!ctx || !pts || !origin || !out || !out_n || stride < 12) return AICP_ERR_INVALID;
  if (n > (size_t)INT32_MAX) return AICP_ERR_INVALID;
  float inv[9], t[3], rpy[3];
  crop_box_frame(origin, inv, t, rpy);
  if (rpy_out)
    for (int q = 0; q < 3; ++q) rpy_out[q] = rpy[q];
  *out_n = 0;
  if (n == 0) return AICP_OK;
  HIPC(hipSetDevice(ctx->device));
  HIPC(ensure(ctx->ref1, n * 16));
  HIPC(ensure(ctx->pin_io, n * 16 + 16));
  pack_xyz4(pts, n, stride, ctx->pin_io.as<float>());
  HIPC(hipMemcpyAsync(ctx->ref1.p, ctx->pin_io.p, n * 16, hipMemcpyHostToDevice, ctx->stream));
  return crop_device(ctx, ctx->ref1.as<float4>(), n, inv, t, mn, mx, out, n, out_n);
}

int aicp_hip_last_nn_timing(const aicp_hip_ctx* ctx, int* n_launches, double* total_ms, double* bytes,
                            uint64_t* queries) {
  if (!ctx) return AICP_ERR_INVALID;
  if (n_launches) *n_launches = ctx->last_nn_launches;
  if (total_ms) *total_ms = ctx->last_nn_ms;
  if (bytes) *bytes = ctx->last_nn_bytes;
  if (queries) *queries = ctx->last_queries;
  return AICP_OK;
}

int aicp_hip_last_phase_ms(const aicp_hip_ctx* ctx, double out_ms[5]) {
  if (!ctx || !out_ms) return AICP_ERR_INVALID;
  for (int i = 0; i < 5; ++i) out_ms[i] = ctx->last_phase[i];
  return AICP_OK;
}

int aicp_hip_knn(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, const float* queries, size_t nq,
                 size_t qstride, int k, float epsilon, float max_dist, int32_t* out_ids, float* out_d2,
                 uint64_t* out_touched) {
  if (!ctx || !pts || !queries || !out_ids || !out_d2 || n == 0 || stride < 12 || qstride < 12) return AICP_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  PairDesc td;
  int rc = upload_tree(ctx, pts, n, stride, td);
  if (rc) return rc;
  hipStream_t st_ = ctx->stream;
  HIPC(ensure(ctx->read_c, nq * 16 + 16));
  HIPC(ensure(ctx->match, nq * (size_t)k * 4 + 4));
  HIPC(ensure(ctx->d2, nq * (size_t)k * 4 + 4));
  HIPC(ensure(ctx->scratch, 16 + kCtrWords * 4));
  HIPC(ensure(ctx->pin_io, std::max<size_t>(nq * 16, nq * (size_t)k * 4) + 16));
  float* h = ctx->pin_io.as<float>();
  pack_xyz4(queries, nq, qstride, h);
  HIPC(hipMemcpyAsync(ctx->read_c.p, h, nq * 16, hipMemcpyHostToDevice, st_));
  HIPC(hipMemsetAsync(ctx->scratch.p, 0, 16 + kCtrWords * 4, st_));
  const float maxE2 = (1 + epsilon) * (1 + epsilon);
  const float maxR2 = max_dist * max_dist;
  if (!launch_knn_generic(st_, (uint32_t)nq, ctx->read_c.as<float4>(), ctx->nodes.as<uint4>(),
                          nullptr, ctx->bpts.as<float4>(), k, maxE2, maxR2,
                          ctx->match.as<int32_t>(), ctx->d2.as<float>(), ctx->scratch.as<unsigned long long>(),
                          (uint32_t*)(ctx->scratch.as<char>() + 16)))
    FAIL(AICP_ERR_UNSUPPORTED, "k must be 1, 4, 10, 20 or 30");
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(st_));
  HIPC(hipMemcpy(out_ids, ctx->match.p, nq * (size_t)k * 4, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(out_d2, ctx->d2.p, nq * (size_t)k * 4, hipMemcpyDeviceToHost));
  if (out_touched) HIPC(hipMemcpy(out_touched, ctx->scratch.p, 16, hipMemcpyDeviceToHost));
  return AICP_OK;
}

int aicp_hip_normals(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, int knn, float* out_normals,
                     int32_t* out_degenerate) {
  if (!ctx || !pts || !out_normals || n == 0 || stride < 12) return AICP_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  PairDesc d;
  int rc = upload_tree(ctx, pts, n, stride, d);
  if (rc) return rc;
  hipStream_t st_ = ctx->stream;
  HIPC(ensure(ctx->state, sizeof(PairState)));
  HIPC(ensure(ctx->bnrm, n * 16));
  HIPC(ensure(ctx->nbids, n * 4 * (size_t)std::max(knn, 1)));
  HIPC(ensure(ctx->ctrs, kCtrWords * 4));
  HIPC(hipMemsetAsync(ctx->ctrs.p, 0, kCtrWords * 4, st_));
  launch_init_state(st_, 1, ctx->desc.as<PairDesc>(), ctx->state.as<PairState>());
  if (!launch_normals(st_, 1, (uint32_t)n, ctx->desc.as<PairDesc>(), ctx->state.as<PairState>(),
                      ctx->nodes.as<uint4>(), nullptr, ctx->bpts.as<float4>(),
                      ctx->bnrm.as<float4>(), knn, ctx->nbids.as<int32_t>(), ctx->ctrs.as<uint32_t>(),
                      ctx->opt.normals_knn_engine))
    FAIL(AICP_ERR_UNSUPPORTED, "knn must be 10, 20 or 30");
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(st_));
  std::vector<float> nb(4 * n), bp(4 * n);
  HIPC(hipMemcpy(nb.data(), ctx->bnrm.p, n * 16, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(bp.data(), ctx->bpts.p, n * 16, hipMemcpyDeviceToHost));
  PairState st;
  HIPC(hipMemcpy(&st, ctx->state.p, sizeof(st), hipMemcpyDeviceToHost));
  for (size_t j = 0; j < n; ++j) {
    int32_t id;
    std::memcpy(&id, &bp[4 * j + 3], 4);  // bucket position -> input index
    for (int k = 0; k < 3; ++k) out_normals[3 * (size_t)id + k] = nb[4 * j + k];
  }
  if (out_degenerate) *out_degenerate = st.degenerate;
  return AICP_OK;
}

int aicp_hip_dists_quantile(aicp_hip_ctx* ctx, const float* d2, size_t n, float quantile, float* out_limit) {
  if (!ctx || !d2 || !out_limit || n == 0 || n >= (1ull << 31)) return AICP_ERR_INVALID;
  if (!(quantile >= 0.f && quantile <= 1.f)) return AICP_ERR_INVALID;  // "quantile must be between 0 and 1"
  HIPC(hipSetDevice(ctx->device));
  hipStream_t st_ = ctx->stream;
  PairDesc d{};
  d.n_read = (uint32_t)n;
  d.ratio = quantile;
  HIPC(ensure(ctx->desc, sizeof(PairDesc)));
  HIPC(ensure(ctx->state, sizeof(PairState)));
  HIPC(ensure(ctx->d2, n * 4));
  HIPC(ensure(ctx->pin_io, n * 4));
  std::memcpy(ctx->pin_io.p, d2, n * 4);
  HIPC(hipMemcpyAsync(ctx->desc.p, &d, sizeof(d), hipMemcpyHostToDevice, st_));
  HIPC(hipMemcpyAsync(ctx->d2.p, ctx->pin_io.p, n * 4, hipMemcpyHostToDevice, st_));
  // one pair: blocks of kNNBlock * kSelPerThread readings
  const uint32_t per = kNNBlock * kSelPerThread, nb = (uint32_t)((n + per - 1) / per);
  HIPC(ensure(ctx->qmap, (size_t)nb * 8));
  HIPC(ensure(ctx->pin_desc, (size_t)nb * 8));
  uint32_t* hm = ctx->pin_desc.as<uint32_t>();
  for (uint32_t b = 0; b < nb; ++b) {
    hm[b] = 0;
    hm[nb + b] = b * per;
  }
  HIPC(hipMemcpyAsync(ctx->qmap.p, hm, (size_t)nb * 8, hipMemcpyHostToDevice, st_));
  BlockMap qm{ctx->qmap.as<int32_t>(), ctx->qmap.as<uint32_t>() + nb, nb};
  HIPC(ensure(ctx->sel_hist, kHistBins * 4));
  HIPC(ensure(ctx->sel_cand, n * 4));
  HIPC(ensure(ctx->sel_cnt, 4));
  HIPC(hipMemsetAsync(ctx->sel_hist.p, 0, kHistBins * 4, st_));
  HIPC(hipMemsetAsync(ctx->sel_cnt.p, 0, 4, st_));
  launch_init_state(st_, 1, ctx->desc.as<PairDesc>(), ctx->state.as<PairState>());
  launch_icp_select(st_, qm, 1, ctx->desc.as<PairDesc>(), ctx->state.as<PairState>(), ctx->d2.as<float>(),
                    ctx->sel_hist.as<uint32_t>(), ctx->sel_cand.as<uint32_t>(), ctx->sel_cnt.as<uint32_t>());
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(st_));
  PairState st;
  HIPC(hipMemcpy(&st, ctx->state.p, sizeof(st), hipMemcpyDeviceToHost));
  if (st.status) FAIL(st.status, "no outlier to filter");
  *out_limit = st.limit;
  return AICP_OK;
}

int aicp_hip_solve6(aicp_hip_ctx* ctx, const double* A, const double* b, double* out_x, int32_t* out_path) {
  if (!ctx || !A || !b || !out_x) return AICP_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  HIPC(ensure(ctx->scratch, 8 * (36 + 6 + 6) + 8));
  char* d = ctx->scratch.as<char>();
  HIPC(hipMemcpy(d, A, 36 * 8, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(d + 288, b, 6 * 8, hipMemcpyHostToDevice));
  launch_solve6(ctx->stream, (const double*)d, (const double*)(d + 288), (double*)(d + 336), (int32_t*)(d + 384));
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  HIPC(hipMemcpy(out_x, d + 336, 48, hipMemcpyDeviceToHost));
  int32_t path = 0;
  HIPC(hipMemcpy(&path, d + 384, 4, hipMemcpyDeviceToHost));
  if (out_path) *out_path = path;
  return AICP_OK;
}

void aicp_hip_default_prefilter(aicp_prefilter_params* p) {
  if (!p) return;
  *p = aicp_prefilter_params{};
  p->leaf_size = 0.08f;  // filteringUtils.cpp:12
  p->normal_k = 30;      // :22
  p->neighbours = 15;    // :30
  p->min_cluster_size = 50;
  p->max_cluster_size = 1000000;
  p->smoothness_rad = (float)(3.0 / 180.0 * M_PI);  // :33 (setSmoothnessThreshold(float))
  p->curvature_threshold = 1.0f;
}

// VoxelGrid -> NormalEstimation -> RegionGrowing on the device (kernels_prefilter.hip). Host
// syncs: after the voxel grid (sampled count sizes the tree), per round of two propagation
// launches (fixed-point test), and the final counts.
struct PfRun {  // device results of pf_core
  uint32_t V = 0, n_out = 0, n_clusters = 0;
  const float4* out4 = nullptr;      // kept points, clusters concatenated
  const float4* nrm = nullptr;       // normal + curvature, kd-tree bucket order
  const uint32_t* inv = nullptr;     // sampled index -> bucket position
  const int32_t* cluster_of = nullptr;
};
// host side of pf_core's device-to-host copies, in the context's pinned memory: a copy still in
// flight when pf_core returns early on an error writes into memory that stays valid
struct PfHost {
  PfCtl hc;
  unsigned long long ht[2];
  uint32_t tl_err;
  uint32_t hf[2];
};
struct PfLayout {
  PfCtl* ctl;
  float4* pts4;  // the input, n points
  PfWork W;
};

static int pf_check(aicp_hip_ctx* ctx, const aicp_prefilter_params* prm) {
  if (!(prm->leaf_size > 0.f) || !std::isfinite(prm->leaf_size)) FAIL(AICP_ERR_INVALID, "leaf size must be > 0");
  const int K = prm->normal_k, NB = prm->neighbours;
  if (K != 10 && K != 20 && K != 30) FAIL(AICP_ERR_UNSUPPORTED, "normal_k must be 10, 20 or 30");
  if (NB < 1 || NB > kPfMaxNbrs || NB > K) FAIL(AICP_ERR_UNSUPPORTED, "neighbours must be 1..min(16, normal_k)");
  return AICP_OK;
}

// scratch of the voxel grid and the extraction: ctl | pts4[n] | 9 x (n + 1) words | temp
static int pf_layout(aicp_hip_ctx* ctx, size_t n, PfLayout* L) {
  const size_t wn = (n + 1 + 63) & ~size_t(63);
  const size_t temp_b = pf_temp_bytes(n + 1);
  const size_t off_pts = 256, off_w = off_pts + n * 16, off_temp = off_w + 9 * wn * 4;
  HIPC(ensure(ctx->pf_a, off_temp + temp_b));
  char* A = ctx->pf_a.as<char>();
  uint32_t* wb = (uint32_t*)(A + off_w);
  L->ctl = (PfCtl*)A;
  L->pts4 = (float4*)(A + off_pts);
  L->W = PfWork{wb, wb + wn, wb + 2 * wn, wb + 3 * wn, wb + 4 * wn, wb + 5 * wn, wb + 6 * wn, wb + 7 * wn, wb + 8 * wn,
                A + off_temp, temp_b};
  return AICP_OK;
}

// the whole chain on n points already in the layout's pts4 (enqueued on ctx->stream)
static int pf_core(aicp_hip_ctx* ctx, const aicp_prefilter_params* prm, size_t n, const PfLayout& Lo, PfRun* o) {
  // (the sampled cloud's tree goes to pf_bpts / pf_nodes: a cached reference stays resident)
  hipStream_t s = ctx->stream;
  const int K = prm->normal_k, NB = prm->neighbours;
  for (auto& e : ctx->pf_ev)
    if (!e) HIPC(hipEventCreate(&e));
  hipEvent_t* E = ctx->pf_ev;  // 0 input ready, 1 voxels, 2 kNN start, 3 kNN end, 4 normals, 5 clusters
  PfCtl* dctl = Lo.ctl;
  const PfWork& W = Lo.W;
  HIPC(ensure(ctx->ref1, n * 16));
  HIPC(ensure(ctx->pin_pf, sizeof(PfHost)));
  HIPC(hipStreamSynchronize(s));  // no copy of an earlier call is still in flight into pin_pf
  PfHost& H = *ctx->pin_pf.as<PfHost>();
  PfCtl& hc = H.hc;
  hc = PfCtl{};
  for (int k = 0; k < 3; ++k) hc.lo[k] = 0xFFFFFFFFu;
  HIPC(hipMemcpyAsync(dctl, &hc, sizeof(hc), hipMemcpyHostToDevice, s));
  HIPC(hipStreamSynchronize(s));  // hc is reused as the destination of the read-backs below
  HIPC(hipEventRecord(E[0], s));
  HIPC(launch_pf_voxel(s, (uint32_t)n, Lo.pts4, 1.f / prm->leaf_size, dctl, W, ctx->ref1.as<float4>()));
  HIPC(hipEventRecord(E[1], s));
  HIPC(hipMemcpyAsync(&hc, dctl, sizeof(hc), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (hc.passthrough && hc.n_bad)
    FAIL(AICP_ERR_UNSUPPORTED, "voxel grid overflows 32-bit indices and the cloud has non-finite points");
  const uint32_t V = hc.n_fin ? hc.n_vox : 0u;
  *o = PfRun{};
  o->V = V;
  if (V == 0) return AICP_OK;
  // ---- kd-tree of the sampled cloud and its exact kNN (libnabo order, eps 0, self included)
  PairDesc d{};
  d.n_ref = V;
  d.ratio = 0.5f;
  d.tl_off = 0;
  ident4(d.Tin);
  HIPC(ensure(ctx->desc, sizeof(PairDesc)));
  HIPC(hipMemcpyAsync(ctx->desc.p, &d, sizeof(d), hipMemcpyHostToDevice, s));
  int rc = device_trees_begin(ctx->tb[0], ctx->err, s, 1, V, ctx->desc.as<PairDesc>(), ctx->ref1.as<float4>(), 0, 8,
                              ctx->pf_bpts, ctx->pf_nodes);
  if (rc) return rc;
  rc = device_trees_end(ctx->tb[0], ctx->err, s, 1, V, ctx->desc.as<PairDesc>(), 8, ctx->pf_bpts, ctx->pf_nodes, 0);
  if (rc) return rc;
  HIPC(ensure(ctx->match, (size_t)V * K * 4));
  HIPC(ensure(ctx->ctrs, kCtrWords * 4 + 16));
  HIPC(hipMemsetAsync(ctx->ctrs.p, 0, kCtrWords * 4 + 16, s));
  const float4* bpts = ctx->pf_bpts.as<float4>();
  unsigned long long* dtouch = (unsigned long long*)(ctx->ctrs.as<uint32_t>() + kCtrWords);
  HIPC(hipEventRecord(E[2], s));
  if (!launch_knn_ids(s, 1, V, ctx->desc.as<PairDesc>(), ctx->pf_nodes.as<uint4>(), bpts, K, ctx->match.as<int32_t>(),
                      ctx->ctrs.as<uint32_t>(), dtouch, ctx->opt.normals_knn_engine))
    FAIL(AICP_ERR_UNSUPPORTED, "normal_k must be 10, 20 or 30");
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(E[3], s));
  // ---- per sampled point: inv, nrm (float4), nbp (16), ckey, cval, nob, order_of, em, label,
  // cluster_of, out4 (float4), comp, kth (uint2)
  const size_t vn = ((size_t)V + 63) & ~size_t(63);
  HIPC(ensure(ctx->pf_b, vn * 4 * (1 + 4 + kPfMaxNbrs + 8 + 4 + 2) + 256));
  uint32_t* B = ctx->pf_b.as<uint32_t>();
  uint32_t* inv = B;
  float4* nrm = (float4*)(B + vn);
  int32_t* nbp = (int32_t*)(B + 5 * vn);
  uint32_t* ckey = B + (5 + kPfMaxNbrs) * vn;
  uint32_t* cval = ckey + vn;
  uint32_t* nob = cval + vn;
  uint32_t* order_of = nob + vn;
  uint32_t* em = order_of + vn;
  uint32_t* label = em + vn;
  int32_t* cluster_of = (int32_t*)(label + vn);
  float4* out4 = (float4*)(cluster_of + vn);
  uint32_t* comp = (uint32_t*)(out4 + vn);
  uint2* kth = (uint2*)(comp + vn);
  uint32_t* flags = (uint32_t*)(kth + vn);
  const float vp[3] = {prm->viewpoint[0], prm->viewpoint[1], prm->viewpoint[2]};
  if (!launch_pf_normals(s, V, K, NB, bpts, ctx->ref1.as<float4>(), ctx->match.as<int32_t>(), inv, vp, nrm, nbp,
                         kth, ckey, cval))
    FAIL(AICP_ERR_UNSUPPORTED, "normal_k must be 10, 20 or 30");
  HIPC(hipEventRecord(E[4], s));
  // validatePoint: cosine_threshold = cosf(theta_threshold_)
  const float cos_thr = (float)std::cos((double)prm->smoothness_rad);
  HIPC(launch_pf_order(s, V, NB, W, ckey, cval, inv, bpts, nrm, nbp, kth, cos_thr, prm->curvature_threshold, nob,
                       order_of, em, label));
  // ---- min-label propagation to the fixed point: union-find over mutual edges, then passes
  // until one changes no label (labels only decrease, so this ends; V passes bound any schedule)
  launch_rg_components(s, V, NB, nbp, em, comp, label);
  constexpr int R = 2;
  uint32_t* hf = H.hf;
  for (uint64_t launches = 0;; launches += R) {
    if (launches > (uint64_t)V + 2 * R) FAIL(AICP_ERR_HIP, "region growing did not reach its fixed point");
    HIPC(hipMemsetAsync(flags, 0, R * 4, s));
    for (int r = 0; r < R; ++r) launch_rg_iter(s, V, NB, nbp, em, nob, comp, label, flags + r);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(hf, flags, R * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    ctx->last_pf.propagation_passes = (int)(launches + R);
    if (!hf[R - 1]) break;
  }
  launch_rg_settle(s, V, comp, label);
  launch_rg_count_inf(s, V, label, dctl);
  HIPC(hipMemcpyAsync(&hc, dctl, sizeof(hc), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (hc.n_inf) launch_rg_phaseb(s, V, NB, nbp, em, nob, label);
  HIPC(launch_rg_extract(s, V, (uint32_t)std::max(prm->min_cluster_size, 0),
                         (uint32_t)std::max(prm->max_cluster_size, 0), label, inv, ctx->ref1.as<float4>(), W, out4,
                         cluster_of, dctl));
  HIPC(hipEventRecord(E[5], s));
  HIPC(hipMemcpyAsync(&hc, dctl, sizeof(hc), hipMemcpyDeviceToHost, s));
  unsigned long long* ht = H.ht;
  HIPC(hipMemcpyAsync(ht, dtouch, 16, hipMemcpyDeviceToHost, s));
  const uint32_t& tl_err = H.tl_err;
  HIPC(hipMemcpyAsync(&H.tl_err, &ctx->tb[0].tw.ctl->error, 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (tl_err & 4) FAIL(AICP_ERR_HIP, "pre-filter treelets exceed their allotment");
  aicp_prefilter_stats& ps = ctx->last_pf;
  ps.voxel_ms = ev_ms(E[0], E[1]);
  ps.normals_ms = ev_ms(E[1], E[4]);
  ps.segment_ms = ev_ms(E[4], E[5]);
  ps.device_ms = ev_ms(E[0], E[5]);
  ps.knn_ms = ev_ms(E[2], E[3]);
  ps.knn_queries = V;
  ps.knn_points_touched = ht[0];
  ps.knn_nodes_touched = ht[1];
  if (hc.n_out > V || hc.n_clusters > V) FAIL(AICP_ERR_HIP, "pre-filter: inconsistent cluster counts");
  o->n_out = hc.n_out;
  o->n_clusters = hc.n_clusters;
  o->out4 = out4;
  o->nrm = nrm;
  o->inv = inv;
  o->cluster_of = cluster_of;
  return AICP_OK;
}

int aicp_hip_prefilter(aicp_hip_ctx* ctx, const aicp_prefilter_params* prm, const float* pts, size_t n,
                       size_t stride, float* out, size_t* out_n, float* sampled, int32_t* labels, size_t* n_sampled,
                       size_t* n_clusters) {
  if (!ctx || !prm || !out || !out_n || (n && !pts) || stride < 12 || (stride % 4)) return AICP_ERR_INVALID;
  if (n >= (1ull << 31)) return AICP_ERR_INVALID;
  int rc = pf_check(ctx, prm);
  if (rc) return rc;
  *out_n = 0;
  if (n_sampled) *n_sampled = 0;
  if (n_clusters) *n_clusters = 0;
  ctx->last_pf = aicp_prefilter_stats{};
  if (n == 0) return AICP_OK;
  const auto t_wall = std::chrono::steady_clock::now();
  HIPC(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  PfLayout Lo;
  rc = pf_layout(ctx, n, &Lo);
  if (rc) return rc;
  HIPC(ensure(ctx->pin_io, n * 16 + 64));
  pack_xyz4(pts, n, stride, ctx->pin_io.as<float>());
  HIPC(hipMemcpyAsync(Lo.pts4, ctx->pin_io.p, n * 16, hipMemcpyHostToDevice, s));
  PfRun o;
  rc = pf_core(ctx, prm, n, Lo, &o);
  if (rc) return rc;
  const uint32_t V = o.V;
  if (n_sampled) *n_sampled = V;
  if (V) {
    float* h = ctx->pin_io.as<float>();
    if (o.n_out) HIPC(hipMemcpy(h, o.out4, (size_t)o.n_out * 16, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < o.n_out; ++i)
      for (int k = 0; k < 3; ++k) out[3 * i + k] = h[4 * i + k];
    *out_n = o.n_out;
    if (n_clusters) *n_clusters = o.n_clusters;
    if (labels) HIPC(hipMemcpy(labels, o.cluster_of, (size_t)V * 4, hipMemcpyDeviceToHost));
    if (sampled) {
      std::vector<float> P(4 * (size_t)V), N(4 * (size_t)V);
      std::vector<uint32_t> I(V);
      HIPC(hipMemcpy(P.data(), ctx->ref1.p, (size_t)V * 16, hipMemcpyDeviceToHost));
      HIPC(hipMemcpy(N.data(), o.nrm, (size_t)V * 16, hipMemcpyDeviceToHost));
      HIPC(hipMemcpy(I.data(), o.inv, (size_t)V * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < V; ++i) {
        float* q = sampled + 8 * i;
        const float* nb = &N[4 * (size_t)I[i]];
        q[0] = P[4 * i];
        q[1] = P[4 * i + 1];
        q[2] = P[4 * i + 2];
        q[3] = nb[3];
        q[4] = nb[0];
        q[5] = nb[1];
        q[6] = nb[2];
        q[7] = 0.f;
      }
    }
  }
  ctx->last_pf.wall_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall).count();
  return AICP_OK;
}

// ---- device-resident prior map (localization mode, app.cpp:41-51, 469-493) ------------------
int aicp_hip_map_create(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, aicp_hip_map** out) {
  if (!ctx || !out || (n && !pts) || stride < 12 || (stride % 4) || n > (size_t)INT32_MAX) return AICP_ERR_INVALID;
  *out = nullptr;
  HIPC(hipSetDevice(ctx->device));
  aicp_hip_map* m = new aicp_hip_map();
  if (n) {
    const hipError_t e = ensure(m->pts, n * 16);
    if (e != hipSuccess) {
      delete m;
      ctx->err = std::string("map allocation: ") + hipGetErrorString(e);
      return AICP_ERR_HIP;
    }
    HIPC(ensure(ctx->pin_io, n * 16 + 16));
    pack_xyz4(pts, n, stride, ctx->pin_io.as<float>());
    HIPC(hipMemcpyAsync(m->pts.p, ctx->pin_io.p, n * 16, hipMemcpyHostToDevice, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
  }
  m->n = n;
  *out = m;
  return AICP_OK;
}

void aicp_hip_map_free(aicp_hip_ctx* ctx, aicp_hip_map* map) {
  if (!map) return;
  if (ctx) (void)hipStreamSynchronize(ctx->stream);
  release(map->pts);
  delete map;
}

int aicp_hip_map_size(const aicp_hip_map* map, size_t* n) {
  if (!map || !n) return AICP_ERR_INVALID;
  *n = map->n;
  return AICP_OK;
}

int aicp_hip_map_download(aicp_hip_ctx* ctx, const aicp_hip_map* map, float* out, size_t cap, size_t* out_n) {
  if (!ctx || !map || !out_n || (map->n && !out)) return AICP_ERR_INVALID;
  if (cap < map->n) FAIL(AICP_ERR_INVALID, "map download: output capacity too small");
  HIPC(hipSetDevice(ctx->device));
  *out_n = map->n;
  if (!map->n) return AICP_OK;
  HIPC(ensure(ctx->pin_io, map->n * 16));
  HIPC(hipStreamSynchronize(ctx->stream));
  HIPC(hipMemcpy(ctx->pin_io.p, map->pts.p, map->n * 16, hipMemcpyDeviceToHost));
  const float* h = ctx->pin_io.as<float>();
  for (size_t i = 0; i < map->n; ++i)
    for (int k = 0; k < 3; ++k) out[3 * i + k] = h[4 * i + k];
  return AICP_OK;
}

int aicp_hip_map_crop(aicp_hip_ctx* ctx, const aicp_hip_map* map, float mn, float mx, const float origin[16],
                      float* out, size_t cap, size_t* out_n) {
  if (!ctx || !map || !origin || !out_n || (cap && !out)) return AICP_ERR_INVALID;
  float inv[9], t[3], rpy[3];
  crop_box_frame(origin, inv, t, rpy);
  *out_n = 0;
  if (!map->n) return AICP_OK;
  HIPC(hipSetDevice(ctx->device));
  return crop_device(ctx, map->pts.as<float4>(), map->n, inv, t, mn, mx, out, cap, out_n);
}

// Localization-only batch (localize_against_prior_map): every reading's reference is the map
// cropped around its prior pose on the device (setReference, app.cpp:41-51), written straight
// into the batch's reference array; the overlap is bypassed at 50 % (app.cpp:123-127), so the
// ratio is the auto-tune of 50 (0.5).
int aicp_hip_map_register_batch(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_hip_map* map, float mn,
                                float mx, const aicp_cloud* readings, const float* poses, size_t n, int flags,
                                float* out_T, aicp_icp_stats* stats) {
  if (!ctx || !cfg || !map || !readings || !poses || !out_T || n == 0) return AICP_ERR_INVALID;
  if (!map->n) FAIL(AICP_ERR_INVALID, "empty map");
  if (n > (size_t)kMaxPairs) FAIL(AICP_ERR_UNSUPPORTED, "more than 4096 readings in one batch");
  HIPC(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t ab = crop_args_bytes(), tiles = crop_tiles(map->n);
  const size_t o_args = 0, o_cnt = (n * ab + 255) & ~size_t(255), o_off = o_cnt + n * tiles * 4,
               o_tot = o_off + n * tiles * 4, o_base = o_tot + n * 4, total_b = o_base + n * 4;
  HIPC(ensure(ctx->crop_ws, total_b));
  HIPC(ensure(ctx->pin_crop, n * ab + 2 * n * 4));
  char* ws = ctx->crop_ws.as<char>();
  char* h = ctx->pin_crop.as<char>();
  for (size_t i = 0; i < n; ++i) {
    float inv[9], t[3], rpy[3];
    crop_box_frame(poses + 16 * i, inv, t, rpy);
    pack_crop_args(inv, t, mn, mx, h + i * ab);
  }
  HIPC(hipMemcpyAsync(ws + o_args, h, n * ab, hipMemcpyHostToDevice, s));
  launch_crop_count_multi(s, (int)map->n, (int)n, ws + o_args, map->pts.as<float4>(), (uint32_t*)(ws + o_cnt),
                          (uint32_t*)(ws + o_off), (uint32_t*)(ws + o_tot));
  HIPC(hipGetLastError());
  uint32_t* htot = reinterpret_cast<uint32_t*>(h + n * ab);
  HIPC(hipMemcpyAsync(htot, ws + o_tot, n * 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  // a batch whose references are the crops (pair i: reference i), readings from the host
  std::vector<aicp_pair> pairs(n);
  for (size_t i = 0; i < n; ++i) {
    const aicp_cloud& c = readings[i];
    if (htot[i] == 0) FAIL(AICP_ERR_INVALID, "reading " + std::to_string(i) + ": empty map crop");
    aicp_pair& p = pairs[i];
    p = aicp_pair{};
    p.ref = c.pts;  // not read (references on the device)
    p.n_ref = htot[i];
    p.ref_stride = 16;
    p.read = c.pts;
    p.n_read = c.n;
    p.read_stride = c.stride;
    for (int k = 0; k < 3; ++k) {
      p.ref_origin[k] = poses[16 * i + 12 + k];
      p.read_origin[k] = c.origin[k];
    }
  }
  if (!ctx->mapbatch) ctx->mapbatch = new aicp_hip_batch();
  aicp_hip_batch* B = ctx->mapbatch;
  int rc = upload_pairs(ctx, pairs.data(), n, B, true);
  if (rc) return rc;
  uint32_t* hbase = htot + n;
  for (size_t i = 0; i < n; ++i) hbase[i] = B->rdesc[i].ref_off;
  HIPC(hipMemcpyAsync(ws + o_base, hbase, n * 4, hipMemcpyHostToDevice, s));
  launch_crop_scatter_multi(s, (int)map->n, (int)n, ws + o_args, map->pts.as<float4>(), (const uint32_t*)(ws + o_off),
                            (const uint32_t*)(ws + o_base), B->ref_raw.as<float4>());
  HIPC(hipGetLastError());
  aicp_icp_config c = *cfg;
  c.trimmed_ratio = aicp_hip_autotune_ratio(50.0f);  // octree_overlap_ = 50.0 (app.cpp:123-127)
  return run_batch(ctx, B, &c, 0.0, AICP_RUN_ICP | (flags & AICP_RUN_TIME_NN), out_T, stats, nullptr);
}

int aicp_hip_map_merge(aicp_hip_ctx* ctx, aicp_hip_map* map, const float* pts, size_t n, size_t stride,
                       const float T[16]) {
  if (!ctx || !map || !T || (n && !pts) || stride < 12 || (stride % 4)) return AICP_ERR_INVALID;
  if (map->n + n > (size_t)INT32_MAX) FAIL(AICP_ERR_INVALID, "map merge: more than 2^31 points");
  if (!n) return AICP_OK;
  HIPC(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t need = (map->n + n) * 16;
  if (need > map->pts.cap) {  // grow with copy (ensure() would drop the content)
    DevBuf nb;
    HIPC(ensure(nb, std::max(need, 2 * map->pts.cap)));
    hipError_t e = map->n ? hipMemcpyAsync(nb.p, map->pts.p, map->n * 16, hipMemcpyDeviceToDevice, s) : hipSuccess;
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {  // the map keeps its old buffer; the new one is released
      (void)hipStreamSynchronize(s);
      release(nb);
      FAIL(AICP_ERR_HIP, std::string("map merge: grow copy: ") + hipGetErrorString(e));
    }
    release(map->pts);
    map->pts = nb;
  }
  HIPC(ensure(ctx->scratch, 64 + n * 16));
  HIPC(ensure(ctx->pin_io, n * 16 + 64));
  float* h = ctx->pin_io.as<float>();
  std::memcpy(h, T, 64);
  pack_xyz4(pts, n, stride, h + 16);
  char* d = ctx->scratch.as<char>();
  HIPC(hipMemcpyAsync(d, h, 64 + n * 16, hipMemcpyHostToDevice, s));
  // transformPointCloud (pcl 1.8, common/impl/transforms.hpp): x' = r00 x + r01 y + r02 z + t0
  // in float, in that order (launch_transform: the same expression, no FMA)
  launch_transform(s, (int)n, (const float*)d, (const float4*)(d + 64), map->pts.as<float4>() + map->n);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s));
  map->n += n;
  return AICP_OK;
}

int aicp_hip_map_prefilter(aicp_hip_ctx* ctx, aicp_hip_map* map, const aicp_prefilter_params* prm) {
  if (!ctx || !map || !prm) return AICP_ERR_INVALID;
  int rc = pf_check(ctx, prm);
  if (rc) return rc;
  ctx->last_pf = aicp_prefilter_stats{};
  if (!map->n) return AICP_OK;
  const auto t_wall = std::chrono::steady_clock::now();
  HIPC(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  PfLayout Lo;
  rc = pf_layout(ctx, map->n, &Lo);
  if (rc) return rc;
  HIPC(hipMemcpyAsync(Lo.pts4, map->pts.p, map->n * 16, hipMemcpyDeviceToDevice, s));
  PfRun o;
  rc = pf_core(ctx, prm, map->n, Lo, &o);
  if (rc) return rc;
  // the map becomes the kept points (prior_map_->updateCloud(map_prefiltered), app.cpp:490-492)
  if (o.V && o.n_out) HIPC(hipMemcpyAsync(map->pts.p, o.out4, (size_t)o.n_out * 16, hipMemcpyDeviceToDevice, s));
  HIPC(hipStreamSynchronize(s));
  map->n = o.V ? o.n_out : 0;
  ctx->last_pf.wall_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall).count();
  return AICP_OK;
}

}  // extern "C"

namespace {
// One raw cloud through regionGrowingUniformPlaneSegmentationFilter on the device, moved first
// by T when T is given (pcl::transformPointCloud in float, launch_transform: setAndFilterReading's
// debug branch, app.cpp:90-99). The kept points come back packed xyz (clusters concatenated).
int pf_cloud(aicp_hip_ctx* ctx, const aicp_prefilter_params* prm, const aicp_cloud& c, const float* T,
             std::vector<float>& out) {
  out.clear();
  hipStream_t s = ctx->stream;
  PfLayout Lo;
  int rc = pf_layout(ctx, c.n, &Lo);
  if (rc) return rc;
  HIPC(hipStreamSynchronize(s));  // (pin_io and scratch are free)
  HIPC(ensure(ctx->pin_io, c.n * 16 + 64));
  float* h = ctx->pin_io.as<float>();
  if (T) {
    HIPC(ensure(ctx->scratch, 64 + c.n * 16));
    std::memcpy(h, T, 64);
    pack_xyz4(c.pts, c.n, c.stride, h + 16);
    char* d = ctx->scratch.as<char>();
    HIPC(hipMemcpyAsync(d, h, 64 + c.n * 16, hipMemcpyHostToDevice, s));
    launch_transform(s, (int)c.n, (const float*)d, (const float4*)(d + 64), Lo.pts4);
    HIPC(hipGetLastError());
  } else {
    pack_xyz4(c.pts, c.n, c.stride, h);
    HIPC(hipMemcpyAsync(Lo.pts4, h, c.n * 16, hipMemcpyHostToDevice, s));
  }
  PfRun o;
  rc = pf_core(ctx, prm, c.n, Lo, &o);  // (returns with the stream idle)
  if (rc) return rc;
  if (!o.V || !o.n_out) return AICP_OK;
  HIPC(hipMemcpy(h, o.out4, (size_t)o.n_out * 16, hipMemcpyDeviceToHost));
  out.resize(3 * (size_t)o.n_out);
  for (size_t i = 0; i < o.n_out; ++i)
    for (int k = 0; k < 3; ++k) out[3 * i + k] = h[4 * i + k];
  return AICP_OK;
}

aicp_cloud packed_cloud(const std::vector<float>& p, const double origin[3]) {
  aicp_cloud c{};
  c.pts = p.data();
  c.n = p.size() / 3;
  c.stride = 12;
  for (int k = 0; k < 3; ++k) c.origin[k] = origin[k];
  return c;
}
}  // namespace

extern "C" {

// App's stream from raw clouds in App's order (app.cpp:282-414 with setAndFilterReading,
// app.cpp:77-100): see include/aicp_hip.h.
int aicp_hip_sequence_run_raw(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                              const aicp_prefilter_params* pf, const aicp_cloud* first, const aicp_cloud* readings,
                              size_t n, float* out_T, aicp_sequence_result* out, size_t* n_done) {
  if (!ctx || !cfg || !prm || !pf || !first || (n && (!readings || !out_T || !out)) || !n_done) return AICP_ERR_INVALID;
  *n_done = 0;
  int rc = pf_check(ctx, pf);
  if (rc) return rc;
  const int F = prm->reference_update_frequency;
  if (F < 1) FAIL(AICP_ERR_INVALID, "reference_update_frequency must be >= 1");
  const bool doOvl = prm->flags & AICP_RUN_OVERLAP, debug = prm->flags & AICP_SEQ_DEBUG;
  if (doOvl && !(prm->resolution > 0)) FAIL(AICP_ERR_INVALID, "resolution");
  rc = check_cfg(ctx, cfg, AICP_RUN_ICP | (doOvl ? AICP_RUN_OVERLAP : 0));
  if (rc) return rc;
  auto valid = [](const aicp_cloud& c) {
    return c.pts && c.n >= 1 && c.n < (1ull << 31) && c.stride >= 12 && c.stride % 4 == 0;
  };
  if (!valid(*first)) FAIL(AICP_ERR_INVALID, "invalid first cloud");
  for (size_t i = 0; i < n; ++i)
    if (!valid(readings[i])) FAIL(AICP_ERR_INVALID, "invalid reading " + std::to_string(i));
  HIPC(hipSetDevice(ctx->device));
  // the first cloud: pre-filtered as given (processCloud, app.cpp:293-297)
  std::vector<float> ref;
  rc = pf_cloud(ctx, pf, *first, nullptr, ref);
  if (rc) return rc;
  if (ref.empty()) FAIL(AICP_ERR_INVALID, "the first cloud keeps no point after the pre-filter");
  // a reading the pre-filter empties fails its registration (libpointmatcher throws on an empty
  // cloud), which ends the stream like any registration error (app.cpp:210)
  auto empty_reading = [&](size_t i, int reference) {
    out[i] = aicp_sequence_result{};
    out[i].status = out[i].icp.status = AICP_ERR_INVALID;
    out[i].reference = reference;
    ident4(out_T + 16 * i);
    *n_done = i + 1;
    FAIL(AICP_ERR_INVALID, "reading " + std::to_string(i) + " keeps no point after the pre-filter");
  };
  if (!debug) {  // robot mode: each reading pre-filtered as given (app.cpp:87-88), then the stream
    std::vector<std::vector<float>> kept(n);
    std::vector<aicp_cloud> clouds(n);
    size_t m = n;
    for (size_t i = 0; i < n && m == n; ++i) {
      rc = pf_cloud(ctx, pf, readings[i], nullptr, kept[i]);
      if (rc) return rc;
      if (kept[i].empty()) m = i;
      clouds[i] = packed_cloud(kept[i], readings[i].origin);
    }
    const aicp_cloud c0 = packed_cloud(ref, first->origin);
    rc = aicp_hip_sequence_run(ctx, cfg, prm, &c0, clouds.data(), m, out_T, out, n_done);
    if (rc || m == n) return rc;
    int reference = -1;
    for (size_t i = 0; i < m; ++i)
      if (out[i].is_reference) reference = (int)i;
    return empty_reading(m, reference);
  }
  // debug mode: reading after reading (initialT_ carries every accepted correction)
  float initT[16];
  ident4(initT);
  double ref_origin[3] = {first->origin[0], first->origin[1], first->origin[2]};
  int ref_id = -1, acc = 0;
  const int flags = AICP_RUN_ICP | (doOvl ? AICP_RUN_OVERLAP : 0) | (prm->flags & AICP_RUN_TIME_NN);
  std::vector<float> rd;
  for (size_t i = 0; i < n; ++i) {
    // setAndFilterReading (app.cpp:90-99): the raw reading moved by initialT_, then pre-filtered;
    // its prior pose becomes initialT_iso * prior pose
    double o[3];
    corrected_origin(initT, readings[i].origin, o);
    rc = pf_cloud(ctx, pf, readings[i], initT, rd);
    if (rc) return rc;
    if (rd.empty()) return empty_reading(i, ref_id);
    aicp_pair p{};
    p.ref = ref.data();
    p.n_ref = ref.size() / 3;
    p.ref_stride = 12;
    p.read = rd.data();
    p.n_read = rd.size() / 3;
    p.read_stride = 12;
    for (int k = 0; k < 3; ++k) {
      p.ref_origin[k] = ref_origin[k];
      p.read_origin[k] = o[k];
    }
    aicp_sequence_result& r = out[i];
    r = aicp_sequence_result{};
    r.reference = ref_id;
    float* T = out_T + 16 * i;
    ident4(T);
    // computeOverlap -> ratio -> registerClouds against the resident reference (app.cpp:218-247)
    rc = oneshot(ctx, cfg, &p, 1, doOvl ? prm->resolution : 0.0, flags, T, &r.icp, nullptr);
    if (!rc) rc = r.icp.status;
    r.status = r.icp.status = rc;
    *n_done = i + 1;
    if (rc) {  // the worker ends here (app.cpp:210)
      ctx->err = "reading " + std::to_string(i) + ": status " + std::to_string(rc) + ": " + ctx->err;
      return rc;
    }
    if (correction_rejected(T, prm->max_correction_magnitude)) continue;  // app.cpp:366-373
    r.accepted = 1;
    corrected_origin(T, o, r.corrected_origin);
    if (++acc == F) {  // the corrected reading is the next reference (app.cpp:375-391)
      std::vector<float> next(rd.size());
      for (size_t j = 0; j < rd.size(); j += 3) apply4(T, rd[j], rd[j + 1], rd[j + 2], &next[j]);
      ref.swap(next);
      for (int k = 0; k < 3; ++k) ref_origin[k] = r.corrected_origin[k];
      ref_id = (int)i;
      r.is_reference = 1;
      acc = 0;
    }
    mul4(T, initT, initT);  // initialT_ = correction * initialT_ (app.cpp:414)
  }
  return AICP_OK;
}

int aicp_hip_last_prefilter_stats(const aicp_hip_ctx* ctx, aicp_prefilter_stats* out) {
  if (!ctx || !out) return AICP_ERR_INVALID;
  *out = ctx->last_pf;
  return AICP_OK;
}

}  // extern "C"
