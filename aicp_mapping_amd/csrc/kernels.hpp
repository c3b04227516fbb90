// kernels.hpp — launch wrappers of the HIP kernels (host-callable).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aicp_common.hpp"

namespace aicp {

// Block -> (pair, first local index) tables for a flat grid over per-pair ranges.
struct BlockMap {
  const int32_t* pair;
  const uint32_t* start;
  uint32_t n_blocks;
};

// ---- ICP ---------------------------------------------------------------------------------
void launch_prepare_read(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* read_raw,
                         float4* read_c);
// Spatial (Morton) order of the reading points of every pair, inside each pair's own range
// (kernels_order.hip). keys*/vals*: total entries each; temp: read_order_temp_bytes.
size_t read_order_temp_bytes(size_t n, int n_pairs);
hipError_t launch_read_order(hipStream_t s, BlockMap m, int n_pairs, const PairDesc* pd, const float4* raw,
                             uint32_t total, uint64_t* keys0, uint64_t* keys1, uint32_t* vals0, uint32_t* vals1,
                             void* temp, size_t temp_bytes, float4* out);
void launch_gather_ref(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* ref_raw,
                       const int32_t* perm, float4* bpts);
void launch_init_state(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st);
// SurfaceNormal of the reference points (bucket order); ids: scratch of total_ref * knn;
// ctr: kPersistCtrWords work counters (zeroed on s when the persistent engine runs). engine:
// aicp_hip_options::normals_knn_engine.
// Returns false if knn is unsupported.
bool launch_normals(hipStream_t s, int n_pairs, uint32_t total_ref, const PairDesc* pd, PairState* st,
                    const uint4* nodes, const int32_t* parent, const float4* bpts, float4* bnrm, int knn,
                    int32_t* ids, uint32_t* ctr, int engine);
// the kNN of every reference point in its own tree (bucket order in and out: ids are bucket
// positions of the pair's tree, -1 past the cloud size); eps 0, self included. touched
// (nullable, zeroed): += touched points, inner nodes
bool launch_knn_ids(hipStream_t s, int n_pairs, uint32_t total_ref, const PairDesc* pd, const uint4* nodes,
                    const float4* bpts, int knn, int32_t* ids, uint32_t* ctr, unsigned long long* touched,
                    int engine);
// host_n (nullable): device pointer of mapped host memory that receives the active count;
// done_sig (nullable, signal memory): once no pair is active, the final corrections go to outT
// and *ticket is stored to done_sig (the sequence's next reference waits on it)
void launch_active_list(hipStream_t s, int n_pairs, const PairDesc* pd, const PairState* st,
                        ActiveList* al, uint32_t* ctr, uint32_t* host_n = nullptr, uint64_t* done_sig = nullptr,
                        const uint64_t* ticket = nullptr, float* outT = nullptr, int src_pair = -1);
// Fused ICP iteration (AICP_ICP_FUSE=0 restores one launch per step): the last workgroup of a
// pair to finish the histogram / compaction / reduction runs that pair's find1 / final select /
// update, and the last pair of the group rebuilds the active list for the next iteration (and,
// when none is left, publishes the corrections and the sequence ticket). Four launches per
// iteration (NN, select x2, reduce) instead of eight. Counters start at zero (icp_sync_words per
// pair group) and reset themselves.
struct IcpIterSync {
  uint32_t* sel1;   // per pair (absolute index): histogram workgroups arrived
  uint32_t* sel2;   // per pair: compaction workgroups arrived
  uint32_t* red;    // per pair: reduction workgroups arrived
  uint32_t* pairs;  // pairs of the group done with this iteration
  int np;           // the group's pairs (pd, st point at its first)
  const PairDesc* pd;
  PairState* st;
  ActiveList* al;
  uint32_t* ctr;
  uint32_t* host_n;    // nullable: the active count for the next iteration (mapped host memory)
  uint64_t* done_sig;  // nullable: see launch_active_list
  const uint64_t* ticket;
  float* outT;
  int src_pair = -1;  // >= 0: bit 31 of host_n says whether this pair (of the group) is still active
};
void tree_prof_dump();  // diagnostic builds (AICP_ITER_PROF): k_tr_mid phase times to stderr
void iter_prof_dump();  // diagnostic builds (AICP_ITER_PROF): per-kernel body / tail times to stderr
inline size_t icp_sync_words(size_t n_pairs) { return 3 * n_pairs + 2; }
// sync words laid out for pairs [0, n_pairs): sel1 | sel2 | red | pairs (2: one per group)
IcpIterSync icp_sync_layout(uint32_t* words, size_t n_pairs, int group);
void launch_icp_select_f(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st, const float* d2,
                         uint32_t* hist1, uint32_t* cand, uint32_t* cand_cnt, const IcpIterSync& y);
// from the second iteration on: the select in one launch, its compaction on the previous
// iteration's digit-1 bin (same limit; a missed guess is compacted again by the pair's last
// workgroup, counted in PairState::sel_miss)
// the whole select of each pair in one workgroup (batches of many pairs of <= 65536 readings)
void launch_icp_select_pair(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const float* d2,
                            uint32_t* cand, const IcpIterSync& y);
// force: aicp_hip_options::select_pair (-1 auto, 0 off, 1 on)
bool sel_pair_fits(size_t n_pairs, uint64_t max_read, int force);
void launch_icp_select_fused(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st, const float* d2,
                             uint32_t* hist1, uint32_t* cand, uint32_t* cand_cnt, const IcpIterSync& y);
void launch_icp_reduce_f(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st, const float4* read_c,
                         const int32_t* match, const float* d2, const uint32_t* touched, const float4* bpts,
                         const float4* bnrm, double* slab, const IcpParams& prm, const IcpIterSync& y);
void launch_icp_nn(hipStream_t s, int grid_items, const PairDesc* pd, const PairState* st,
                   const ActiveList* al, const float4* read_c, const uint4* nodes, const uint4* tl,
                   const int32_t* parent, const float4* bpts, const uint2* ptl, int32_t* match, float* d2,
                   uint32_t* touched, uint32_t* ctr, const IcpParams& prm, hipEvent_t e0 = nullptr,
                   hipEvent_t e1 = nullptr);
// TrimmedDist limit per active pair. m: blocks of kNNBlock * kSelPerThread readings;
// hist1: n_pairs * kHistBins zeroed words, cand: total_read words, cand_cnt: n_pairs zeroed
// words (both left zeroed for the next call).
// m covers pairs p0 .. p0 + n_pairs - 1 (absolute pair indices into pd / st / hist1 / cand_cnt).
void launch_icp_select(hipStream_t s, BlockMap m, int n_pairs, const PairDesc* pd, PairState* st,
                       const float* d2, uint32_t* hist1, uint32_t* cand, uint32_t* cand_cnt, int p0 = 0);
void launch_icp_reduce(hipStream_t s, BlockMap m, const PairDesc* pd, const PairState* st,
                       const float4* read_c, const int32_t* match, const float* d2,
                       const uint32_t* touched, const float4* bpts, const float4* bnrm, double* slab);
void launch_icp_update(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const double* slab, const IcpParams& prm);
void launch_finalize(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                     float* outT);

// AICP_NN_PROF builds: print and reset the NN kernel's per-phase cycle shares (stderr)
void nn_prof_dump();

// ---- kernel-level entry points ----------------------------------------------------------
bool launch_knn_generic(hipStream_t s, uint32_t nq, const float4* q, const uint4* nodes,
                        const int32_t* parent, const float4* bpts, int k, float maxE2,
                        float maxR2, int32_t* ids, float* d2, unsigned long long* touched,
                        uint32_t* ctr);
void launch_transform(hipStream_t s, int n, const float* T, const float4* in, float4* out);
// kernels_crop.hip: order-preserving oriented box crop (getPointsInOrientedBox).
size_t crop_tiles(size_t n);
void launch_crop_box(hipStream_t s, int n, const float inv[9], const float t[3], float mn, float mx,
                     const float4* pts, uint32_t* tile_cnt, uint32_t* tile_off, uint32_t* total,
                     float4* out);
// many crops of one map (one per localization reading): args = n_crops packed CropBoxArgs
// (pack_crop_args, crop_args_bytes each); tile_cnt / tile_off: n_crops * crop_tiles(n) words;
// totals: n_crops words. The scatter writes crop c at out + base_of[c], in input order.
size_t crop_args_bytes();
void pack_crop_args(const float inv[9], const float t[3], float mn, float mx, void* dst);
void launch_crop_count_multi(hipStream_t s, int n, int n_crops, const void* args, const float4* pts,
                             uint32_t* tile_cnt, uint32_t* tile_off, uint32_t* totals);
void launch_crop_scatter_multi(hipStream_t s, int n, int n_crops, const void* args, const float4* pts,
                               const uint32_t* tile_off, const uint32_t* base_of, float4* out);
void launch_solve6(hipStream_t s, const double* A, const double* b, double* x, int32_t* path);

// ---- kd-tree construction (kernels_tree.hip) ---------------------------------------------
struct TreeWork {
  float4* W[2];          // points being partitioned (ping-pong), total
  int32_t* segof[2];     // segment of each position at the current / next level, total
  TreeSeg* seg[2];       // segments of the current / next level, max_seg
  uint32_t* flag;        // total + 2
  uint32_t* X1;          // scans, total + 2
  uint32_t* X2;
  uint32_t* posL;        // partner positions, total
  uint32_t* posR;
  NodeEvent* ev;         // 2 * total slots (leaf: first position; inner: total + split position)
  uint8_t* valid;        // 2 * total
  SubSeg* subs;          // wave-subtree segments, max_seg
  SubSeg* mids;          // mid-size segments (kSubMax < count <= kMidMax), max_seg
  uint32_t* ecnt;        // nodes ending at each position, total + 2
  uint64_t* sums;        // 6 per pair (128-bit fixed-point coordinate sums), then 6 per tree_sum_tiles tile
  int32_t* pair_depth;   // per pair
  TreeCtl* ctl;
  void* scan_temp;
  size_t scan_temp_bytes;
  size_t max_seg;
  int n_pairs;
  uint64_t* lb;          // look-back words of the build's scans (lb_bytes), zeroed by launch_tree_prepare
  size_t lb_stride;      // words per scan
  uint32_t mid_max;      // segments up to this size leave the global levels (kMidMax; kSubMax: no mid builder)
  uint32_t lvl_min;      // the level-synchronous subtree builder from this many points (aicp_hip_options)
};
uint32_t tree_mid_max();
hipError_t set_lb_force_stall(int on);  // aicp_hip_test_force_scan_stall
size_t tree_sum_tiles(size_t n);  // k_tr_sum's tiles over n points
size_t tree_scan_temp_bytes(size_t n);
size_t lb_bytes(uint32_t total);
size_t lb_stride_words(uint32_t total);
// centroid (center = 1) + frames in pd, centred points, root segments
// matcher treelets of n_refs trees (rd[r].tl_off / tl_cap set by the host) of the build w (its
// look-back words and control block; cap = 2 * its points + 2): rank: cap + 1 words; errors into
// w.ctl->error (bit 4)
hipError_t launch_treelets(hipStream_t s, int n_refs, uint32_t cap, const PairDesc* rd, const uint4* nodes,
                           int bucket, uint32_t* rank, uint4* tl, uint2* link, const TreeWork& w);
// part 1: only what does not read the points (zeroed work space; frames when center = 0); part 2:
// the rest; 0: all
hipError_t launch_tree_prepare(hipStream_t s, int n_pairs, uint32_t total, PairDesc* pd, const float4* raw,
                               int center, const TreeWork& w, float4* bpts, int bucket, int part = 0);
// one level: nodes at depth `level` are split (their children get depth level + 1)
// last: the final planned level -- children above kSubMax points also go to the subtree
// kernel (its global-memory path) instead of a next level
hipError_t launch_tree_level(hipStream_t s, int level, uint32_t total, const TreeWork& w, float4* bpts,
                             int bucket, bool last);
// mid-size segments, one workgroup each: nodes split in LDS until the pieces fit the subtree builders
hipError_t launch_tree_mid(hipStream_t s, uint32_t total, const TreeWork& w, float4* bpts, int bucket);
// subtrees of the segments with <= kSubMax points, one wave each (grid-stride over the device count)
hipError_t launch_tree_subtrees(hipStream_t s, uint32_t total, const TreeWork& w, float4* bpts,
                                int bucket);
// node records (preorder) and PairDesc node_off / n_nodes / tree_depth
hipError_t launch_tree_finish(hipStream_t s, int n_pairs, uint32_t total, PairDesc* pd, const TreeWork& w,
                              uint4* nodes);

// pairs -> their shared reference's centroid / tree fields (+ T_refMean_dataIn), and its
// SurfaceNormal degenerate count
void launch_pairs_from_refs(hipStream_t s, int n_pairs, PairDesc* pd, const PairDesc* rd);
// normals of the raw-coordinate tree's bucket order -> bnrm in the matcher tree's order
void launch_normals_to_matcher(hipStream_t s, int n_refs, uint32_t total, const PairDesc* rd, const float4* bpts,
                               const float4* bpts_raw, const float4* nrm_raw, uint32_t* inv, float4* bnrm);
void launch_pairs_degenerate(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const PairState* rst);
void launch_pairs_degenerate_part(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const PairState* rst,
                                  int what);

// ---- overlap ------------------------------------------------------------------------------
// Clouds: the reference side runs over overlap groups (one per distinct reference cloud and
// origin; pd = group descriptors, st = group states), the reading side over pairs.
// sides: 1 = reference origin, 2 = reading origin
void launch_ovl_init(hipStream_t s, int n, const PairDesc* pd, PairState* st, double res, int sides);
void launch_ovl_bbox(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                     const float4* pts, int side, double res);
// od[i]: the map of entry i (group or pair) of the side being marked; max_blocks > 0: at most
// that many workgroups, each marking every max_blocks-th block of the map
void launch_ovl_mark(hipStream_t s, BlockMap m, const PairDesc* pd, const OvlDesc* od, PairState* st,
                     const float4* pts, int side, double res, uint8_t* maps, bool filter,
                     unsigned max_blocks = 0);
// |A| per group (gst.ovl_counts[0]), |B| and |A∩B| per pair (st.ovl_counts[1], [2])
void launch_ovl_count(hipStream_t s, int n_pairs, int n_groups, const PairDesc* pd, const OvlDesc* od_read,
                      const OvlDesc* od_ref, PairState* st, PairState* gst, const uint8_t* maps);
// the parts of launch_ovl_count: |S| of n maps into st[i].ovl_counts[slot]; |A∩B| per pair
// wide: many workgroups per map (the one-shot call of a single pair)
void launch_ovl_popcount(hipStream_t s, int n, const OvlDesc* od, PairState* st, int slot, const uint8_t* maps,
                         bool wide = false);
void launch_ovl_intersect(hipStream_t s, int n_pairs, const PairDesc* pd, const OvlDesc* od_read, const OvlDesc* od_ref,
                          PairState* st, const uint8_t* maps, bool wide = false);
void launch_ovl_finish(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st, const PairState* gst,
                       int set_ratio);

// ---- sparse overlap (kernels_overlap_sparse.hip): sorted key words instead of voxel maps -------
size_t ovl_sparse_scan_bytes(size_t n_points);
size_t ovl_sparse_sort_bytes(size_t n_keys);
// per point key counts (cnt, n_points slots) and their exclusive prefix (off)
hipError_t launch_ovl_sparse_count(hipStream_t s, uint32_t n_blocks, const uint32_t* blk_cloud,
                                   const uint32_t* blk_start, const OvlCloud* clouds, const float4* ref,
                                   const float4* read, double res, uint32_t n_points, uint32_t* cnt, uint64_t* off,
                                   void* temp, size_t temp_bytes);
// keys -> sorted words -> |S| of every cloud (gst[g].ovl_counts[0], st[p].ovl_counts[1]) and
// |A ∩ B| per pair (st[p].ovl_counts[2]); clouds: n_groups groups then n_pairs readings
hipError_t launch_ovl_sparse_sets(hipStream_t s, uint32_t n_blocks, const uint32_t* blk_cloud,
                                  const uint32_t* blk_start, const OvlCloud* clouds, const float4* ref,
                                  const float4* read, double res, const uint64_t* off, uint64_t n_keys,
                                  uint64_t* keys0, uint64_t* keys1, void* temp, size_t temp_bytes, int n_groups,
                                  int n_pairs, const PairDesc* pd, unsigned long long* per_cloud,
                                  unsigned long long* per_pair, PairState* gst, PairState* st);

// The stream's sorted-key overlap: one side of a window (its readings, or its reference) as a
// key list of `cap` words, cap = a host bound of the keys (no read-back of the true count).
struct OvlKeySide {
  OvlCloud* clouds;            // n_clouds (device)
  int n_clouds;
  const uint32_t* blk_cloud;   // n_blocks blocks of 256 points
  const uint32_t* blk_start;
  uint32_t n_blocks;
  uint32_t n_points;           // count slots (clouds[c].slot + j)
  uint32_t* cnt;               // n_points
  uint64_t* off;               // n_points
  uint64_t cap;
  uint64_t* keys0;             // cap each
  uint64_t* keys1;             // sorted
  void* temp;                  // ovl_keys_temp_bytes
  size_t temp_bytes;
  unsigned long long* per_cloud;  // n_clouds
};
size_t ovl_keys_temp_bytes(size_t n_points, size_t cap, int n_clouds);
// keys of the side's clouds (points at pts + clouds[c].pts_off), sorted; |S_c| into
// st[c].ovl_counts[slot]; origin0 (nullable, 3 device doubles): clouds[0].origin := origin0 first.
// A cloud whose keys exceed cap reports st[c].ovl_err.
hipError_t launch_ovl_keys(hipStream_t s, const OvlKeySide& k, const double* origin0, const float4* pts,
                           double res, PairState* st, int slot);
// |A ∩ B| of every reading of rd against the reference side (one cloud) into st[p].ovl_counts[2]
hipError_t launch_ovl_keys_intersect(hipStream_t s, const OvlKeySide& rd, const OvlKeySide& ref,
                                     unsigned long long* per_pair, PairState* st);

// ---- frame-to-reference stream (kernels_sequence.hip) ---------------------------------------
// gd->ref_origin = translation of fromMatrix4fToIsometry3d(T) * prior pose of src (1 thread);
// T (src's correction, written by another stream's kernel) is copied to Tcopy for the transform
// that follows on the same stream
// the next reference: its origin into gd, Tcopy = T, out = T * in (k_transform's arithmetic);
// src_st (nullable): T from the source's state and frames instead (k_finalize's product)
void launch_seq_ref_points(hipStream_t s, int n, PairDesc* gd, const PairDesc* src, const PairState* src_st,
                           const float* T, float* Tcopy, const float4* in, float4* out);
// the window's descriptors, states and corrections into the sequence's arrays (np readings)
void launch_seq_commit(hipStream_t s, int np, const PairDesc* d, const PairState* st, const float* T, PairDesc* gd,
                       PairState* gst, float* gT);
// a[0, na), b[0, nb), c[0, nc) = 0 in one launch
void launch_zero_words3(hipStream_t s, uint32_t* a, size_t na, uint32_t* b, size_t nb, uint32_t* c, size_t nc);
// debug working mode (app.cpp:87-96, 414), one thread each: hist := initT, d's prior origin :=
// translation of initT * prior pose; then outT := d's correction and, if it is accepted,
// initT := correction * initT
void launch_debug_prep(hipStream_t s, PairDesc* d, const float* initT, float* hist);
void launch_debug_post(hipStream_t s, const PairDesc* d, PairState* st, float* outT, float* initT, float max_corr);
// od[i] (min, dim, bytes) from st[i].ovl_bbox; od[i].off preset; bytes > cap[i]: ovl_err, empty map
void launch_ovl_size(hipStream_t s, int n, PairState* st, OvlDesc* od, const uint64_t* cap);
// zero the n maps of od[] (device-side sizes, each at most max_bytes)
void launch_ovl_clear(hipStream_t s, int n, const OvlDesc* od, uint8_t* maps, uint64_t max_bytes);

// ---- pre-filter (kernels_prefilter.hip): regionGrowingUniformPlaneSegmentationFilter -------
constexpr int kPfMaxNbrs = 16;  // RegionGrowing neighbours per point (edge mask bits)
struct PfCtl {                  // device control block; lo = 0xFFFFFFFF, everything else 0 at start
  uint32_t lo[3], hi[3];        // order-preserving bits of the finite points' min / max
  uint32_t n_fin, n_bad;        // finite / non-finite input points
  int32_t minb[3];              // VoxelGrid min_b_
  uint32_t mul1, mul2;          // divb_mul_[1], divb_mul_[2]
  float inv;                    // inverse leaf size
  uint32_t passthrough;         // PCL's integer-overflow guard fired: the cloud passes unfiltered
  uint32_t n_vox;               // sampled points V
  uint32_t n_inf;               // points left for k_rg_phaseb
  uint32_t n_seg, n_clusters, n_out;
};
struct PfWork {  // scratch, n (+1) words each
  uint32_t *k0, *k1, *v0, *v1, *flag, *scan, *keep, *kpts, *koff;
  void* temp;
  size_t temp_bytes;
};
size_t pf_temp_bytes(size_t n);
// VoxelGrid: ctl->n_vox centroids into sampled (ascending voxel index)
hipError_t launch_pf_voxel(hipStream_t s, uint32_t n, const float4* pts, float inv, PfCtl* ctl, const PfWork& w,
                           float4* sampled);
// NormalEstimation from the kNN of the sampled tree (bucket order); k in {10, 20, 30}
// ids: launch_knn_ids output (bucket positions)
bool launch_pf_normals(hipStream_t s, uint32_t V, int k, int nnb, const float4* bpts, const float4* sampled,
                       const int32_t* ids, uint32_t* inv, const float vp[3], float4* nrm, int32_t* nbp, uint2* kth,
                       uint32_t* ckey, uint32_t* cval);
// seed order, edge masks and initial labels
hipError_t launch_pf_order(hipStream_t s, uint32_t V, int nnb, const PfWork& w, const uint32_t* ckey,
                           const uint32_t* cval, const uint32_t* inv, const float4* bpts, const float4* nrm,
                           const int32_t* nbp, const uint2* kth, float cos_thr, float curv_thr, uint32_t* nob,
                           uint32_t* order_of, uint32_t* em, uint32_t* label);
// union-find over mutual edges (marked in em bits 17..): comp[x] = component root, roots start at their members' minimum
void launch_rg_components(hipStream_t s, uint32_t V, int nnb, const int32_t* nbp, uint32_t* em, uint32_t* comp,
                          uint32_t* label);
void launch_rg_iter(hipStream_t s, uint32_t V, int nnb, const int32_t* nbp, const uint32_t* em, const uint32_t* nob,
                    const uint32_t* comp, uint32_t* label, uint32_t* changed);
void launch_rg_settle(hipStream_t s, uint32_t V, const uint32_t* comp, uint32_t* label);
void launch_rg_count_inf(hipStream_t s, uint32_t V, const uint32_t* label, PfCtl* ctl);
void launch_rg_phaseb(hipStream_t s, uint32_t V, int nnb, const int32_t* nbp, const uint32_t* em, const uint32_t* nob,
                      uint32_t* label);
// clusters of min..max points: out (creation order, ascending index), cluster of every point
hipError_t launch_rg_extract(hipStream_t s, uint32_t V, uint32_t min_size, uint32_t max_size, const uint32_t* label,
                             const uint32_t* inv, const float4* sampled, const PfWork& w, float4* out,
                             int32_t* cluster_of, PfCtl* ctl);

}  // namespace aicp
