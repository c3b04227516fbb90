// aicp_common.hpp — data layout shared by the host orchestrator and the HIP kernels.
//
// HBM layout (one batch = P pairs, every array concatenated over pairs, offsets in PairDesc):
//   read_raw  float4[ΣN]  reading xyz as given (w unused)
//   read_c    float4[ΣN]  reading in the reference-mean frame (T_refMean_dataIn applied once)
//   ref_raw   float4[ΣM]  reference xyz as given (overlap input)
//   bpts      float4[ΣM]  centred reference points in kd-tree bucket order, w = input id bits
//   bnrm      float4[ΣM]  SurfaceNormal normals in bucket order (w = 0)
//   nodes     uint4[ΣW]   kd-tree node records, preorder (left child = n + 1):
//                           inner: x = cut (float bits), y = cd | right << 2, z = parent
//                           leaf : x = bucket count,     y = 3  | bucket_start << 2, z = parent
//                         (16 B: a node record and a bucket point load with one instruction)
//                         w = depth
//   tl        uint4[Σ(4M + 1)] matcher tree as two-level treelet records (kernels_tree.hip)
//   ptl       uint32[Σ(4M + 1)] per treelet: node id of its root's parent
//   match     int32[ΣN]   bucket position of the NN of each reading point
//   d2        float[ΣN]   squared NN distance
// Bucket positions are local to the pair (ref_off added by the kernels).
#pragma once
#include <stdint.h>

// ---- diagnostic builds ----------------------------------------------------------------------
// The product library carries no counters. -DAICP_DIAG=1 builds a diagnostic library
// (tools/variants.sh NAME "-DAICP_DIAG=1 -DAICP_QLAT_PROF=1"), whose counters are chosen with
//   AICP_XCD_PROF   per-XCD-group first start / last end and query cost of each NN launch
//   AICP_QLAT_PROF  per-query NN latency / completion-time histograms
//   AICP_NN_PROF    per-phase s_memtime cycles of the NN's persistent waves
//   AICP_ITER_PROF  bodies and serial tails of the ICP iteration kernels, k_tr_mid phases
// and printed with the context option profile = 1. Without AICP_DIAG each is 0 whatever the
// command line says.
#ifndef AICP_DIAG
#define AICP_DIAG 0
#endif
#if !AICP_DIAG
#undef AICP_XCD_PROF
#undef AICP_QLAT_PROF
#undef AICP_NN_PROF
#undef AICP_ITER_PROF
#endif
#ifndef AICP_XCD_PROF
#define AICP_XCD_PROF 0
#endif
#ifndef AICP_QLAT_PROF
#define AICP_QLAT_PROF 0
#endif
#ifndef AICP_NN_PROF
#define AICP_NN_PROF 0
#endif
#ifndef AICP_ITER_PROF
#define AICP_ITER_PROF 0
#endif

namespace aicp {

constexpr int kHistBins = 2048;     // radix-select digit 1/2 (11 bits)
constexpr int kHist3Bins = 1024;    // digit 3 (10 bits)
constexpr int kNNBlock = 256;       // NN / reduce kernel block
constexpr int kReducePerThread = 4; // reading points per thread and chunk in the reduce kernel
#ifndef AICP_REDUCE_CHUNKS
#define AICP_REDUCE_CHUNKS 1
#endif
constexpr int kReduceChunks = AICP_REDUCE_CHUNKS;  // chunks per reduce thread (2 and 4 measured no faster than 1)
constexpr int kSelPerThread = 16;   // reading points per thread in the select passes
constexpr int kRedCols = 30;        // 21 unique A entries + 6 b + kept + NN touch counts (2)
constexpr int kFarStack = 48;       // max nested far descents (= max tree depth supported)
constexpr int kHistRing = 32;       // differential checker history ring
constexpr uint32_t kLeaf = 3;
constexpr int kMaxPairs = 4096;     // pairs per batch
constexpr int kXcdGroups = 8;       // work groups of the persistent kernels (one per XCD)
constexpr int kCtrStride = 16;      // words between work counters (64 B: one counter per line)
// A persistent kernel's work counters: per XCD group kHeads heads (the group's slot range cut
// into kHeads contiguous parts, so that no more than ~1/kHeads of the group's waves pull from
// one word: a word serves ~88 returning atomics per us, MI355X_MICROARCH.md "dequeue") and one
// word of exhausted-head bits.
#ifndef AICP_NN_HEADS
#define AICP_NN_HEADS 8  // (C2 NN per launch, rocprofv3: 2 heads 75.2, 4 heads 70.6, 8 heads 68.0-68.7 us)
#endif
constexpr int kHeads = AICP_NN_HEADS;
constexpr int kGroupCtrs = kHeads + 1;
constexpr int kPersistCtrWords = kXcdGroups * kGroupCtrs * kCtrStride;  // one persistent kernel's counters
constexpr int kKnnCtrOff = kPersistCtrWords;                            // the normals kNN's, after the ICP NN's
constexpr int kCtrWords = 2 * kPersistCtrWords;                         // ICP NN counters, normals kNN

// One entry of the active list: what a wave of the NN kernel holds in scalar registers while it
// serves a 64-slot chunk of the entry's pair (32 bytes: one scalar load).
struct NnEntry {
  uint32_t off;                // first slot of the pair in the work space
  uint32_t n_read, read_off;   // the pair's readings
  uint32_t tl_off, node_off;   // its matcher tree (treelets / node records)
  uint32_t ref_off;            // its reference points
  int32_t pair;
  uint32_t pad;
};

// Compacted list of the pairs still iterating (k_active_list), consumed by the persistent
// NN kernel: slot s of the work space belongs to pair[e] with off[e] <= s < off[e+1]. The
// chunk table that follows the struct in the same allocation (al_chunks) names the entry of
// every 64-slot chunk, so a wave finds its chunk's context with two dependent scalar loads
// (chunk table, entry) instead of a binary search over off[] plus a PairDesc load.
struct ActiveList {
  uint32_t n;
  uint32_t total;
  uint32_t pad[6];
  NnEntry ent[kMaxPairs];
  uint32_t off[kMaxPairs + 1];
  int32_t pair[kMaxPairs];
};
// the u16 chunk table behind the active list: entry of chunk c (slots [64 c, 64 c + 64))
__host__ __device__ inline uint16_t* al_chunks(ActiveList* al) { return reinterpret_cast<uint16_t*>(al + 1); }
__host__ __device__ inline const uint16_t* al_chunks(const ActiveList* al) {
  return reinterpret_cast<const uint16_t*>(al + 1);
}
// bytes of an active list whose work space holds n_read readings in n_pairs pairs (each pair's
// range padded to a multiple of 64 slots)
inline size_t active_list_bytes(uint64_t n_read, uint64_t n_pairs) {
  return sizeof(ActiveList) + 2 * (size_t)(n_read / 64 + n_pairs + 1) + 4;
}

struct PairDesc {
  uint32_t ref_off, n_ref;      // into ref arrays (ref_raw, bpts, bnrm)
  uint32_t read_off, n_read;    // into reading arrays
  uint32_t node_off, n_nodes;   // into nodes/parent
  uint32_t red_blk_off, n_red_blk;  // reduce blocks of this pair (slab rows)
  float Tin[16];                // initial transform T0 (column-major)
  float Tinit[16];              // T_refMean_dataIn (column-major)
  float Tmean[16];              // T_refIn_refMean
  float mean[3];                // reference centroid (float)
  float ratio;                  // configured trimmed ratio (overridden by overlap)
  int32_t tree_depth;
  int32_t ref_id;               // index of the pair's (deduplicated) reference cloud
  int32_t ogroup;               // overlap group: distinct (reference cloud, reference origin)
  uint32_t tl_off, tl_cap;      // matcher treelets (kernels_tree.hip): first record, records allotted
  double ref_origin[3], read_origin[3];
};

// Overlap voxel maps of a pair (AICP_RUN_OVERLAP): one byte per voxel of the padded key box.
// Kept apart from PairDesc so the overlap (its own stream) never rewrites descriptors the
// kd-tree stream is filling in.
struct OvlDesc {
  int32_t min[3];   // key of voxel (0,0,0), a multiple of the brick extent on each axis
  int32_t dim[3];   // box extent in voxels, a multiple of the brick extent on each axis
  uint64_t off;     // byte offset of this cloud's map in the map arena
  uint64_t bytes;   // map bytes (multiple of 128)
};

// Maps are bricked: 8 x 8 x 2 voxels (key axes 0, 1, 2) per 128-byte brick, bricks in (0, 1, 2)
// row-major order, voxels inside a brick at ((a & 7) << 4) | ((b & 7) << 1) | (c & 1). A ray
// crosses a brick in several steps, so its marks land on ~1/8 of the 128-byte lines a linear
// layout (a new line for every step along axis 0 or 1) has them on, and the lines of a scan's
// near-sensor voxels are shared by more rays. Boxes start on brick boundaries of the key lattice,
// so the 16-byte word s of a brick holds the same voxels (a & 7 = s) in every map.
constexpr int kOvlBrick0 = 8, kOvlBrick1 = 8, kOvlBrick2 = 2, kOvlBrickBytes = 128;
// the padded box of keys [lo, hi] (lo > hi: empty) on one axis of brick extent b
__host__ __device__ inline void ovl_axis(int lo, int hi, int b, int32_t& mn, int32_t& dim) {
  if (lo > hi) lo = hi = 0;  // nothing inside the key range
  const int l = lo - 2, h = hi + 3;  // two voxels of padding below, two above (exclusive end + 1)
  mn = (int32_t)((l >= 0 ? l / b : -((-l + b - 1) / b)) * b);
  dim = (int32_t)(((h - mn) + b - 1) / b * b);
}
// map bytes of a box (the bricks cover it exactly)
__host__ __device__ inline uint64_t ovl_bytes(const int32_t dim[3]) {
  return (uint64_t)dim[0] * (uint64_t)dim[1] * (uint64_t)dim[2];
}
// byte of the voxel at box coordinates (a, b, c), 0 <= a < dim[0] ...
__host__ __device__ inline uint64_t ovl_index(uint32_t a, uint32_t b, uint32_t c, uint32_t dim1, uint32_t dim2) {
  const uint64_t brick = ((uint64_t)(a >> 3) * (dim1 >> 3) + (b >> 3)) * (dim2 >> 1) + (c >> 1);
  return brick * kOvlBrickBytes + (((a & 7u) << 4) | ((b & 7u) << 1) | (c & 1u));
}

// One cloud of the sparse overlap path (kernels_overlap_sparse.hip): an overlap group's reference
// (side 0, points in ref_raw) or a pair's reading (side 1, points in the sorted readings).
struct OvlCloud {
  uint32_t pts_off, n;
  uint32_t side, pad;
  double origin[3];
  uint64_t slot;  // first per-point key-count slot
};

struct PairState {
  float T[16];          // T_iter, column-major
  float limit;          // trimmed distance limit of the current iteration
  float ratio;          // trimmed ratio in use
  int32_t active;       // 1 while iterating
  int32_t status;       // AICP_* code
  int32_t iters;
  int32_t converged;
  int32_t kept;
  int32_t n_finite;
  int32_t hist_count;   // entries pushed into the checker ring
  int32_t degenerate;
  float inlier_ratio;
  float overlap;        // percent, -1 if not computed
  uint64_t touched_pts, touched_nodes;  // libnabo PointCountTouched / inner nodes, all iterations
  uint64_t ovl_counts[3];
  int32_t ovl_bbox[6];  // kmin[3], kmax[3] (union of both clouds)
  int32_t ovl_err;
  uint32_t sel_b1, sel_r1;  // trimmed select: digit-1 bin of the k-th value and its rank in it
  uint32_t sel_miss;    // fused selects whose guessed bin was not the k-th value's (k_sel_fused)
  double qh[kHistRing][4];
  double th[kHistRing][3];
  // per history entry i >= 1: |angdist(q_i, q_i-1)| and |t_i - t_i-1|, computed once when entry
  // i is pushed (the Differential checker sums the last smoothLength of them every iteration)
  double dq[kHistRing], dt[kHistRing];
};

// ---- device kd-tree construction (kernels_tree.hip) ----------------------------------------
// A segment = a node still to split at the current level (count > bucket).
struct TreeSeg {
  uint32_t first, count;   // global point positions
  int32_t pair, depth;
  float mn[3], mx[3];      // node box (libnabo implicit bounds)
  int32_t cd;
  float ideal;             // (mx[cd] + mn[cd]) / 2
  uint32_t lo, hi;         // ordered-int min / max of the points' cd coordinate
  uint32_t br1, br2, left;
  int32_t child[2];        // next-level segment index; -1 leaf child; -2 subtree (SubSeg) child
  int32_t parent_f, parent_depth;  // the parent node's first position and depth (-1: root)
  uint32_t bmn[3], bmx[3]; // root only: ordered-int box of the centred points
};

// One record per node, in a slot of its own: a leaf at its first position, an inner node at
// total + its split position (first + left), which no other node shares; the preorder index
// is computed afterwards.
struct NodeEvent {
  uint32_t f, c;           // point range [f, f + c), global positions
  int32_t depth, pair;
  uint32_t cut_bits;
  int32_t cd;              // kLeaf for a leaf
  uint32_t left;           // left child point count
  uint32_t parent_f;
  int32_t parent_depth;    // -1 at the root
};

// A segment small enough for one wave to finish its whole subtree in LDS (k_tr_subtree).
#ifndef AICP_SUBMAX
#define AICP_SUBMAX 1024
#endif
constexpr int kSubMax = AICP_SUBMAX;  // largest segment one wave finishes in LDS (k_tr_subtree)
struct SubSeg {
  uint32_t f, c;
  int32_t pair, depth;
  float mn[3], mx[3];
  uint32_t parent_f;
  int32_t parent_depth;
};

// A segment of at most kMidMax points is split in one workgroup's LDS (k_tr_mid) down to
// segments of <= kSubMax points; larger ones by the global levels.
#ifndef AICP_MIDMAX
#define AICP_MIDMAX 8192
#endif
constexpr int kMidMax = AICP_MIDMAX;

struct TreeCtl {
  uint32_t nseg[kFarStack + 2];  // segments per global level
  uint32_t n_small;              // SubSeg entries
  uint32_t n_mid;                // mid-size segments (k_tr_mid)
  uint32_t n_big;                // of which above kSubMax points (planned build too shallow)
  int32_t error;
};

struct IcpParams {
  float maxE2;     // (1 + eps)^2, float
  float maxR2;     // maxDist^2
  int32_t max_iter;
  int32_t smooth;
  float min_rot, min_trans;
  int32_t knn_normals;
  int32_t prof_slot;  // diagnostic builds (AICP_XCD_PROF): the launch's record slot
};

}  // namespace aicp
