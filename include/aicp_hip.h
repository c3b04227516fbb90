/*
 * aicp_hip.h — C-ABI of the MI355X-native ICP registration core (libaicp_hip.so).
 *
 * This is the drop-in boundary that replaces the in-process C++ virtual interfaces
 * of aicp_core (reference paths relative to zbqq/aicp_mapping):
 *
 *   aicp::AbstractRegistrator   aicp_core/include/aicp_registration/abstract_registrator.hpp:8-19
 *     registerClouds(ref, read, Matrix4f&)   -> aicp_hip_register / aicp_hip_register_batch
 *     getOutputReading(cloud)                -> aicp_hip_transform
 *     updateConfigParams(path)               -> aicp_hip_parse_pm_yaml
 *   aicp::AbstractOverlapper    aicp_core/include/aicp_overlap/abstract_overlapper.hpp:13-19
 *     computeOverlap(...) + getOverlap()     -> aicp_hip_overlap / aicp_hip_overlap_batch
 *   App::computeRegistration ratio auto-tune aicp_core/src/registration/app.cpp:197-205
 *     + replaceRatioConfigFile               aicp_core/src/utils/fileIO.cpp:179-214
 *                                            -> aicp_hip_autotune_ratio,
 *                                               aicp_hip_replace_ratio_config_file,
 *                                               aicp_hip_align_batch (overlap -> ratio -> ICP on device)
 *
 * Conventions
 *   - Plain C, no exceptions cross this boundary; every entry point returns an AICP_* code.
 *   - Host memory is caller-owned. Point arrays are AoS float x,y,z at a byte stride, so a
 *     pcl::PointXYZ array (16 B per point) passes zero-copy with stride = 16.
 *   - Counts are explicit (the reference uses cloud.width, cloudIO.cpp:83).
 *   - Transforms are column-major float[16], so Eigen::Matrix4f::data() passes through.
 *   - A context owns one HIP stream and a device arena; use one context per host thread
 *     (the reference calls its registrator from a single worker thread, app.cpp:528-550).
 */
#ifndef AICP_HIP_H_
#define AICP_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes --------------------------------------------------------------------- */
#define AICP_OK 0
#define AICP_ERR_CONVERGENCE 1  /* maps PM::ConvergenceError ("no outlier to filter",
                                   "no point to minimize", NaN in the differential checker) */
#define AICP_ERR_INVALID 2      /* invalid argument / config (reference: exit(1),
                                   pointmatcher_registration.cpp:60-64,96-100) */
#define AICP_ERR_HIP 3          /* HIP runtime failure or extension unavailable */
#define AICP_ERR_UNSUPPORTED 4  /* chain element or size not supported by this core */
#define AICP_ERR_TRANSFORMATION 5 /* maps PM::TransformationError: a transform applied to the
                                     reading has |1 - det R| > 0.001 (RigidTransformation::
                                     checkParameters; the initial T, every T_iter, the final T) */

typedef struct aicp_hip_ctx aicp_hip_ctx;
typedef struct aicp_hip_batch aicp_hip_batch;

/* The libpointmatcher chain subset of icp_autotuned_default.yaml:9-51. */
typedef struct {
  int32_t knn_normals;    /* SurfaceNormalDataPointsFilter.knn            (20)   */
  float nn_epsilon;       /* KDTreeMatcher.epsilon                        (3.16) */
  float nn_max_dist;      /* KDTreeMatcher.maxDist                        (inf)  */
  float trimmed_ratio;    /* TrimmedDistOutlierFilter.ratio               (0.70) */
  int32_t max_iter;       /* CounterTransformationChecker.maxIterationCount (20) */
  float min_diff_rot;     /* DifferentialTransformationChecker.minDiffRotErr (1e-3) */
  float min_diff_trans;   /* DifferentialTransformationChecker.minDiffTransErr (1e-2) */
  int32_t smooth_length;  /* DifferentialTransformationChecker.smoothLength (4) */
  int32_t bucket_size;    /* libnabo kd-tree bucketSize                    (8)   */
  int32_t knn_match;      /* KDTreeMatcher.knn; only 1 is supported        (1)   */
} aicp_icp_config;

typedef struct {
  int32_t status;            /* AICP_* code of this pair                          */
  int32_t iterations;        /* ICP iterations executed (IterationsCount)         */
  int32_t converged;         /* 1: differential checker stopped, 0: counter limit */
  int32_t degenerate_normals;/* SurfaceNormal rank-deficient points (reference)   */
  float inlier_ratio;        /* weightedPointUsedRatio of the last iteration      */
  float trimmed_ratio;       /* ratio actually used                               */
  float overlap_percent;     /* octree-equivalent overlap, -1 if not computed     */
  int32_t tree_depth;        /* depth of the matcher kd-tree                      */
  uint64_t nn_points_touched;/* libnabo PointCountTouched over all iterations     */
  uint64_t nn_nodes_touched; /* inner nodes descended over all iterations         */
  uint64_t overlap_keys[3];  /* |S_ref|, |S_read|, |S_ref ∩ S_read|                */
} aicp_icp_stats;

typedef struct {
  const float* ref;      /* reference cloud, x,y,z at ref_stride bytes            */
  uint64_t n_ref;
  uint64_t ref_stride;   /* bytes between points: 12 packed, 16 / 32 / 48 =      */
                         /* pcl::PointXYZ / PointXYZRGB / PointXYZRGBNormal rows   */
  const float* read;     /* reading cloud                                         */
  uint64_t n_read;
  uint64_t read_stride;
  const float* init_T;   /* nullable = identity; column-major 4x4                 */
  double ref_origin[3];  /* sensor origin of the reference (pose translation)     */
  double read_origin[3]; /* sensor origin of the reading                          */
} aicp_pair;

/* One cloud with its sensor origin (the sequence and localization entry points). */
typedef struct {
  const float* pts;      /* x, y, z at `stride` bytes */
  uint64_t n;
  uint64_t stride;
  double origin[3];      /* prior pose translation = sensor origin (octrees_overlap.cpp:229-230) */
} aicp_cloud;

/* flags for aicp_hip_align_batch / aicp_hip_batch_run */
#define AICP_RUN_OVERLAP 1      /* compute overlap and auto-tune the trimmed ratio */
#define AICP_RUN_ICP 2          /* run the ICP registration                        */
#define AICP_RUN_TIME_NN 4      /* record HIP events around every NN launch        */

/* ---- context ---------------------------------------------------------------------------- */
int aicp_hip_create(int device, aicp_hip_ctx** out);
void aicp_hip_destroy(aicp_hip_ctx* ctx);
const char* aicp_hip_last_error(const aicp_hip_ctx* ctx);
const char* aicp_hip_version(void);
/* Provenance of this binary: "src <sha256 prefix of its sources and Makefile> arch <gfx> extra
 * <extra compile flags>" (aicp_mapping_amd/csrc/Makefile); aicp_mapping_amd._lib.source_hash()
 * computes the same hash from a source tree. */
const char* aicp_hip_build_info(void);

/* Context options: the engine and schedule switches the tests and A/B measurements use. The
 * library reads no environment variable; a context starts with aicp_hip_default_options' values
 * (the product path) and keeps what aicp_hip_set_options gives it until the next call. No option
 * changes a result: every engine and schedule gives the same transforms, statistics and counts
 * (the tests compare them). Replaces nothing in the reference. */
typedef struct {
  int32_t profile;            /* 1: host and device phase times (and the counters of the diagnostic
                                 build, -DAICP_DIAG=1) on stderr; the timing events it records
                                 shift the schedule slightly */
  int32_t nn_engine;          /* 0: treelet records where they fit (bucketSize <= 15, <= 4 M
                                 reference points); 1: node records (Trav<1>) always */
  int32_t overlap_path;       /* 0: voxel maps within their memory budget, sorted key lists above;
                                 1: sorted key lists always */
  int32_t normals_knn_engine; /* SurfaceNormal kNN: 0: one octet of lanes per query up to 300 000
                                 queries, one lane above; 1: octets always; 2: one lane always */
  int32_t select_pair;        /* trimmed select: -1: one workgroup per pair from 256 pairs on
                                 (readings <= 65536 each); 0: never; 1: whenever it fits */
  int32_t select_fused_from;  /* ICP iteration from which the chip-wide select runs as one launch
                                 (0: never); 3 */
  int32_t raw_tree_first;     /* batch path: -1: the raw-coordinate tree before the matcher tree
                                 from 4 M reference points on; 0: never; 1: always */
  int32_t raw_first_at;       /* with the raw tree first, the matcher tree starts after the raw
                                 tree's global levels (2) or after the whole raw tree (1); 2 */
  int32_t no_early_exit;      /* 1: every ICP loop enqueues maxIterationCount iterations (tests:
                                 the polled early exit must not change results) */
  int32_t tree_plan;          /* kd-tree global levels: 0: planned from the cloud size; k > 0: k
                                 levels (tests: a too-shallow plan); -1: host-polled build */
  uint32_t tree_lvl_min;      /* the level-synchronous subtree builder from this many points of a
                                 build on; 4194304 */
  int32_t reference_cache;    /* 1: the one-shot calls keep their reference (and last reading)
                                 resident for the next call, identified by a byte compare against a
                                 host copy (aicp_hip_reference_cache_stats); 0: nothing is kept,
                                 copied or compared between calls */
  uint32_t oneshot_keep_mib;  /* device copies of a one-shot call's inputs are kept for the next
                                 call up to this size (MiB), released above it; 4096 */
  int32_t early_reference;    /* stream (non-debug): 1: the next reference starts once its source
                                 reading's registration has stopped, while the window's other
                                 readings still iterate; 0: once the whole window's loop ends; 1 */
  uint64_t read_order_min;    /* Morton order of a batch's readings from this many points on;
                                 200000 */
} aicp_hip_options;
void aicp_hip_default_options(aicp_hip_options* out);
int aicp_hip_set_options(aicp_hip_ctx* ctx, const aicp_hip_options* opt);
int aicp_hip_get_options(const aicp_hip_ctx* ctx, aicp_hip_options* out);
/* Test hook, process-wide on the calling thread's device: on != 0 sends every tile but the first
 * of the kd-tree builds' single-pass scans down the path a stalled look-back takes (the exact
 * prefix recomputed, error 16 reported: the call returns AICP_ERR_HIP and nothing faults). */
int aicp_hip_test_force_scan_stall(int on);

/* ---- configuration (host-only; the reference re-parses the chain per call) -------------- */
void aicp_hip_default_config(aicp_icp_config* out);
/* Parses the libpointmatcher chain subset (pointmatcher_registration.cpp:59-66).
 * Unsupported chain elements yield AICP_ERR_UNSUPPORTED. */
int aicp_hip_parse_pm_yaml(const char* path, aicp_icp_config* out);
/* Text rewrite of "ratio: " + 4 chars, byte-for-byte as fileIO.cpp:179-214. */
int aicp_hip_replace_ratio_config_file(const char* in_path, const char* out_path, float ratio);
/* clamp(overlap/100, .25, .70) (app.cpp:197-202) then the 6-significant-digit text
 * round trip of replaceRatioConfigFile + lexical_cast<float>. */
float aicp_hip_autotune_ratio(float overlap_percent);

/* ---- registration / overlap (host buffers) ---------------------------------------------- */
int aicp_hip_register(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_pair* pair,
                      float out_T[16], aicp_icp_stats* stats /* nullable */);
int aicp_hip_register_batch(aicp_hip_ctx* ctx, const aicp_icp_config* cfg,
                            const aicp_pair* pairs, size_t n_pairs,
                            float* out_T /* 16*n */, aicp_icp_stats* stats /* n, nullable */);
int aicp_hip_overlap(aicp_hip_ctx* ctx, const aicp_pair* pair, double resolution,
                     float* out_overlap_percent);
int aicp_hip_overlap_batch(aicp_hip_ctx* ctx, const aicp_pair* pairs, size_t n_pairs,
                           double resolution, float* out_overlap_percent /* n */,
                           aicp_icp_stats* stats /* n, nullable: overlap_keys */);
/* Reference cache of the one-shot calls above (register*, overlap*, align_batch). App registers
 * reading after reading against one reference (app.cpp:72-73; a new one every
 * reference_update_frequency readings, app.cpp:383-391) and calls computeOverlap then
 * registerClouds per reading (app.cpp:132-135, 205-210). When every pair of a call passes the same
 * reference array as the previous call -- (pointer, count, stride) equal and the points
 * byte-identical to a copy the context keeps -- the reference's centroid, kd-trees, treelets and
 * normals (ICP), and its voxel map for the same origin and resolution (overlap), stay resident in
 * the context and are reused; the reference is not uploaded again. Any other call that rewrites
 * those buffers (a batch with several references, the kernel-level entry points, the
 * pre-filter) drops the cache. Results are the same as without it.
 * out: tree hits, tree builds, overlap-map hits, overlap-map builds since the context's creation. */
int aicp_hip_reference_cache_stats(const aicp_hip_ctx* ctx, uint64_t out[4]);
/* App::runAicpPipeline hot path (app.cpp:218-247): overlap -> auto-tuned ratio -> ICP,
 * all on device, one launch sequence for the whole batch. cfg->trimmed_ratio is ignored
 * when flags has AICP_RUN_OVERLAP. */
int aicp_hip_align_batch(aicp_hip_ctx* ctx, const aicp_icp_config* cfg,
                         const aicp_pair* pairs, size_t n_pairs, double resolution, int flags,
                         float* out_T /* 16*n */, aicp_icp_stats* stats /* n, nullable */);
/* ---- several GPUs from one host process (C5) ----------------------------------
 * Independent pairs shard across devices with no data-path exchange: one context and one host
 * thread per device, longest-processing-time shards by n_read * log2(n_ref), and the per-pair
 * results written at the pairs' own indices (the gather). Replaces nothing in the reference,
 * which registers one pair at a time on the CPU (app.cpp:528-550); it is the C++ host's form of
 * bench.py's torch.distributed path. devices = NULL: devices 0..n_devices-1 (n_devices <= 0:
 * every visible device); a device may be listed more than once (several contexts on one GPU). */
typedef struct aicp_hip_multi aicp_hip_multi;
int aicp_hip_multi_create(const int* devices, int n_devices, aicp_hip_multi** out);
void aicp_hip_multi_destroy(aicp_hip_multi* m);
int aicp_hip_multi_size(const aicp_hip_multi* m);
aicp_hip_ctx* aicp_hip_multi_context(aicp_hip_multi* m, int i);
const char* aicp_hip_multi_last_error(const aicp_hip_multi* m);
/* aicp_hip_align_batch over the devices; out_device (n, nullable): the device of each pair */
int aicp_hip_multi_align_batch(aicp_hip_multi* m, const aicp_icp_config* cfg, const aicp_pair* pairs,
                               size_t n_pairs, double resolution, int flags, float* out_T /* 16*n */,
                               aicp_icp_stats* stats /* n, nullable */, int* out_device /* n, nullable */);

/* getOutputReading: out = T * in (float, pad row 1), pointmatcher_registration.cpp:128-131. */
int aicp_hip_transform(aicp_hip_ctx* ctx, const float T[16], const float* in, size_t n,
                       size_t stride, float* out /* packed xyz, 3*n */);

/* Localization-only map crop, getPointsInOrientedBox (aicp_core/src/utils/filteringUtils.cpp:619-637,
 * called at app.cpp:41-51): pcl::CropBox with the cube [min, max]^3, rotation =
 * origin.R.eulerAngles(0,1,2) and translation = origin.t (origin: Matrix4f, col-major). Kept
 * points are written packed xyz in input order to out (capacity n points); *out_n = count.
 * Non-finite points are dropped. rpy_out (nullable) receives the box angles. */
int aicp_hip_crop_box(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, float min,
                      float max, const float origin[16], float* out /* 3*n */, size_t* out_n,
                      float* rpy_out /* 3, nullable */);

/* Pre-filter regionGrowingUniformPlaneSegmentationFilter (aicp_core/src/utils/filteringUtils.cpp:5-45,
 * called at app.cpp:109,295,491 and app_ros.cpp:309; the XYZRGBNormal overload :51-103 adds the
 * viewpoint, the sampled cloud with normals and the clusters): pcl::VoxelGrid (leaf 0.08) ->
 * pcl::NormalEstimation (k 30) -> pcl::RegionGrowing (15 neighbours, 3 deg, curvature 1.0,
 * clusters of 50..1e6 points). Rules for PCL's unspecified orders: DESIGN.md §4.4. */
typedef struct {
  float leaf_size;           /* VoxelGrid leaf, all three axes (0.08) */
  int32_t normal_k;          /* NormalEstimation k: 10, 20 or 30 (30) */
  int32_t neighbours;        /* RegionGrowing neighbours, <= min(16, normal_k) (15) */
  int32_t min_cluster_size;  /* 50 */
  int32_t max_cluster_size;  /* 1000000 */
  float smoothness_rad;      /* 3.0 / 180.0 * M_PI as float */
  float curvature_threshold; /* 1.0 */
  float viewpoint[3];        /* NormalEstimation viewpoint ((0,0,0): the first overload) */
} aicp_prefilter_params;
void aicp_hip_default_prefilter(aicp_prefilter_params* out);
/* out: the clusters' points concatenated (clusters in creation order, each in sampled-cloud
 * order), packed xyz, capacity n points; *out_n = count. Optional (nullable, capacity n):
 * sampled = 8 floats per sampled point {x, y, z, curvature, nx, ny, nz, 0}; labels = cluster of
 * each sampled point (-1: in no kept cluster). A cloud whose voxel grid would overflow 32-bit
 * indices passes unfiltered (as in PCL), which requires finite points (else
 * AICP_ERR_UNSUPPORTED). */
int aicp_hip_prefilter(aicp_hip_ctx* ctx, const aicp_prefilter_params* prm, const float* pts, size_t n,
                       size_t stride, float* out /* 3*n */, size_t* out_n, float* sampled /* 8*n */,
                       int32_t* labels /* n */, size_t* n_sampled /* nullable */,
                       size_t* n_clusters /* nullable */);

/* Timing of the last aicp_hip_prefilter (HIP events on the context stream). */
typedef struct {
  double voxel_ms;          /* VoxelGrid: bounds, keys, sort, centroids */
  double normals_ms;        /* kd-tree of the sampled cloud, kNN, normals */
  double segment_ms;        /* RegionGrowing: seed order, union-find, propagation (with its host
                               round trips), cluster extraction */
  double device_ms;         /* input uploaded -> clusters ready */
  double wall_ms;           /* the whole call: host packing, PCIe both ways */
  double knn_ms;            /* the kNN kernel alone */
  uint64_t knn_queries;     /* sampled points */
  uint64_t knn_points_touched, knn_nodes_touched;
  int32_t propagation_passes;
  int32_t pad;
} aicp_prefilter_stats;
int aicp_hip_last_prefilter_stats(const aicp_hip_ctx* ctx, aicp_prefilter_stats* out);

/* ---- device-resident prior map (localization mode) ------------------------------------------
 * App keeps prior_map_ and, per reading, crops it around the prior pose (setReference,
 * app.cpp:41-51), appends the aligned reference reading every reference_update_frequency clouds
 * (merge_aligned_clouds_to_map, app.cpp:469-483: *merged = *prior_map + *output, output =
 * transformPointCloud(read_prefiltered, correction)) and pre-filters the whole map every 30
 * clouds (app.cpp:485-493). The map stays in HBM: crop, merge and pre-filter run on it without
 * re-uploading it. */
typedef struct aicp_hip_map aicp_hip_map;
int aicp_hip_map_create(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, aicp_hip_map** out);
void aicp_hip_map_free(aicp_hip_ctx* ctx, aicp_hip_map* map);
int aicp_hip_map_size(const aicp_hip_map* map, size_t* n);
/* the map's points, packed xyz (capacity cap points) */
int aicp_hip_map_download(aicp_hip_ctx* ctx, const aicp_hip_map* map, float* out, size_t cap, size_t* out_n);
/* getPointsInOrientedBox on the map (aicp_hip_crop_box semantics), kept points to out */
int aicp_hip_map_crop(aicp_hip_ctx* ctx, const aicp_hip_map* map, float min, float max, const float origin[16],
                      float* out /* 3*cap */, size_t cap, size_t* out_n);
/* Localization-only batch (localize_against_prior_map, app.cpp:41-51,123-127): reading i is
 * registered against the map cropped on the device to [min, max]^3 around its prior pose
 * poses[16 i .. 16 i + 15] (getPointsInOrientedBox, Matrix4f column-major); the crop goes straight
 * into the batch's reference array (no host round trip). The overlap is fixed at 50 %, so the
 * trimmed ratio is aicp_hip_autotune_ratio(50) = 0.5 whatever cfg->trimmed_ratio says.
 * flags: AICP_RUN_TIME_NN only. An empty crop is AICP_ERR_INVALID. */
int aicp_hip_map_register_batch(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_hip_map* map, float min,
                                float max, const aicp_cloud* readings, const float* poses /* 16*n */, size_t n,
                                int flags, float* out_T /* 16*n */, aicp_icp_stats* stats /* n, nullable */);
/* map += T * pts (pcl::transformPointCloud, T column-major float[16]) */
int aicp_hip_map_merge(aicp_hip_ctx* ctx, aicp_hip_map* map, const float* pts, size_t n, size_t stride,
                       const float T[16]);
/* map = regionGrowingUniformPlaneSegmentationFilter(map) (aicp_hip_prefilter on device data) */
int aicp_hip_map_prefilter(aicp_hip_ctx* ctx, aicp_hip_map* map, const aicp_prefilter_params* prm);

/* ---- device-resident batches (inputs uploaded once, run many times) ----------------------- */
int aicp_hip_batch_upload(aicp_hip_ctx* ctx, const aicp_pair* pairs, size_t n_pairs,
                          aicp_hip_batch** out);
int aicp_hip_batch_run(aicp_hip_ctx* ctx, aicp_hip_batch* batch, const aicp_icp_config* cfg,
                       double resolution, int flags, float* out_T /* 16*n */,
                       aicp_icp_stats* stats /* n, nullable */);
void aicp_hip_batch_free(aicp_hip_ctx* ctx, aicp_hip_batch* batch);
/* Timing of the last batch_run with AICP_RUN_TIME_NN: NN launches, their total duration
 * (HIP events on the context stream), and the algorithmic bytes they moved. */
int aicp_hip_last_nn_timing(const aicp_hip_ctx* ctx, int* n_launches, double* total_ms,
                            double* algorithmic_bytes, uint64_t* queries);
/* Phase times (ms, HIP events) of the last batch_run: [0] overlap (stream 1), [1] raw-
 * coordinate kd-tree + SurfaceNormal (stream 2), [2] centroid + matcher kd-tree (stream 2),
 * [3] icp loop, [4] total wall time. [0] runs concurrently with [1]-[2]. */
int aicp_hip_last_phase_ms(const aicp_hip_ctx* ctx, double out_ms[5]);

/* ---- App's frame-to-reference stream (app.cpp:282-414, robot working mode) ---------------------
 * The first cloud becomes the reference (app.cpp:285-312). Every reading is registered against
 * the current reference (overlap -> auto-tuned ratio -> ICP, app.cpp:218-247); a correction with
 * |t_i| > max_correction_magnitude drops the reading (app.cpp:366-373); an accepted reading is
 * transformed by its correction (pcl::transformPointCloud, float) and, when it is the
 * reference_update_frequency-th accepted reading since the last reference update, it becomes the
 * next reference with the translation of its corrected pose correction * prior pose as sensor
 * origin (app.cpp:375-391, aligned_cloud.cpp:61-70, common.cpp:4-23). A registration error ends
 * the stream, as the uncaught exception ends App's worker (app.cpp:210).
 * Inputs are host buffers (pre-filtered clouds, as App passes read_prefiltered); everything
 * from the upload to the corrections runs on the device, the next reference included. */

/* aicp_sequence_params.flags: App's "debug" working_mode (aicp.launch:36). Each reading is first
 * transformed by initialT_ (pcl::transformPointCloud, float) and its prior pose becomes
 * initialT_ * prior pose (app.cpp:87-96); after each accepted reading initialT_ = correction *
 * initialT_ (app.cpp:414; identity at the start). The readings then depend on each other one by
 * one, so the device registers them one after the other (the reference trees are still built
 * once per window). Without the flag: "robot" mode, the node's default (aicp_ros_node.cpp:14).
 * Filter order: this entry point takes pre-filtered clouds in both modes and moves them by
 * initialT_ afterwards. App moves the RAW reading first and pre-filters the moved cloud
 * (setAndFilterReading, app.cpp:87-99); the 0.08 m VoxelGrid is aligned to the world frame, so the
 * two orders keep different points unless initialT_ is the identity. App's exact order is
 * aicp_hip_sequence_run_raw below; this entry point is the robot-mode fast path. */
#define AICP_SEQ_DEBUG 8

typedef struct {
  int32_t reference_update_frequency; /* 5 (aicp.launch:61) */
  float max_correction_magnitude;     /* 1.0 (aicp.launch:63; aicp_ros_node.cpp:28 default 0.5) */
  double resolution;                  /* octomapResolution (0.2, aicp_config.yaml:21) */
  int32_t flags;                      /* AICP_RUN_OVERLAP: per-reading overlap + auto-tuned ratio
                                         (else cfg->trimmed_ratio); AICP_RUN_TIME_NN; AICP_SEQ_DEBUG */
} aicp_sequence_params;

typedef struct {
  int32_t status;          /* AICP_* of this reading's registration */
  int32_t accepted;        /* 0: dropped, some |t_i| > max_correction_magnitude */
  int32_t reference;       /* cloud it was registered against: -1 the first cloud, else a reading */
  int32_t is_reference;    /* 1: it became the next reference */
  double corrected_origin[3]; /* translation of correction * prior pose (accepted readings; in debug
                                 mode the prior pose is initialT_ * the reading's prior pose) */
  aicp_icp_stats icp;
} aicp_sequence_result;

typedef struct {
  int32_t windows;         /* reference windows run (incl. re-runs after a misprediction) */
  int32_t replans;         /* re-plans after a dropped reading or an error */
  double wall_ms;          /* the whole call: packing, H2D, device work, D2H */
  double device_ms;        /* first upload enqueued -> last correction (HIP events) */
} aicp_sequence_timing;

void aicp_hip_default_sequence_params(aicp_sequence_params* out);
/* out_T: 16 floats per reading (correction, column-major); out: per reading; *n_done = readings
 * processed (all of them unless a registration error ended the stream at reading n_done - 1). */
int aicp_hip_sequence_run(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                          const aicp_cloud* first, const aicp_cloud* readings, size_t n_readings,
                          float* out_T /* 16*n */, aicp_sequence_result* out /* n */, size_t* n_done);
int aicp_hip_last_sequence_timing(const aicp_hip_ctx* ctx, aicp_sequence_timing* out);

/* App's stream from RAW clouds, in App's own order (processCloud, app.cpp:282-414 with
 * setAndFilterReading, app.cpp:77-100): the first cloud is pre-filtered as given (app.cpp:293-297)
 * and becomes the reference. Robot mode: every reading is pre-filtered as given on the device,
 * then the kept points run through aicp_hip_sequence_run. Debug mode (prm->flags AICP_SEQ_DEBUG):
 * reading after reading, the RAW reading is moved by initialT_ on the device
 * (pcl::transformPointCloud, float), the moved cloud is pre-filtered there, its prior pose becomes
 * initialT_ * prior pose, and it is registered against the current reference (overlap ->
 * auto-tuned ratio -> ICP; the reference's trees stay resident across readings); then the drop
 * test, the reference update and initialT_ = correction * initialT_ (app.cpp:362-414). The
 * pre-filter's region growing is host-driven, so debug mode takes host round trips per reading.
 * pf: the pre-filter (aicp_hip_default_prefilter). A reading the pre-filter empties ends the
 * stream with AICP_ERR_INVALID as its status (libpointmatcher throws on an empty cloud).
 * Results as aicp_hip_sequence_run (corrected_origin from initialT_ * prior pose in debug mode);
 * aicp_hip_last_sequence_timing describes robot mode's inner aicp_hip_sequence_run only. */
int aicp_hip_sequence_run_raw(aicp_hip_ctx* ctx, const aicp_icp_config* cfg, const aicp_sequence_params* prm,
                              const aicp_prefilter_params* pf, const aicp_cloud* first, const aicp_cloud* readings,
                              size_t n_readings, float* out_T /* 16*n */, aicp_sequence_result* out /* n */,
                              size_t* n_done);

/* ---- kernel-level entry points (parity tests and diagnostics) --------------------------- */
/* kd-tree over pts (as given, no centring) + k-NN of queries: libnabo
 * KDTreeUnbalancedPtInLeavesImplicitBoundsStackOpt order, ALLOW_SELF_MATCH.
 * ids are input indices of pts; unmatched = -1 with dist +inf. */
int aicp_hip_knn(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride,
                 const float* queries, size_t nq, size_t qstride, int k, float epsilon,
                 float max_dist, int32_t* out_ids /* k*nq */, float* out_d2 /* k*nq */,
                 uint64_t* out_touched /* nullable */);
/* SurfaceNormal descriptor (knn, keepNormals) of pts in input order. */
int aicp_hip_normals(aicp_hip_ctx* ctx, const float* pts, size_t n, size_t stride, int knn,
                     float* out_normals /* 3*n */, int32_t* out_degenerate /* nullable */);
/* Matches::getDistsQuantile on the device (radix select). */
int aicp_hip_dists_quantile(aicp_hip_ctx* ctx, const float* d2, size_t n, float quantile,
                            float* out_limit);
/* solvePossiblyUnderdeterminedLinearSystem on the device (A row-major 6x6, double). */
int aicp_hip_solve6(aicp_hip_ctx* ctx, const double* A, const double* b, double* out_x,
                    int32_t* out_path /* 0 LLT, 1 QR min-norm, 2 eigen pseudo-inverse */);

#ifdef __cplusplus
}
#endif

#endif /* AICP_HIP_H_ */
