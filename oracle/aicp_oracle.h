/*
 * aicp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (C++17, single thread, no dependencies) of the reference hot path:
 * libpointmatcher 1.2.x ICP chain of icp_autotuned_default.yaml, libnabo's
 * KDTreeUnbalancedPtInLeavesImplicitBoundsStackOpt, and octomap's ray insertion as used by
 * aicp_core's OctreesOverlap. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 *
 * PARITY UNPINNED: libpointmatcher, libnabo and octomap are third-party libraries that are
 * not vendored in the reference and are absent from this image; the reference's only test
 * (aicp_core/test/aicp_test.cpp) needs external data. No golden vector pins this boundary.
 * The restatement is checked against independent numpy/scipy computations instead
 * (tests/test_oracle.py) and the fixtures it generates are committed under tests/golden/.
 */
#ifndef AICP_ORACLE_H_
#define AICP_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ao_tree ao_tree;

typedef struct {
  int32_t knn_normals;
  float nn_epsilon;
  float nn_max_dist;
  float trimmed_ratio;
  int32_t max_iter;
  float min_diff_rot;
  float min_diff_trans;
  int32_t smooth_length;
  int32_t bucket_size;
  int32_t normals_on_centered; /* 0: reference semantics (normals on raw ref coords, own
                                  tree); 1: normals from the centred matcher tree (the
                                  device design) */
} ao_icp_config;

#define AO_TRACE_MAX 64
typedef struct {
  int32_t status;             /* 0 ok, 1 convergence error, 2 invalid,
                                 5 TransformationError (|1 - det R| > 0.001)      */
  int32_t iterations;
  int32_t converged;          /* differential checker fired                          */
  int32_t degenerate_normals;
  float inlier_ratio;
  float mean[3];              /* reference centroid used for centring               */
  int32_t tree_depth;
  int32_t tree_nodes;
  uint64_t nn_points_touched;
  uint64_t nn_nodes_touched;
  /* per iteration trace */
  float limit[AO_TRACE_MAX];
  int32_t kept[AO_TRACE_MAX];
  int32_t solve_path[AO_TRACE_MAX];
  float T_iter[AO_TRACE_MAX][16]; /* column-major, after the update of iteration i */
  double A0[36];                  /* normal equations of iteration 0 (row-major)    */
  double b0[6];
} ao_icp_stats;

/* kd-tree (libnabo order) over n points of dim 3 read at a float stride. */
int ao_tree_build(const float* pts, int64_t n, int64_t stride_floats, int bucket, ao_tree** out);
void ao_tree_free(ao_tree* t);
int ao_tree_info(const ao_tree* t, int32_t* n_nodes, int32_t* depth, int32_t* n_leaves);
/* Preorder export: cd (0..2 inner, 3 leaf), cut value (inner) / bucket start (leaf),
 * right child (inner) / bucket count (leaf); bucket_ids = point ids in bucket order. */
int ao_tree_export(const ao_tree* t, int32_t* cd, float* cut, int32_t* right_or_count,
                   int32_t* bucket_start, int32_t* bucket_ids);
int ao_tree_knn(const ao_tree* t, const float* q, int64_t nq, int64_t qstride_floats, int k,
                float epsilon, int allow_self, float max_radius, int32_t* ids, float* d2,
                uint64_t* touched_points, uint64_t* touched_nodes);

/* The two-pass partition of buildNodes, sequential form and the prefix-count form used by a
 * parallel build; both return the permutation of values (for cross-checking). */
int ao_partition_sequential(float* v, int32_t* idx, int32_t count, float cut, int32_t* br1,
                            int32_t* br2);
int ao_partition_parallel(float* v, int32_t* idx, int32_t count, float cut, int32_t* br1,
                          int32_t* br2);

/* SurfaceNormalDataPointsFilter (knn, epsilon 0, keepNormals, keepDensities). */
int ao_surface_normals(const float* pts, int64_t n, int64_t stride_floats, int knn,
                       float* normals /* 3n */, float* densities /* n, nullable */,
                       int32_t* degenerate);

/* Matches::getDistsQuantile + TrimmedDist limit. err=1 -> "no outlier to filter". */
float ao_dists_quantile(const float* d2, int64_t n, float quantile, int32_t* err);

/* solvePossiblyUnderdeterminedLinearSystem (A row-major). path: 0 LLT, 1 QR min-norm,
 * 2 eigen pseudo-inverse (stands for the double JacobiSVD fallback). */
int ao_solve6(const double* A, const double* b, double* x, int32_t* path);

/* Full ICP (ICP::compute + computeWithTransformedReference). T0 nullable. */
int ao_icp(const float* ref, int64_t m, int64_t ref_stride_floats, const float* read,
           int64_t n, int64_t read_stride_floats, const float* T0, const ao_icp_config* cfg,
           float* T_out, ao_icp_stats* stats);

/* OctreesOverlap::computeOverlap: counts[0] = |S_ref|, [1] = |S_read|, [2] = overlap. */
int ao_overlap(const float* ref, int64_t m, int64_t ref_stride_floats, const double* ref_origin,
               const float* read, int64_t n, int64_t read_stride_floats,
               const double* read_origin, double resolution, float* overlap_percent,
               uint64_t* counts);
/* Ray keys of one ray (computeRayKeys) packed as k0<<32|k1<<16|k2; returns count or -1. */
int64_t ao_ray_keys(const float origin[3], const float end[3], double resolution,
                    uint64_t* out, int64_t cap);

/* App::computeRegistration ratio auto-tune + replaceRatioConfigFile text round trip. */
float ao_autotune_ratio(float overlap_percent);
float ao_quantize_ratio(float ratio);

/* getPointsInOrientedBox (filteringUtils.cpp:619-637): pcl::CropBox with min/max cube,
 * rotation = origin.R.eulerAngles(0,1,2), translation = origin.t. origin is col-major float[16]
 * (Matrix4f). Kept points in input order; out_n = count. rpy_out (nullable) = the angles. */
int ao_crop_box(const float* pts, int64_t n, int64_t stride_floats, float mn, float mx,
                const float origin[16], float* out_xyz, int64_t* out_n, float* rpy_out);

/* Pre-filter regionGrowingUniformPlaneSegmentationFilter (filteringUtils.cpp:5-45): VoxelGrid ->
 * NormalEstimation -> RegionGrowing, restated in prefilter_oracle.cpp (rules for PCL's unspecified
 * orders there). sampled: optional, 8 floats per sampled point {x, y, z, curvature, nx, ny, nz,
 * cluster}; labels: optional, cluster per sampled point (-1: none); out: 3 floats per kept point,
 * clusters concatenated. All capacities n. Returns 0, 2 (invalid), 3 (PCL would pass a cloud with
 * non-finite points through unfiltered). */
typedef struct {
  float leaf;
  int32_t normal_k;
  int32_t neighbours;
  int32_t min_cluster;
  int32_t max_cluster;
  float cos_smoothness; /* cosf(theta) of validatePoint */
  float curvature;
  float viewpoint[3];
} ao_prefilter_params;
int ao_prefilter(const float* pts, int64_t n, int64_t stride_floats, const ao_prefilter_params* prm,
                 float* sampled, int32_t* labels, int64_t* n_sampled, int64_t* n_clusters, float* out,
                 int64_t* n_out);

#ifdef __cplusplus
}
#endif
#endif
