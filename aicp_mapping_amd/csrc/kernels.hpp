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
void launch_gather_ref(hipStream_t s, BlockMap m, const PairDesc* pd, const float4* ref_raw,
                       const int32_t* perm, float4* bpts);
void launch_init_state(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       uint32_t* hist1);
// knn: normals of the reference points (bucket order). Returns false if knn unsupported.
bool launch_normals(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                    const uint2* nodes, const int32_t* parent, const float4* bpts, float4* bnrm,
                    int knn);
void launch_icp_nn(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                   const float4* read_c, const uint2* nodes, const int32_t* parent,
                   const float4* bpts, int32_t* match, float* d2, uint32_t* hist1,
                   const IcpParams& prm);
void launch_icp_select(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const float* d2, const uint32_t* hist1);
void launch_icp_reduce(hipStream_t s, BlockMap m, const PairDesc* pd, const PairState* st,
                       const float4* read_c, const int32_t* match, const float* d2,
                       const float4* bpts, const float4* bnrm, double* slab);
void launch_icp_update(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const double* slab, uint32_t* hist1, const IcpParams& prm);
void launch_finalize(hipStream_t s, int n_pairs, const PairDesc* pd, const PairState* st,
                     float* outT);

// ---- kernel-level entry points ----------------------------------------------------------
bool launch_knn_generic(hipStream_t s, int nq, const float4* q, const uint2* nodes,
                        const int32_t* parent, const float4* bpts, int k, float maxE2,
                        float maxR2, int32_t* ids, float* d2, unsigned long long* touched);
void launch_hist_d2(hipStream_t s, BlockMap m, const PairDesc* pd, const float* d2,
                    uint32_t* hist1);
void launch_transform(hipStream_t s, int n, const float* T, const float4* in, float4* out);
void launch_solve6(hipStream_t s, const double* A, const double* b, double* x, int32_t* path);

// ---- overlap -------------------------------------------------------------------------------
void launch_ovl_init(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                     double res);
void launch_ovl_bbox(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                     const float4* pts, int side, double res);
void launch_ovl_mark(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                     const float4* pts, int side, double res, uint32_t* bitmap);
void launch_ovl_count(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                      const uint32_t* bitmap);
void launch_ovl_finish(hipStream_t s, int n_pairs, PairState* st, int set_ratio);

}  // namespace aicp
