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
void launch_init_state(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st);
// SurfaceNormal of the reference points (bucket order); ids: scratch of total_ref * knn;
// ctr: zeroed work counter. Returns false if knn is unsupported.
bool launch_normals(hipStream_t s, int n_pairs, uint32_t total_ref, const PairDesc* pd, PairState* st,
                    const uint4* nodes, const int32_t* parent, const float4* bpts, float4* bnrm, int knn,
                    int32_t* ids, uint32_t* ctr);
void launch_active_list(hipStream_t s, int n_pairs, const PairDesc* pd, const PairState* st,
                        ActiveList* al, uint32_t* ctr);
void launch_icp_nn(hipStream_t s, int grid_items, const PairDesc* pd, const PairState* st,
                   const ActiveList* al, const float4* read_c, const uint4* nodes,
                   const int32_t* parent, const float4* bpts, int32_t* match, float* d2,
                   uint32_t* touched, uint32_t* ctr, const IcpParams& prm);
void launch_icp_select(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const float* d2);
void launch_icp_reduce(hipStream_t s, BlockMap m, const PairDesc* pd, const PairState* st,
                       const float4* read_c, const int32_t* match, const float* d2,
                       const uint32_t* touched, const float4* bpts, const float4* bnrm, double* slab);
void launch_icp_update(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                       const double* slab, const IcpParams& prm);
void launch_finalize(hipStream_t s, int n_pairs, const PairDesc* pd, const PairState* st,
                     float* outT);

// ---- kernel-level entry points ----------------------------------------------------------
bool launch_knn_generic(hipStream_t s, uint32_t nq, const float4* q, const uint4* nodes,
                        const int32_t* parent, const float4* bpts, int k, float maxE2,
                        float maxR2, int32_t* ids, float* d2, unsigned long long* touched,
                        uint32_t* ctr);
void launch_transform(hipStream_t s, int n, const float* T, const float4* in, float4* out);
void launch_solve6(hipStream_t s, const double* A, const double* b, double* x, int32_t* path);

// ---- overlap -------------------------------------------------------------------------------
void launch_ovl_init(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                     double res);
void launch_ovl_bbox(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                     const float4* pts, int side, double res);
void launch_ovl_mark(hipStream_t s, BlockMap m, const PairDesc* pd, PairState* st,
                     const float4* pts, int side, double res, uint8_t* maps);
void launch_ovl_count(hipStream_t s, int n_pairs, const PairDesc* pd, PairState* st,
                      const uint8_t* maps);
void launch_ovl_finish(hipStream_t s, int n_pairs, PairState* st, int set_ratio);

}  // namespace aicp
