// kernels_sequence.hip — the device side of App's frame-to-reference stream (sequence.cpp).
//
// The next reference is built from the last reading of a window without a host round trip:
// k_seq_ref_points writes its sensor origin (the corrected pose's translation, app.cpp:375-391)
// into the overlap group descriptor and the corrected cloud,
// and the voxel maps of the overlap are sized on the device (k_ovl_size) inside a slot whose
// capacity the host bounds from the source cloud's extent (a rigid motion keeps its diameter).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "aicp_common.hpp"
#include "icp_math.hpp"
#include "kernels.hpp"

namespace aicp {

// The new reference from the window's last reading in one launch (two kernels before, back to
// back on the matcher stream's critical path). gd: the new window's overlap group; src: the
// reading that becomes the reference; T: its correction (column-major, the finalize output).
// Every workgroup reads T; workgroup 0 also writes its copy and the reference's sensor origin
// (the corrected pose's translation, app.cpp:375-391), and each point is moved by apply4 exactly
// as k_transform moves it (pcl::transformPointCloud's float order).
// src_st (nullable): the source's state in the previous window, whose loop may still be running
// (the source pair itself has stopped): its correction is k_finalize's product of the frames and
// the ICP transform, computed here with the same operations instead of read from T.
__global__ __launch_bounds__(256) void k_seq_ref_points(int n, PairDesc* gd, const PairDesc* __restrict__ src,
                                                        const PairState* __restrict__ src_st, const float* T,
                                                        float* Tcopy, const float4* __restrict__ in,
                                                        float4* __restrict__ out) {
  __shared__ float Ts[16];
  if (src_st) {
    if (threadIdx.x == 0) {  // (system-scope loads, as for T: written by another stream's kernels)
      auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
      float St[16], Tm[16], Ti[16], tmp[16], Tf[16];
      for (int k = 0; k < 16; ++k) {
        St[k] = ld(src_st->T + k);
        Tm[k] = ld(src->Tmean + k);
        Ti[k] = ld(src->Tinit + k);
      }
      mul4(Tm, St, tmp);
      mul4(tmp, Ti, Tf);
      for (int k = 0; k < 16; ++k) Ts[k] = Tf[k];
    }
  } else if (threadIdx.x < 16) {
    Ts[threadIdx.x] = __hip_atomic_load(T + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  float Tl[16];
  for (int k = 0; k < 16; ++k) Tl[k] = Ts[k];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (int k = 0; k < 16; ++k) Tcopy[k] = Tl[k];
    double o[3];
    corrected_origin(Tl, src->read_origin, o);
    for (int k = 0; k < 3; ++k) gd->ref_origin[k] = o[k];
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  float q[3];
  apply4(Tl, p.x, p.y, p.z, q);
  out[i] = make_float4(q[0], q[1], q[2], 1.f);
}

// App's debug working mode (app.cpp:87-96): before reading d is registered, initT (initialT_) is
// kept in hist (its value before this reading, for a re-plan) and the reading's prior pose
// becomes initialT_ * prior pose: its translation is the overlap's sensor origin
// (fromMatrix4fToIsometry3d, common.cpp:4-23, as for a correction). The points follow with
// k_transform(initT).
__global__ void k_debug_prep(PairDesc* d, const float* initT, float* hist) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float T[16];
  for (int k = 0; k < 16; ++k) T[k] = initT[k];
  for (int k = 0; k < 16; ++k) hist[k] = T[k];
  double o[3];
  corrected_origin(T, d->read_origin, o);
  for (int k = 0; k < 3; ++k) d->read_origin[k] = o[k];
}

// the reading's correction (k_finalize's arithmetic and rigidity check) and, when it is accepted
// (|t_i| <= max_correction_magnitude, app.cpp:366-373), initialT_ = correction * initialT_
// (app.cpp:414: a dropped reading returns before that line)
__global__ void k_debug_post(const PairDesc* __restrict__ d, PairState* st, float* outT, float* initT,
                             float max_corr) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float tmp[16], T[16];
  mul4(d->Tmean, st->T, tmp);
  mul4(tmp, d->Tinit, T);
  for (int i = 0; i < 16; ++i) outT[i] = T[i];
  if (st->status == 0 && !rigid_ok(T)) st->status = 5;
  if (st->status != 0 || correction_rejected(T, max_corr)) return;
  float I[16], N[16];
  for (int i = 0; i < 16; ++i) I[i] = initT[i];
  mul4(T, I, N);
  for (int i = 0; i < 16; ++i) initT[i] = N[i];
}

// one map per entry from the key box in st[i].ovl_bbox (k_ovl_init + k_ovl_bbox), padded by 2
// voxels below and 2 above like the batch path's host sizing; od[i].off is preset by the host.
// A box beyond cap[i] bytes is reported (ovl_err) and gets an empty map: every mark and lookup
// then fails its bounds test, so nothing is stored outside the slot.
__global__ void k_ovl_size(int n, PairState* st, OvlDesc* od, const uint64_t* __restrict__ cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  OvlDesc& o = od[i];
  const int br[3] = {kOvlBrick0, kOvlBrick1, kOvlBrick2};
  for (int k = 0; k < 3; ++k) ovl_axis(st[i].ovl_bbox[k], st[i].ovl_bbox[3 + k], br[k], o.min[k], o.dim[k]);
  o.bytes = ovl_bytes(o.dim);
  if (o.bytes > cap[i]) {
    for (int k = 0; k < 3; ++k) o.dim[k] = 0;
    o.bytes = 0;
    st[i].ovl_err = 1;
  }
}

// zero the n maps of od[] (sizes known on the device only), 16 B per store
__global__ __launch_bounds__(256) void k_ovl_clear(int n, const OvlDesc* __restrict__ od, uint8_t* maps) {
  for (int m = 0; m < n; ++m) {
    const OvlDesc& o = od[m];
    uint4* p = (uint4*)(maps + o.off);
    const uint64_t n16 = o.bytes / 16;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n16; w += (uint64_t)gridDim.x * blockDim.x)
      p[w] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// word copies of the three arrays (one block; a window holds at most kMaxPairs readings)
__global__ __launch_bounds__(256) void k_seq_commit(int np, const uint32_t* __restrict__ d, const uint32_t* __restrict__ st,
                                                    const uint32_t* __restrict__ T, uint32_t* gd, uint32_t* gst,
                                                    uint32_t* gT) {
  const uint32_t nd = (uint32_t)np * (sizeof(PairDesc) / 4), ns = (uint32_t)np * (sizeof(PairState) / 4),
                 nt = (uint32_t)np * 16;
  for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) gd[i] = d[i];
  for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) gst[i] = st[i];
  for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) gT[i] = T[i];
}

// up to three word arrays zeroed by one launch (the loop's histogram, counts and hand-off words:
// three hipMemsetAsync calls were five fill kernels of ~5 us each on the window's critical stream)
__global__ __launch_bounds__(256) void k_zero_words3(uint32_t* a, uint32_t na, uint32_t* b, uint32_t nb, uint32_t* c,
                                                     uint32_t nc) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < na + nb + nc; i += stride) {
    if (i < na) a[i] = 0u;
    else if (i < na + nb) b[i - na] = 0u;
    else c[i - na - nb] = 0u;
  }
}

void launch_zero_words3(hipStream_t s, uint32_t* a, size_t na, uint32_t* b, size_t nb, uint32_t* c, size_t nc) {
  const size_t n = na + nb + nc;
  if (!n) return;
  const unsigned g = (unsigned)std::min<size_t>(256, (n + 255) / 256);
  k_zero_words3<<<g, 256, 0, s>>>(a, (uint32_t)na, b, (uint32_t)nb, c, (uint32_t)nc);
}

void launch_seq_commit(hipStream_t s, int np, const PairDesc* d, const PairState* st, const float* T, PairDesc* gd,
                       PairState* gst, float* gT) {
  static_assert(sizeof(PairDesc) % 4 == 0 && sizeof(PairState) % 4 == 0, "word copies");
  if (np > 0)
    k_seq_commit<<<1, 256, 0, s>>>(np, (const uint32_t*)d, (const uint32_t*)st, (const uint32_t*)T, (uint32_t*)gd,
                                   (uint32_t*)gst, (uint32_t*)gT);
}
void launch_seq_ref_points(hipStream_t s, int n, PairDesc* gd, const PairDesc* src, const PairState* src_st,
                           const float* T, float* Tcopy, const float4* in, float4* out) {
  k_seq_ref_points<<<(unsigned)std::max(1, (n + 255) / 256), 256, 0, s>>>(n, gd, src, src_st, T, Tcopy, in, out);
}
void launch_debug_prep(hipStream_t s, PairDesc* d, const float* initT, float* hist) {
  k_debug_prep<<<1, 64, 0, s>>>(d, initT, hist);
}
void launch_debug_post(hipStream_t s, const PairDesc* d, PairState* st, float* outT, float* initT, float max_corr) {
  k_debug_post<<<1, 64, 0, s>>>(d, st, outT, initT, max_corr);
}
void launch_ovl_size(hipStream_t s, int n, PairState* st, OvlDesc* od, const uint64_t* cap) {
  if (n) k_ovl_size<<<(n + 63) / 64, 64, 0, s>>>(n, st, od, cap);
}
void launch_ovl_clear(hipStream_t s, int n, const OvlDesc* od, uint8_t* maps, uint64_t max_bytes) {
  if (!n || !max_bytes) return;
  const uint64_t blocks = (max_bytes / 16 + 255) / 256;
  k_ovl_clear<<<(unsigned)(blocks < 2048 ? (blocks ? blocks : 1) : 2048), 256, 0, s>>>(n, od, maps);
}

}  // namespace aicp
