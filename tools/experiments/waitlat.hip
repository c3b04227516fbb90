// waitlat.hip — latency of hipStreamWaitValue64 released by a kernel's store to signal memory
// (diagnostic for the sequence's device-side window dependency). Stream A: a kernel that spins
// for ~`us` microseconds and then stores the ticket; stream B: wait-value, then a kernel that
// records the realtime clock. Prints the producer's store time and the consumer's start time.
// Build: hipcc --offload-arch=gfx950 -O2 tools/waitlat.hip -o tools/waitlat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void producer(uint64_t* sig, uint64_t ticket, uint64_t spin_ticks, uint64_t* ts) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(8);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  __threadfence_system();
  __hip_atomic_store(sig, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  ts[0] = t1;
}

__global__ void consumer(uint64_t* ts) {
  if (threadIdx.x == 0) ts[1] = __builtin_amdgcn_s_memrealtime();
}

int main(int argc, char** argv) {
  const int us = argc > 1 ? std::atoi(argv[1]) : 500;
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  std::printf("CanUseStreamWaitValue %d\n", can);
  uint64_t* sig = nullptr;
  CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
  uint64_t* ts = nullptr;
  CK(hipMalloc(&ts, 16));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamWriteValue64(a, sig, 0, 0));
  CK(hipStreamSynchronize(a));
  for (int r = 1; r <= 8; ++r) {
    // consumer first in host order would be the unsafe order; keep producer first
    producer<<<1, 64, 0, a>>>(sig, (uint64_t)r, (uint64_t)us * 100, ts);  // 100 MHz realtime clock
    CK(hipStreamWaitValue64(b, sig, (uint64_t)r, hipStreamWaitValueGte, ~0ull));
    consumer<<<1, 64, 0, b>>>(ts);
    CK(hipStreamSynchronize(b));
    CK(hipStreamSynchronize(a));
    uint64_t h[2];
    CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
    std::printf("round %d: store -> consumer start %.2f us\n", r, (double)(h[1] - h[0]) / 100.0);
  }
  // event-based wait for comparison
  hipEvent_t e;
  CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (int r = 0; r < 4; ++r) {
    producer<<<1, 64, 0, a>>>(sig, 100 + r, (uint64_t)us * 100, ts);
    CK(hipEventRecord(e, a));
    CK(hipStreamWaitEvent(b, e, 0));
    consumer<<<1, 64, 0, b>>>(ts);
    CK(hipStreamSynchronize(b));
    uint64_t h[2];
    CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
    std::printf("event round %d: store -> consumer start %.2f us\n", r, (double)(h[1] - h[0]) / 100.0);
  }
  return 0;
}
