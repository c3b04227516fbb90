// gather_bench.hip — per-CU throughput of dependent gathers on MI355X, to model the NN kernel's
// bound: wave-instructions per CU per microsecond as a function of distinct cache lines per
// instruction (64 / lanes_per_line), bytes per lane and table size (L1 / L2 / MALL resident).
// Not part of the product. Build: hipcc --offload-arch=gfx950 -O3 gather_bench.hip -o gather_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

template <int W>
__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ table, uint32_t mask, int iters, int lpl,
                                                uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint32_t grp = (uint32_t)(lane / lpl);
  uint32_t line = mix(wave * 131u + grp) & mask;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    const size_t idx = (size_t)line * 4 + (lane & 3);
    uint32_t v;
    if (W == 16) { const uint4 t = table[idx]; v = t.x ^ t.w; }
    else if (W == 8) { const uint2 t = reinterpret_cast<const uint2*>(table)[2 * idx]; v = t.x ^ t.y; }
    else { v = reinterpret_cast<const uint32_t*>(table)[4 * idx]; }
    acc += v;
    line = mix(v ^ (grp * 2654435761u)) & mask;
  }
  out[blockIdx.x * 256u + threadIdx.x] = acc;
}

int main() {
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, dev));
  const int cus = pr.multiProcessorCount;
  const size_t maxb = 256ull << 20;
  uint4* tab;
  CK(hipMalloc(&tab, maxb));
  std::vector<uint4> h(maxb / 16);
  for (size_t i = 0; i < h.size(); ++i) {
    const uint32_t r = (uint32_t)((i / 4) * 2654435761ull + 12345);
    h[i] = make_uint4(r, 0, 0, 0);  // the four 16-B words of a 64-B line carry the same next key
  }
  CK(hipMemcpy(tab, h.data(), maxb, hipMemcpyHostToDevice));
  const int blocks = cus * 8;  // 32 waves per CU
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 2000;
  printf("cus %d, 32 waves/CU, %d dependent loads per lane\n", cus, iters);
  printf("%10s %4s %6s %12s %14s\n", "table", "W", "lines", "us", "instr/CU/us");
  for (size_t tb : {16ull << 10, 2ull << 20, 64ull << 20, 256ull << 20}) {
    const uint32_t lines = (uint32_t)(tb / 64);
    const uint32_t mask = lines - 1;
    for (int W : {16, 8, 4})
      for (int lpl : {1, 2, 4, 8, 16, 64}) {
        auto run = [&]() {
          if (W == 16) k_gather<16><<<blocks, 256>>>(tab, mask, iters, lpl, out);
          else if (W == 8) k_gather<8><<<blocks, 256>>>(tab, mask, iters, lpl, out);
          else k_gather<4><<<blocks, 256>>>(tab, mask, iters, lpl, out);
        };
        run();
        CK(hipEventRecord(a));
        run();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double instr_per_cu = (double)blocks * 4 * iters / cus;
        printf("%9zuK %4d %6d %12.1f %14.2f\n", tb >> 10, W, 64 / lpl, ms * 1e3, instr_per_cu / (ms * 1e3));
      }
  }
  return 0;
}
