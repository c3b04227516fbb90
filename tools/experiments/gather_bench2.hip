// gather_bench2.hip — which load shape should the NN kernel's dependent gathers use? Per-CU
// wave-instructions/us of a chain of dependent gathers where every lane reads one 16-byte record
// (64-B blocks shared by `lpl` lanes at 16-B strides, as octets and Morton-coherent descents do),
// read as: one dwordx4, one dwordx3 (12 B), two dwordx2 (x,y then z,w), one dwordx2 (8 B only),
// one dword. Reports records/CU/us, i.e. per lane-record, not per instruction.
// Not part of the product. Build: hipcc --offload-arch=gfx950 -O3 gather_bench2.hip -o gather_bench2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

template <int V>
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
    if (V == 0) {  // dwordx4
      const uint4 t = table[idx];
      v = t.x ^ t.w;
    } else if (V == 1) {  // dwordx3
      const uint32_t* p = reinterpret_cast<const uint32_t*>(table + idx);
      const uint3 t = *reinterpret_cast<const uint3*>(p);
      v = t.x ^ t.z;
    } else if (V == 2) {  // two dwordx2
      const uint2* p = reinterpret_cast<const uint2*>(table + idx);
      const uint2 a = p[0], b = p[1];
      v = a.x ^ b.y;
    } else if (V == 3) {  // one dwordx2
      const uint2 a = reinterpret_cast<const uint2*>(table + idx)[0];
      v = a.x ^ a.y;
    } else {  // dword
      v = reinterpret_cast<const uint32_t*>(table + idx)[0];
    }
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
  const size_t maxb = 64ull << 20;
  uint4* tab;
  CK(hipMalloc(&tab, maxb));
  std::vector<uint4> h(maxb / 16);
  for (size_t i = 0; i < h.size(); ++i) {
    const uint32_t r = (uint32_t)((i / 4) * 2654435761ull + 12345);
    h[i] = make_uint4(r, 0, 0, 0);  // every word of a record carries the block's next key (x ^ w = x)
    h[i].w = 0;
  }
  CK(hipMemcpy(tab, h.data(), maxb, hipMemcpyHostToDevice));
  const int blocks = cus * 8;  // 32 waves per CU
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 1000;
  const char* names[] = {"dwordx4", "dwordx3", "2xdwordx2", "dwordx2", "dword"};
  printf("cus %d, 32 waves/CU, %d dependent record reads per lane; lane-records per CU per us\n", cus, iters);
  printf("%8s %10s %6s %10s %12s\n", "table", "shape", "lines", "us", "rec/CU/us");
  for (size_t tb : {16ull << 10, 2ull << 20, 64ull << 20}) {
    const uint32_t mask = (uint32_t)(tb / 64) - 1;
    for (int V = 0; V < 5; ++V)
      for (int lpl : {1, 4, 8, 16}) {
        auto run = [&]() {
          switch (V) {
            case 0: k_gather<0><<<blocks, 256>>>(tab, mask, iters, lpl, out); break;
            case 1: k_gather<1><<<blocks, 256>>>(tab, mask, iters, lpl, out); break;
            case 2: k_gather<2><<<blocks, 256>>>(tab, mask, iters, lpl, out); break;
            case 3: k_gather<3><<<blocks, 256>>>(tab, mask, iters, lpl, out); break;
            default: k_gather<4><<<blocks, 256>>>(tab, mask, iters, lpl, out); break;
          }
        };
        run();
        CK(hipEventRecord(a));
        run();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double rec_per_cu = (double)blocks * 256 * iters / cus;
        printf("%7zuK %10s %6d %10.1f %12.1f\n", tb >> 10, names[V], 64 / lpl, ms * 1e3, rec_per_cu / (ms * 1e3));
      }
  }
  return 0;
}
