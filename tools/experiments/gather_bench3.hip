// gather_bench3.hip — the NN kernel's own gather shapes, as dependent chains (32 waves/CU):
//   bucket shapes (an octet of 8 lanes reads one owner's bucket; 8 owners per instruction):
//     oct16x4  8 points of 16 B (float4), lane i reads point i           -> 128 B per owner
//     oct8x2   8 points' (x, y) of 8 B, lane i reads entry i              ->  64 B per owner
//     oct4x1   8 points' z of 4 B                                          ->  32 B per owner
//     oct8x2+4 oct8x2 then oct4x1 from a second array (xy + z)
//   node shapes (every lane its own random record):
//     node16   one 16-B record (dwordx4)      node12  12 B (dwordx3)
//     node8    8 B (dwordx2)                  node8x3 three dwordx2 of one 32-B record
// Reports lane-loads (one per lane per chain step) per CU per us and cycles per wave-step.
// Not part of the product. Build: hipcc --offload-arch=gfx950 -O3 gather_bench3.hip -o gather_bench3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

template <int V>
__global__ __launch_bounds__(256) void k_chain(const uint32_t* __restrict__ t, uint32_t mask, int iters, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint32_t own = V < 4 ? (uint32_t)(lane >> 3) : (uint32_t)lane;
  const uint32_t i = lane & 7;
  uint32_t rec = mix(wave * 131u + own) & mask;  // 128-B record index
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    const uint32_t* base = t + (size_t)rec * 32;  // 128 B records
    uint32_t v;
    if (V == 0) { const uint4 a = reinterpret_cast<const uint4*>(base)[i]; v = a.x ^ a.w; }
    else if (V == 1) { const uint2 a = reinterpret_cast<const uint2*>(base)[i]; v = a.x ^ a.y; }
    else if (V == 2) { v = base[i]; }
    else if (V == 3) { const uint2 a = reinterpret_cast<const uint2*>(base)[i]; const uint32_t z = base[16 + i]; v = a.x ^ a.y ^ z; }
    else if (V == 4) { const uint4 a = reinterpret_cast<const uint4*>(base)[0]; v = a.x ^ a.w; }
    else if (V == 5) { const uint3 a = *reinterpret_cast<const uint3*>(base); v = a.x ^ a.z; }
    else if (V == 6) { const uint2 a = reinterpret_cast<const uint2*>(base)[0]; v = a.x ^ a.y; }
    else { const uint2* p = reinterpret_cast<const uint2*>(base); const uint2 a = p[0], b = p[1], c = p[2]; v = a.x ^ b.y ^ c.x; }
    // the octet's next record comes from its lane 0's value (all lanes read the same key)
    acc += v;
    rec = mix(v ^ (own * 2654435761u)) & mask;
  }
  out[blockIdx.x * 256u + threadIdx.x] = acc;
}

int main() {
  CK(hipSetDevice(0));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  const size_t maxb = 64ull << 20;
  uint32_t* tab;
  CK(hipMalloc(&tab, maxb));
  std::vector<uint32_t> h(maxb / 4, 0);
  for (size_t r = 0; r < h.size() / 32; ++r) {
    const uint32_t k = (uint32_t)(r * 2654435761ull + 12345);
    for (int w = 0; w < 32; ++w) h[32 * r + w] = (w & 1) ? 0u : k;  // even words carry the key, odd words 0
  }
  // every shape's xor of the words it reads equals the key: x ^ w (x4: w = 0), x ^ z (x3: z = k)...
  for (size_t r = 0; r < h.size() / 32; ++r) {
    const uint32_t k = h[32 * r];
    for (int w = 0; w < 32; ++w) h[32 * r + w] = 0;
    h[32 * r + 0] = k;  // shapes reading word 0 of entry i: set each entry's first word
    for (int e = 0; e < 8; ++e) { h[32 * r + 4 * e] = k; h[32 * r + 2 * e] = k; }
  }
  CK(hipMemcpy(tab, h.data(), maxb, hipMemcpyHostToDevice));
  const int blocks = cus * 8;
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 1000;
  const char* names[] = {"oct16x4", "oct8x2", "oct4x1", "oct8x2+4", "node16", "node12", "node8", "node8x3"};
  printf("cus %d, 32 waves/CU, %d dependent steps per lane\n", cus, iters);
  printf("%8s %10s %10s %14s %14s\n", "table", "shape", "us", "lane-ld/CU/us", "cyc/wave-step");
  for (size_t tb : {2ull << 20, 64ull << 20}) {
    const uint32_t mask = (uint32_t)(tb / 128) - 1;
    for (int V = 0; V < 8; ++V) {
      auto run = [&]() {
        switch (V) {
          case 0: k_chain<0><<<blocks, 256>>>(tab, mask, iters, out); break;
          case 1: k_chain<1><<<blocks, 256>>>(tab, mask, iters, out); break;
          case 2: k_chain<2><<<blocks, 256>>>(tab, mask, iters, out); break;
          case 3: k_chain<3><<<blocks, 256>>>(tab, mask, iters, out); break;
          case 4: k_chain<4><<<blocks, 256>>>(tab, mask, iters, out); break;
          case 5: k_chain<5><<<blocks, 256>>>(tab, mask, iters, out); break;
          case 6: k_chain<6><<<blocks, 256>>>(tab, mask, iters, out); break;
          default: k_chain<7><<<blocks, 256>>>(tab, mask, iters, out); break;
        }
      };
      run();
      CK(hipEventRecord(a));
      run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double lanes_per_cu = (double)blocks * 256 * iters / cus;
      const double steps_per_cu = lanes_per_cu / 64;
      printf("%7zuK %10s %10.1f %14.1f %14.1f\n", tb >> 10, names[V], ms * 1e3, lanes_per_cu / (ms * 1e3),
             ms * 1e-3 * 2.4e9 / steps_per_cu);
    }
  }
  return 0;
}
