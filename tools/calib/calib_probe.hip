// Probe-rate calibration for the chain walk (k4_tile): how fast can the chip
// serve N independent random 16-B reads, as a function of the table's size and
// of how many distinct entries the reads touch?  The walk probes one chain-table
// entry per non-CLIENT span (~5e7 per 10^8 mesh spans) over ~4.8e5 distinct
// chains; this times exactly that access shape with nothing else in the kernel
// (4 loads in flight per thread, power-of-two masks, no divisions).
// Diagnostic only: nothing of the engine runs here.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mixr(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

// reads: n; entry of read i = mix(hot(i)) & mask, hot(i) uniform in [0, hot)
__global__ void __launch_bounds__(256) k_probe(const uint4 *__restrict__ t, uint64_t mask, uint32_t hot, uint64_t n,
                                               uint32_t *__restrict__ out) {
  uint32_t s = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
  for (uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4; i0 < n; i0 += stride) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t h = mixr(i0 + q + 0x9E3779B97F4A7C15ull);
      const uint32_t id = (uint32_t)(((h & 0xFFFFFFFFull) * hot) >> 32);
      v[q] = t[mixr((uint64_t)id * 0x632BE59BD9B4E019ull + 1) & mask];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) s ^= v[q].x ^ v[q].w;
  }
  if (s == 0x12345678u) out[0] = s;
}

int main() {
  const uint64_t n = 50000000ull;
  const uint64_t maxb = 256ull << 20;
  uint4 *t = nullptr;
  uint32_t *out = nullptr;
  if (hipMalloc(&t, maxb) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(t, 0, maxb) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const uint64_t sizes[] = {2ull << 20, 8ull << 20, 16ull << 20, 32ull << 20, 128ull << 20};
  const uint32_t hots[] = {480000u, 0u};
  int grids[] = {2048, 8192};
  printf("[\n");
  bool first = true;
  for (uint64_t sz : sizes)
    for (uint32_t h0 : hots)
      for (int g : grids) {
        const uint64_t slots = sz / 16;
        const uint32_t hot = h0 ? h0 : (uint32_t)(slots > 0xFFFFFFFFull ? 0xFFFFFFFFull : slots);
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          (void)hipEventRecord(e0, 0);
          hipLaunchKernelGGL(k_probe, dim3(g), dim3(256), 0, 0, t, slots - 1, hot, n, out);
          (void)hipEventRecord(e1, 0);
          if (hipEventSynchronize(e1) != hipSuccess) return 2;
          float ms = 0;
          (void)hipEventElapsedTime(&ms, e0, e1);
          if (ms < best) best = ms;
        }
        printf("%s {\"table_bytes\": %llu, \"distinct\": %u, \"grid\": %d, \"reads\": %llu, \"ms\": %.4f, "
               "\"G_reads_per_s\": %.2f}\n",
               first ? "" : ",", (unsigned long long)sz, hot, g, (unsigned long long)n, best, n / (best * 1e6));
        first = false;
      }
  printf("]\n");
  (void)hipFree(t);
  (void)hipFree(out);
  return 0;
}
