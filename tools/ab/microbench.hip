// Diagnostic micro-benchmarks for directory/partition write patterns (not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// each block = one tile, writes P words: strided (p*ntiles + tile) or contiguous (tile*P + p)
__global__ void dir_write(uint32_t *dir, uint32_t P, uint32_t ntiles, int strided) {
  uint32_t tile = blockIdx.x;
  for (uint32_t p = threadIdx.x; p < P; p += blockDim.x) {
    uint64_t idx = strided ? (uint64_t)p * ntiles + tile : (uint64_t)tile * P + p;
    dir[idx] = p ^ tile;
  }
}
// scattered 8B writes: each thread writes D words to a random partition region (like key emit)
__global__ void scatter_write(unsigned long long *pool, uint64_t region, uint32_t P, uint32_t n, int sorted) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t p = sorted ? (blockIdx.x % P) : (uint32_t)((i * 2654435761u) % P);
  uint64_t base = (uint64_t)p * region + ((uint64_t)blockIdx.x / P) * blockDim.x * 4 + threadIdx.x * 4;
  for (int d = 0; d < 4; ++d) pool[(base + d) % (region * P)] = i + d;
}
__global__ void stream_read(const uint4 *a, uint64_t n4, unsigned long long *sink) {
  uint4 acc = {0, 0, 0, 0};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = a[i]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x12345 && acc.y == 7) atomicAdd(sink, 1ull);
}

int main() {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float ms;
  const uint32_t ntiles = 48828;
  for (uint32_t P : {59u, 512u}) {
    uint32_t *dir; CK(hipMalloc(&dir, (size_t)P * ntiles * 4));
    for (int strided = 1; strided >= 0; --strided) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a)); hipLaunchKernelGGL(dir_write, dim3(ntiles), dim3(512), 0, 0, dir, P, ntiles, strided);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      }
      printf("dir_write P=%u strided=%d: %.3f ms (%.1f MB)\n", P, strided, ms, P * (double)ntiles * 4 / 1e6);
    }
    CK(hipFree(dir));
  }
  {
    const uint32_t n = 50000000, P = 512; uint64_t region = (uint64_t)n * 4 / P + 4096;
    unsigned long long *pool; CK(hipMalloc(&pool, region * P * 8));
    for (int sorted = 0; sorted < 2; ++sorted) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a)); hipLaunchKernelGGL(scatter_write, dim3((n + 255) / 256), dim3(256), 0, 0, pool, region, P, n, sorted);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      }
      printf("scatter_write 4x8B per thread, sorted=%d: %.3f ms -> %.0f GB/s payload\n", sorted, ms, n * 32.0 / ms / 1e6);
    }
    CK(hipFree(pool));
  }
  {
    uint64_t bytes = 4ull << 30; uint4 *buf; unsigned long long *sink;
    CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&sink, 8)); CK(hipMemset(buf, 1, bytes));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a)); hipLaunchKernelGGL(stream_read, dim3(8192), dim3(256), 0, 0, buf, bytes / 16, sink);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("stream_read 4 GiB: %.3f ms -> %.0f GB/s\n", ms, bytes / ms / 1e6);
  }
  return 0;
}
