// Diagnostic micro-benchmarks (not product code): what a global edge-key set
// costs on MI355X when it lives in L2/MALL, versus materialising the keys.
//   probe_lin   : u64 linear-probing table, read-only hits (keys present)
//   probe_bkt   : 64-B buckets of 8 keys (one line per probe)
//   write_scat  : 8-B stores, every lane to a different run (emit today)
//   write_runs  : the same keys written as runs of R consecutive keys by
//                 consecutive lanes (LDS-sorted emit)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);               \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t keyof(uint64_t i) { return mix64(i + 77) | 1; }

__global__ void build_lin(unsigned long long *t, uint64_t cap, uint32_t K) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  uint64_t k = keyof(i), p = __umul64hi(mix64(k), cap);
  for (;;) {
    unsigned long long c = atomicCAS(&t[p], 0ull, k);
    if (c == 0 || c == k) return;
    p = p + 1 == cap ? 0 : p + 1;
  }
}
__global__ void probe_lin(const unsigned long long *t, uint64_t cap, uint32_t K, uint64_t nprobe,
                          unsigned long long *miss) {
  uint64_t m = 0;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < nprobe; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = keyof(mix64(j) % K), p = __umul64hi(mix64(k), cap);
    for (int z = 0; z < 64; ++z) {
      uint64_t c = t[p];
      if (c == k) break;
      if (c == 0) {
        ++m;
        break;
      }
      p = p + 1 == cap ? 0 : p + 1;
    }
  }
  if (m) atomicAdd(miss, m);
}
// buckets of 8 u64 (64 B); two choices
__global__ void build_bkt(unsigned long long *t, uint32_t nb, uint32_t K, unsigned int *fill) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  uint64_t k = keyof(i), h = mix64(k);
  uint32_t b1 = (uint32_t)__umul64hi(h, nb), b2 = (uint32_t)__umul64hi(mix64(h), nb);
  uint32_t b = fill[b1] <= fill[b2] ? b1 : b2;
  uint32_t s = atomicAdd(&fill[b], 1u);
  if (s >= 8) {
    b = b ^ b1 ^ b2;
    s = atomicAdd(&fill[b], 1u);
  }
  if (s < 8) t[(uint64_t)b * 8 + s] = k;
}
__global__ void probe_bkt(const unsigned long long *t, uint32_t nb, uint32_t K, uint64_t nprobe,
                          unsigned long long *miss) {
  uint64_t m = 0;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < nprobe; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = keyof(mix64(j) % K), h = mix64(k);
    uint32_t b1 = (uint32_t)__umul64hi(h, nb);
    const ulonglong4 *q = reinterpret_cast<const ulonglong4 *>(t + (uint64_t)b1 * 8);
    ulonglong4 x = q[0], y = q[1];
    bool f = x.x == k || x.y == k || x.z == k || x.w == k || y.x == k || y.y == k || y.z == k || y.w == k;
    if (!f) {
      uint32_t b2 = (uint32_t)__umul64hi(mix64(h), nb);
      q = reinterpret_cast<const ulonglong4 *>(t + (uint64_t)b2 * 8);
      x = q[0];
      y = q[1];
      f = x.x == k || x.y == k || x.z == k || x.w == k || y.x == k || y.y == k || y.z == k || y.w == k;
    }
    m += !f;
  }
  if (m) atomicAdd(miss, m);
}
// each lane writes R keys to its own random run
__global__ void write_scat(unsigned long long *pool, uint64_t nruns, uint32_t R) {
  uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j >= nruns) return;
  uint64_t r = mix64(j) % nruns;
  for (uint32_t d = 0; d < R; ++d) pool[r * R + d] = j + d;
}
// consecutive lanes write consecutive keys of runs of R
__global__ void write_runs(unsigned long long *pool, uint64_t nruns, uint32_t R) {
  uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (e >= nruns * R) return;
  uint64_t j = e / R, d = e % R;
  uint64_t r = mix64(j) % nruns;
  pool[r * R + d] = e;
}

int main() {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  unsigned long long *miss;
  CK(hipMalloc(&miss, 8));
  const uint64_t NP = 210000000ull;
  for (uint32_t K : {900000u, 3000000u}) {
    for (double load : {0.3, 0.5}) {
      uint64_t cap = (uint64_t)(K / load);
      unsigned long long *t;
      CK(hipMalloc(&t, cap * 8));
      CK(hipMemset(t, 0, cap * 8));
      hipLaunchKernelGGL(build_lin, dim3((K + 255) / 256), dim3(256), 0, 0, t, cap, K);
      for (uint32_t grid : {2048u, 8192u}) {
        for (int rep = 0; rep < 2; ++rep) {
          CK(hipMemset(miss, 0, 8));
          CK(hipEventRecord(a));
          hipLaunchKernelGGL(probe_lin, dim3(grid), dim3(256), 0, 0, t, cap, K, NP, miss);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          CK(hipEventElapsedTime(&ms, a, b));
        }
        unsigned long long h = 0;
        CK(hipMemcpy(&h, miss, 8, hipMemcpyDeviceToHost));
        printf("probe_lin K=%u load=%.1f table=%.1f MB grid=%u: %.3f ms = %.1f G probes/s (miss %llu)\n", K, load,
               cap * 8 / 1e6, grid, ms, NP / ms / 1e6, h);
      }
      CK(hipFree(t));
    }
    {
      uint32_t nb = (uint32_t)(K / 8 / 0.7);
      unsigned long long *t;
      unsigned int *fill;
      CK(hipMalloc(&t, (uint64_t)nb * 64));
      CK(hipMalloc(&fill, (uint64_t)nb * 4));
      CK(hipMemset(t, 0, (uint64_t)nb * 64));
      CK(hipMemset(fill, 0, (uint64_t)nb * 4));
      hipLaunchKernelGGL(build_bkt, dim3((K + 255) / 256), dim3(256), 0, 0, t, nb, K, fill);
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(miss, 0, 8));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(probe_bkt, dim3(8192), dim3(256), 0, 0, t, nb, K, NP, miss);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
      }
      unsigned long long h = 0;
      CK(hipMemcpy(&h, miss, 8, hipMemcpyDeviceToHost));
      printf("probe_bkt K=%u table=%.1f MB: %.3f ms = %.1f G probes/s (miss %llu)\n", K, nb * 64 / 1e6, ms,
             NP / ms / 1e6, h);
      CK(hipFree(t));
      CK(hipFree(fill));
    }
  }
  {
    const uint64_t nkeys = 210000000ull;
    unsigned long long *pool;
    CK(hipMalloc(&pool, nkeys * 8 + 4096));
    for (uint32_t R : {1u, 4u, 8u, 16u, 64u}) {
      uint64_t nruns = nkeys / R;
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(write_scat, dim3((nruns + 255) / 256), dim3(256), 0, 0, pool, nruns, R);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
      }
      printf("write_scat R=%u: %.3f ms = %.0f GB/s\n", R, ms, nkeys * 8 / ms / 1e6);
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(write_runs, dim3((nkeys + 255) / 256), dim3(256), 0, 0, pool, nruns, R);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
      }
      printf("write_runs R=%u: %.3f ms = %.0f GB/s\n", R, ms, nkeys * 8 / ms / 1e6);
    }
    CK(hipFree(pool));
  }
  return 0;
}
