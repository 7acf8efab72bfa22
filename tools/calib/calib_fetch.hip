// Calibration of rocprofv3's FETCH_SIZE for the access shapes the walk uses
// (MI355X_MICROARCH.md: "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").  Three kernels, each its own
// launch, run under `rocprofv3 --pmc FETCH_SIZE`:
//   k_stream   every 16-B word of a 1 GiB buffer once, coalesced (the
//              window's column loads)
//   k_rand64   N uniformly random 16-B reads from a 64 MiB table (the chain
//              table's probes: one 16-byte entry per probe, MALL-resident)
//   k_rand1g   N uniformly random 16-B reads from a 1 GiB table (beyond the MALL)
// tools/calib/calib_fetch.py divides each launch's FETCH_SIZE by its known
// bytes (1 GiB; N * 16).  Diagnostic only: nothing of the engine runs here.
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

__global__ void __launch_bounds__(256) k_stream(const uint4 *__restrict__ a, uint64_t n16, uint32_t *__restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;  // (keeps the loads; never true for a zeroed buffer)
}

__global__ void __launch_bounds__(256) k_rand(const uint4 *__restrict__ t, uint64_t slots, uint64_t n,
                                              uint32_t *__restrict__ out) {
  uint32_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = t[mixr(i + 0x9E3779B97F4A7C15ull) % slots];
    s ^= v.x ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

int main() {
  const uint64_t big = 1ull << 30, small = 64ull << 20, n = 50000000ull;
  uint4 *a = nullptr, *t = nullptr;
  uint32_t *out = nullptr;
  if (hipMalloc(&a, big) != hipSuccess || hipMalloc(&t, small) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, big) != hipSuccess || hipMemset(t, 0, small) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return 1;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, a, big / 16, out);
    hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, t, small / 16, n, out);  // 64 MiB table
    hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, a, big / 16, n, out);    // 1 GiB table
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"stream_bytes\": %llu, \"rand_reads\": %llu, \"rand_bytes_each\": 16}\n", (unsigned long long)big,
         (unsigned long long)n);
  (void)hipFree(a);
  (void)hipFree(t);
  (void)hipFree(out);
  return 0;
}
