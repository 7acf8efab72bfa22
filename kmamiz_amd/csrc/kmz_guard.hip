// kmz_guard.hip -- the multi-GPU sharding guard.
//
// Sharding by whole traces is exact when every parent link stays inside its
// shard.  The reference's span map is global (Traces.ts:117-123), so a span
// whose parentId is missing from its own shard but present on another one
// would be joined there by the reference.  Each rank lists its unresolved
// parent ids (parentId set, no span with that id in the shard: dp == NONE
// after the window join), the ranks exchange those lists, and each rank
// counts how many of the other ranks' ids occur among its own span ids.  A
// nonzero total means the shards are not independent; the caller re-runs
// unsharded.  For Zipkin's Trace[][] (and the synthetic configs) the lists
// are empty and nothing is exchanged.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_kernels.h"

namespace kmz {

__global__ void __launch_bounds__(256) k_unresolved(const uint64_t *__restrict__ pid, const uint32_t *__restrict__ dp,
                                                    uint32_t n, unsigned long long *__restrict__ out, uint64_t cap,
                                                    unsigned long long *__restrict__ count) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (pid[i] == 0 || dp[i] != NONE) continue;
    const unsigned long long x = atomicAdd(count, 1ull);
    if (out && x < cap) out[x] = pid[i];
  }
}

__global__ void __launch_bounds__(256) k_ids_insert(const unsigned long long *__restrict__ ids, uint64_t m,
                                                    unsigned long long *__restrict__ set, uint64_t cap) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = ids[i];
    if (k == 0) continue;  // padding
    uint64_t pos = slot_of(k, cap);
    for (uint64_t z = 0; z < cap; ++z) {
      const unsigned long long c = atomicCAS(&set[pos], 0ull, k);
      if (c == 0 || c == k) break;
      pos = pos + 1 == cap ? 0 : pos + 1;
    }
  }
}

__global__ void __launch_bounds__(256) k_ids_count(const uint64_t *__restrict__ sid, uint32_t n,
                                                   const unsigned long long *__restrict__ set, uint64_t cap,
                                                   unsigned long long *__restrict__ found) {
  uint32_t c = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t k = sid[i];
    if (k == 0) continue;
    uint64_t pos = slot_of(k, cap);
    for (uint64_t z = 0; z < cap; ++z) {
      const unsigned long long v = set[pos];
      if (v == k) {
        ++c;
        break;
      }
      if (v == 0) break;
      pos = pos + 1 == cap ? 0 : pos + 1;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(found, (unsigned long long)c);
}

void launch_unresolved(hipStream_t s, const uint64_t *pid, const uint32_t *dp, uint32_t n, unsigned long long *out,
                       uint64_t cap, unsigned long long *count) {
  if (!n) return;
  const uint32_t g = std::min<uint32_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_unresolved, dim3(g), dim3(256), 0, s, pid, dp, n, out, cap, count);
}

void launch_ids_count(hipStream_t s, const unsigned long long *ids, uint64_t m, unsigned long long *set, uint64_t cap,
                      const uint64_t *sid, uint32_t n, unsigned long long *found) {
  const uint32_t gi = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((m + 255) / 256, 4096));
  if (m) hipLaunchKernelGGL(k_ids_insert, dim3(gi), dim3(256), 0, s, ids, m, set, cap);
  if (!n) return;
  const uint32_t g = std::min<uint32_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_ids_count, dim3(g), dim3(256), 0, s, sid, n, set, cap, found);
}

}  // namespace kmz
