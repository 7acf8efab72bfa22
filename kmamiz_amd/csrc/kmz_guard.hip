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
// are empty and nothing is exchanged.  The other half of the global map's
// semantics, ids repeated across shards, is checked by routing (below).
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

// ---- cross-shard repeated span ids ------------------------------------------
// The reference's span map is global (Traces.ts:117-123): an id that occurs in
// two shards collapses to one row there.  Each rank routes the id_hash of its
// span ids to an owner rank (id_owner: a range of the hash
// space), the ranks exchange them (all-to-all), and each owner runs the
// uniqueness certificate over what it received (kmz_id_repeats).  Every
// shard's own ids are unique already (its certificate), so a repeat among the
// received values is an id shared by two shards.
//   k_route_hist     per chunk: owner histogram in LDS
//   k_route_scan     one workgroup: each (chunk, owner)'s output offset
//   k_route_scatter  per chunk: the hashes to their owner's segment
constexpr uint32_t RT_T = 256, RT_MAXW = 1024;

__global__ void __launch_bounds__(RT_T) k_route_hist(const uint64_t *__restrict__ sid, uint32_t n, uint32_t chunk,
                                                     uint32_t world, uint32_t *__restrict__ hist) {
  __shared__ uint32_t h[RT_MAXW];
  for (uint32_t r = threadIdx.x; r < world; r += RT_T) h[r] = 0;
  __syncthreads();
  const uint32_t b = blockIdx.x * chunk, e = min(n, b + chunk);
  for (uint32_t i = b + threadIdx.x; i < e; i += RT_T) atomicAdd(&h[id_owner(id_hash(sid[i]), world)], 1u);
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < world; r += RT_T) hist[(uint64_t)blockIdx.x * world + r] = h[r];
}

// hist[chunk][owner] -> exclusive output offsets (owner-major); tot[owner] = its count.
// fixed (segw > 0): offsets within the owner's own segment of segw words,
// whose word 0 gets the count (kmz_route_ids_fixed: no counts exchange)
__global__ void __launch_bounds__(RT_T) k_route_scan(uint32_t *__restrict__ hist, uint32_t nchunks, uint32_t world,
                                                     unsigned long long *__restrict__ tot, uint64_t segw,
                                                     unsigned long long *__restrict__ out) {
  __shared__ unsigned long long seg[RT_MAXW];
  for (uint32_t r = threadIdx.x; r < world; r += RT_T) {
    unsigned long long a = 0;
    for (uint32_t c = 0; c < nchunks; ++c) {
      const uint32_t x = hist[(uint64_t)c * world + r];
      hist[(uint64_t)c * world + r] = (uint32_t)a;  // (a shard holds < 2^32 spans)
      a += x;
    }
    seg[r] = a;
    tot[r] = a;
    if (segw) out[(uint64_t)r * segw] = a;
  }
  if (segw) return;  // (segments are the owners' own: no global offsets)
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0;
    for (uint32_t r = 0; r < world; ++r) {
      const unsigned long long x = seg[r];
      seg[r] = a;
      a += x;
    }
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < world; r += RT_T)
    for (uint32_t c = 0; c < nchunks; ++c) hist[(uint64_t)c * world + r] += (uint32_t)seg[r];
}

__global__ void __launch_bounds__(RT_T) k_route_scatter(const uint64_t *__restrict__ sid, uint32_t n, uint32_t chunk,
                                                        uint32_t world, const uint32_t *__restrict__ off,
                                                        unsigned long long *__restrict__ out, uint64_t segw) {
  __shared__ uint32_t cur[RT_MAXW];
  for (uint32_t r = threadIdx.x; r < world; r += RT_T) cur[r] = off[(uint64_t)blockIdx.x * world + r];
  __syncthreads();
  const uint32_t b = blockIdx.x * chunk, e = min(n, b + chunk);
  for (uint32_t i = b + threadIdx.x; i < e; i += RT_T) {  // (order inside a segment is free: the check is a set test)
    const uint64_t h = id_hash(sid[i]);
    const uint32_t r = id_owner(h, world), x = atomicAdd(&cur[r], 1u);
    if (!segw)
      out[x] = h;
    else if (x + 1 < segw)  // (a full segment: its count says so, the exchange is redone exactly)
      out[(uint64_t)r * segw + 1 + x] = h;
  }
}

// Fixed segments in one pass (kmz_route_ids_fixed): each workgroup holds its
// 4096 hashes in registers, ranks them per owner with LDS atomics, reserves
// each owner's run in that owner's segment with one device atomic, and writes
// them; a last tiny kernel stores the counts into the segments' word 0.  8 B
// read + 8 B written per id (the hist/scan/scatter form reads the ids twice).
constexpr uint32_t RF_PT = 16, RF_CH = RT_T * RF_PT;

__global__ void __launch_bounds__(RT_T) k_route_fixed(const uint64_t *__restrict__ sid, uint32_t n, uint32_t world,
                                                      uint64_t segw, unsigned long long *__restrict__ cur,
                                                      unsigned long long *__restrict__ out) {
  __shared__ uint32_t h[RT_MAXW];
  __shared__ unsigned long long base[RT_MAXW];
  for (uint32_t r = threadIdx.x; r < world; r += RT_T) h[r] = 0;
  const uint32_t b = blockIdx.x * RF_CH;
  uint64_t v[RF_PT];
#pragma unroll
  for (int q = 0; q < (int)RF_PT; ++q) {  // every load in flight before the first hash
    const uint32_t i = b + q * RT_T + threadIdx.x;
    v[q] = i < n ? sid[i] : 0;
  }
  __syncthreads();
  uint32_t ow[RF_PT], rk[RF_PT];
#pragma unroll
  for (int q = 0; q < (int)RF_PT; ++q) {
    const uint32_t i = b + q * RT_T + threadIdx.x;
    v[q] = id_hash(v[q]);
    ow[q] = id_owner(v[q], world);
    rk[q] = i < n ? atomicAdd(&h[ow[q]], 1u) : 0u;
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < world; r += RT_T)
    if (h[r]) base[r] = atomicAdd(&cur[r], (unsigned long long)h[r]);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < (int)RF_PT; ++q) {
    const uint32_t i = b + q * RT_T + threadIdx.x;
    const unsigned long long x = base[ow[q]] + rk[q];
    if (i < n && x + 1 < segw) out[(uint64_t)ow[q] * segw + 1 + x] = v[q];  // (full: its count says so)
  }
}

__global__ void __launch_bounds__(RT_T) k_route_counts(uint32_t world, uint64_t segw,
                                                       const unsigned long long *__restrict__ cur, uint32_t stride,
                                                       unsigned long long *__restrict__ out) {
  for (uint32_t r = threadIdx.x; r < world; r += RT_T) out[(uint64_t)r * segw] = cur[(uint64_t)r * stride];
}

void launch_route_counts(hipStream_t s, uint32_t world, uint64_t segw, const unsigned long long *cur, uint32_t stride,
                         unsigned long long *out) {
  hipLaunchKernelGGL(k_route_counts, dim3(1), dim3(RT_T), 0, s, world, segw, cur, stride, out);
}

bool launch_route_fixed(hipStream_t s, const uint64_t *sid, uint32_t n, uint32_t world, uint64_t segw,
                        unsigned long long *cur, unsigned long long *out) {
  if (world == 0 || world > RT_MAXW || segw < 2) return false;
  if (hipMemsetAsync(cur, 0, (size_t)world * 8, s) != hipSuccess) return false;
  if (n) hipLaunchKernelGGL(k_route_fixed, dim3((n + RF_CH - 1) / RF_CH), dim3(RT_T), 0, s, sid, n, world, segw, cur, out);
  launch_route_counts(s, world, segw, cur, 1, out);
  return true;
}

uint32_t route_chunks(uint32_t n) { return std::max<uint32_t>(1, std::min<uint32_t>(1024, (n + 4095) / 4096)); }

bool launch_route(hipStream_t s, const uint64_t *sid, uint32_t n, uint32_t world, uint32_t *hist,
                  unsigned long long *tot, unsigned long long *out, uint64_t segw) {
  if (world == 0 || world > RT_MAXW) return false;
  const uint32_t g = route_chunks(n), chunk = (n + g - 1) / g;
  hipLaunchKernelGGL(k_route_hist, dim3(g), dim3(RT_T), 0, s, sid, n, chunk, world, hist);
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(RT_T), 0, s, hist, g, world, tot, segw, out);
  if (n) hipLaunchKernelGGL(k_route_scatter, dim3(g), dim3(RT_T), 0, s, sid, n, chunk, world, hist, out, segw);
  return true;
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
