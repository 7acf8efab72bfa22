// kmz_shard.hip -- traceId sharding (shard = h(traceId) mod G)
// and the local -> global flatten-index map of a non-contiguous shard.
//
// A rank that owns the traces with shard_of(traceId) == rank holds them in
// their global order, each trace's spans contiguous, so the map from its local
// flatten index to the global one (Traces.ts:29) is monotone.  Every order key
// the path keeps is a MIN of flatten indices (a group's first span,
// RealtimeDataList.ts:23-45; an endpoint's first row, Traces.ts:117-127), and
// a monotone map commutes with MIN: the run works on local indices and only
// the G + E result keys are mapped afterwards (k_remap_index), never the spans.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_kernels.h"

namespace kmz {

static uint32_t grid_of(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192)); }

// sel[t] = spans of trace t0+t if it belongs to `rank`, else 0
__global__ void __launch_bounds__(256) k_shard_select(uint64_t t0, uint64_t nt, uint32_t world, uint32_t rank,
                                                      const uint64_t *__restrict__ cnt, uint64_t *__restrict__ sel) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t hi, lo;
    synth_trace_id(t0 + t, &hi, &lo);
    sel[t] = shard_of(hi, lo, world) == rank ? cnt[t] : 0;
  }
}

// the rank's traces, each at its local offset with its global flatten index
template <int CONFIG>
__global__ void __launch_bounds__(256) k_synth_fill_shard(uint64_t seed, uint64_t t0, uint64_t nt, uint32_t world,
                                                          uint32_t rank, const uint64_t *__restrict__ goff,
                                                          const uint64_t *__restrict__ loff, uint64_t gbase,
                                                          const uint32_t *__restrict__ dur_table, SynthOut out) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t hi, lo;
    synth_trace_id(t0 + t, &hi, &lo);
    if (shard_of(hi, lo, world) == rank) synth_trace<CONFIG>(seed, t0 + t, gbase + goff[t], loff[t], dur_table, &out);
  }
}

__global__ void __launch_bounds__(256) k_add_base(uint64_t *__restrict__ v, uint64_t n, uint64_t base) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] += base;
}

// v[i * stride] = (map(v >> shift) << shift) | (v & low bits), NONE64 kept.
// map(x) = gstart[k] + (x - lstart[k]) for the last run k with lstart[k] <= x
// (lstart non-decreasing; runs of empty or foreign traces repeat a start and
// are skipped by taking the last one).
__global__ void __launch_bounds__(256) k_remap_index(unsigned long long *__restrict__ v, uint64_t n, uint32_t stride,
                                                     uint32_t shift, const uint64_t *__restrict__ lstart,
                                                     const uint64_t *__restrict__ gstart, uint64_t nruns) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long w = v[i * stride];
    if (w == ~0ull) continue;
    const uint64_t x = w >> shift;
    uint64_t a = 0, b = nruns;  // first run with lstart > x
    while (a < b) {
      const uint64_t m = (a + b) >> 1;
      if (lstart[m] <= x)
        a = m + 1;
      else
        b = m;
    }
    if (a == 0) continue;  // (cannot happen: lstart[0] == 0)
    const uint64_t g = gstart[a - 1] + (x - lstart[a - 1]);
    v[i * stride] = (g << shift) | (w & ((1ull << shift) - 1));
  }
}

void launch_shard_select(hipStream_t s, uint64_t t0, uint64_t nt, uint32_t world, uint32_t rank, const uint64_t *cnt,
                         uint64_t *sel) {
  if (nt) hipLaunchKernelGGL(k_shard_select, dim3(grid_of(nt)), dim3(256), 0, s, t0, nt, world, rank, cnt, sel);
}

void launch_synth_fill_shard(hipStream_t s, int config, uint64_t seed, uint64_t t0, uint64_t nt, uint32_t world,
                             uint32_t rank, const uint64_t *goff, const uint64_t *loff, uint64_t gbase,
                             const uint32_t *dur_table, SynthOut out) {
  if (!nt) return;
  const dim3 g(grid_of(nt)), b(256);
  if (config == 2)
    hipLaunchKernelGGL(k_synth_fill_shard<2>, g, b, 0, s, seed, t0, nt, world, rank, goff, loff, gbase, dur_table, out);
  else if (config == 5)
    hipLaunchKernelGGL(k_synth_fill_shard<5>, g, b, 0, s, seed, t0, nt, world, rank, goff, loff, gbase, dur_table, out);
  else
    hipLaunchKernelGGL(k_synth_fill_shard<3>, g, b, 0, s, seed, t0, nt, world, rank, goff, loff, gbase, dur_table, out);
}

void launch_add_base(hipStream_t s, uint64_t *v, uint64_t n, uint64_t base) {
  if (n && base) hipLaunchKernelGGL(k_add_base, dim3(grid_of(n)), dim3(256), 0, s, v, n, base);
}

// v[i] = base + i
__global__ void __launch_bounds__(256) k_iota(unsigned long long *__restrict__ v, uint64_t n, uint64_t base) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = base + i;
}

void launch_iota(hipStream_t s, unsigned long long *v, uint64_t n, uint64_t base) {
  if (n) hipLaunchKernelGGL(k_iota, dim3(grid_of(n)), dim3(256), 0, s, v, n, base);
}

void launch_remap_index(hipStream_t s, unsigned long long *v, uint64_t n, uint32_t stride, uint32_t shift,
                        const uint64_t *lstart, const uint64_t *gstart, uint64_t nruns) {
  if (n && nruns)
    hipLaunchKernelGGL(k_remap_index, dim3(grid_of(n)), dim3(256), 0, s, v, n, stride, shift, lstart, gstart, nruns);
}

}  // namespace kmz
