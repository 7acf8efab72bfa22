// kmz_order.hip -- exact entry order of the reduced dependency graph
// (KMZ_RUN_DEP_ORDER).
//
// The cache layer keeps EndpointDependencies in reduced form: one merged row
// per endpoint, EndpointDependencies.ts:499-542 (combineWith) + 91-112 (trim).
// Its JSON is fixed by the per-row lists of Traces.ts:145-190 and the order in
// which combineWith meets them.  For every entry of the merged graph:
//   dependingBy (side 0) of desc endpoint d, ancestor endpoint a, distance k:
//     r* = the first row of d whose walk has a at distance k;
//     the entry carries ToEndpointInfo of that ancestor span; within r*'s
//     list it sits at its distance (upperMap is filled in walk order).
//   dependingOn (side 1) of anc endpoint a, descendant endpoint d, distance k:
//     r* = the first row of a that a row of d reaches at distance k;
//     within r*'s lowerMap the entry sits where its FIRST such descendant was
//     inserted (rows insert in row order) and carries the LAST one's info.
// Lexicographic minima over the relations give all of it with 64-bit atomics
// (one 32-B table slot per entry key):
//   A0 = min (row(s) << 32 | q)                         side 0
//   A1 = min (row(q) << 32 | row(s)),  B1 = min (row(q) << 32 | ~row(s))   side 1
// (row() = local first-occurrence position; s walks, q is its ancestor).
// One relation is one step of a row's walk over the run's cparent links; the
// value is compared before the atomic, so once the early rows have landed the
// later ones mostly just read (rows are visited in position order).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_kernels.h"

namespace kmz {

static uint32_t grid_of(uint64_t n, uint32_t cap) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, cap));
}

// one 32-B slot per entry: {key, A, B, -}; empty key = ~0 (a key is < 2^63),
// so the table is cleared by one 0xFF memset and a probe + its minima share a
// cache line
struct alignas(32) OrdSlot {
  unsigned long long key, a, b, pad;
};

__device__ __forceinline__ OrdSlot *ord_slot(uint64_t key, OrdSlot *__restrict__ tab, uint64_t ecap,
                                             unsigned int *__restrict__ counters) {
  uint64_t p = slot_of(key, ecap);
  for (uint64_t t = 0; t < ecap; ++t) {
    unsigned long long c = tab[p].key;
    if (c == key) return &tab[p];
    if (c == ~0ull) {
      c = atomicCAS(&tab[p].key, ~0ull, (unsigned long long)key);
      if (c == ~0ull || c == key) return &tab[p];
    }
    p = p + 1 == ecap ? 0 : p + 1;
  }
  atomicOr(&counters[C_FLAGS], F_TABLE_FULL);
  return nullptr;
}

__device__ __forceinline__ void min_to(unsigned long long *a, uint64_t v) {
  if (*(volatile unsigned long long *)a > v) atomicMin(a, (unsigned long long)v);
}

// one thread per span; rows (rowpos != NONE64) walk their cparent chain
__global__ void __launch_bounds__(256) k_dep_order(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                   const uint32_t *__restrict__ cparent,
                                                   const unsigned long long *__restrict__ rowpos, uint32_t n,
                                                   const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                   uint32_t n_ep, uint64_t index_base, OrdSlot *__restrict__ tab,
                                                   uint64_t ecap, unsigned int *__restrict__ counters) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long rp = rowpos[i];
    if (rp == ~0ull) continue;
    const uint64_t r = rp - index_base;
    const uint32_t sh = shape[i];
    const uint32_t d = sh < n_shapes ? dep_ep[sh] : NONE;
    if (d >= n_ep) continue;  // (flagged by the walk already)
    uint32_t q = cparent[i];
    for (uint64_t k = 1; q < n && k <= MAX_DEPTH; ++k) {
      const uint32_t sq = shape[q];
      const uint32_t a = sq < n_shapes ? dep_ep[sq] : NONE;
      if (a >= n_ep) break;
      const uint64_t key = ((uint64_t)a << 40) | ((uint64_t)d << 16) | (k << 1);
      OrdSlot *e = ord_slot(key, tab, ecap, counters);
      if (e) min_to(&e->a, (r << 32) | q);
      if (kind[q] == KIND_SERVER) {
        const uint64_t rq = rowpos[q] - index_base;
        e = ord_slot(key | 1, tab, ecap, counters);
        if (e) {
          min_to(&e->a, (rq << 32) | r);
          min_to(&e->b, (rq << 32) | (~r & 0xFFFFFFFFull));
        }
      }
      q = cparent[q];
    }
  }
}

// value span of each row position (repeated ids: the row of an id is its last
// occurrence, at its first position)
__global__ void __launch_bounds__(256) k_row_value(const unsigned long long *__restrict__ rowpos, uint32_t n,
                                                   uint64_t index_base, uint32_t *__restrict__ val) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long rp = rowpos[i];
    if (rp != ~0ull) val[rp - index_base] = i;
  }
}

// compact the table into kmz_dep_entry records (+ the first rows' ts/shape)
__global__ void __launch_bounds__(256) k_dep_order_out(const OrdSlot *__restrict__ tab, uint64_t ecap,
                                                       const uint32_t *__restrict__ val, const int64_t *__restrict__ ts,
                                                       const uint32_t *__restrict__ shape, uint64_t index_base,
                                                       kmz_dep_entry *__restrict__ out,
                                                       unsigned long long *__restrict__ count,
                                                       const unsigned long long *__restrict__ ep_first, uint32_t n_ep,
                                                       int64_t *__restrict__ row_ts, uint32_t *__restrict__ row_shape) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < ecap; p += stride) {
    const OrdSlot sl = tab[p];
    const uint64_t key = sl.key;
    if (key == ~0ull) continue;
    kmz_dep_entry e;
    e.key = key;
    uint32_t span;
    if (key & 1) {
      const uint32_t rq = (uint32_t)(sl.a >> 32), rs = (uint32_t)sl.a, rl = ~(uint32_t)sl.b;
      span = val ? val[rl] : rl;
      e.row = index_base + rq;
      e.pos = index_base + rs;
    } else {
      const uint32_t rs = (uint32_t)(sl.a >> 32);
      span = (uint32_t)sl.a;
      e.row = index_base + rs;
      e.pos = e.row;
    }
    e.span = index_base + span;
    e.ts = ts[span];
    e.shape = shape[span];
    e.pad = 0;
    out[atomicAdd(count, 1ull)] = e;
  }
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_ep; x += stride) {
    const unsigned long long f = ep_first[x];
    if (f == ~0ull) {
      row_ts[x] = INT64_MIN;
      row_shape[x] = NONE;
    } else {
      const uint32_t r = (uint32_t)((f >> 1) - index_base);
      const uint32_t s = val ? val[r] : r;
      row_ts[x] = ts[s];
      row_shape[x] = shape[s];
    }
  }
}

uint64_t dep_order_slot_bytes() { return sizeof(OrdSlot); }

void launch_dep_order(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                      const uint32_t *cparent, const unsigned long long *rowpos, uint32_t n, const uint32_t *dep_ep,
                      uint32_t n_shapes, uint32_t n_ep, uint64_t index_base, void *tab, uint64_t ecap, uint32_t *val,
                      const unsigned long long *ep_first, kmz_dep_entry *out, unsigned long long *count,
                      int64_t *row_ts, uint32_t *row_shape, unsigned int *counters) {
  OrdSlot *t = static_cast<OrdSlot *>(tab);
  if (val) hipLaunchKernelGGL(k_row_value, dim3(grid_of(n, 16384)), dim3(256), 0, s, rowpos, n, index_base, val);
  hipLaunchKernelGGL(k_dep_order, dim3(grid_of(n, 16384)), dim3(256), 0, s, kind, shape, cparent, rowpos, n, dep_ep,
                     n_shapes, n_ep, index_base, t, ecap, counters);
  hipLaunchKernelGGL(k_dep_order_out, dim3(grid_of(std::max<uint64_t>(ecap, n_ep), 16384)), dim3(256), 0, s, t, ecap,
                     val, ts, shape, index_base, out, count, ep_first, n_ep, row_ts, row_shape);
}

}  // namespace kmz
