// kmz_kernels.hip -- the four hot-path kernels for gfx950 (MI355X).
//
//   K1 build    span-id -> row hash table in HBM (8-byte {tag, index} slots,
//               verified through the span_id column, which is trace-local)
//   K1 fixup    duplicate span ids: last occurrence wins the value, the first
//               keeps the position (JS Map semantics, Traces.ts:117-123)
//   K2 resolve  parent join + CLIENT contraction: for every non-CLIENT span the
//               first non-CLIENT ancestor row (Traces.ts:128-137)
//   K3 stats    segmented (endpoint x status) reduction of exact integer
//               moments, LDS-privatised per workgroup (Traces.ts:27-106,
//               RealtimeDataList.ts:22-118)
//   K4 walk     ancestor traversal over the contracted links: dependency
//               edge triples (LDS-deduplicated, then a global hash set),
//               per-endpoint lastUsage / first row / external (Traces.ts:138-208)
//
// All integer work is exact; the only floating point (finalisation) is shared
// with the host through kmz_common.h and compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include "kmz_kernels.h"

namespace kmz {

// ---------------------------------------------------------------------------
// wave helpers (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ void wave_add_u64(unsigned long long *dst, uint64_t v) {
  // sum over the active lanes, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane_id() == (uint32_t)__ffsll((long long)__ballot(1)) - 1) atomicAdd(dst, (unsigned long long)v);
}

// ---------------------------------------------------------------------------
// K1: build the span-id table
// ---------------------------------------------------------------------------
// slot = tag(key) << 32 | (index + 1); 0 = empty.  Insert claims an empty slot
// with one 64-bit CAS; a slot whose tag matches is verified against
// span_id[index] (the winner's row, usually in the same trace => cached).
// Every thread carries KQ independent inserts in lockstep so that their slot
// loads / CASes overlap (the probe chains are latency bound).
constexpr int KQ = 4;

__global__ void __launch_bounds__(256) k_build(const uint64_t *__restrict__ sid, uint32_t n,
                                               unsigned long long *__restrict__ table, uint64_t cap,
                                               DupEntry *__restrict__ dups, uint32_t dup_cap,
                                               unsigned int *__restrict__ counters) {
  const uint64_t tile = (uint64_t)blockDim.x * KQ;
  for (uint64_t b = (uint64_t)blockIdx.x * tile; b < n; b += (uint64_t)gridDim.x * tile) {
    uint64_t key[KQ], val[KQ], pos[KQ];
    uint32_t tag[KQ], idx[KQ];
    bool act[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      uint64_t i = b + (uint64_t)q * blockDim.x + threadIdx.x;
      act[q] = i < n;
      idx[q] = (uint32_t)i;
      key[q] = act[q] ? sid[i] : 0;
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      if (act[q] && key[q] == 0) {
        atomicOr(&counters[C_FLAGS], F_ZERO_ID);
        act[q] = false;
      }
      tag[q] = tag_of(key[q]);
      val[q] = ((uint64_t)tag[q] << 32) | (uint64_t)(idx[q] + 1);
      pos[q] = slot_of(key[q], cap);
    }
    for (uint64_t probe = 0; probe < cap; ++probe) {
      bool any = false;
      uint64_t cur[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) cur[q] = act[q] ? table[pos[q]] : 0;
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        if (act[q] && cur[q] == 0) cur[q] = atomicCAS(&table[pos[q]], 0ull, (unsigned long long)val[q]);
      uint32_t w[KQ];
      uint64_t wk[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        w[q] = (uint32_t)cur[q] - 1;
        wk[q] = 0;
        if (!act[q]) continue;
        if (cur[q] == 0) {  // claimed
          act[q] = false;
          continue;
        }
        if ((uint32_t)(cur[q] >> 32) == tag[q]) wk[q] = sid[w[q]];
      }
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        if (!act[q]) continue;
        if ((uint32_t)(cur[q] >> 32) == tag[q] && wk[q] == key[q]) {  // duplicate id: defer to the fixup
          uint32_t d = atomicAdd(&counters[C_DUPS], 1u);
          if (d < dup_cap) {
            dups[d].pos = (uint32_t)pos[q];
            dups[d].idx = idx[q];
            dups[d].winner = w[q];
          } else {
            atomicOr(&counters[C_FLAGS], F_DUP_OVERFLOW);
          }
          act[q] = false;
          continue;
        }
        pos[q] = (pos[q] + 1 == cap) ? 0 : pos[q] + 1;
        any = true;
      }
      if (!any) break;
      if (probe + 1 == cap) atomicOr(&counters[C_FLAGS], F_TABLE_FULL);
    }
  }
}

// Duplicate ids: slot index := max occurrence (the Map value), dupmap[pos] :=
// min occurrence (the Map position).
__global__ void __launch_bounds__(256) k_fixup(const DupEntry *__restrict__ dups, const unsigned int *__restrict__ counters,
                                               uint32_t dup_cap, unsigned long long *__restrict__ table,
                                               unsigned int *__restrict__ dkey, unsigned int *__restrict__ dval,
                                               uint32_t dcap) {
  uint32_t nd = min(counters[C_DUPS], dup_cap);
  uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < nd; e += stride) {
    DupEntry d = dups[e];
    uint64_t cur = table[d.pos];
    atomicMax(&table[d.pos], (unsigned long long)((cur & 0xFFFFFFFF00000000ull) | (uint64_t)(d.idx + 1)));
    uint32_t first = min(d.idx, d.winner);
    uint32_t h = (uint32_t)slot_of(d.pos, dcap);
    for (uint32_t p = 0; p < dcap; ++p) {
      uint32_t k = dkey[h];
      if (k == 0) k = atomicCAS(&dkey[h], 0u, d.pos + 1);
      if (k == 0 || k == d.pos + 1) {
        atomicMin(&dval[h], first);
        break;
      }
      h = (h + 1 == dcap) ? 0 : h + 1;
    }
  }
}

__device__ __forceinline__ uint32_t lookup(uint64_t key, const uint64_t *__restrict__ sid,
                                           const unsigned long long *__restrict__ table, uint64_t cap) {
  uint32_t tag = tag_of(key);
  uint64_t pos = slot_of(key, cap);
  for (uint64_t probe = 0; probe < cap; ++probe) {
    uint64_t cur = table[pos];
    if (cur == 0) return NONE;
    if ((uint32_t)(cur >> 32) == tag) {
      uint32_t w = (uint32_t)cur - 1;
      if (sid[w] == key) return w;
    }
    pos = (pos + 1 == cap) ? 0 : pos + 1;
  }
  return NONE;
}

__device__ __forceinline__ uint32_t dup_first(uint64_t pos, const unsigned int *__restrict__ dkey,
                                              const unsigned int *__restrict__ dval, uint32_t dcap) {
  uint32_t h = (uint32_t)slot_of(pos, dcap);
  for (uint32_t p = 0; p < dcap; ++p) {
    uint32_t k = dkey[h];
    if (k == 0) return NONE;
    if (k == (uint32_t)pos + 1) return dval[h];
    h = (h + 1 == dcap) ? 0 : h + 1;
  }
  return NONE;
}

// ---------------------------------------------------------------------------
// K2: parent join + CLIENT contraction
// ---------------------------------------------------------------------------
// cparent[i] = the row reached from span i's parentId after skipping CLIENT
// spans (Traces.ts:131-137), KMZ_NONE when the walk ends.  CLIENT spans never
// start or continue a walk past themselves, so they get NONE.  A CLIENT-only
// loop yields CYC; it is an error only when a row's walk reaches it (K4), as
// the reference only loops on chains it actually walks.
__global__ void __launch_bounds__(256) k_resolve(const uint64_t *__restrict__ sid, const uint64_t *__restrict__ pid,
                                                 const uint8_t *__restrict__ kind, uint32_t n,
                                                 const unsigned long long *__restrict__ table, uint64_t cap,
                                                 uint32_t *__restrict__ cparent, unsigned int *__restrict__ counters) {
  // KQ spans per thread walk their lookups in lockstep: one slot load per
  // pending lookup per round, then the candidate's (span_id, kind, parent_id)
  // together, so every round keeps KQ independent chains in flight.
  const uint64_t tile = (uint64_t)blockDim.x * KQ;
  for (uint64_t b = (uint64_t)blockIdx.x * tile; b < n; b += (uint64_t)gridDim.x * tile) {
    uint64_t p[KQ], pos[KQ];
    uint32_t tag[KQ], res[KQ], hops[KQ];
    bool act[KQ];
    uint8_t k0[KQ];
    uint64_t p0[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      uint64_t i = b + (uint64_t)q * blockDim.x + threadIdx.x;
      k0[q] = i < n ? kind[i] : KIND_CLIENT;
      p0[q] = i < n ? pid[i] : 0;
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      p[q] = k0[q] != KIND_CLIENT ? p0[q] : 0;
      act[q] = p[q] != 0;
      res[q] = NONE;
      hops[q] = 0;
      tag[q] = tag_of(p[q]);
      pos[q] = slot_of(p[q], cap);
    }
    for (uint32_t round = 0; round < 4 * MAX_DEPTH; ++round) {
      uint64_t cur[KQ];
      bool any = false;
#pragma unroll
      for (int q = 0; q < KQ; ++q) cur[q] = act[q] ? table[pos[q]] : 0;
      uint64_t vs[KQ], vp[KQ];
      uint8_t vk[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        vs[q] = 0;
        vp[q] = 0;
        vk[q] = 0;
        if (act[q] && cur[q] != 0 && (uint32_t)(cur[q] >> 32) == tag[q]) {
          uint32_t w = (uint32_t)cur[q] - 1;
          vs[q] = sid[w];
          vk[q] = kind[w];
          vp[q] = pid[w];
        }
      }
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        if (!act[q]) continue;
        if (cur[q] == 0) {  // parent id absent: the walk stops (Traces.ts:133)
          act[q] = false;
          continue;
        }
        if ((uint32_t)(cur[q] >> 32) == tag[q] && vs[q] == p[q]) {
          uint32_t w = (uint32_t)cur[q] - 1;
          if (vk[q] != KIND_CLIENT) {
            res[q] = w;
            act[q] = false;
            continue;
          }
          // CLIENT: skip it and continue with its parent (Traces.ts:134-137)
          if (++hops[q] > MAX_DEPTH) {  // only an error if a row's walk reaches it (K4)
            res[q] = CYC;
            act[q] = false;
            continue;
          }
          p[q] = vp[q];
          if (p[q] == 0) {
            act[q] = false;
            continue;
          }
          tag[q] = tag_of(p[q]);
          pos[q] = slot_of(p[q], cap);
          any = true;
          continue;
        }
        pos[q] = (pos[q] + 1 == cap) ? 0 : pos[q] + 1;
        any = true;
      }
      if (!any) break;
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      uint64_t i = b + (uint64_t)q * blockDim.x + threadIdx.x;
      if (i < n) cparent[i] = res[q];
    }
  }
}

// ---------------------------------------------------------------------------
// K3: (endpoint x status) reduction
// ---------------------------------------------------------------------------
// Per SERVER span (every occurrence, Traces.ts:28-31): g = ep * n_status + status,
//   count += 1, s1 += d, s2a += lo32(d*d), s2b += hi32(d*d),
//   tsmax = max(ts ^ 2^63), first = min(global index).
// Workgroups privatise the accumulators in LDS: DIRECT indexes them by g when
// all groups fit, HASHED keeps an open-addressing LDS table of recently seen
// groups and falls back to global atomics when it is full.
struct GroupAcc {
  unsigned long long *cnt, *s1, *s2a, *s2b, *tsx, *fst;
};

__device__ __forceinline__ void acc_global(const GroupAcc &a, uint32_t g, uint64_t d, uint64_t tsx, uint64_t gi) {
  uint64_t dd = d * d;
  atomicAdd(&a.cnt[g], 1ull);
  atomicAdd(&a.s1[g], (unsigned long long)d);
  atomicAdd(&a.s2a[g], (unsigned long long)(dd & 0xFFFFFFFFull));
  atomicAdd(&a.s2b[g], (unsigned long long)(dd >> 32));
  atomicMax(&a.tsx[g], (unsigned long long)tsx);
  atomicMin(&a.fst[g], (unsigned long long)gi);
}

constexpr uint32_t K3_DIRECT_MAX = 1024;  // groups held directly in LDS (48 KiB)
constexpr uint32_t K3_HASH_CAP = 1024;    // LDS hash entries (52 KiB)

template <bool DIRECT>
__global__ void __launch_bounds__(256) k_stats(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                               const uint16_t *__restrict__ status,
                                               const uint32_t *__restrict__ dur, const int64_t *__restrict__ ts,
                                               uint32_t n, uint32_t chunk, const uint32_t *__restrict__ ep_of_shape,
                                               uint32_t n_shapes, uint32_t n_ep, uint32_t n_status, uint64_t index_base,
                                               GroupAcc acc, unsigned int *__restrict__ counters,
                                               unsigned long long *__restrict__ n_server) {
  __shared__ unsigned long long l_cnt[K3_HASH_CAP], l_s1[K3_HASH_CAP], l_s2a[K3_HASH_CAP], l_s2b[K3_HASH_CAP],
      l_tsx[K3_HASH_CAP], l_fst[K3_HASH_CAP];
  __shared__ unsigned int l_key[DIRECT ? 1 : K3_HASH_CAP];
  const uint32_t G = n_ep * n_status;
  const uint32_t slots = DIRECT ? G : K3_HASH_CAP;
  for (uint32_t s = threadIdx.x; s < slots; s += blockDim.x) {
    l_cnt[s] = 0;
    l_s1[s] = 0;
    l_s2a[s] = 0;
    l_s2b[s] = 0;
    l_tsx[s] = 0;
    l_fst[s] = ~0ull;
    if (!DIRECT) l_key[s] = 0;
  }
  __syncthreads();
  uint64_t c0 = (uint64_t)blockIdx.x * chunk;
  uint32_t end = (uint32_t)min<uint64_t>(c0 + chunk, n);
  uint32_t servers = 0;
  for (uint32_t i = (uint32_t)c0 + threadIdx.x; i < end; i += blockDim.x) {
    if (kind[i] != KIND_SERVER) continue;
    ++servers;
    uint32_t sh = shape[i];
    uint32_t st = status[i];
    uint32_t ep = sh < n_shapes ? (ep_of_shape ? ep_of_shape[sh] : sh) : NONE;  // null map: group by shape
    if (ep >= n_ep || st >= n_status) {
      atomicOr(&counters[C_FLAGS], F_RANGE);
      continue;
    }
    uint32_t g = ep * n_status + st;
    uint64_t d = dur[i];
    uint64_t dd = d * d;
    uint64_t tsx = (uint64_t)ts[i] ^ TS_BIAS;
    uint64_t gi = index_base + i;
    uint32_t s = NONE;
    if (DIRECT) {
      s = g;
    } else {
      uint32_t h = (g * 2654435761u) >> 22;  // 10 bits
      for (uint32_t p = 0; p < 32; ++p) {
        uint32_t k = l_key[h];
        if (k == 0) k = atomicCAS(&l_key[h], 0u, g + 1);
        if (k == 0 || k == g + 1) {
          s = h;
          break;
        }
        h = (h + 1) & (K3_HASH_CAP - 1);
      }
    }
    if (s == NONE) {
      acc_global(acc, g, d, tsx, gi);
      continue;
    }
    atomicAdd(&l_cnt[s], 1ull);
    atomicAdd(&l_s1[s], (unsigned long long)d);
    atomicAdd(&l_s2a[s], (unsigned long long)(dd & 0xFFFFFFFFull));
    atomicAdd(&l_s2b[s], (unsigned long long)(dd >> 32));
    atomicMax(&l_tsx[s], (unsigned long long)tsx);
    atomicMin(&l_fst[s], (unsigned long long)gi);
  }
  wave_add_u64(n_server, servers);
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < slots; s += blockDim.x) {
    if (l_cnt[s] == 0) continue;
    uint32_t g = DIRECT ? s : l_key[s] - 1;
    atomicAdd(&acc.cnt[g], l_cnt[s]);
    atomicAdd(&acc.s1[g], l_s1[s]);
    atomicAdd(&acc.s2a[g], l_s2a[s]);
    atomicAdd(&acc.s2b[g], l_s2b[s]);
    atomicMax(&acc.tsx[g], l_tsx[s]);
    atomicMin(&acc.fst[g], l_fst[s]);
  }
}

// ---------------------------------------------------------------------------
// K4: ancestor traversal
// ---------------------------------------------------------------------------
constexpr uint32_t K4_TSET = 2048;      // LDS triple set (16 KiB)
constexpr uint32_t K4_EP_DIRECT = 2048; // endpoints privatised in LDS (32 KiB)

__device__ __forceinline__ void triple_global(uint64_t key, unsigned long long *__restrict__ trip, uint64_t tcap,
                                              unsigned int *__restrict__ counters) {
  uint64_t pos = eslot(key, tcap);
  // bounded probing: at load <= 0.7 a run of 256 occupied slots does not occur;
  // if it does, the table is (being) overfilled and the host retries bigger
  for (uint64_t p = 0; p < 256; ++p) {
    uint64_t cur = trip[pos];
    if (cur == key) return;
    if (cur == 0) {
      cur = atomicCAS(&trip[pos], 0ull, (unsigned long long)key);
      if (cur == 0) {
        uint32_t c = atomicAdd(&counters[C_TRIPLES], 1u) + 1;
        if ((uint64_t)c * 10 > tcap * 7) atomicOr(&counters[C_FLAGS], F_TRIPLE_OVERFLOW);
        return;
      }
      if (cur == key) return;
    }
    pos = eset_next(pos, tcap);  // (sliced probing, kmz_common.h)
  }
  atomicOr(&counters[C_FLAGS], F_TRIPLE_OVERFLOW);
}

template <bool EP_DIRECT>
__global__ void __launch_bounds__(256) k_walk(const uint64_t *__restrict__ sid, const uint8_t *__restrict__ kind,
                                              const uint32_t *__restrict__ shape, const int64_t *__restrict__ ts,
                                              const uint32_t *__restrict__ cparent, uint32_t n, uint32_t chunk,
                                              const uint32_t *__restrict__ dep_ep, uint32_t n_shapes, uint32_t n_ep,
                                              uint64_t index_base, const unsigned long long *__restrict__ table,
                                              uint64_t cap, const unsigned int *__restrict__ dkey,
                                              const unsigned int *__restrict__ dval, uint32_t dcap,
                                              unsigned long long *__restrict__ trip, uint64_t tcap,
                                              unsigned long long *__restrict__ ep_ts,
                                              unsigned long long *__restrict__ ep_first,
                                              unsigned long long *__restrict__ rowpos_out,
                                              unsigned int *__restrict__ counters,
                                              unsigned long long *__restrict__ stats64, uint32_t ablate) {
  __shared__ unsigned long long l_set[K4_TSET];
  __shared__ unsigned long long l_ts[EP_DIRECT ? K4_EP_DIRECT : 1], l_first[EP_DIRECT ? K4_EP_DIRECT : 1];
  for (uint32_t s = threadIdx.x; s < K4_TSET; s += blockDim.x) l_set[s] = 0;
  if (EP_DIRECT)
    for (uint32_t s = threadIdx.x; s < n_ep; s += blockDim.x) {
      l_ts[s] = 0;
      l_first[s] = ~0ull;
    }
  __syncthreads();
  const bool have_dups = counters[C_DUPS] != 0;
  uint64_t c0 = (uint64_t)blockIdx.x * chunk;
  uint32_t end = (uint32_t)min<uint64_t>(c0 + chunk, n);
  uint64_t rel = 0, rows = 0;
  uint32_t maxd = 0;
  for (uint32_t i = (uint32_t)c0 + threadIdx.x; i < end; i += blockDim.x) {
    uint64_t rp = NONE64;
    if (kind[i] == KIND_SERVER) {
      uint32_t first = i;
      bool is_row = true;
      if (have_dups) {  // the row of an id is its LAST occurrence, at its FIRST position
        uint32_t last = lookup(sid[i], sid, table, cap);
        if (last != i) {
          is_row = false;
        } else {
          uint64_t pos = slot_of(sid[i], cap);
          // find the slot index of this key for the dupmap
          for (uint64_t p = 0; p < cap; ++p) {
            uint64_t cur = table[pos];
            if ((uint32_t)cur - 1 == i) break;
            pos = (pos + 1 == cap) ? 0 : pos + 1;
          }
          uint32_t f = dup_first(pos, dkey, dval, dcap);
          if (f != NONE) first = f;
        }
      }
      if (is_row) {
        ++rows;
        rp = index_base + first;
        uint32_t sh = shape[i];
        uint32_t es = sh < n_shapes ? dep_ep[sh] : NONE;
        if (es >= n_ep) {
          atomicOr(&counters[C_FLAGS], F_RANGE);
        } else {
          uint32_t cur = cparent[i];
          uint64_t fkey = (rp << 1) | (cur != NONE ? 1ull : 0ull);
          uint64_t tsx = (uint64_t)ts[i] ^ TS_BIAS;
          if (EP_DIRECT) {
            atomicMax(&l_ts[es], (unsigned long long)tsx);
            atomicMin(&l_first[es], (unsigned long long)fkey);
          } else if (!(ablate & 4)) {
            atomicMax(&ep_ts[es], (unsigned long long)tsx);
            atomicMin(&ep_first[es], (unsigned long long)fkey);
          }
          uint32_t d = 0;
          while (cur != NONE) {
            ++d;
            if (d > MAX_DEPTH || cur == CYC) {
              atomicOr(&counters[C_FLAGS], F_CYCLE);
              break;
            }
            uint8_t ka = kind[cur];
            uint32_t sa = shape[cur];
            uint32_t ea = sa < n_shapes ? dep_ep[sa] : NONE;
            if (ea >= n_ep) {
              atomicOr(&counters[C_FLAGS], F_RANGE);
              break;
            }
            uint64_t key = ((uint64_t)ea << 40) | ((uint64_t)es << 16) | ((uint64_t)d << 1) |
                           (ka == KIND_SERVER ? 1ull : 0ull);
            // LDS dedup, then the global set
            uint32_t h = (uint32_t)(mix64(key) >> 53);  // 11 bits
            bool done = (ablate & 1) != 0;  // diagnostic: skip edge-key dedup
            for (uint32_t p = 0; p < 8; ++p) {
              uint64_t c = l_set[h];
              if (c == key) {
                done = true;
                break;
              }
              if (c == 0) {
                c = atomicCAS(&l_set[h], 0ull, (unsigned long long)key);
                if (c == 0) break;  // new in this workgroup
                if (c == key) {
                  done = true;
                  break;
                }
              }
              h = (h + 1) & (K4_TSET - 1);
            }
            if (!done && !(ablate & 2)) triple_global(key, trip, tcap, counters);
            if (ka != KIND_SERVER) {  // non-SERVER ancestors are not rows: count their use here
              uint64_t tsa = (uint64_t)ts[cur] ^ TS_BIAS;
              if (EP_DIRECT)
                atomicMax(&l_ts[ea], (unsigned long long)tsa);
              else
                atomicMax(&ep_ts[ea], (unsigned long long)tsa);
            }
            cur = cparent[cur];
          }
          rel += d;
          maxd = max(maxd, d);
        }
      }
    }
    if (rowpos_out) rowpos_out[i] = rp;
  }
  wave_add_u64(&stats64[S_ROWS], rows);
  wave_add_u64(&stats64[S_REL], rel);
  for (int off = 32; off > 0; off >>= 1) maxd = max(maxd, (uint32_t)__shfl_xor(maxd, off, 64));
  if (lane_id() == 0 && maxd) atomicMax(&stats64[S_MAXD], (unsigned long long)maxd);
  if (EP_DIRECT) {
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < n_ep; s += blockDim.x) {
      if (l_ts[s]) atomicMax(&ep_ts[s], l_ts[s]);
      if (l_first[s] != ~0ull) atomicMin(&ep_first[s], l_first[s]);
    }
  }
}

// ---------------------------------------------------------------------------
// finalisation / compaction
// ---------------------------------------------------------------------------
// Each workgroup finalises whole chunks of FZ_CH groups; with `bcnt` (one
// chunk per workgroup) it also counts the chunk's used groups (combined > 0)
// for k_used_scatter.
constexpr uint32_t FZ_T = 256, FZ_PT = 4, FZ_CH = FZ_T * FZ_PT;
__global__ void __launch_bounds__(FZ_T) k_finalize(GroupAcc acc, uint32_t G, kmz_group *__restrict__ out,
                                                   uint32_t *__restrict__ bcnt) {
  __shared__ uint32_t wsum[FZ_T / 64];
  for (uint64_t base = (uint64_t)blockIdx.x * FZ_CH; base < G; base += (uint64_t)gridDim.x * FZ_CH) {
    uint32_t used = 0;
#pragma unroll
    for (uint32_t q = 0; q < FZ_PT; ++q) {
      const uint64_t g = base + q * FZ_T + threadIdx.x;
      if (g >= G) continue;
      kmz_group r;
      r.combined = acc.cnt[g];
      r.first = acc.fst[g];
      r.latest_timestamp = (int64_t)(acc.tsx[g] ^ TS_BIAS);
      finalize_moments(acc.cnt[g], acc.s1[g], acc.s2a[g], acc.s2b[g], &r.mean, &r.cv);
      out[g] = r;
      used += r.combined != 0;
    }
    if (bcnt) {  // (one chunk per workgroup)
      for (int o = 32; o > 0; o >>= 1) used += __shfl_xor(used, o, 64);
      if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = used;
      __syncthreads();
      if (threadIdx.x == 0) bcnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
  }
}

// The used groups in ascending id, compacted (kmz_fetch_used copies only
// them: a 2 500-trace tick touches 7-19 % of the groups, and the dense copy
// was most of its fetch).  Workgroup b: its chunk's offset = the used counts
// of the chunks before it (at most 2^12 of them), then the chunk's used
// groups in order by wave ballots; the last workgroup stores the total.
__global__ void __launch_bounds__(FZ_T) k_used_scatter(const kmz_group *__restrict__ dense, uint32_t G,
                                                       const uint32_t *__restrict__ bcnt, uint32_t *__restrict__ ids,
                                                       kmz_group *__restrict__ used,
                                                       unsigned long long *__restrict__ total) {
  __shared__ uint32_t wsum[FZ_T / 64];
  __shared__ uint32_t wpre[FZ_PT][FZ_T / 64];
  const uint32_t b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t pre = 0;
  for (uint32_t k = threadIdx.x; k < b; k += FZ_T) pre += bcnt[k];
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  bool f[FZ_PT];
  uint64_t m[FZ_PT];
#pragma unroll
  for (uint32_t q = 0; q < FZ_PT; ++q) {
    const uint64_t g = (uint64_t)b * FZ_CH + q * FZ_T + threadIdx.x;
    f[q] = g < G && dense[g].combined != 0;
    m[q] = __ballot(f[q]);
    if (lane == 0) wpre[q][w] = __popcll(m[q]);
  }
  if (lane == 0) wsum[w] = pre;
  __syncthreads();
  uint32_t off = wsum[0] + wsum[1] + wsum[2] + wsum[3];  // the chunks before this one
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (uint32_t q = 0; q < FZ_PT; ++q) {
    uint32_t at = off;
    for (uint32_t v = 0; v < w; ++v) at += wpre[q][v];
    if (f[q]) {
      const uint64_t g = (uint64_t)b * FZ_CH + q * FZ_T + threadIdx.x;
      const uint32_t pos = at + (uint32_t)__popcll(m[q] & lt);
      ids[pos] = (uint32_t)g;
      used[pos] = dense[g];
    }
    for (uint32_t v = 0; v < FZ_T / 64; ++v) off += wpre[q][v];
  }
  if (b + 1 == gridDim.x && threadIdx.x == 0) *total = off;
}

// K3 runs once per batch over (shape x status).  The endpoint groups of either
// realtime identity (Traces.ts:32-46 / 73-99) are unions of shape groups; the
// integer moments, max timestamp and min first index combine exactly.
__global__ void __launch_bounds__(256) k_collapse_groups(const unsigned long long *__restrict__ sg, uint32_t n_shapes,
                                                         uint32_t S, const uint32_t *__restrict__ map, uint32_t n_ep,
                                                         unsigned long long *__restrict__ grp,
                                                         unsigned int *__restrict__ counters) {
  const uint64_t Gs = (uint64_t)n_shapes * S, G = (uint64_t)n_ep * S;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < Gs; x += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = sg[x];
    if (!c) continue;
    const uint32_t sh = (uint32_t)(x / S), st = (uint32_t)(x % S);
    const uint32_t e = map[sh];
    if (e >= n_ep) {
      atomicOr(&counters[C_FLAGS], F_RANGE);
      continue;
    }
    const uint64_t g = (uint64_t)e * S + st;
    atomicAdd(&grp[g], c);
    atomicAdd(&grp[G + g], sg[Gs + x]);
    atomicAdd(&grp[2 * G + g], sg[2 * Gs + x]);
    atomicAdd(&grp[3 * G + g], sg[3 * Gs + x]);
    atomicMax(&grp[4 * G + g], sg[4 * Gs + x]);
    atomicMin(&grp[5 * G + g], sg[5 * Gs + x]);
  }
}

// Rows of a batch with unique span ids are its SERVER spans, so the per
// dependency endpoint lastUsage (max timestamp of its rows) and first row (min
// index) are unions of shape groups too; `external` is read off the first
// row's contracted parent (Traces.ts:182-190, EndpointDependencies.ts:508-541).
__global__ void __launch_bounds__(256) k_collapse_endpoints(const unsigned long long *__restrict__ sg, uint32_t n_shapes,
                                                            uint32_t S, const uint32_t *__restrict__ dep_map,
                                                            uint32_t n_dep, const uint32_t *__restrict__ cparent,
                                                            uint64_t index_base,
                                                            unsigned long long *__restrict__ ep_ts,
                                                            unsigned long long *__restrict__ ep_first,
                                                            unsigned int *__restrict__ counters) {
  const uint64_t Gs = (uint64_t)n_shapes * S;
  for (uint32_t sh = blockIdx.x * blockDim.x + threadIdx.x; sh < n_shapes; sh += gridDim.x * blockDim.x) {
    unsigned long long tsx = 0, fst = ~0ull;
    for (uint32_t st = 0; st < S; ++st) {
      const uint64_t x = (uint64_t)sh * S + st;
      if (!sg[x]) continue;
      tsx = max(tsx, sg[4 * Gs + x]);
      fst = min(fst, sg[5 * Gs + x]);
    }
    if (fst == ~0ull) continue;
    const uint32_t e = dep_map ? dep_map[sh] : sh;
    if (e >= n_dep) {
      atomicOr(&counters[C_FLAGS], F_RANGE);
      continue;
    }
    atomicMax(&ep_ts[e], tsx);
    const uint32_t cp = cparent[fst - index_base];
    atomicMin(&ep_first[e], (fst << 1) | (cp != NONE ? 1ull : 0ull));
  }
}

// Edge-set compaction: each workgroup takes chunks of CP_CH slots, each wave
// a contiguous quarter of the chunk, CP_PL slots per lane held in registers
// (every load in flight at once, one read of the table); the wave counts its
// keys by ballots, the workgroup reserves the chunk's output range with ONE
// atomic, and each wave writes its keys in slot order, one ballot prefix per
// 64 slots (no barrier inside the loop).  Output order is free (the keys are
// a set).  (The form with a second, cache-resident read of the slice and two
// barriers per 256 slots took 148 us on config 5's 2^25-slot set.)
constexpr uint32_t CP_T = 256, CP_PL = 32, CP_CH = CP_T * CP_PL;
__global__ void __launch_bounds__(CP_T) k_compact(const unsigned long long *__restrict__ trip, uint64_t tcap,
                                                  unsigned long long *__restrict__ out,
                                                  unsigned long long *__restrict__ count) {
  __shared__ uint32_t wsum[CP_T / 64];
  __shared__ unsigned long long wbase[CP_T / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1;
  for (uint64_t c0 = (uint64_t)blockIdx.x * CP_CH; c0 < tcap; c0 += (uint64_t)gridDim.x * CP_CH) {
    const uint64_t wb = c0 + (uint64_t)w * (CP_CH / (CP_T / 64));
    unsigned long long k[CP_PL];
#pragma unroll
    for (uint32_t j = 0; j < CP_PL; ++j) {
      const uint64_t p = wb + j * 64 + lane;
      k[j] = p < tcap ? trip[p] : 0ull;
    }
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < CP_PL; ++j) c += (uint32_t)__popcll(__ballot(k[j] != 0));
    if (lane == 0) wsum[w] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (uint32_t v = 0; v < CP_T / 64; ++v) t += wsum[v];
      unsigned long long b = t ? atomicAdd(count, (unsigned long long)t) : 0ull;
      for (uint32_t v = 0; v < CP_T / 64; ++v) {
        wbase[v] = b;
        b += wsum[v];
      }
    }
    __syncthreads();
    unsigned long long run = wbase[w];
#pragma unroll
    for (uint32_t j = 0; j < CP_PL; ++j) {
      const uint64_t m = __ballot(k[j] != 0);
      if (k[j]) out[run + __popcll(m & lt)] = k[j];
      run += __popcll(m);
    }
    __syncthreads();  // (wsum / wbase reused by the next chunk)
  }
}

// ---------------------------------------------------------------------------
// synthetic generation
// ---------------------------------------------------------------------------
template <int CONFIG>
__global__ void __launch_bounds__(256) k_synth_count(uint64_t seed, uint64_t t0, uint64_t nt, uint64_t *__restrict__ cnt) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x)
    cnt[t] = synth_trace<CONFIG>(seed, t0 + t, 0, 0, nullptr, nullptr);
}

template <int CONFIG>
__global__ void __launch_bounds__(256) k_synth_fill(uint64_t seed, uint64_t t0, uint64_t nt,
                                                    const uint64_t *__restrict__ off, uint64_t gbase,
                                                    const uint32_t *__restrict__ dur_table, SynthOut out) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x)
    synth_trace<CONFIG>(seed, t0 + t, gbase + off[t], off[t], dur_table, &out);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline uint32_t grid_for(uint64_t work, uint32_t cap_blocks = 8192) {
  uint64_t b = (work + 255) / 256;
  if (b < 1) b = 1;
  return (uint32_t)(b < cap_blocks ? b : cap_blocks);
}

void launch_build(hipStream_t s, const uint64_t *sid, uint32_t n, unsigned long long *table, uint64_t cap,
                  DupEntry *dups, uint32_t dup_cap, unsigned int *counters) {
  if (!n) return;
  hipLaunchKernelGGL(k_build, dim3(grid_for((n + KQ - 1) / KQ)), dim3(256), 0, s, sid, n, table, cap, dups, dup_cap,
                     counters);
}
void launch_fixup(hipStream_t s, const DupEntry *dups, const unsigned int *counters, uint32_t dup_cap,
                  unsigned long long *table, unsigned int *dkey, unsigned int *dval, uint32_t dcap) {
  hipLaunchKernelGGL(k_fixup, dim3(grid_for(dup_cap, 1024)), dim3(256), 0, s, dups, counters, dup_cap, table, dkey, dval,
                     dcap);
}
void launch_resolve(hipStream_t s, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind, uint32_t n,
                    const unsigned long long *table, uint64_t cap, uint32_t *cparent, unsigned int *counters) {
  if (!n) return;
  hipLaunchKernelGGL(k_resolve, dim3(grid_for((n + KQ - 1) / KQ)), dim3(256), 0, s, sid, pid, kind, n, table, cap,
                     cparent, counters);
}

static inline uint32_t chunk_for(uint32_t n, uint32_t min_chunk) {
  // >= ~2048 workgroups for a full chip when n allows it, chunks of >= min_chunk
  uint32_t c = (n + 2047) / 2048;
  if (c < min_chunk) c = min_chunk;
  return (c + 255) / 256 * 256;
}

void launch_stats(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status, const uint32_t *dur,
                  const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape, uint32_t n_shapes, uint32_t n_ep,
                  uint32_t n_status, uint64_t index_base, unsigned long long *grp, unsigned int *counters,
                  unsigned long long *n_server) {
  if (!n) return;
  uint64_t G = (uint64_t)n_ep * n_status;
  GroupAcc a{grp, grp + G, grp + 2 * G, grp + 3 * G, grp + 4 * G, grp + 5 * G};
  if (G <= K3_DIRECT_MAX) {
    uint32_t chunk = chunk_for(n, (uint32_t)(4 * G > 1024 ? 4 * G : 1024));
    uint32_t blocks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_stats<true>, dim3(blocks), dim3(256), 0, s, kind, shape, status, dur, ts, n, chunk, ep_of_shape,
                       n_shapes, n_ep, n_status, index_base, a, counters, n_server);
  } else {
    uint32_t chunk = chunk_for(n, 4096);
    uint32_t blocks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_stats<false>, dim3(blocks), dim3(256), 0, s, kind, shape, status, dur, ts, n, chunk,
                       ep_of_shape, n_shapes, n_ep, n_status, index_base, a, counters, n_server);
  }
}

void launch_walk(hipStream_t s, const uint64_t *sid, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                 const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                 uint64_t index_base, const unsigned long long *table, uint64_t cap, const unsigned int *dkey,
                 const unsigned int *dval, uint32_t dcap, unsigned long long *trip, uint64_t tcap,
                 unsigned long long *ep_ts, unsigned long long *ep_first, unsigned long long *rowpos,
                 unsigned int *counters, unsigned long long *stats64, uint32_t ablate) {
  if (!n) return;
  if (n_ep <= K4_EP_DIRECT) {
    uint32_t chunk = chunk_for(n, 4 * n_ep > 1024 ? 4 * n_ep : 1024);
    uint32_t blocks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_walk<true>, dim3(blocks), dim3(256), 0, s, sid, kind, shape, ts, cparent, n, chunk, dep_ep,
                       n_shapes, n_ep, index_base, table, cap, dkey, dval, dcap, trip, tcap, ep_ts, ep_first, rowpos,
                       counters, stats64, ablate);
  } else {
    uint32_t chunk = chunk_for(n, 1024);
    uint32_t blocks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_walk<false>, dim3(blocks), dim3(256), 0, s, sid, kind, shape, ts, cparent, n, chunk, dep_ep,
                       n_shapes, n_ep, index_base, table, cap, dkey, dval, dcap, trip, tcap, ep_ts, ep_first, rowpos,
                       counters, stats64, ablate);
  }
}

// Several buffer fills in one launch (a run's per-buffer hipMemsetAsync calls
// were 13 fill kernels, ~3 us of GPU time each at a production tick):
// blockIdx.y = the segment; 16-byte stores where the segment is aligned.
__global__ void __launch_bounds__(256) k_fill(FillArgs a) {
  const uint32_t k = blockIdx.y;
  if (k >= a.n) return;
  uint8_t *p = reinterpret_cast<uint8_t *>(a.p[k]);
  const uint64_t bytes = a.bytes[k];
  const uint32_t v = a.val[k] & 0xFFu;
  const uint32_t w = v | (v << 8) | (v << 16) | (v << 24);
  const uint64_t head = (16 - ((uintptr_t)p & 15)) & 15;
  const uint64_t h = head < bytes ? head : bytes;
  const uint64_t n16 = (bytes - h) / 16;
  uint4 *q = reinterpret_cast<uint4 *>(p + h);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
    q[i] = make_uint4(w, w, w, w);
  if (blockIdx.x == 0) {  // unaligned head and tail bytes
    if (threadIdx.x < h) p[threadIdx.x] = (uint8_t)v;
    const uint64_t t0 = h + n16 * 16;
    if (t0 + threadIdx.x < bytes) p[t0 + threadIdx.x] = (uint8_t)v;
  }
}

// up to 4 device-to-device copies of 8-byte-multiple, 8-byte-aligned ranges in
// one launch (kmz_fetch_begin's snapshot: one launch instead of three blits
// on the critical path of a pipelined step)
__global__ void __launch_bounds__(256) k_copy8(CopyArgs a) {
  const uint32_t k = blockIdx.y;
  if (k >= a.n) return;
  const unsigned long long *__restrict__ src = static_cast<const unsigned long long *>(a.src[k]);
  unsigned long long *__restrict__ dst = static_cast<unsigned long long *>(a.dst[k]);
  const uint64_t n8 = a.bytes[k] / 8;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

bool launch_copy8(hipStream_t s, const CopyArgs &a) {
  if (!a.n) return true;
  uint64_t mx = 0;
  for (uint32_t k = 0; k < a.n; ++k) {
    if ((a.bytes[k] | (uintptr_t)a.src[k] | (uintptr_t)a.dst[k]) & 7) return false;
    mx = std::max<uint64_t>(mx, a.bytes[k]);
  }
  const uint32_t gx = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((mx / 8 + 255) / 256, 1024));
  hipLaunchKernelGGL(k_copy8, dim3(gx, a.n), dim3(256), 0, s, a);
  return true;
}

void launch_fill(hipStream_t s, const FillArgs &a) {
  if (!a.n) return;
  uint64_t mx = 0;
  for (uint32_t k = 0; k < a.n; ++k) mx = std::max<uint64_t>(mx, a.bytes[k]);
  const uint32_t gx = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((mx / 16 + 255) / 256, 2048));
  hipLaunchKernelGGL(k_fill, dim3(gx, a.n), dim3(256), 0, s, a);
}

uint32_t used_chunks(uint32_t G) { return (G + FZ_CH - 1) / FZ_CH; }

void launch_finalize(hipStream_t s, unsigned long long *grp, uint32_t G, kmz_group *out, const GroupsUsed *u) {
  if (!G) return;
  GroupAcc a{grp, grp + G, grp + 2ull * G, grp + 3ull * G, grp + 4ull * G, grp + 5ull * G};
  if (u && used_chunks(G) <= USED_MAX_CHUNKS) {
    const uint32_t nb = used_chunks(G);
    hipLaunchKernelGGL(k_finalize, dim3(nb), dim3(FZ_T), 0, s, a, G, out, u->bcnt);
    hipLaunchKernelGGL(k_used_scatter, dim3(nb), dim3(FZ_T), 0, s, out, G, u->bcnt, u->ids, u->groups, u->total);
  } else {
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(G, 1024)), dim3(FZ_T), 0, s, a, G, out, (uint32_t *)nullptr);
  }
}

void launch_collapse_groups(hipStream_t s, const unsigned long long *sg, uint32_t n_shapes, uint32_t S,
                            const uint32_t *map, uint32_t n_ep, unsigned long long *grp, unsigned int *counters) {
  const uint64_t Gs = (uint64_t)n_shapes * S;
  if (!Gs) return;
  hipLaunchKernelGGL(k_collapse_groups, dim3(grid_for(Gs, 2048)), dim3(256), 0, s, sg, n_shapes, S, map, n_ep, grp,
                     counters);
}

void launch_collapse_endpoints(hipStream_t s, const unsigned long long *sg, uint32_t n_shapes, uint32_t S,
                               const uint32_t *dep_map, uint32_t n_dep, const uint32_t *cparent, uint64_t index_base,
                               unsigned long long *ep_ts, unsigned long long *ep_first, unsigned int *counters) {
  if (!n_shapes) return;
  hipLaunchKernelGGL(k_collapse_endpoints, dim3(grid_for(n_shapes, 2048)), dim3(256), 0, s, sg, n_shapes, S, dep_map,
                     n_dep, cparent, index_base, ep_ts, ep_first, counters);
}

void launch_compact(hipStream_t s, const unsigned long long *trip, uint64_t tcap, unsigned long long *out,
                    unsigned long long *count) {
  // (one CP_CH-slot chunk per workgroup up to 2^13 workgroups: config 5's
  // 2^25-slot set in 512 workgroups was a 256-step dependent loop each, 0.28 ms)
  const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, (tcap + CP_CH - 1) / CP_CH));
  hipLaunchKernelGGL(k_compact, dim3(g), dim3(CP_T), 0, s, trip, tcap, out, count);
}

void launch_synth_count(hipStream_t s, int config, uint64_t seed, uint64_t t0, uint64_t nt, uint64_t *cnt) {
  if (!nt) return;
  if (config == 2)
    hipLaunchKernelGGL(k_synth_count<2>, dim3(grid_for(nt)), dim3(256), 0, s, seed, t0, nt, cnt);
  else if (config == 5)
    hipLaunchKernelGGL(k_synth_count<5>, dim3(grid_for(nt)), dim3(256), 0, s, seed, t0, nt, cnt);
  else
    hipLaunchKernelGGL(k_synth_count<3>, dim3(grid_for(nt)), dim3(256), 0, s, seed, t0, nt, cnt);
}

void launch_synth_fill(hipStream_t s, int config, uint64_t seed, uint64_t t0, uint64_t nt, const uint64_t *off,
                       uint64_t gbase, const uint32_t *dur_table, SynthOut out) {
  if (!nt) return;
  if (config == 2)
    hipLaunchKernelGGL(k_synth_fill<2>, dim3(grid_for(nt)), dim3(256), 0, s, seed, t0, nt, off, gbase, dur_table, out);
  else if (config == 5)
    hipLaunchKernelGGL(k_synth_fill<5>, dim3(grid_for(nt)), dim3(256), 0, s, seed, t0, nt, off, gbase, dur_table, out);
  else
    hipLaunchKernelGGL(k_synth_fill<3>, dim3(grid_for(nt)), dim3(256), 0, s, seed, t0, nt, off, gbase, dur_table, out);
}

}  // namespace kmz
