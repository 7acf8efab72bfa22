// kmz_part.hip -- partitioned (atomic-free) K3 for large key spaces (the
// 20k-endpoint mesh and up).
//
// K3P  (endpoint x status) reduction when G > 1024 groups:
//   produce: each 2048-span tile bins its SERVER records by group partition
//            (1024 groups each) in LDS and writes them contiguously into its
//            own tile region + a dense [partition][tile] directory word;
//   reduce:  slice workgroups of one partition accumulate the records in LDS
//            (direct-indexed, 48 B per group) and write dense slice partials;
//   combine: sum / max / min over slices -> the 6 x G u64 group partials.
//   No global atomics, bit-deterministic.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include "kmz_kernels.h"

namespace kmz {

// ---------------------------------------------------------------------------
// block-wide exclusive scan of cnt[0..P) into off[0..P) (P <= 2 * blockDim)
// ---------------------------------------------------------------------------
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan_pairs(const uint32_t *cnt, uint32_t *off, uint32_t P,
                                                          uint32_t *wave_tot) {
  const uint32_t t = threadIdx.x;
  uint32_t a = 2 * t < P ? cnt[2 * t] : 0;
  uint32_t b = 2 * t + 1 < P ? cnt[2 * t + 1] : 0;
  uint32_t s = a + b;
  uint32_t lane = t & 63, wv = t >> 6;
  uint32_t x = s;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wave_tot[wv] = x;
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < THREADS / 64; ++w) {
      uint32_t v = wave_tot[w];
      wave_tot[w] = acc;
      acc += v;
    }
    wave_tot[THREADS / 64] = acc;
  }
  __syncthreads();
  uint32_t excl = wave_tot[wv] + x - s;
  const uint32_t total = wave_tot[THREADS / 64];
  if (2 * t < P) off[2 * t] = excl;
  if (2 * t + 1 < P) off[2 * t + 1] = excl + a;
  __syncthreads();  // off[] is read by other threads (and wave_tot is reused) after the return
  return total;
}

// ===========================================================================
// K3P
// ===========================================================================
// one SERVER span's record: 8 bytes
//   bits  0-9   group within its partition (K3R = 1024 groups per partition)
//   bits 10-16  the span's 16-span block within the tile (index / 16)
//   bits 17-36  duration (us, < 2^20)
//   bits 37-63  timestamp - the tile's least SERVER timestamp (us, < 2^27: 134 s)
// (16-byte records {timestamp, duration, group | index} until round 3: the
// record round trip was half of K3's HBM traffic.)  The reduce keeps a group's
// first block; k3_first_fix then finds the group's first span inside that
// block (16 spans read per group), so the first index stays exact without
// the 11 index bits, which would have cost the group bits (256-group
// partitions made the runs per (tile, partition) four times shorter, the
// directory four times larger and the reduce slower than with 16-byte
// records) or the timestamp's range (the synthetic meshes spread a tile's
// traces over 30 s).  (A first index kept by produce with a device atomicMin
// behind a plain read cost 0.2 ms at 10^8 spans: the read sees its XCD's
// stale L2 copy, so nearly every span took the atomic.)  A span whose
// duration or time offset does not fit is an escape: produce lists its index,
// k3_escape adds it into a block of escape partials with device atomics, and
// k3_escape_fold folds that block into the group partials.  Escapes are rare
// (requests of a second or more; a tile spread over more than two minutes).
#ifndef KMZ_K3T
#define KMZ_K3T 2048
#endif
constexpr uint32_t K3T = KMZ_K3T;  // spans per tile
constexpr uint32_t K3R = 1024;    // groups per partition
constexpr uint32_t K3PMAX = 256;  // partitions (G <= 2^18)
constexpr int K3PT = K3T / 4;     // producer threads (four spans each)
constexpr uint32_t K3_GB = 10, K3_CB = 7, K3_DB = 20, K3_TB = 27;
constexpr uint32_t K3BS = K3T >> K3_CB;  // spans per block (16)
constexpr uint32_t K3F = 6;  // partial fields: count, sum d, sum d^2 (two limbs), max timestamp, first block
static_assert(K3R == (1u << K3_GB) && K3_GB + K3_CB + K3_DB + K3_TB == 64 && K3BS * (1u << K3_CB) == K3T,
              "record fields");
static_assert(K3PT <= 1024, "producer threads");
__device__ __forceinline__ uint64_t k3_rec(uint32_t gl, uint32_t li, uint32_t d, uint64_t toff) {
  return (uint64_t)gl | ((uint64_t)(li / K3BS) << K3_GB) | ((uint64_t)d << (K3_GB + K3_CB)) | (toff << (64 - K3_TB));
}
__device__ __forceinline__ uint32_t k3_rec_g(uint64_t x) { return (uint32_t)x & (K3R - 1); }
__device__ __forceinline__ uint32_t k3_rec_blk(uint64_t x) { return (uint32_t)(x >> K3_GB) & ((1u << K3_CB) - 1); }
__device__ __forceinline__ uint32_t k3_rec_d(uint64_t x) {
  return (uint32_t)(x >> (K3_GB + K3_CB)) & ((1u << K3_DB) - 1);
}
__device__ __forceinline__ uint64_t k3_rec_toff(uint64_t x) { return x >> (64 - K3_TB); }
constexpr uint32_t K3_BPT = 1u << K3_CB;  // blocks per tile

__global__ void __launch_bounds__(K3PT) k3_produce(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                   const uint16_t *__restrict__ status, const uint32_t *__restrict__ dur,
                                                   const int64_t *__restrict__ ts, uint32_t n,
                                                   const uint32_t *__restrict__ ep_of_shape, uint32_t n_shapes,
                                                   uint32_t n_ep, uint32_t n_status, uint32_t P, uint32_t ntiles,
                                                   uint32_t S, uint32_t tps, uint64_t *__restrict__ pool,
                                                   uint32_t *__restrict__ dir, uint64_t *__restrict__ tbase,
                                                   uint32_t *__restrict__ esc, unsigned int *__restrict__ counters,
                                                   uint32_t *__restrict__ tile_servers) {
  __shared__ uint32_t cnt[K3PMAX], off[K3PMAX];
  __shared__ uint32_t wave_tot[K3PT / 64 + 1];
  __shared__ unsigned long long wmin[K3PT / 64];
  __shared__ uint64_t stage[K3T];
  const uint32_t tile = blockIdx.x, t0 = tile * K3T;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int PER = K3T / K3PT;
  // every column of the tile in flight at once (clamped, unconditional loads)
  uint8_t kd[PER];
  uint32_t sh[PER], du[PER];
  uint16_t st[PER];
  int64_t tv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = min(t0 + k * K3PT + threadIdx.x, n - 1);
    kd[k] = kind[i];
    sh[k] = shape[i];
    st[k] = status[i];
    du[k] = dur[i];
    tv[k] = ts[i];
  }
  for (uint32_t p = threadIdx.x; p < P; p += K3PT) cnt[p] = 0;
  // the tile's least SERVER timestamp (order-preserving unsigned form): the
  // records' time base
  unsigned long long mn = ~0ull;
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (t0 + k * K3PT + threadIdx.x < n && kd[k] == KIND_SERVER) mn = min(mn, (unsigned long long)((uint64_t)tv[k] ^ TS_BIAS));
  for (int o = 32; o > 0; o >>= 1) mn = min(mn, (unsigned long long)__shfl_xor(mn, o, 64));
  if (lane == 0) wmin[w] = mn;
  __syncthreads();
  uint64_t base = ~0ull;
  for (int k = 0; k < K3PT / 64; ++k) base = min(base, (uint64_t)wmin[k]);
  uint32_t pp[PER], rr[PER];
  uint64_t rec[PER];
  uint32_t servers = 0, flags = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t li = k * K3PT + threadIdx.x;
    pp[k] = NONE;
    bool escape = false;
    if (t0 + li < n && kd[k] == KIND_SERVER) {
      ++servers;
      const uint32_t ep = sh[k] < n_shapes ? (ep_of_shape ? ep_of_shape[sh[k]] : sh[k]) : NONE;  // null map: by shape
      if (ep >= n_ep || st[k] >= n_status) {
        flags |= F_RANGE;
      } else {
        const uint32_t g = ep * n_status + st[k];
        const uint64_t toff = ((uint64_t)tv[k] ^ TS_BIAS) - base;
        if (du[k] < (1u << K3_DB) && toff < (1ull << K3_TB)) {
          pp[k] = g / K3R;
          rec[k] = k3_rec(g % K3R, li, du[k], toff);
          rr[k] = atomicAdd(&cnt[pp[k]], 1u);
        } else {
          escape = true;
        }
      }
    }
    // escapes: one list reservation per wave
    const uint64_t em = __ballot(escape);
    if (em) {
      uint32_t eb = 0;
      if (lane == 0) eb = atomicAdd(&counters[C_K3ESC], (uint32_t)__popcll(em));
      eb = __shfl(eb, 0, 64);
      if (escape) esc[eb + __popcll(em & ((1ull << lane) - 1))] = t0 + li;
    }
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  __syncthreads();
  uint32_t total = block_excl_scan_pairs<K3PT>(cnt, off, P, wave_tot);
  // directory: [partition][slice][tile within the slice], so a reduce
  // workgroup's words are contiguous (slice s holds tiles s, s + S, ...)
  for (uint32_t p = threadIdx.x; p < P; p += K3PT)
    dir[((uint64_t)p * S + tile % S) * tps + tile / S] = (off[p] << 16) | cnt[p];
  if (threadIdx.x == 0) tbase[tile] = base;
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (pp[k] != NONE) stage[off[pp[k]] + rr[k]] = rec[k];
  __syncthreads();
  // coalesced copy of the partition-sorted tile into its region (16 bytes a lane)
  const uint4 *src = reinterpret_cast<const uint4 *>(stage);
  uint4 *dst = reinterpret_cast<uint4 *>(pool + (uint64_t)tile * K3T);
  for (uint32_t x = threadIdx.x; 2 * x < total; x += K3PT) dst[x] = src[x];
  // realtime-row count: per tile, summed later (no same-address atomics)
  for (int o = 32; o > 0; o >>= 1) servers += __shfl_xor(servers, o, 64);
  if (lane == 0) wave_tot[w] = servers;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < K3PT / 64; ++k) t += wave_tot[k];
    tile_servers[tile] = t;
  }
}

// the escapes (spans without a record) into the escape block E [6][G]:
// device atomics, one span at a time (rare)
__global__ void __launch_bounds__(256) k3_escape(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                 const uint16_t *__restrict__ status, const uint32_t *__restrict__ dur,
                                                 const int64_t *__restrict__ ts, const uint32_t *__restrict__ ep_of_shape,
                                                 uint32_t n_shapes, uint32_t n_status, uint64_t index_base,
                                                 const uint32_t *__restrict__ esc, const unsigned int *__restrict__ counters,
                                                 unsigned long long *__restrict__ E, uint32_t G) {
  const uint32_t m = counters[C_K3ESC];
  for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < m; x += gridDim.x * 256) {
    const uint32_t i = esc[x];
    const uint32_t sh = shape[i];
    const uint32_t ep = ep_of_shape ? ep_of_shape[sh] : sh;  // (checked by produce: a listed span is in range)
    const uint32_t g = ep * n_status + status[i];
    const uint64_t d = dur[i], dd = d * d;
    atomicAdd(&E[g], 1ull);
    atomicAdd(&E[G + g], (unsigned long long)d);
    atomicAdd(&E[2ull * G + g], (unsigned long long)(dd & 0xFFFFFFFFull));
    atomicAdd(&E[3ull * G + g], (unsigned long long)(dd >> 32));
    atomicMax(&E[4ull * G + g], (unsigned long long)((uint64_t)ts[i] ^ TS_BIAS));
    atomicMin(&E[5ull * G + g], (unsigned long long)(index_base + i));
    (void)kind;
    (void)n_shapes;
  }
}

// E into the group partials, one thread per group, canonical limbs kept
__global__ void __launch_bounds__(256) k3_escape_fold(const unsigned int *__restrict__ counters,
                                                      const unsigned long long *__restrict__ E, uint32_t G,
                                                      unsigned long long *__restrict__ grp) {
  if (counters[C_K3ESC] == 0) return;
  for (uint32_t g = blockIdx.x * 256 + threadIdx.x; g < G; g += gridDim.x * 256) {
    if (E[g] == 0) continue;
    grp[g] += E[g];
    grp[G + g] += E[G + g];
    const unsigned long long s2a = grp[2ull * G + g] + E[2ull * G + g], s2b = grp[3ull * G + g] + E[3ull * G + g];
    grp[2ull * G + g] = s2a & 0xFFFFFFFFull;
    grp[3ull * G + g] = s2b + (s2a >> 32);
    grp[4ull * G + g] = max(grp[4ull * G + g], E[4ull * G + g]);
    grp[5ull * G + g] = min(grp[5ull * G + g], E[5ull * G + g]);
  }
}

// sum / max of per-tile counters: a few workgroups, one atomic per workgroup
// and field (replaces per-tile same-address atomics)
__global__ void __launch_bounds__(1024) k_tile_sum(const uint32_t *__restrict__ v, uint32_t ntiles, uint32_t stride,
                                                   uint32_t fields, unsigned long long *__restrict__ out,
                                                   uint32_t max_field) {
  __shared__ unsigned long long red[16][4];
  unsigned long long acc[4] = {0, 0, 0, 0};
  for (uint32_t t = blockIdx.x * 1024 + threadIdx.x; t < ntiles; t += gridDim.x * 1024)
    for (uint32_t f = 0; f < fields; ++f) {
      uint64_t x = v[(uint64_t)t * stride + f];
      acc[f] = (f == max_field) ? max(acc[f], (unsigned long long)x) : acc[f] + x;
    }
  for (uint32_t f = 0; f < fields; ++f)
    for (int o = 32; o > 0; o >>= 1) {
      unsigned long long y = __shfl_xor(acc[f], o, 64);
      acc[f] = (f == max_field) ? max(acc[f], y) : acc[f] + y;
    }
  if ((threadIdx.x & 63) == 0)
    for (uint32_t f = 0; f < fields; ++f) red[threadIdx.x >> 6][f] = acc[f];
  __syncthreads();
  if (threadIdx.x < fields) {
    unsigned long long r = 0;
    for (int w = 0; w < 16; ++w) r = (threadIdx.x == max_field) ? max(r, red[w][threadIdx.x]) : r + red[w][threadIdx.x];
    if (threadIdx.x == max_field)
      atomicMax(&out[threadIdx.x], r);
    else if (r)
      atomicAdd(&out[threadIdx.x], r);
  }
}

static inline uint32_t tile_sum_blocks(uint32_t ntiles) { return std::min<uint32_t>(64, (ntiles + 1023) / 1024 + 0); }

// slice s of partition p: tiles s, s+S, ...  -> part[(s*K3F + f) * G + g].
// Each wave takes 64 of the slice's tiles at a time (one directory word and
// time base per lane), scans their run lengths across the lanes, and spreads
// the concatenation of the runs over its lanes (coalesced 8-byte reads, four
// per lane in flight); a record finds its run by a binary search over the
// wave's 64 run starts in LDS.
//
// PACK (a slice holds < 2^22 records: ceil(ntiles / S) * K3T < 2^22): four
// LDS atomics per record instead of six --
//   a_cs  += 2^42 + d       count in bits 42..63, sum of durations < 2^20 in
//                           bits 0..41 (< 2^22 of them: no carry)
//   a_s2  += d^2            (d < 2^20: d^2 < 2^40, the sum < 2^62)
//   a_tsx  max, a_fst min   the first block as a u32 within the slice / item
// (every record's duration is < 2^20: wider ones are escapes).  Written out in
// the unpacked partial format (s2 split into lo32 / hi32 limbs, the first
// block global); k3_first_fix turns blocks into span indices.
#ifndef KMZ_K3RT
#define KMZ_K3RT 512  // (256 -> 512: the balanced reduce 0.23 -> 0.20 ms on the mesh, profiles/r05/ab)
#endif
constexpr int K3RT = KMZ_K3RT;  // balanced-reduce threads per workgroup
constexpr uint32_t K3RB = 64;  // runs per wave batch (one per lane)
#ifndef KMZ_K3_U
#define KMZ_K3_U 4  // records per lane in flight in k3_reduce_bal's record loop
#endif
#ifndef KMZ_K3_SEARCH
#define KMZ_K3_SEARCH 0  // 1: round 4's binary search for a record's run (A/B)
#endif
#ifndef KMZ_K3_COND
#define KMZ_K3_COND 1  // max / min atomics only when a plain read says they move
#endif
// one record into the LDS accumulators: fb is its block within the slice /
// item (PACK) or its global block
template <bool PACK>
__device__ __forceinline__ void k3_accumulate(uint64_t x, uint64_t tsx, uint64_t fb, unsigned long long *a0,
                                              unsigned long long *a1, unsigned long long *a2, unsigned long long *a3,
                                              unsigned long long *a_tsx, unsigned long long *a_fst,
                                              uint32_t *a_fst32) {
  const uint32_t kl = k3_rec_g(x);
  const uint64_t d = k3_rec_d(x), dd = d * d;
  if (PACK) {
    atomicAdd(&a0[kl], (1ull << 42) + d);
    atomicAdd(&a1[kl], (unsigned long long)dd);
  } else {
    atomicAdd(&a0[kl], 1ull);
    atomicAdd(&a1[kl], (unsigned long long)d);
    atomicAdd(&a2[kl], (unsigned long long)(dd & 0xFFFFFFFFull));
    atomicAdd(&a3[kl], (unsigned long long)(dd >> 32));
  }
#if KMZ_K3_COND
  // max and min only move one way: a plain LDS read that already dominates
  // this record makes its atomic a no-op, so it is skipped (a stale read can
  // only cost an unneeded atomic)
  if (tsx > a_tsx[kl]) atomicMax(&a_tsx[kl], (unsigned long long)tsx);
  if (PACK) {
    if ((uint32_t)fb < a_fst32[kl]) atomicMin(&a_fst32[kl], (uint32_t)fb);
  } else {
    if (fb < a_fst[kl]) atomicMin(&a_fst[kl], (unsigned long long)fb);
  }
#else
  atomicMax(&a_tsx[kl], (unsigned long long)tsx);
  if (PACK)
    atomicMin(&a_fst32[kl], (uint32_t)fb);
  else
    atomicMin(&a_fst[kl], (unsigned long long)fb);
#endif
}

// one accumulator block out: packed or unpacked LDS sums -> the K3F partial
// fields at b[f * stride] (the first block: `fst`, already global)
template <bool PACK>
__device__ __forceinline__ void k3_write_partial(const unsigned long long *acc, uint32_t k, unsigned long long fst,
                                                 unsigned long long *__restrict__ b, uint64_t stride) {
  if (PACK) {
    const unsigned long long cs = acc[k], s2 = acc[K3R + k];
    b[0] = cs >> 42;
    b[stride] = cs & ((1ull << 42) - 1);
    b[2 * stride] = s2 & 0xFFFFFFFFull;
    b[3 * stride] = s2 >> 32;
  } else {
    b[0] = acc[k];
    b[stride] = acc[K3R + k];
    b[2 * stride] = acc[2 * K3R + k] & 0xFFFFFFFFull;  // (canonical limbs)
    b[3 * stride] = acc[3 * K3R + k] + (acc[2 * K3R + k] >> 32);
  }
  b[4 * stride] = acc[4 * K3R + k];
  b[5 * stride] = fst;
}

template <bool PACK>
__global__ void __launch_bounds__(K3RT) k3_reduce(const uint64_t *__restrict__ pool, const uint32_t *__restrict__ dir,
                                                  const uint64_t *__restrict__ tbase, uint32_t ntiles, uint32_t S,
                                                  uint32_t G, unsigned long long *__restrict__ part) {
  __shared__ unsigned long long acc[K3F * K3R];
  constexpr uint32_t NW = K3RT / 64;
  __shared__ uint32_t r_pre[NW][K3RB], r_off[NW][K3RB];  // per wave: run starts in the batch, pool offsets
  __shared__ uint64_t r_tb[NW][K3RB];                    // ... and the runs' time bases
  unsigned long long *a0 = acc, *a1 = acc + K3R, *a2 = acc + 2 * K3R, *a3 = acc + 3 * K3R, *a_tsx = acc + 4 * K3R,
                     *a_fst = acc + 5 * K3R;
  uint32_t *a_fst32 = reinterpret_cast<uint32_t *>(a_fst);
  const uint32_t s = blockIdx.x, p = blockIdx.y;
  for (uint32_t k = threadIdx.x; k < K3F * K3R; k += K3RT) acc[k] = k < 5 * K3R ? 0ull : ~0ull;
  __syncthreads();
  const uint32_t tps = (ntiles + S - 1) / S;
  const uint32_t *row = dir + ((uint64_t)p * S + s) * tps;  // this slice's tiles, in order
  constexpr uint32_t U = 4;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t step = (uint64_t)S * NW;  // consecutive tiles of this wave
  for (uint64_t k0 = (uint64_t)s + (uint64_t)w * S; k0 < ntiles; k0 += step * K3RB) {
    // this lane's run: tile k0 + lane * step
    const uint64_t k = k0 + lane * step;
    const uint32_t x = k < ntiles ? row[(k - s) / S] : 0;
    const uint32_t o = x >> 16;
    const uint32_t c = (o + (x & 0xFFFF) <= K3T) ? (x & 0xFFFF) : 0;  // a well-formed directory never exceeds the tile
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    r_pre[w][lane] = incl - c;
    r_off[w][lane] = (uint32_t)(k < ntiles ? k : 0) * K3T + o;  // (ntiles * K3T < 2^32: n < 2^32)
    r_tb[w][lane] = c ? tbase[k] : 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    for (uint32_t q0 = 0; q0 < total; q0 += 64 * U) {
      uint64_t xr[U];
      uint32_t run[U];
      bool v[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t q = q0 + u * 64 + lane;
        v[u] = q < total;
        uint32_t j = 0;  // the last run starting at or before q
#pragma unroll
        for (uint32_t b = 32; b; b >>= 1)
          if (r_pre[w][j + b] <= q) j += b;
        run[u] = j;
        xr[u] = pool[v[u] ? r_off[w][j] + (q - r_pre[w][j]) : 0];
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (!v[u]) continue;
        // this slice's tiles are s, s + S, ...: (k - s) / S numbers them
        const uint64_t fb = PACK ? (uint64_t)(((uint32_t)((k0 - s) / S) + run[u] * (uint32_t)(step / S)) * K3_BPT +
                                              k3_rec_blk(xr[u]))
                                 : (k0 + run[u] * step) * K3_BPT + k3_rec_blk(xr[u]);
        k3_accumulate<PACK>(xr[u], r_tb[w][run[u]] + k3_rec_toff(xr[u]), fb, a0, a1, a2, a3, a_tsx, a_fst, a_fst32);
      }
    }
    __builtin_amdgcn_wave_barrier();  // r_pre / r_off / r_tb are rewritten by the next batch
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < K3R; k += K3RT) {
    uint64_t g = (uint64_t)p * K3R + k;
    if (g >= G) break;
    unsigned long long *b = part + (uint64_t)s * K3F * G + g;
    const uint32_t f = a_fst32[k];
    const unsigned long long fst =
        PACK ? (f == ~0u ? ~0ull : ((uint64_t)s + (uint64_t)(f / K3_BPT) * S) * K3_BPT + f % K3_BPT) : a_fst[k];
    k3_write_partial<PACK>(acc, k, fst, b, G);
  }
}

// ---------------------------------------------------------------------------
// Balanced K3 reduce.  Partitions are far from equal: config 5's hot
// endpoints put 6.2x the mean record count into one partition (the mesh: 1.8x),
// so with a fixed number of slices per partition the hot partitions' slices
// set the kernel's length.  Here the directory is [partition][tile]; k3_psum
// counts each partition's records, k3_plan gives partition p
// S_p = ceil(T_p / target) work items (about K3_ITEMS in all, each a
// contiguous tile range of its partition: records are spread evenly over the
// tiles), and k3_reduce_bal runs one workgroup per item.  k3_combine_bal folds
// the items of each partition.
// ---------------------------------------------------------------------------
constexpr uint32_t K3_ITEMS = 1536;       // an upper bound: 2 rounds of 3 workgroups per CU on 256 CUs
constexpr uint32_t K3_ITEM_MIN = 4096;    // records: below that an item is not worth its partial write-out

// per-partition record counts from the [partition][tile] directory, each row
// summed by K3_PSUM_SPLIT workgroups into partial sums (one workgroup per
// partition reading its whole ~10^5-word row took ~0.08 ms at 10^8 spans)
constexpr uint32_t K3_PSUM_SPLIT = 16;
__global__ void __launch_bounds__(256) k3_psum(const uint32_t *__restrict__ dir, uint32_t ntiles,
                                               uint32_t *__restrict__ tot) {
  __shared__ uint32_t red[4];
  const uint32_t *row = dir + (uint64_t)blockIdx.x * ntiles;
  const uint32_t per = (ntiles + K3_PSUM_SPLIT - 1) / K3_PSUM_SPLIT;
  const uint32_t k0 = blockIdx.y * per, k1 = min(ntiles, k0 + per);
  uint32_t s = 0;
  for (uint32_t kb = k0; kb < k1; kb += 8 * 256) {  // eight loads in flight per thread
    uint32_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t k = kb + u * 256 + threadIdx.x;
      x[u] = k < k1 ? row[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t o = x[u] >> 16, c = x[u] & 0xFFFF;
      s += (o + c <= K3T) ? c : 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tot[(uint64_t)blockIdx.x * K3_PSUM_SPLIT + blockIdx.y] = red[0] + red[1] + red[2] + red[3];
}

// one workgroup: S_p and the exclusive scan item_off[0..P] (P <= K3PMAX)
__global__ void __launch_bounds__(1024) k3_plan(const uint32_t *__restrict__ tot, uint32_t P, uint32_t ntiles,
                                                uint32_t nitems, uint32_t *__restrict__ item_off) {
  __shared__ unsigned long long rsum[16];
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t c = 0;
  if (t < P)
    for (uint32_t j = 0; j < K3_PSUM_SPLIT; ++j) c += tot[(uint64_t)t * K3_PSUM_SPLIT + j];
  unsigned long long r = c;
  for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
  if (lane == 0) rsum[w] = r;
  __syncthreads();
  unsigned long long R = 0;
  for (int k = 0; k < 16; ++k) R += rsum[k];
  const unsigned long long target = max((R + nitems - 1) / nitems, (unsigned long long)K3_ITEM_MIN);
  const uint32_t sp = t < P ? (uint32_t)min((c + target - 1) / target, (unsigned long long)ntiles) : 0;
  const uint32_t s1 = t < P ? max(sp, 1u) : 0;
  uint32_t x = s1;  // inclusive scan over the workgroup
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t k = 0; k < w; ++k) before += wsum[k];
  if (t < P) item_off[t] = before + x - s1;
  if (t == P - 1) item_off[P] = before + x;
}

// item -> (partition, tile range); partials [item][K3F][K3R].  The packed
// accumulators of k3_reduce are used when the item holds < 2^22 records
// (counted first from its directory words: records need not be spread evenly,
// e.g. input sorted by endpoint), else the unpacked ones.  The record loop is
// instantiated for each accumulator form and chosen once per workgroup (as the
// fixed-slice k3_reduce<PACK> is compiled), not per record.
template <bool PACK>
__device__ __forceinline__ void k3_reduce_items(const uint64_t *__restrict__ pool, const uint32_t *__restrict__ row,
                                                const uint64_t *__restrict__ tbase, uint64_t tb, uint64_t te,
                                                unsigned long long *acc, uint32_t (*r_pre)[K3RB],
                                                uint32_t (*r_off)[K3RB], uint64_t (*r_tb)[K3RB],
                                                uint8_t (*r_tile)[K3RB], unsigned long long *r_mask) {
  constexpr uint32_t NW = K3RT / 64;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long *a0 = acc, *a1 = acc + K3R, *a2 = acc + 2 * K3R, *a3 = acc + 3 * K3R, *a_tsx = acc + 4 * K3R,
                     *a_fst = acc + 5 * K3R;
  uint32_t *a_fst32 = reinterpret_cast<uint32_t *>(a_fst);
  constexpr uint32_t U = KMZ_K3_U;
  // each batch's directory words are loaded during the batch before it.
  // (Every load here is unconditional, its index clamped into the item, and
  // masked after: a load under a branch made the compiler wait for it at the
  // merge -- the next batch's words right after their issue, the time base
  // before the records -- three round trips per batch instead of one.)
  if (te <= tb) return;  // (an empty item: nothing loaded)
  const uint64_t tl = te - 1;  // the item's last tile
  const uint64_t k00 = tb + (uint64_t)w * K3RB + lane;
  uint32_t xn = row[k00 < te ? k00 : tl];
  xn = k00 < te ? xn : 0;
  for (uint64_t k0 = tb + (uint64_t)w * K3RB; k0 < te; k0 += (uint64_t)NW * K3RB) {
    const uint64_t k = k0 + lane;  // this lane's run: tile k
    const uint32_t x = xn;
    // (the time base first: its wait, counted in order, then leaves the next
    // batch's directory word in flight)
    const uint64_t tbk = tbase[k < te ? k : tl];
    const uint64_t kn = k + (uint64_t)NW * K3RB;
    xn = row[kn < te ? kn : tl];
    xn = kn < te ? xn : 0;
    const uint32_t o = x >> 16;
    const uint32_t c = (o + (x & 0xFFFF) <= K3T) ? (x & 0xFFFF) : 0;
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    // the non-empty runs, compacted (so that no two share a start): run i's
    // start, pool offset, time base and tile
    const uint64_t ne = __ballot(c != 0);
    const uint32_t ci = __popcll(ne & ((1ull << lane) - 1)), pre = incl - c;
    if (c) {
      r_pre[w][ci] = pre;
      r_off[w][ci] = (uint32_t)k * K3T + o;
      r_tb[w][ci] = tbk;
      r_tile[w][ci] = lane;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // a record's run without a search: per 64 records [b, b + 64), the runs
    // starting inside set their bit of a start mask (lane i holds compacted
    // run i's start); run(q) = (runs starting before b) + popcount of the
    // mask's bits <= q - b, minus one
    const uint32_t nr = (uint32_t)__popcll(ne);
    const uint32_t mypre = lane < nr ? r_pre[w][lane] : 0xFFFFFFFFu;
    for (uint32_t q0 = 0; q0 < total; q0 += 64 * U) {
      uint64_t xr[U];
      uint32_t run[U];
      bool v[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t b = q0 + u * 64, q = b + lane;
        v[u] = q < total;
#if KMZ_K3_SEARCH  // (round 4: a binary search over the run starts, six dependent LDS reads)
        uint32_t jj = 0;
#pragma unroll
        for (uint32_t bb = 32; bb; bb >>= 1)
          if (jj + bb < nr && r_pre[w][jj + bb] <= q) jj += bb;
#else
        const uint32_t sft = mypre - b;  // (wraps for runs starting before b)
        // the wave's start mask in LDS: cleared by lane 0, one OR per run
        // starting in [b, b + 64), read back by every lane (one wave's LDS
        // operations complete in order)
        if (lane == 0) r_mask[w] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (sft < 64) atomicOr(&r_mask[w], 1ull << sft);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const uint64_t m = r_mask[w];
        const uint32_t before = (uint32_t)__popcll(__ballot(mypre < b));
        uint32_t jj = before + (uint32_t)__popcll(m & (~0ull >> (63 - lane))) - 1;
        jj = v[u] ? jj : 0;  // (a lane past the records: any run, its load is not used)
#endif
        run[u] = jj;
        xr[u] = pool[v[u] ? r_off[w][jj] + (q - r_pre[w][jj]) : 0];
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (!v[u]) continue;
        const uint64_t tile = k0 + r_tile[w][run[u]];
        const uint64_t fb = PACK ? (uint64_t)((uint32_t)(tile - tb) * K3_BPT + k3_rec_blk(xr[u]))
                                 : tile * K3_BPT + k3_rec_blk(xr[u]);
        k3_accumulate<PACK>(xr[u], r_tb[w][run[u]] + k3_rec_toff(xr[u]), fb, a0, a1, a2, a3, a_tsx, a_fst, a_fst32);
      }
    }
    __builtin_amdgcn_wave_barrier();  // r_pre / r_off / r_tb are rewritten by the next batch
  }
}

__global__ void __launch_bounds__(K3RT) k3_reduce_bal(const uint64_t *__restrict__ pool, const uint32_t *__restrict__ dir,
                                                      const uint64_t *__restrict__ tbase, uint32_t ntiles, uint32_t P,
                                                      const uint32_t *__restrict__ item_off, uint32_t G, uint32_t upk,
                                                      unsigned long long *__restrict__ part) {
  __shared__ unsigned long long acc[K3F * K3R];
  constexpr uint32_t NW = K3RT / 64;
  __shared__ uint32_t r_pre[NW][K3RB], r_off[NW][K3RB], wred[NW];
  __shared__ uint64_t r_tb[NW][K3RB];
  __shared__ uint8_t r_tile[NW][K3RB];
  __shared__ unsigned long long r_mask[NW];
  const uint32_t item = blockIdx.x;
  if (item >= item_off[P]) return;  // (the grid is an upper bound; uniform over the workgroup)
  uint32_t lo = 0, hi = P;  // the partition: item_off[p] <= item < item_off[p + 1]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (item_off[mid] <= item) lo = mid; else hi = mid;
  }
  const uint32_t p = lo, j = item - item_off[p], sp = item_off[p + 1] - item_off[p];
  const uint64_t tb = (uint64_t)j * ntiles / sp, te = (uint64_t)(j + 1) * ntiles / sp;
  const uint32_t *row = dir + (uint64_t)p * ntiles;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t nrec = 0;
  for (uint64_t kb = tb; kb < te; kb += 8 * K3RT) {  // eight loads in flight per thread
    uint32_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t k = kb + u * K3RT + threadIdx.x;
      x[u] = k < te ? row[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) nrec += ((x[u] >> 16) + (x[u] & 0xFFFF) <= K3T) ? (x[u] & 0xFFFF) : 0;
  }
  for (int o = 32; o > 0; o >>= 1) nrec += __shfl_xor(nrec, o, 64);
  if (lane == 0) wred[w] = nrec;
  for (uint32_t k = threadIdx.x; k < K3F * K3R; k += K3RT) acc[k] = k < 5 * K3R ? 0ull : ~0ull;
  __syncthreads();
  uint32_t tot = 0;
  for (uint32_t k = 0; k < NW; ++k) tot += wred[k];
  const bool pack = tot < (1u << 22) && !upk;  // (upk: test knob)
  // packed: cs, s2, -, -, tsx, fst32 (u32) -- unpacked: cnt, s1, s2a, s2b, tsx, fst
  if (pack)
    k3_reduce_items<true>(pool, row, tbase, tb, te, acc, r_pre, r_off, r_tb, r_tile, r_mask);
  else
    k3_reduce_items<false>(pool, row, tbase, tb, te, acc, r_pre, r_off, r_tb, r_tile, r_mask);
  __syncthreads();
  unsigned long long *b = part + (uint64_t)item * K3F * K3R;
  for (uint32_t k = threadIdx.x; k < K3R; k += K3RT) {
    if ((uint64_t)p * K3R + k >= G) break;
    if (pack) {
      const uint32_t f = reinterpret_cast<const uint32_t *>(acc + 5 * K3R)[k];
      k3_write_partial<true>(acc, k, f == ~0u ? ~0ull : tb * K3_BPT + f, b + k, K3R);
    } else {
      k3_write_partial<false>(acc, k, acc[5 * K3R + k], b + k, K3R);
    }
  }
}

// the items of each partition folded (the first block: k3_first_fix next)
__global__ void __launch_bounds__(256) k3_combine_bal(const unsigned long long *__restrict__ part,
                                                      const uint32_t *__restrict__ item_off, uint32_t G,
                                                      unsigned long long *__restrict__ grp) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const uint32_t p = g / K3R, k = g % K3R;
    unsigned long long c = 0, s1 = 0, s2a = 0, s2b = 0, tsx = 0, fst = ~0ull;
    // (unrolled: a hot partition has many items, and one item's six loads at
    // a time left the kernel waiting on one round trip per item)
#pragma unroll 4
    for (uint32_t it = item_off[p]; it < item_off[p + 1]; ++it) {
      const unsigned long long *b = part + (uint64_t)it * K3F * K3R + k;
      c += b[0];
      s1 += b[K3R];
      s2a += b[2 * K3R];
      s2b += b[3 * K3R];
      tsx = max(tsx, b[4 * K3R]);
      fst = min(fst, b[5 * K3R]);
    }
    grp[g] = c;
    grp[G + g] = s1;
    grp[2ull * G + g] = s2a & 0xFFFFFFFFull;  // canonical limbs: S2 = s2a + 2^32 s2b with s2a < 2^32,
    grp[3ull * G + g] = s2b + (s2a >> 32);     // whatever split the items' sums had
    grp[4ull * G + g] = tsx;
    grp[5ull * G + g] = fst;
  }
}

__global__ void __launch_bounds__(256) k3_combine(const unsigned long long *__restrict__ part, uint32_t S, uint32_t G,
                                                  unsigned long long *__restrict__ grp) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    unsigned long long c = 0, s1 = 0, s2a = 0, s2b = 0, tsx = 0, fst = ~0ull;
    for (uint32_t s = 0; s < S; ++s) {
      const unsigned long long *b = part + (uint64_t)s * K3F * G + g;
      c += b[0];
      s1 += b[G];
      s2a += b[2ull * G];
      s2b += b[3ull * G];
      tsx = max(tsx, b[4ull * G]);
      fst = min(fst, b[5ull * G]);
    }
    grp[g] = c;
    grp[G + g] = s1;
    grp[2ull * G + g] = s2a & 0xFFFFFFFFull;  // (canonical limbs, as k3_combine_bal)
    grp[3ull * G + g] = s2b + (s2a >> 32);
    grp[4ull * G + g] = tsx;
    grp[5ull * G + g] = fst;
  }
}

// a group's first block -> its first span: the first SERVER span of the
// block in the group (one exists: the block's record came from it; an
// escaped span of the group earlier in the block is found the same way)
__global__ void __launch_bounds__(256) k3_first_fix(const uint8_t *__restrict__ kind,
                                                    const uint32_t *__restrict__ shape,
                                                    const uint16_t *__restrict__ status, uint32_t n,
                                                    const uint32_t *__restrict__ ep_of_shape, uint32_t n_shapes,
                                                    uint32_t n_status, uint64_t index_base, uint32_t G,
                                                    unsigned long long *__restrict__ grp,
                                                    unsigned int *__restrict__ counters) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const unsigned long long blk = grp[5ull * G + g];
    if (blk == ~0ull) continue;
    const uint64_t i0 = blk * K3BS;
    unsigned long long f = ~0ull;
    for (uint32_t j = 0; j < K3BS && i0 + j < n; ++j) {
      const uint64_t i = i0 + j;
      if (kind[i] != KIND_SERVER || shape[i] >= n_shapes) continue;
      const uint32_t ep = ep_of_shape ? ep_of_shape[shape[i]] : shape[i];
      if ((uint64_t)ep * n_status + status[i] == g) {
        f = index_base + i;
        break;
      }
    }
    if (f == ~0ull) atomicOr(&counters[C_FLAGS], F_RANGE);  // (cannot happen for a well-formed run)
    grp[5ull * G + g] = f;
  }
}

// ===========================================================================
// K3S: (endpoint x status) reduction for small key spaces (G <= 1024, e.g.
// Bookinfo's 18 groups): every workgroup reduces one contiguous chunk in LDS
// (one copy of the accumulators per wave while G <= 256, so lanes only
// contend within their wave) and writes its partials; no global atomics, no
// shared counter (a per-wave atomic on one n_server word serialises ~4k
// waves).  k3_combine_small folds the chunks: one workgroup per group.
// ===========================================================================
constexpr int KS_T = 256;
__global__ void __launch_bounds__(KS_T) k3_small(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                 const uint16_t *__restrict__ status, const uint32_t *__restrict__ dur,
                                                 const int64_t *__restrict__ ts, uint32_t n, uint32_t chunk,
                                                 const uint32_t *__restrict__ ep_of_shape, uint32_t n_shapes,
                                                 uint32_t n_ep, uint32_t n_status, uint64_t index_base,
                                                 uint32_t copies, unsigned int *__restrict__ counters,
                                                 unsigned long long *__restrict__ part,
                                                 uint32_t *__restrict__ wg_servers) {
  extern __shared__ unsigned long long sm[];
  __shared__ uint32_t wsrv[KS_T / 64];
  const uint32_t G = n_ep * n_status;
  for (uint32_t k = threadIdx.x; k < copies * 6 * G; k += KS_T) sm[k] = (k / G) % 6 == 5 ? ~0ull : 0ull;
  __syncthreads();
  unsigned long long *a = sm + (copies > 1 ? (threadIdx.x >> 6) : 0) * 6 * G;
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
  const uint32_t end = (uint32_t)min<uint64_t>(c0 + chunk, n);
  uint32_t servers = 0, flags = 0;
  for (uint32_t i = (uint32_t)c0 + threadIdx.x; i < end; i += KS_T) {
    if (kind[i] != KIND_SERVER) continue;
    ++servers;
    const uint32_t sh = shape[i], st = status[i];
    const uint32_t ep = sh < n_shapes ? (ep_of_shape ? ep_of_shape[sh] : sh) : NONE;  // null map: by shape
    if (ep >= n_ep || st >= n_status) {
      flags |= F_RANGE;
      continue;
    }
    const uint32_t g = ep * n_status + st;
    const uint64_t d = dur[i], dd = d * d;
    atomicAdd(&a[g], 1ull);
    atomicAdd(&a[G + g], (unsigned long long)d);
    atomicAdd(&a[2 * G + g], (unsigned long long)(dd & 0xFFFFFFFFull));
    atomicAdd(&a[3 * G + g], (unsigned long long)(dd >> 32));
    atomicMax(&a[4 * G + g], (unsigned long long)((uint64_t)ts[i] ^ TS_BIAS));
    atomicMin(&a[5 * G + g], (unsigned long long)(index_base + i));
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) servers += __shfl_xor(servers, o, 64);
  if ((threadIdx.x & 63) == 0) wsrv[threadIdx.x >> 6] = servers;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < KS_T / 64; ++w) t += wsrv[w];
    wg_servers[blockIdx.x] = t;
  }
  for (uint32_t k = threadIdx.x; k < 6 * G; k += KS_T) {
    const uint32_t f = k / G;
    unsigned long long v = sm[k];
    for (uint32_t c = 1; c < copies; ++c) {
      const unsigned long long x = sm[c * 6 * G + k];
      v = f < 4 ? v + x : (f == 4 ? max(v, x) : min(v, x));
    }
    part[(uint64_t)blockIdx.x * 6 * G + k] = v;
  }
}

__global__ void __launch_bounds__(256) k3_combine_small(const unsigned long long *__restrict__ part, uint32_t S,
                                                        uint32_t G, unsigned long long *__restrict__ grp) {
  __shared__ unsigned long long red[4][6];
  const uint32_t g = blockIdx.x;
  unsigned long long v[6] = {0, 0, 0, 0, 0, ~0ull};
  for (uint32_t s = threadIdx.x; s < S; s += 256) {
    const unsigned long long *b = part + (uint64_t)s * 6 * G + g;
#pragma unroll
    for (int f = 0; f < 4; ++f) v[f] += b[(uint64_t)f * G];
    v[4] = max(v[4], b[4ull * G]);
    v[5] = min(v[5], b[5ull * G]);
  }
#pragma unroll
  for (int f = 0; f < 6; ++f)
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long y = __shfl_xor(v[f], o, 64);
      v[f] = f < 4 ? v[f] + y : (f == 4 ? max(v[f], y) : min(v[f], y));
    }
  if ((threadIdx.x & 63) == 0)
    for (int f = 0; f < 6; ++f) red[threadIdx.x >> 6][f] = v[f];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int f = threadIdx.x;
    unsigned long long r = red[0][f];
    for (int w = 1; w < 4; ++w) r = f < 4 ? r + red[w][f] : (f == 4 ? max(r, red[w][f]) : min(r, red[w][f]));
    grp[(uint64_t)f * G + g] = r;
  }
}

uint32_t k3_small_blocks(uint32_t n) { return std::max<uint32_t>(1, std::min<uint32_t>(1024, (n + 1023) / 1024)); }

void launch_k3_small(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                     const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                     uint32_t n_shapes, uint32_t n_ep, uint32_t n_status, uint64_t index_base,
                     unsigned int *counters, unsigned long long *n_server, unsigned long long *part,
                     uint32_t *tile_tmp, unsigned long long *grp) {
  const uint32_t G = n_ep * n_status;
  if (!n || !G) return;
  const uint32_t nb = k3_small_blocks(n), chunk = (n + nb - 1) / nb;
  const uint32_t copies = G <= 256 ? KS_T / 64 : 1;
  hipLaunchKernelGGL(k3_small, dim3(nb), dim3(KS_T), (size_t)copies * 6 * G * 8, s, kind, shape, status, dur, ts, n,
                     chunk, ep_of_shape, n_shapes, n_ep, n_status, index_base, copies, counters, part, tile_tmp);
  hipLaunchKernelGGL(k3_combine_small, dim3(G), dim3(256), 0, s, part, nb, G, grp);
  hipLaunchKernelGGL(k_tile_sum, dim3(std::max<uint32_t>(1, tile_sum_blocks(nb))), dim3(1024), 0, s, tile_tmp, nb, 1u, 1u,
                     n_server, 99u);
}

void launch_k3_produce(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                       const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                       uint32_t n_shapes, uint32_t n_ep, uint32_t n_status, uint32_t S, unsigned int *counters,
                       unsigned long long *n_server, void *pool, uint32_t *dir, uint32_t *tile_tmp) {
  if (!n || !n_ep) return;
  const uint32_t G = n_ep * n_status, P = (G + K3R - 1) / K3R, ntiles = (n + K3T - 1) / K3T;
  uint64_t *rec = static_cast<uint64_t *>(pool);
  hipLaunchKernelGGL(k3_produce, dim3(ntiles), dim3(K3PT), 0, s, kind, shape, status, dur, ts, n, ep_of_shape,
                     n_shapes, n_ep, n_status, P, ntiles, S, (ntiles + S - 1) / S, rec, dir, k3_tbase(pool, n),
                     k3_esc(pool, n), counters, tile_tmp);
  hipLaunchKernelGGL(k_tile_sum, dim3(std::max<uint32_t>(1, tile_sum_blocks(ntiles))), dim3(1024), 0, s, tile_tmp, ntiles, 1u, 1u,
                     n_server, 99u);
}

void launch_k3_reduce(hipStream_t s, uint32_t n, uint32_t G, const void *pool, const uint32_t *dir,
                      unsigned long long *part, uint32_t S, unsigned long long *grp) {
  if (!n || !G) return;
  const uint32_t P = (G + K3R - 1) / K3R, ntiles = (n + K3T - 1) / K3T;
#ifndef KMZ_K3_PACK
#define KMZ_K3_PACK 1
#endif
  // packed accumulators while a slice's records stay below 2^22 (counts and
  // in-slice first indices fit their fields)
  // one slice: its partials are the group partials ([6][G], the same layout)
  unsigned long long *dst = S == 1 ? grp : part;
  const uint64_t *rec = static_cast<const uint64_t *>(pool);
  const uint64_t *tb = k3_tbase(const_cast<void *>(pool), n);
  if (KMZ_K3_PACK && (uint64_t)((ntiles + S - 1) / S) * K3T < (1ull << 22))
    hipLaunchKernelGGL(k3_reduce<true>, dim3(S, P), dim3(K3RT), 0, s, rec, dir, tb, ntiles, S, G, dst);
  else
    hipLaunchKernelGGL(k3_reduce<false>, dim3(S, P), dim3(K3RT), 0, s, rec, dir, tb, ntiles, S, G, dst);
  if (S > 1)
    hipLaunchKernelGGL(k3_combine, dim3((G + 255) / 256 < 2048 ? (G + 255) / 256 : 2048), dim3(256), 0, s, part, S,
                       G, grp);
}

// workgroups of k3_reduce_bal the device keeps resident (CUs x occupancy),
// queried once per device; 768 (256 CUs x 3) if the query fails
static uint32_t k3_resident() {
  static std::mutex mu;
  static uint32_t cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 768;
  std::lock_guard<std::mutex> lk(mu);
  if (!cached[dev]) {
    int cus = 0, occ = 0;
    uint32_t g = 768;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k3_reduce_bal, K3RT, 0) == hipSuccess && occ > 0)
      g = (uint32_t)cus * (uint32_t)occ;
    cached[dev] = g;
  }
  return cached[dev];
}

// balanced: per-partition record counts, the item plan, one workgroup per item
void launch_k3_reduce_bal(hipStream_t s, uint32_t n, uint32_t G, const void *pool,
                          const uint32_t *dir, uint32_t *plan, unsigned long long *part, unsigned long long *grp,
                          bool unpacked) {
  if (!n || !G) return;
  const uint32_t P = (G + K3R - 1) / K3R, ntiles = (n + K3T - 1) / K3T;
  uint32_t *tot = plan, *item_off = plan + (uint64_t)P * K3_PSUM_SPLIT;
  hipLaunchKernelGGL(k3_psum, dim3(P, K3_PSUM_SPLIT), dim3(256), 0, s, dir, ntiles, tot);
  // items: Σ_p ceil(T_p / target) <= nitems + P, so nitems = 2 rounds of the
  // resident workgroups less P keeps the rounding's extra items out of a third,
  // nearly empty round (the mesh: 1595 items for 1536 slots took 0.35 ms)
  const uint32_t slots = std::min<uint32_t>(K3_ITEMS, 2 * k3_resident());
  const uint32_t nitems = slots > P + 256 ? slots - P : 256;
  hipLaunchKernelGGL(k3_plan, dim3(1), dim3(1024), 0, s, tot, P, ntiles, nitems, item_off);
  hipLaunchKernelGGL(k3_reduce_bal, dim3(k3_bal_items(G)), dim3(K3RT), 0, s, static_cast<const uint64_t *>(pool), dir,
                     k3_tbase(const_cast<void *>(pool), n), ntiles, P, item_off, G, unpacked ? 1u : 0u, part);
  hipLaunchKernelGGL(k3_combine_bal, dim3((G + 255) / 256 < 2048 ? (G + 255) / 256 : 2048), dim3(256), 0, s, part,
                     item_off, G, grp);
}

uint32_t k3_plan_words(uint32_t P) { return P * K3_PSUM_SPLIT + P + 1; }
uint32_t k3_bal_items(uint32_t G) { return K3_ITEMS + (G + K3R - 1) / K3R; }  // an upper bound of the plan's items
uint64_t k3_bal_part_bytes(uint32_t G) { return (uint64_t)k3_bal_items(G) * K3F * K3R * 8; }
uint64_t k3_slice_part_bytes(uint32_t G, uint32_t S) { return (uint64_t)S * K3F * G * 8; }
uint32_t k3_partitions(uint32_t G) { return (G + K3R - 1) / K3R; }
uint32_t k3_pmax() { return K3PMAX; }
// the record pool: [tile][K3T] records, then each tile's time base (u64), then
// the escape list (u32 span indices, as many as spans at worst)
uint64_t k3_pool_bytes(uint32_t n) {
  const uint64_t nt = (n + K3T - 1) / K3T;
  return nt * K3T * 8 + nt * 8 + ((uint64_t)n + 4) * 4;
}
uint64_t *k3_tbase(void *pool, uint32_t n) { return static_cast<uint64_t *>(pool) + (uint64_t)((n + K3T - 1) / K3T) * K3T; }
uint32_t *k3_esc(void *pool, uint32_t n) {
  return reinterpret_cast<uint32_t *>(k3_tbase(pool, n) + (n + K3T - 1) / K3T);
}

void launch_k3_first(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status, uint32_t n,
                     const uint32_t *ep_of_shape, uint32_t n_shapes, uint32_t n_status, uint64_t index_base,
                     uint32_t G, unsigned long long *grp, unsigned int *counters) {
  if (!n || !G) return;
  hipLaunchKernelGGL(k3_first_fix, dim3(std::min<uint32_t>((G + 255) / 256, 2048)), dim3(256), 0, s, kind, shape,
                     status, n, ep_of_shape, n_shapes, n_status, index_base, G, grp, counters);
}

void launch_k3_escapes(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                       const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                       uint32_t n_shapes, uint32_t n_status, uint64_t index_base, void *pool,
                       const unsigned int *counters, unsigned long long *E, uint32_t G, unsigned long long *grp) {
  if (!n || !G) return;
  hipLaunchKernelGGL(k3_escape, dim3(256), dim3(256), 0, s, kind, shape, status, dur, ts, ep_of_shape, n_shapes,
                     n_status, index_base, k3_esc(pool, n), counters, E, G);
  hipLaunchKernelGGL(k3_escape_fold, dim3(std::min<uint32_t>((G + 255) / 256, 2048)), dim3(256), 0, s, counters, E, G,
                     grp);
}
uint32_t k3_tiles(uint32_t n) { return (n + K3T - 1) / K3T; }
uint64_t k3_dir_words(uint32_t n, uint32_t P, uint32_t S) {
  const uint64_t nt = k3_tiles(n);
  return (uint64_t)P * S * ((nt + S - 1) / S);
}

void launch_tile_sum(hipStream_t s, const uint32_t *v, uint32_t ntiles, uint32_t stride, uint32_t fields,
                     unsigned long long *out, uint32_t max_field) {
  hipLaunchKernelGGL(k_tile_sum, dim3(std::max<uint32_t>(1, tile_sum_blocks(ntiles))), dim3(1024), 0, s, v, ntiles, stride,
                     fields, out, max_field);
}

}  // namespace kmz
