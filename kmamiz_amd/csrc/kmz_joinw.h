// kmz_joinw.h -- the window join's tile geometry and LDS helpers, shared by
// k_join_window (kmz_join.hip) and the fused join + chain walk (kmz_fuse.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kmz_kernels.h"

namespace kmz {

constexpr uint32_t JT = 2048, JH = 256, JW = JT + 2 * JH, JTT = 512;
static_assert(JW < 4096, "local index + 1 must fit an entry's 12 bits");
constexpr uint16_t L_NONE = 0xFFFF, L_MISS = 0xFFFE;
// certificate pass 1: 2^6 bins per join tile; 2^8 (CERT_B1W) past ~10^8 ids,
// so that pass 2 still writes runs of ~8 records per sub-bin (cert_plan)
constexpr uint32_t CERT_B1 = 6, CERT_BINS = 1u << CERT_B1, CERT_B1W = 8;
// certificate pass 1's ranks from LDS atomics (1) or from 6 wave ballots
// per span (0: 1.09 against 1.00 ms for k_join_window on config 3)
#ifndef KMZ_RANK_ATOMIC
#define KMZ_RANK_ATOMIC 1
#endif

// exclusive scan of LDS u32 array a[0..m) in place, any m <= 64 * blockDim.x
__device__ __forceinline__ void block_scan_lds(uint32_t *a, uint32_t m, uint32_t *wsum) {
  const uint32_t per = (m + blockDim.x - 1) / blockDim.x;
  const uint32_t b = threadIdx.x * per, e = min(m, b + per);
  uint32_t s = 0;
  for (uint32_t k = b; k < e; ++k) s += a[k];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = s;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
      uint32_t t = wsum[k];
      wsum[k] = acc;
      acc += t;
    }
  }
  __syncthreads();
  uint32_t run = wsum[w] + x - s;
  for (uint32_t k = b; k < e; ++k) {
    uint32_t t = a[k];
    a[k] = run;
    run += t;
  }
  __syncthreads();
}

// LDS hash of a window: two-choice buckets of 8 u16 entries (one 16-byte LDS
// read each), entry = fingerprint (4 bits of a multiplicative hash of the id) << 12 | local index + 1.
// A lookup reads its two buckets and compares 16 fingerprints; only a
// fingerprint hit reads the 64-bit id.  Entries that find both buckets full go
// to a small stash that lookups scan (broadcast reads) when it is not empty.
// No probe loops: constant work per span, no wave waiting on its unluckiest lane.
constexpr uint32_t JB = 1024;     // buckets (8192 entries, load <= 0.31)
static_assert(JB * 16 >= JT * 8, "the buckets double as the tile's certificate staging");
constexpr uint32_t JSTASH = 64;
// Window-hash placement: two 32-bit multiplicative hashes of the folded id.
// Placement quality only affects speed (an overfull bucket pair goes to the
// stash, a full stash to the table path); exactness comes from comparing the
// full 64-bit ids, and the certificate keeps its own bijective cert_hash.
static_assert(JB == 1024, "bucket indices are the top 10 bits of the 32-bit hashes");
// the certificate's hash of a span id: a bijection of the 64-bit ids (an odd
// multiplier, then an xorshift), so equal hashes are equal ids; its top bits
// pick the bin and sub-bin, its low bits the check's bucket.  (mix64's second
// multiply and shifts bought nothing here: one multiply spreads sequential
// ids over the top bits, the xorshift brings them to the low bits.)  0 -> 0.
__device__ __forceinline__ uint64_t cert_hash(uint64_t x) { return id_hash(x); }  // (kmz_common.h)
__device__ __forceinline__ uint32_t jfold(uint64_t id) { return (uint32_t)id ^ (uint32_t)(id >> 32); }
__device__ __forceinline__ uint32_t jb1(uint32_t x) { return (x * 0x9E3779B1u) >> 22; }
__device__ __forceinline__ uint32_t jb2(uint32_t x) { return (x * 0x85EBCA77u) >> 22; }
// fingerprints are 1..15: an empty entry (0) never matches one, so a lookup
// compares fingerprints only
__device__ __forceinline__ uint32_t jfp(uint32_t x) { return max(((x * 0x9E3779B1u) >> 18) & 0xF, 1u); }

// k_join_window's hash: one 32-bit multiply of the folded id; the bucket is
// its top 10 bits, the 8-bit fingerprint (1..255: an empty slot's byte is 0)
// the next 8
__device__ __forceinline__ uint32_t jh8(uint32_t x) { return x * 0x9E3779B1u; }
__device__ __forceinline__ uint32_t jbk8(uint32_t h) { return h >> 22; }
__device__ __forceinline__ uint32_t jfp8(uint32_t h) { return max((h >> 14) & 0xFFu, 1u); }

// lanes of this wave whose `v` (B bits) equals mine, among `valid` lanes
template <int B>
__device__ __forceinline__ uint64_t match_bits(uint32_t v, uint64_t valid) {
  uint64_t m = valid;
#pragma unroll
  for (int bit = 0; bit < B; ++bit) {
    const uint64_t b = __ballot((v >> bit) & 1);
    m &= ((v >> bit) & 1) ? b : ~b;
  }
  return m;
}
__device__ __forceinline__ uint64_t match6(uint32_t v, uint64_t valid) { return match_bits<6>(v, valid); }

}  // namespace kmz
