// kmz_chainw.h -- chain signatures, the chain table and the edge-key set:
// the device helpers of the chain walk, shared by k4_chain (kmz_chain.hip) and
// the fused join + chain walk (kmz_fuse.hip).  See kmz_chain.hip for the
// exactness argument.
#pragma once
#include <hip/hip_runtime.h>

#include "kmz_kernels.h"

namespace kmz {

constexpr uint16_t W_NONE = 0xFFFF, W_CYC = 0xFFFE, W_OUT = 0xFFFD;
constexpr uint32_t WIN_DEPTH = 255;  // deeper in-window ancestries take the pending path
constexpr uint32_t PROBE_MAX = 512;
// bound of a wait on another lane's publish (chain_put returning 0).  The
// publish is the instruction after that lane's claim, so a wait this long
// means something is wrong; it raises F_SPIN (the run is redone exactly) and
// never drops a check, a row or a key.  KMZ_ABLATE bit 11 (test knob) makes
// the bound 0, i.e. every wait "runs out".
constexpr uint32_t SPIN_MAX = 1u << 20;
__host__ __device__ __forceinline__ uint32_t spin_bound(uint32_t ablate) { return (ablate & (1u << 11)) ? 0u : SPIN_MAX; }
constexpr uint32_t IMAP = 256;  // LDS map: one inserting leader per distinct new chain
#ifndef KMZ_SIG_MIX
#define KMZ_SIG_MIX 0
#endif
constexpr uint32_t SIG_R = 21;  // fold rotation (odd: x ^ rotl(x, R) is 2-to-1 only on {x, ~x})
// per-slot byte: kind in bits 0-1, state in bits 2-3 (state written only by the slot's owner)
constexpr uint8_t S_NONE = 0, S_DONE = 1, S_PUT = 2, S_PEND = 3;
__device__ __forceinline__ uint8_t kf_kind(uint8_t b) { return b & 3; }
__device__ __forceinline__ uint8_t kf_st(uint8_t b) { return b >> 2; }
__device__ __forceinline__ uint8_t kf_make(uint8_t kind, uint8_t st) { return (uint8_t)(kind | (st << 2)); }

// A chain element's 64-bit value: an injective function of (endpoint, on) --
// one 32 x 64-bit multiply by an odd constant of (endpoint << 1 | on) ^ seed
// (endpoints past 2^30 are all "none") -- cheap enough that the walk computes
// it per step from the endpoint instead of reading it from LDS (the walk's
// window records are 8 bytes).  Injectivity is what the chain table's
// exactness argument needs (kmz_chain.hip); the odd multiplier spreads the
// bits the table's home slot is taken from.  (Until round 5: mix64, two 64-bit
// multiplies, kept in 16-byte LDS records.)
__host__ __device__ __forceinline__ uint64_t sig_elem(uint32_t ep, bool on, uint64_t seed) {
  const uint32_t x = (((ep < EPK_NONE ? ep : EPK_NONE) << 1) | (on ? 1u : 0u)) ^ (uint32_t)seed;
  return (uint64_t)x * 0x9E3779B97F4A7C15ull;
}
constexpr uint64_t ROOT_SIG = ~0ull;  // the "parent sig" of a root
__device__ __forceinline__ uint64_t rotl64(uint64_t x, uint32_t r) {
  r &= 63;
  return r ? (x << r) | (x >> (64 - r)) : x;
}
// one fold step: the ancestors a1 (nearest) .. aD give
//   acc = rotl^(D-1)(e(a1)) ^ ... ^ rotl(e(aD-1)) ^ e(aD)
__device__ __forceinline__ uint64_t sig_step(uint64_t acc, uint64_t el) {
  return ((acc << SIG_R) | (acc >> (64 - SIG_R))) ^ el;
}
// The finish is an xor with a depth and seed constant: a bijection for each
// depth, which is all the exactness argument needs.  Placement mixes once
// more (sig_place); a final mix64 of both sigs (two 64-bit multiplies per sig,
// two sigs per span) cost 4 % of k4_chain (mesh 1.33 against 1.28 ms).
// 0 marks an unwritten word and ROOT_SIG a root's parent: a sig equal to
// either is treated as a collision (another seed)
__device__ __forceinline__ uint64_t sig_final(uint64_t acc, uint32_t d, uint64_t seed, uint32_t *flags) {
#if KMZ_SIG_MIX
  const uint64_t z = mix64(acc ^ ((uint64_t)d * 0x632BE59BD9B4E019ull) ^ (seed << 1));
#else
  const uint64_t z = acc ^ ((uint64_t)d * 0x632BE59BD9B4E019ull) ^ (seed << 1);
#endif
  if (z == 0 || z == ROOT_SIG) *flags |= F_SIG;
  return z;
}
// Placement of a sig (the chain table's home slot, the walk's LDS leader
// map): an xorshift and one multiply, so that every bit of the sig reaches the
// top bits -- the fold of Fibonacci-hashed elements leaves some low-quality
// bits (low bits of a product) rotated into the top ones.  Placement only:
// identity is the whole sig.
__device__ __forceinline__ uint64_t sig_place(uint64_t sig) { return (sig ^ (sig >> 29)) * 0xBF58476D1CE4E5B9ull; }
// home slot: the placement's high bits (ccap is a power of two)
__device__ __forceinline__ uint64_t cslot(uint64_t sig, uint64_t ccap) {
  return sig_place(sig) >> (64 - __builtin_ctzll(ccap));
}

__device__ __forceinline__ uint64_t edge_key(uint32_t ea, uint32_t es, uint32_t d, bool on) {
  return ((uint64_t)ea << 40) | ((uint64_t)es << 16) | ((uint64_t)d << 1) | (on ? 1ull : 0ull);
}

// the global edge-key set (one insert per key of a NEW chain only); its size
// is counted by the compaction
__device__ __forceinline__ void edge_insert(uint64_t key, unsigned long long *__restrict__ trip, uint64_t tcap,
                                           uint32_t *flags) {
  // an overfull set makes every insert probe PROBE_MAX slots: once this
  // thread has seen it, the run is repeated with a larger set anyway
  if (*flags & F_TRIPLE_OVERFLOW) return;
  uint64_t pos = eslot(key, tcap);
  for (uint32_t z = 0; z < PROBE_MAX; ++z) {
    uint64_t cur = trip[pos];
    if (cur == key) return;
    if (cur == 0) {
      cur = atomicCAS(&trip[pos], 0ull, (unsigned long long)key);
      if (cur == 0 || cur == key) return;
    }
    pos = eset_next(pos, tcap);
  }
  *flags |= F_TRIPLE_OVERFLOW;
}

// Chain table entry words: [0] sig, [1] parent sig (ROOT_SIG at a root).
// Both are written once with a nonzero value, so a reader needs no ordering
// between them: an entry is published once both are nonzero.
// Insert (or join) the chain `sig`.  Returns 1 inserted, 2 found (and
// checked), 0 not yet decidable (the winner has not published), -1 probe bound.
// A slot this call claims is appended to the run's written list (gpos, counted
// in counters[C_WPOS]) so that it can be cleared after the run.
__device__ __forceinline__ int chain_put(unsigned long long *__restrict__ ctab, uint64_t ccap, uint64_t sig,
                                         uint64_t psig, uint32_t *flags, uint32_t *__restrict__ gpos,
                                         uint32_t gcap, unsigned int *__restrict__ counters) {
  if (*flags & F_CHAIN_OVERFLOW) return -1;  // (this thread found the table full: the run is repeated larger)
  uint64_t pos = cslot(sig, ccap);
  for (uint32_t z = 0; z < PROBE_MAX; ++z) {
    unsigned long long *e = ctab + 2 * pos;
    const unsigned long long c = atomicCAS(&e[0], 0ull, (unsigned long long)sig);
    if (c == 0) {
      atomicExch(&e[1], (unsigned long long)psig);
      const uint32_t x = atomicAdd(&counters[C_WPOS], 1u);  // (rare paths only)
      if (x < gcap)
        gpos[x] = (uint32_t)pos;
      else
        *flags |= F_CTAB_DIRTY;
      return 1;
    }
    if (c == sig) {
      const unsigned long long ps = atomicAdd(&e[1], 0ull);  // memory-side read
      if (ps == 0) return 0;
      if (ps != psig) *flags |= F_SIG;
      return 2;
    }
    pos = pos + 1 == ccap ? 0 : pos + 1;
  }
  *flags |= F_CHAIN_OVERFLOW;
  return -1;
}

}  // namespace kmz
