// kmz_common.h -- host+device helpers shared by the kernels, the C ABI and the
// host-side finaliser.  Everything here is integer or correctly-rounded fp64
// arithmetic (compiled with -ffp-contract=off) so host and device agree bit
// for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KMZ_HD __host__ __device__ __forceinline__

namespace kmz {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t CYC = 0xFFFFFFFEu;  // cparent of a span whose CLIENT chain loops
constexpr uint64_t NONE64 = ~0ull;
constexpr uint64_t TS_BIAS = 1ull << 63;  // signed -> order-preserving unsigned
constexpr uint32_t MAX_DEPTH = 1u << 14;  // cycle guard (reference: unbounded)

// error bits (device-side, folded into kmz_info.flags)
constexpr uint32_t F_CYCLE = 1u;
constexpr uint32_t F_ZERO_ID = 2u;
constexpr uint32_t F_RANGE = 4u;
constexpr uint32_t F_DUP_OVERFLOW = 8u;
constexpr uint32_t F_TRIPLE_OVERFLOW = 16u;
constexpr uint32_t F_TABLE_FULL = 32u;
constexpr uint32_t F_CHAIN_OVERFLOW = 64u;
constexpr uint32_t F_CTAB_DIRTY = 512u;     // (informational) the chain table could not be cleared by list
constexpr uint32_t F_STAGE_FULL = 1024u;    // (informational) K4 key staging overflowed: keys went straight to the edge set
constexpr uint32_t F_MISS_OVERFLOW = 256u;  // the window join's miss table is too small (grown, run again)
constexpr uint32_t F_SIG = 128u;  // a 64-bit ancestry hash collision (K4 retries with another seed)
// a K4 wait on another lane's chain-table publish ran out of its bound: the
// entry's check (and for a pending row its counts and keys) did not happen, so
// the run is repeated on the exact per-row walk (kmz_run)
constexpr uint32_t F_SPIN = 2048u;

// splitmix64 finaliser: a bijection on u64 with mix64(0) == 0.
KMZ_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

KMZ_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// traceId -> shard (shard = h(traceId) mod G).  (hi, lo) is the
// 128-bit value of a canonical lowercase-hex traceId (hi = 0 for 16-digit
// ids; other strings are hashed by kmz_trace_shard).  A multiply-shift range
// reduction instead of a modulo: uniform for any world size.
KMZ_HD uint64_t shard_hash(uint64_t hi, uint64_t lo) { return mix64(hi ^ mix64(lo ^ 0x4B4D5A5348415244ull)); }
KMZ_HD uint32_t shard_of(uint64_t hi, uint64_t lo, uint32_t world) {
  return (uint32_t)mulhi64(shard_hash(hi, lo), world);
}

// The uniqueness certificate's hash of a span id (kmz_join.hip) and the
// cross-shard id routing (kmz_guard.hip): a bijection of the 64-bit ids (an
// odd multiplier, then an xorshift), so equal hashes are equal ids; 0 -> 0.
KMZ_HD uint64_t id_hash(uint64_t x) {
  x *= 0x9E3779B97F4A7C15ull;
  return x ^ (x >> 29);
}
// owner rank of a hashed id among `world` ranks (a range of the hash space;
// the host mirror in dist.py computes the same in numpy uint64)
KMZ_HD uint32_t id_owner(uint64_t h, uint32_t world) { return (uint32_t)(((h >> 32) * world) >> 32); }

// position of key k in a table of `cap` slots (any cap, no pow2 rounding)
KMZ_HD uint64_t slot_of(uint64_t k, uint64_t cap) { return mulhi64(mix64(k ^ 0x5bd1e9955bd1e995ull), cap); }
KMZ_HD uint32_t tag_of(uint64_t k) { return (uint32_t)(mix64(k + 0x9e3779b97f4a7c15ull) >> 32); }

// Edge-key sets (the run's `trip` table) probe linearly inside slices of
// ESLICE slots: a key's probe sequence wraps within the slice of its home
// slot, so every slice is a self-contained table (kmz_chain.hip builds each
// one in LDS from the keys partitioned to it).  A cap that is not a multiple
// of ESLICE probes the whole table.
constexpr uint64_t ESLICE = 8192;
// Edge keys are ancestor << 40 | descendant << 16 | distance << 1 | on.  A key
// with both endpoints < 2^16 and distance < 32 is *compact*: its 38-bit code
// (anc 16 | desc 16 | d 5 | on 1) times an odd constant mod 2^38 is a
// bijection of the codes, so the 38 bits x38 name the key, and a key staged
// in a slice known from x38's top bits needs only x38's low 32 bits
// (kmz_chain.hip: direct enumeration stages 4-byte keys).
constexpr uint64_t EK_PHI = 0x9E3779B97F4A7C15ull;
constexpr uint64_t EK_M38 = (1ull << 38) - 1;
constexpr uint64_t ek_inv64(uint64_t a) {  // a^-1 mod 2^64 (a odd): Newton, 6 steps
  uint64_t x = a;
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}
constexpr uint64_t EK_PHI_INV = ek_inv64(EK_PHI);
static_assert(EK_PHI * EK_PHI_INV == 1, "inverse of the edge-key multiplier");
KMZ_HD bool ekey_compact(uint64_t k) {
  return (k >> 56) == 0 && ((k >> 32) & 0xFF) == 0 && ((k >> 6) & 0x3FF) == 0;  // anc, desc < 2^16, d < 32
}
KMZ_HD uint64_t ekey_code(uint64_t k) {  // (compact keys)
  return ((k >> 40) << 22) | (((k >> 16) & 0xFFFF) << 6) | (k & 63);
}
KMZ_HD uint64_t ekey_x38(uint64_t k) { return (ekey_code(k) * EK_PHI) & EK_M38; }
KMZ_HD uint64_t ekey_from_x38(uint64_t x) {
  const uint64_t c = (x * EK_PHI_INV) & EK_M38;
  return ((c >> 22) << 40) | (((c >> 6) & 0xFFFF) << 16) | (c & 63);
}
// the edge set's hash of a key: x38 in the top bits for compact keys, the
// 64-bit Fibonacci product for the others (any fixed function of the key will
// do: the set compares whole keys)
KMZ_HD uint64_t ekey_hash(uint64_t k) { return ekey_compact(k) ? ekey_x38(k) << 26 : k * EK_PHI; }
// home slot of an edge key, range-reduced like slot_of.  For a power-of-two
// cap it is the hash's top log2(cap) bits.
KMZ_HD uint64_t eslot(uint64_t k, uint64_t cap) { return mulhi64(ekey_hash(k), cap); }
KMZ_HD uint64_t eset_next(uint64_t pos, uint64_t cap) {
  if (cap % ESLICE) return pos + 1 == cap ? 0 : pos + 1;
  return (pos & ~(ESLICE - 1)) | ((pos + 1) & (ESLICE - 1));
}

// ---- JS number semantics ----------------------------------------------------
// Math.round: nearest, ties toward +inf (ECMA-262 Math.round)
KMZ_HD double js_round(double x) {
  double r = floor(x);
  if (x - r >= 0.5) r += 1.0;
  return r;
}
// Utils.ToPrecise (src/utils/Utils.ts:311-313)
KMZ_HD double to_precise(double x) {
  const double eps = 2.220446049250313e-16;  // Number.EPSILON
  double t = x + eps;  // add and multiply round separately (-ffp-contract=off)
  double u = t * 1e14;
  return js_round(u) / 1e14;
}

KMZ_HD double u128_to_double(uint64_t hi, uint64_t lo) {
  // (double)hi * 2^64 + (double)lo : <= 1 ulp from the exact value
  return (double)hi * 18446744073709551616.0 + (double)lo;
}

// Finalise one (endpoint x status) group from exact integer moments of the
// durations d_i (us):  n, S1 = sum d, S2 = sum d^2 = s2a + s2b * 2^32.
//   mean_ms = S1 / (1000 n)                       (RealtimeDataList.ts:100-118
//   cv      = sqrt(n*S2 - S1^2) / S1               computes the same quantities
// both exact-then-rounded, so they differ from the reference's sequential
// Welford only by the reference's own rounding (<= ~1e-15 relative).
KMZ_HD void finalize_moments(uint64_t n, uint64_t s1, uint64_t s2a, uint64_t s2b, double *mean_out,
                             double *cv_out) {
  if (n == 0) {
    *mean_out = 0.0;
    *cv_out = 0.0;
    return;
  }
  // S2 = s2a + s2b<<32 as 128-bit (hi, lo)
  uint64_t lo = s2a + (s2b << 32);
  uint64_t carry = lo < s2a ? 1ull : 0ull;
  uint64_t hi = (s2b >> 32) + carry;
  // n * S2 (n < 2^32, S2 < 2^96 -> < 2^128)
  uint64_t p_lo = n * lo;
  uint64_t p_hi = mulhi64(n, lo) + n * hi;
  // S1^2
  uint64_t q_lo = s1 * s1;
  uint64_t q_hi = mulhi64(s1, s1);
  // n*S2 - S1^2 >= 0 (Cauchy-Schwarz)
  uint64_t r_lo = p_lo - q_lo;
  uint64_t borrow = p_lo < q_lo ? 1ull : 0ull;
  uint64_t r_hi = p_hi - q_hi - borrow;
  double mean = (double)s1 / ((double)n * 1000.0);
  double cv = 0.0;
  if (s1 != 0) {
    double num = u128_to_double(r_hi, r_lo);
    cv = sqrt(num) / (double)s1;
  }
  *mean_out = to_precise(mean);
  *cv_out = to_precise(cv);
}

}  // namespace kmz
