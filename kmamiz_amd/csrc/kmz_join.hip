// kmz_join.hip -- K1': the span-id parent join without a global hash table.
//
// The reference builds one Map over every span of the batch (Traces.ts:117-123)
// and then resolves each parentId through it, skipping CLIENT spans
// (Traces.ts:128-137).  A global HBM hash table makes that two random accesses
// per span into a table far larger than the MALL; on MI355X that is bound by
// random-line throughput, not bandwidth.  Parents are, however, almost always
// a few rows away (Zipkin returns a trace's spans together), so:
//
//   k_join_window   tile of JT spans + JH halo on each side in LDS: an LDS
//                   hash of the window's span ids, each span's parent found
//                   in the window (dp), CLIENT contraction inside the window
//                   (cparent).  Chains that leave the window are PEND, parent
//                   ids not in the window MISS.  The same kernel scatters the
//                   tile's hashed ids into 64 bins (pass 1 of the certificate).
//   k_cert_split    pass 2: each bin chunk is split into 2^B2 sub-bins.
//   k_cert_check    pass 3: exact duplicate check of each sub-bin in LDS.
//
// A window hit is the Map's answer only if the id occurs once in the whole
// batch; the certificate proves that (cert_hash is a bijection, so equal hashes
// are equal ids).  If any id repeats, the host runs the global table path
// (kmz_kernels.hip: K1 build/fixup, K2 resolve), which implements the Map's
// last-value/first-position rule.  MISS parents are looked up with a
// semi-join of the missing ids against all span ids (k_miss_*), and PEND
// chains are finished over the global dp array (k_pend).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_joinw.h"

namespace kmz {

#ifndef KMZ_CERT_PQ
#define KMZ_CERT_PQ 8
#endif
constexpr uint32_t CERT_PQ = KMZ_CERT_PQ;  // pass 2: records per thread (chunks of PQ * 1024 records of one bin)
constexpr uint32_t CERT_SET = 8192;    // pass-3 LDS set (u64), sub-bins <= 6144 records

__host__ __device__ uint32_t join_tiles(uint32_t n) { return (n + JT - 1) / JT; }

__device__ unsigned long long g_join_dbg[16];  // diagnostic phase clocks (KMZ_ABLATE bit 23 only)
#define KMZ_JSTAMP(k)                                           \
  if (dbg_t) {                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0 && tprev) tacc[k] += t_ - tprev;       \
    tprev = t_;                                                 \
  }

// (A persistent form of this kernel, the next tile's window loaded while the
// current tile contracts and bins, measured 1.62 against 1.18 ms on config 3.)
// Its window: the tile and KH spans either side.  A parent further out is a
// MISS (the semi-join), a chain leaving the window PEND (k_pend): slower for
// those spans, never a different answer.  (KH = 128: mesh 3.328 -> 3.310 ms,
// config 5 7.31 -> 8.22 ms, its longer traces leaving more parents outside;
// profiles/r05/ab/halo, halop.)
#ifndef KMZ_JOIN_HALO
#define KMZ_JOIN_HALO 256
#endif
constexpr uint32_t KH = KMZ_JOIN_HALO, KW = JT + 2 * KH;
static_assert(KW <= JW, "the window hash is sized for JW slots");
template <uint32_t B1>
__global__ void __launch_bounds__(JTT, 6) k_join_window(const uint64_t *__restrict__ sid, const uint64_t *__restrict__ pid,
                                                     const uint8_t *__restrict__ kind, uint32_t n,
                                                     uint32_t *__restrict__ cparent, uint32_t *__restrict__ dp,
                                                     unsigned long long *__restrict__ pool1,
                                                     uint16_t *__restrict__ jdir,
                                                     unsigned int *__restrict__ counters, uint32_t ablate,
                                                     const JoinRoute rt) {
  constexpr uint32_t NW = JTT / 64, BINS = 1u << B1;
  const bool route = rt.out != nullptr;  // (kmz_route_ids_join: pass 1 bins by owner into the segments)
  __shared__ uint64_t lsid[KW];
  // the window's LDS hash (kmz_joinw.h jh8): per bucket 8 entries (local
  // index + 1, u16) and their 8-bit fingerprints in one u64, so that a lookup
  // tests all 8 with a few 32-bit operations (a zero-byte test) instead of
  // decoding 16 packed entries; fill counts are bytes, four per word.  A
  // bucket's count wraps past 255 ids (its carry lands in the neighbour's
  // byte), and an insert that then reads 0..7 would write a slot already
  // written -- two threads could leave a fingerprint of one id beside the
  // index of another.  No tile ever answers from such a table: 256 ids in one
  // bucket put >= 248 of them past its 8 slots, i.e. past the 64-entry stash,
  // which sets `ovf` (CERT_OVF): the run is redone on the table path.  (Below the
  // wrap, a lookup compares whole ids, so a fingerprint collision only costs
  // a further candidate.)  After the lookups
  // the entries become the certificate's staging and the fingerprints its
  // per-wave bin counters (pass 1)
  __shared__ uint4 lidx[JB];
  __shared__ unsigned long long lfp[JB];
  __shared__ uint32_t lcnt4[JB / 4];
  uint32_t *const wcnt = reinterpret_cast<uint32_t *>(lfp);
  constexpr uint32_t WCAP = JB * 2;  // u32 words of the pass-1 counters
  static_assert(BINS * NW <= WCAP, "pass-1 counters fit the fingerprint words");
  // per window slot: its parent's local index (12 bits, or X_NONE / X_MISS)
  // | X_CLIENT when the slot itself is a CLIENT span (no separate kind array:
  // 2.5 KB of LDS, the third workgroup per CU)
  __shared__ uint16_t ldp[KW];
  constexpr uint32_t X_NONE = 0xFFF, X_MISS = 0xFFE, X_CLIENT = 0x8000;
  static_assert(KW < X_MISS, "local indices stay below the markers");
  __shared__ uint32_t wsum[NW];
  __shared__ uint32_t stash[JSTASH];  // fingerprint << 16 | local index + 1
  __shared__ uint32_t nstash;
  constexpr int PW = (KW + JTT - 1) / JTT, PT = JT / JTT;  // (slots past KW: w0 + jl >= w1)
  const uint32_t t0 = blockIdx.x * JT, t1 = min(n, t0 + JT);
  const uint32_t w0 = t0 > KH ? t0 - KH : 0, w1 = min(n, t1 + KH);
  const bool dbg_t = (ablate & (1u << 23)) != 0;
  unsigned long long tprev = 0, tacc[6] = {0, 0, 0, 0, 0, 0};
  KMZ_JSTAMP(0);
  for (uint32_t k = threadIdx.x; k < JB; k += JTT) lfp[k] = 0;
  for (uint32_t k = threadIdx.x; k < JB / 4; k += JTT) lcnt4[k] = 0;
  if (threadIdx.x == 0) nstash = 0;
  // one round of window loads (ids, kinds, parent ids), all in flight together
  uint64_t s[PW], p[PW];
  uint8_t k[PW];
#pragma unroll
  for (int q = 0; q < PW; ++q) {  // clamped and unconditional: no branch between the loads
    const uint32_t j = w0 + q * JTT + threadIdx.x, jj = min(j, n - 1);
    s[q] = sid[jj];
    p[q] = pid[jj];
    k[q] = kind[jj];
  }
#pragma unroll
  for (int q = 0; q < PW; ++q)
    if (w0 + q * JTT + threadIdx.x >= w1) {
      s[q] = p[q] = 0;
      k[q] = 0;
    }
  uint32_t hs[PW];
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const uint32_t jl = q * JTT + threadIdx.x;
    hs[q] = jh8(jfold(s[q]));
    if (w0 + jl < w1) lsid[jl] = s[q];
  }
  __syncthreads();
  KMZ_JSTAMP(0);
  bool ovf = false;
  uint8_t *const lfp8 = reinterpret_cast<uint8_t *>(lfp);
  uint16_t *const lidx16 = reinterpret_cast<uint16_t *>(lidx);
  if (!(ablate & 256)) {  // insert: a slot of the id's bucket, else the stash
    // (in lockstep over the thread's PW ids: the slot claims in flight together)
    uint32_t sq[PW];
    bool iq[PW];
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      iq[q] = w0 + q * JTT + threadIdx.x < w1 && s[q] != 0;
      const uint32_t b = jbk8(hs[q]), sh = (b & 3) * 8;
      sq[q] = iq[q] ? (atomicAdd(&lcnt4[b >> 2], 1u << sh) >> sh) & 0xFF : 0u;
    }
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      const uint32_t jl = q * JTT + threadIdx.x;
      if (!iq[q]) continue;
      const uint32_t b = jbk8(hs[q]);
      if (sq[q] < 8) {
        lfp8[b * 8 + sq[q]] = (uint8_t)jfp8(hs[q]);
        lidx16[b * 8 + sq[q]] = (uint16_t)(jl + 1);
      } else {
        const uint32_t t = atomicAdd(&nstash, 1u);
        if (t < JSTASH)
          stash[t] = (jfp8(hs[q]) << 16) | (jl + 1);
        else
          ovf = true;  // this tile cannot answer: the table path runs
      }
    }
  }
  __syncthreads();
  KMZ_JSTAMP(1);
  const uint32_t ns = min(nstash, JSTASH);
  // window parents: tile spans, and CLIENT spans of the halo (chains pass
  // through them).  The PW lookups of a thread go in lockstep, each step's
  // LDS reads in flight together: the bucket's fingerprints; the first
  // candidate's entry; its id.  Further candidates (an 8-bit fingerprint
  // collision) and the stash are the rare tail.
  uint32_t hq[PW], eq[PW];
  uint64_t cq[PW];
  bool nq[PW];
  uint16_t rq[PW];
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const uint32_t jl = q * JTT + threadIdx.x, j = w0 + jl;
    nq[q] = j < w1 && p[q] != 0 && ((j >= t0 && j < t1) || k[q] == KIND_CLIENT) && !(ablate & 512);
    rq[q] = nq[q] ? X_MISS : X_NONE;
    hq[q] = jh8(jfold(p[q]));
    const uint64_t w = lfp[nq[q] ? jbk8(hq[q]) : 0];
    uint32_t pat = jfp8(hq[q]);
    pat |= pat << 8;
    pat |= pat << 16;
    // exact zero-byte test of fingerprints ^ pattern: bit 7 of a byte of
    // ~y & 0x80.. is set iff that byte matched (no carry crosses a byte)
    const uint32_t xl = (uint32_t)w ^ pat, xh = (uint32_t)(w >> 32) ^ pat;
    const uint32_t yl = ((xl & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | xl;
    const uint32_t yh = ((xh & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | xh;
    const uint64_t cand = ((uint64_t)(~yh & 0x80808080u) << 32) | (uint64_t)(~yl & 0x80808080u);
    cq[q] = nq[q] ? cand : 0;
  }
#pragma unroll
  for (int q = 0; q < PW; ++q)  // the first candidate's entry (local index + 1)
    eq[q] = cq[q] ? lidx16[jbk8(hq[q]) * 8 + (__builtin_ctzll(cq[q]) >> 3)] : 0;
#pragma unroll
  for (int q = 0; q < PW; ++q) {  // its id
    const bool hit = eq[q] && lsid[eq[q] ? eq[q] - 1 : 0] == p[q];
    if (hit) rq[q] = (uint16_t)(eq[q] - 1);
    if (!hit) cq[q] &= cq[q] - 1;  // (the rest, if the first was a fingerprint collision)
    else cq[q] = 0;
  }
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const uint32_t jl = q * JTT + threadIdx.x;
    if (w0 + jl >= w1) continue;
    uint32_t r = rq[q];
    uint64_t cand = cq[q];
    while (cand) {  // (rare) further candidates
      const uint32_t t = __builtin_ctzll(cand) >> 3;
      cand &= cand - 1;
      const uint32_t en = lidx16[jbk8(hq[q]) * 8 + t];
      if (lsid[en - 1] == p[q]) {
        r = en - 1;
        break;
      }
    }
    if (nq[q] && r == X_MISS) {
      const uint32_t f = jfp8(hq[q]);
      for (uint32_t t = 0; t < ns; ++t) {
        const uint32_t en = stash[t];
        if ((en >> 16) == f && lsid[(en & 0xFFFF) - 1] == p[q]) r = (en & 0xFFFF) - 1;
      }
    }
    ldp[jl] = (uint16_t)(r | (k[q] == KIND_CLIENT ? X_CLIENT : 0u));
  }
  if (ovf) atomicOr(&counters[C_CERT], CERT_OVF);
  __syncthreads();
  KMZ_JSTAMP(2);
  // tile: CLIENT contraction inside the window (Traces.ts:131-137), lockstep
  uint32_t miss = 0, pend = 0, zero = 0;
  uint64_t hv[PT];
  {
    uint32_t j[PT], cp[PT], hops[PT], d0[PT];
    bool act[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t i = t0 + q * JTT + threadIdx.x, il = i - w0;
      const bool ok = i < t1;
      const uint32_t e0 = ok ? ldp[il] : X_NONE;
      d0[q] = e0 & 0xFFF;
      act[q] = ok && !(e0 & X_CLIENT);
      j[q] = d0[q];
      cp[q] = NONE;
      hops[q] = 0;
    }
    for (;;) {
      bool any = false;
      uint32_t ej[PT];
#pragma unroll
      for (int q = 0; q < PT; ++q) ej[q] = (act[q] && j[q] < KW) ? ldp[j[q]] : 0;
#pragma unroll
      for (int q = 0; q < PT; ++q) {
        if (!act[q]) continue;
        if (j[q] >= KW) {  // markers (a compare, not a switch: see Window::next in kmz_part.hip)
          cp[q] = j[q] == X_NONE ? NONE : PEND;
          act[q] = false;
        } else if (!(ej[q] & X_CLIENT)) {
          cp[q] = w0 + j[q];
          act[q] = false;
        } else if (++hops[q] > MAX_DEPTH) {
          cp[q] = CYC;
          act[q] = false;
        } else {
          j[q] = ej[q] & 0xFFF;
          any = true;
        }
      }
      if (!any) break;
    }
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t i = t0 + q * JTT + threadIdx.x;
      hv[q] = 0;
      if (i >= t1) continue;
      cparent[i] = cp[q];
      dp[i] = d0[q] == X_NONE ? NONE : (d0[q] == X_MISS ? MISSV : w0 + d0[q]);
      miss += d0[q] == X_MISS;
      pend += cp[q] == PEND;
      const uint64_t key = lsid[i - w0];
      zero += key == 0;
      hv[q] = cert_hash(key);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    miss += __shfl_xor(miss, o, 64);
    pend += __shfl_xor(pend, o, 64);
    zero += __shfl_xor(zero, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (miss) atomicAdd(&counters[C_MISS], miss);
    if (pend) atomicAdd(&counters[C_PEND], pend);
    if (zero) atomicOr(&counters[C_FLAGS], F_ZERO_ID);
  }
  KMZ_JSTAMP(3);
  if (ablate & 64) return;  // diagnostic: no certificate pass 1
  // certificate pass 1: the tile's hashed ids into 2^B1 bins.  Ranks come
  // from per-wave bin counters (LDS atomics with return), or where the LDS
  // has no room for them (2^8 bins) from wave ballots.  (Routing: into the
  // owner ranks' bins instead, world <= 2^B1.)
  auto bin_of = [&](uint64_t h) -> uint32_t { return route ? id_owner(h, rt.world) : (uint32_t)(h >> (64 - B1)); };
  for (uint32_t e = threadIdx.x; e < BINS * NW; e += JTT) wcnt[e] = 0;
  __syncthreads();  // the hash entries are free from here on
  uint64_t *stg = reinterpret_cast<uint64_t *>(lidx);
  static_assert(JB * 16 >= JT * 8, "the hash entries hold the tile's certificate staging");
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t rk[PT];
#if KMZ_RANK_ATOMIC
  if constexpr (2 * BINS * NW <= WCAP) {
    // wave-major counters (a wave's 64 lanes spread over the banks; the
    // order within a bin is immaterial to the certificate), transposed to
    // bin-major for the scan.  The 6 ballots per span this replaces were an
    // eighth of the kernel's VALU instructions.
    uint32_t *const wmaj = wcnt + BINS * NW;
    for (uint32_t e = threadIdx.x; e < BINS * NW; e += JTT) wmaj[e] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t i = t0 + q * JTT + threadIdx.x;
      rk[q] = i < t1 ? atomicAdd(&wmaj[w * BINS + bin_of(hv[q])], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < BINS * NW; e += JTT) wcnt[e] = wmaj[(e % NW) * BINS + e / NW];
  } else
#endif
  {
#pragma unroll
  for (int q = 0; q < PT; ++q) {
    const uint32_t i = t0 + q * JTT + threadIdx.x;
    const bool ok = i < t1;
    const uint32_t bin = bin_of(hv[q]);
    const uint64_t peers = match_bits<B1>(bin, __ballot(ok));
    uint32_t prior = 0;
    if (ok) prior = wcnt[bin * NW + w];
    rk[q] = prior + __popcll(peers & lt);
    if (ok && (peers & lt) == 0) wcnt[bin * NW + w] = prior + __popcll(peers);
  }
  }
  __syncthreads();
  block_scan_lds(wcnt, BINS * NW, wsum);  // bin-major, wave-minor offsets
  uint32_t *const rbase = lcnt4;  // (routing: each owner's run in its segment; the fill counts are free)
  static_assert(JB / 4 >= BINS, "an owner run base per pass-1 bin");
  if (route) {
    // each owner's run of this tile reserved in its segment by one device
    // atomic, issued before the staging so that its round trip overlaps it
    for (uint32_t r = threadIdx.x; r < rt.world; r += JTT) {
      const uint32_t o = wcnt[r * NW], e = r + 1 < BINS ? wcnt[(r + 1) * NW] : t1 - t0;
      rbase[r] = e > o ? (uint32_t)atomicAdd(&rt.cur[(uint64_t)r * ROUTE_CUR_STRIDE], (unsigned long long)(e - o)) : 0u;
    }
  } else {
    // tile-major output, bins in order: no global atomics; the bin offsets go
    // to the tile's directory row for pass 2
    for (uint32_t b = threadIdx.x; b < BINS; b += JTT) jdir[(uint64_t)blockIdx.x * BINS + b] = (uint16_t)wcnt[b * NW];
  }
#pragma unroll
  for (int q = 0; q < PT; ++q) {
    const uint32_t i = t0 + q * JTT + threadIdx.x;
    if (i < t1) stg[wcnt[bin_of(hv[q]) * NW + w] + rk[q]] = hv[q];
  }
  __syncthreads();
  if (route) {
    for (uint32_t e = threadIdx.x; e < t1 - t0; e += JTT) {
      const uint64_t x = stg[e];
      const uint32_t r = id_owner(x, rt.world);
      const uint64_t pos = (uint64_t)rbase[r] + (e - wcnt[r * NW]);
      if (pos + 1 < rt.segw) rt.out[(uint64_t)r * rt.segw + 1 + pos] = x;  // (full: its count says so)
    }
  } else {
    for (uint32_t e = threadIdx.x; e < t1 - t0; e += JTT) pool1[(uint64_t)t0 + e] = stg[e];
  }
  KMZ_JSTAMP(4);
  if (dbg_t && threadIdx.x == 0)
    for (int kk = 0; kk < 5; ++kk) atomicAdd(&g_join_dbg[kk], tacc[kk]);
}

// Certificate pass 1 over a plain array of values (no join): the cross-shard
// repeated-id guard (kmz_guard.hip) checks the routed id hashes it received
// with the same split + check.  Each value is hashed once more (cert_hash,
// still a bijection): the routing fixed the top bits of the values a rank
// receives, and the bins need them uniform.  Same tile-major layout as
// k_join_window's pass 1 (pool1, jdir).
// One tile of pass 1: cnt (<= JT) values from v into pool1 tile `tile`, its
// bin starts into jdir.
__device__ __forceinline__ void cert_bin_tile(const unsigned long long *__restrict__ v, uint32_t cnt, uint32_t tile,
                                              unsigned long long *__restrict__ pool1, uint16_t *__restrict__ jdir) {
  constexpr uint32_t NW = JTT / 64, PT = JT / JTT;
  __shared__ uint64_t stg[JT];
  __shared__ uint32_t wcnt[CERT_BINS * NW], wsum[NW];
  for (uint32_t e = threadIdx.x; e < CERT_BINS * NW; e += JTT) wcnt[e] = 0;
  uint64_t hv[PT];
#pragma unroll
  for (int q = 0; q < (int)PT; ++q) {
    const uint32_t i = q * JTT + threadIdx.x;
    hv[q] = i < cnt ? cert_hash(v[i]) : 0;
  }
  __syncthreads();
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t rk[PT];
#pragma unroll
  for (int q = 0; q < (int)PT; ++q) {
    const bool ok = q * JTT + threadIdx.x < cnt;
    const uint32_t bin = (uint32_t)(hv[q] >> (64 - CERT_B1));
    const uint64_t peers = match6(bin, __ballot(ok));
    uint32_t prior = 0;
    if (ok) prior = wcnt[bin * NW + w];
    rk[q] = prior + __popcll(peers & lt);
    if (ok && (peers & lt) == 0) wcnt[bin * NW + w] = prior + __popcll(peers);
  }
  __syncthreads();
  block_scan_lds(wcnt, CERT_BINS * NW, wsum);
  if (threadIdx.x < CERT_BINS) jdir[(uint64_t)tile * CERT_BINS + threadIdx.x] = (uint16_t)wcnt[threadIdx.x * NW];
#pragma unroll
  for (int q = 0; q < (int)PT; ++q)
    if (q * JTT + threadIdx.x < cnt) stg[wcnt[(uint32_t)(hv[q] >> (64 - CERT_B1)) * NW + w] + rk[q]] = hv[q];
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < cnt; e += JTT) pool1[(uint64_t)tile * JT + e] = stg[e];
}

__global__ void __launch_bounds__(JTT) k_cert_bin(const unsigned long long *__restrict__ v, uint32_t n,
                                                  unsigned long long *__restrict__ pool1, uint16_t *__restrict__ jdir) {
  const uint32_t t0 = blockIdx.x * JT;
  cert_bin_tile(v + t0, min(n - t0, JT), blockIdx.x, pool1, jdir);
}

// The same over the guard's fixed segments as received (kmz_id_repeats_seg):
// segment r = [count, values...] of segw words; tps tiles per segment, tile
// sizes (a segment's last tiles short or empty) into tsz for the split.  The
// largest count any source sent (the next segment size; >= segw: it
// overflowed) into *maxc.
__global__ void __launch_bounds__(JTT) k_cert_bin_seg(const unsigned long long *__restrict__ segs, uint32_t world,
                                                      uint64_t segw, uint32_t tps,
                                                      unsigned long long *__restrict__ pool1,
                                                      uint16_t *__restrict__ jdir, uint16_t *__restrict__ tsz,
                                                      unsigned long long *__restrict__ maxc) {
  const uint32_t r = blockIdx.x / tps, lt = blockIdx.x % tps;
  const unsigned long long c = segs[(uint64_t)r * segw];
  const uint64_t have = c < segw - 1 ? c : segw - 1, b0 = (uint64_t)lt * JT;
  const uint32_t cnt = have > b0 ? (uint32_t)min<uint64_t>(JT, have - b0) : 0u;
  if (lt == 0 && threadIdx.x == 0) atomicMax(maxc, c);
  if (threadIdx.x == 0) tsz[blockIdx.x] = (uint16_t)cnt;
  cert_bin_tile(segs + (uint64_t)r * segw + 1 + b0, cnt, blockIdx.x, pool1, jdir);
}

void launch_cert_bin(hipStream_t s, const unsigned long long *v, uint32_t n, unsigned long long *pool1,
                     uint16_t *jdir) {
  if (!n) return;
  hipLaunchKernelGGL(k_cert_bin, dim3(join_tiles(n)), dim3(JTT), 0, s, v, n, pool1, jdir);
}

void launch_cert_bin_seg(hipStream_t s, const unsigned long long *segs, uint32_t world, uint64_t segw, uint32_t tps,
                         unsigned long long *pool1, uint16_t *jdir, uint16_t *tsz, unsigned long long *maxc) {
  hipLaunchKernelGGL(k_cert_bin_seg, dim3(world * tps), dim3(JTT), 0, s, segs, world, segw, tps, pool1, jdir, tsz,
                     maxc);
}

// pass 2: for one bin, the runs of TPC tiles -> 2^B2 sub-bins (dynamic LDS:
// PQ * 1024 u64 staging + 2 * 2^B2 u32).  (Reserving four sub-bins per
// 64-bit atomic, as 16-bit fields, measured 0.59 against 0.57 ms on config 3:
// the per-sub-bin reservations are not what bounds this pass.)  (PQ = 16, i.e. runs twice as long
// per sub-bin, measured slower: 0.59 against 0.55 ms on config 3.)
// With 2^8 pass-1 bins (B1 = 8, batches past ~10^8 ids) a chunk takes 4x the
// tiles (tile runs of ~8 records); a record then finds its tile run by a
// binary search over the run starts instead of the byte map.
template <int PQ, uint32_t B1>
__global__ void __launch_bounds__(1024) k_cert_split(const unsigned long long *__restrict__ pool1,
                                                     const uint16_t *__restrict__ jdir, uint32_t n, uint32_t chunks,
                                                     uint32_t B2, unsigned long long *__restrict__ pool2,
                                                     uint32_t cap2, unsigned int *__restrict__ cur2,
                                                     unsigned int *__restrict__ counters,
                                                     const uint16_t *__restrict__ tsz) {
  constexpr uint32_t BINS = 1u << B1;
  // ~32 ids per tile run at 64 bins, ~8 at 256
  constexpr uint32_t CERT_CHUNK = PQ * 1024, CERT_TPC = (PQ * 24) << (B1 - CERT_B1);
  constexpr bool MAP = CERT_TPC <= 256;  // record -> tile by a byte map (else a binary search)
  static_assert(CERT_TPC <= 1024, "one thread per tile run");
  extern __shared__ uint64_t dyn[];
  __shared__ uint32_t wsum[16], tcnt[CERT_TPC], toff[CERT_TPC];
  __shared__ uint8_t tof[MAP ? CERT_CHUNK : 1];  // record -> its tile in the chunk
  uint64_t *stg = dyn;
  const uint32_t M = 1u << B2;
  uint32_t *cnt = reinterpret_cast<uint32_t *>(dyn + CERT_CHUNK), *base = cnt + M;
  const uint32_t b = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const uint32_t ntiles = join_tiles(n), T0 = ch * CERT_TPC;
  if (T0 >= ntiles) return;
  const uint32_t nt = min(CERT_TPC, ntiles - T0);
  for (uint32_t k = threadIdx.x; k < M; k += blockDim.x) cnt[k] = 0;
  uint32_t c = 0;
  if (threadIdx.x < CERT_TPC) {
    uint32_t o = 0;
    if (threadIdx.x < nt) {
      // (three unconditional loads, in flight together: a load under a branch
      // -- tsz only for the guard's segment tiles, the next bin's offset only
      // below the last bin -- made the compiler wait for it at the merge,
      // before issuing the next)
      const uint32_t t = T0 + threadIdx.x;
      const uint16_t *row = jdir + (uint64_t)t * BINS;
      o = row[b];
      const uint32_t e1 = row[b + 1 < BINS ? b + 1 : b];
      const uint32_t tz = (tsz ? tsz : jdir)[t];
      const uint32_t tsize = tsz ? tz : min(JT, n - t * JT);  // (tsz: the guard's segment tiles)
      const uint32_t e = b + 1 < BINS ? e1 : tsize;
      c = e - o;
    }
    tcnt[threadIdx.x] = c;
    toff[threadIdx.x] = o;
  }
  __syncthreads();
  const uint32_t last = tcnt[CERT_TPC - 1];
  block_scan_lds(tcnt, CERT_TPC, wsum);  // tcnt := position of the tile's run in the chunk
  const uint32_t cn = tcnt[CERT_TPC - 1] + last;
  if (cn > CERT_CHUNK) {  // cannot happen for hashed ids short of ~20 sigma
    if (threadIdx.x == 0) atomicOr(&counters[C_CERT], CERT_OVF);
    return;
  }
  // record -> tile map: each tile's thread writes its run (one LDS lookup per
  // record below instead of a binary search of dependent LDS reads)
  if (MAP && threadIdx.x < nt)
    for (uint32_t j = 0, p = tcnt[threadIdx.x]; j < c; ++j) tof[p + j] = (uint8_t)threadIdx.x;
  __syncthreads();
  auto tile_of = [&](uint32_t e) -> uint32_t {
    if (MAP) return tof[e];
    uint32_t lo = 0;  // the last run starting at or before e (empty runs share the next one's start)
#pragma unroll
    for (uint32_t step = 512; step; step >>= 1)
      if (lo + step < nt && tcnt[lo + step] <= e) lo += step;
    return lo;
  };
  // gather the chunk's records straight into registers: every load is in
  // flight before any is used
  uint64_t h[PQ];
  uint32_t rk[PQ];
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const uint32_t e = q * 1024 + threadIdx.x;
    h[q] = 0;
    if (e < cn) {
      const uint32_t lo = tile_of(e);
      h[q] = pool1[(uint64_t)(T0 + lo) * JT + toff[lo] + (e - tcnt[lo])];
    }
  }
  const uint32_t sh = 64 - B1 - B2;
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const uint32_t e = q * 1024 + threadIdx.x;
    rk[q] = e < cn ? atomicAdd(&cnt[(uint32_t)(h[q] >> sh) & (M - 1)], 1u) : 0;
  }
  __syncthreads();
  // each sub-bin's global run, reserved with one device atomic; the returned
  // bases are stored to LDS only after the scan and the LDS scatter below, so
  // the atomics' round trip overlaps them (barriers here wait for LDS only)
  static_assert((1u << 12) <= 4 * 1024, "M <= 4 sub-bins per thread");
  uint32_t rb[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u) {
    const uint32_t k = u * 1024 + threadIdx.x;
    const uint32_t c = k < M ? cnt[k] : 0;
    if (c) rb[u] = atomicAdd(&cur2[(b << B2) | k], c);
  }
  block_scan_lds(cnt, M, wsum);  // cnt := local offsets (its first barrier orders the reads above)
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const uint32_t e = q * 1024 + threadIdx.x;
    if (e < cn) stg[cnt[(uint32_t)(h[q] >> sh) & (M - 1)] + rk[q]] = h[q];
  }
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u) {
    const uint32_t k = u * 1024 + threadIdx.x;
    if (k < M) base[k] = rb[u];
  }
  __syncthreads();
  bool ovf = false;
  for (uint32_t e = threadIdx.x; e < cn; e += blockDim.x) {
    const uint64_t x = stg[e];
    const uint32_t sb = (uint32_t)(x >> sh) & (M - 1);
    const uint32_t pos = base[sb] + e - cnt[sb];
    if (pos < cap2)
      pool2[(uint64_t)((b << B2) | sb) * cap2 + pos] = x;
    else
      ovf = true;
  }
  if (ovf) atomicOr(&counters[C_CERT], CERT_OVF);
}

// pass 2b (past 2^29 ids): each level-2 sub-bin, CERT_CHUNK records at a
// time, split again by the next B3 hash bits.  A single pass 2 into the
// 2^12 sub-bins 10^9 ids need wrote runs of ~2 records per chunk and sub-bin
// (8.6 ms at 10^9 against 0.54 ms at 10^8); two passes of 2^6 write runs of
// ~128.  Same ranking, reservations and write-out as k_cert_split.
template <int PQ>
__global__ void __launch_bounds__(1024) k_cert_resplit(const unsigned long long *__restrict__ pin, uint32_t cap_in,
                                                       const unsigned int *__restrict__ cur_in, uint32_t chunks,
                                                       uint32_t sh, uint32_t B3, unsigned long long *__restrict__ pout,
                                                       uint32_t cap_out, unsigned int *__restrict__ cur_out,
                                                       unsigned int *__restrict__ counters) {
  constexpr uint32_t CH = PQ * 1024;
  extern __shared__ uint64_t dyn[];
  __shared__ uint32_t wsum[16];
  uint64_t *stg = dyn;
  const uint32_t M = 1u << B3;
  uint32_t *cnt = reinterpret_cast<uint32_t *>(dyn + CH), *base = cnt + M;
  const uint32_t b = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const uint32_t m = min(cur_in[b], cap_in), e0 = ch * CH;
  if (e0 >= m) return;  // (uniform over the workgroup)
  const uint32_t cn = min(CH, m - e0);
  const unsigned long long *src = pin + (uint64_t)b * cap_in + e0;
  uint64_t h[PQ];
  uint32_t rk[PQ];
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const uint32_t e = q * 1024 + threadIdx.x;
    h[q] = e < cn ? src[e] : 0;
  }
  for (uint32_t k = threadIdx.x; k < M; k += blockDim.x) cnt[k] = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const uint32_t e = q * 1024 + threadIdx.x;
    rk[q] = e < cn ? atomicAdd(&cnt[(uint32_t)(h[q] >> sh) & (M - 1)], 1u) : 0;
  }
  __syncthreads();
  uint32_t rb = 0;  // (M <= 1024: one sub-bin per thread)
  {
    const uint32_t c = threadIdx.x < M ? cnt[threadIdx.x] : 0;
    if (c) rb = atomicAdd(&cur_out[(b << B3) | threadIdx.x], c);
  }
  block_scan_lds(cnt, M, wsum);
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
    const uint32_t e = q * 1024 + threadIdx.x;
    if (e < cn) stg[cnt[(uint32_t)(h[q] >> sh) & (M - 1)] + rk[q]] = h[q];
  }
  if (threadIdx.x < M) base[threadIdx.x] = rb;
  __syncthreads();
  bool ovf = false;
  for (uint32_t e = threadIdx.x; e < cn; e += blockDim.x) {
    const uint64_t x = stg[e];
    const uint32_t sb = (uint32_t)(x >> sh) & (M - 1);
    const uint32_t pos = base[sb] + e - cnt[sb];
    if (pos < cap_out)
      pout[(uint64_t)((b << B3) | sb) * cap_out + pos] = x;
    else
      ovf = true;
  }
  if (ovf) atomicOr(&counters[C_CERT], CERT_OVF);
}

// pass 3: exact duplicate check of one sub-bin, without probe loops.  Every
// hashed id goes to bucket (low bits of the hash) of an LDS table of 8-slot
// buckets: one returning LDS add gives its slot, one store places it; ids
// past a bucket's 8 slots go to an overflow list.  Equal ids share a bucket,
// so after one barrier each thread compares the pairs of its buckets' slots,
// and each overflow id its bucket's slots and the other overflow ids.
// cert_plan keeps a sub-bin at ~3 ids per bucket (a handful overflow).
constexpr uint32_t CK_NB = 1024, CK_S = 8;  // buckets, slots per bucket (32 KB of words; 64 KB of ids)
#ifndef KMZ_CK_OVF
#define KMZ_CK_OVF 256
#endif
constexpr uint32_t CK_OVF = KMZ_CK_OVF;     // overflow ids (2 KB)
// threads per pass-3 workgroup: with 8-byte slots (76 KB of LDS, two
// workgroups per CU) 1024 threads (six ids each) kept twice the waves of 512
// in flight: check 0.296 -> 0.257 ms on config 3 (profiles/r04/ab/cct/).
// With the 32-bit words (39 KB) four workgroups of 512 fit: 0.253 -> 0.238 ms
// at 10^8, 2.41 -> 2.11 ms at 10^9 (profiles/r06/ab/ckfp2*; the words at
// 1024 threads were slower than the 8-byte slots, 0.262 ms).
#ifndef KMZ_CCT
#define KMZ_CCT 512
#endif
constexpr int CCT = KMZ_CCT;
constexpr int CK_PER = 6144 / CCT;          // ids per thread: sub-bins <= CCT * CK_PER = 6144 (cert_plan)
static_assert(CCT * CK_PER >= CERT_SET * 3 / 4, "a sub-bin must fit the workgroup's registers");
// (A persistent form that loads the next sub-bin's ids while checking the
// current one measured slower: 0.31 against 0.275 ms on config 3.)
#ifndef KMZ_CK_FP
#define KMZ_CK_FP 1
#endif
// (An open-addressing form -- each id claims the first free slot from its
// home by an LDS compare-and-swap -- measured slower than the 8-slot buckets.)
#if KMZ_CK_FP
// The buckets hold 32-bit words instead of the ids: the 19 hash bits above
// the bucket's 10 (a fingerprint) and the id's 13-bit position in the
// sub-bin.  The pair test compares words' fingerprints; only a fingerprint
// hit (~2^-19 per pair, a few hundred per 10^8 ids) reads the two ids back
// from the pool and compares them whole, so the verdict stays exact.  Half
// the LDS bytes written and read, and 32-bit compares.
constexpr uint32_t CK_FPSH = 13;  // word = fp19 << 13 | position
static_assert(CCT * CK_PER <= (1u << CK_FPSH), "positions fit the word");
__device__ __forceinline__ uint32_t ck_fp(uint64_t h) { return (uint32_t)(h >> 10) & 0x7FFFFu; }
__global__ void __launch_bounds__(CCT) k_cert_check(const unsigned long long *__restrict__ pool, uint32_t cap,
                                                   const unsigned int *__restrict__ cur, uint32_t cur_stride,
                                                   unsigned int *__restrict__ counters) {
  __shared__ uint4 bkt4[CK_NB * CK_S / 4];
  __shared__ uint32_t bcnt[CK_NB];
  __shared__ unsigned long long ovf[CK_OVF];
  __shared__ uint32_t novf;
  uint32_t *bkt = reinterpret_cast<uint32_t *>(bkt4);
  const uint32_t sb = blockIdx.x;
  const uint32_t m = min(cur[(uint64_t)sb * cur_stride], cap);
  if (m == 0) return;
  const unsigned long long *src = pool + (uint64_t)sb * cap;
  uint64_t h[CK_PER];
#pragma unroll
  for (int q = 0; q < CK_PER; ++q) {  // every load in flight while the counters are cleared
    const uint32_t e = q * CCT + threadIdx.x;
    h[q] = e < m ? src[e] : 0;
  }
  for (uint32_t k = threadIdx.x; k < CK_NB; k += CCT) bcnt[k] = 0;
  if (threadIdx.x == 0) novf = 0;
  __syncthreads();
  bool lost = false;
#pragma unroll
  for (int q = 0; q < CK_PER; ++q) {
    if (h[q] == 0) continue;  // padding (and cert_hash(0) == 0: span id 0, reported as F_ZERO_ID)
    const uint32_t b = (uint32_t)h[q] & (CK_NB - 1);
    const uint32_t slot = atomicAdd(&bcnt[b], 1u);
    if (slot < CK_S) {
      // a bucket is 32 B (8 banks): slot s at position s ^ ((b >> 3) & 7), so
      // the first slots of the buckets spread over all 64 banks
      bkt[b * CK_S + (slot ^ ((b >> 3) & 7))] = (ck_fp(h[q]) << CK_FPSH) | (q * CCT + threadIdx.x);
    } else {
      const uint32_t o = atomicAdd(&novf, 1u);
      if (o < CK_OVF) ovf[o] = h[q];
      else lost = true;
    }
  }
  __syncthreads();
  bool dup = false;
  for (uint32_t b = threadIdx.x; b < CK_NB; b += CCT) {
    const uint32_t c = min(bcnt[b], CK_S);
    if (c < 2) continue;
    // lanes b and b + 8 start on different halves of their buckets (same
    // banks otherwise within a ds_read_b128 group)
    const uint32_t r = (b >> 3) & 1, sw = (b >> 3) & 7;
    const uint4 v0 = bkt4[b * 2 + r], v1 = bkt4[b * 2 + (r ^ 1)];
    const uint32_t x[CK_S] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    bool ok[CK_S];
#pragma unroll
    for (uint32_t j = 0; j < CK_S; ++j) ok[j] = ((((j >> 2) ^ r) << 2 | (j & 3)) ^ sw) < c;
    bool hit = false;
#pragma unroll
    for (uint32_t i = 0; i < CK_S; ++i)
#pragma unroll
      for (uint32_t j = i + 1; j < CK_S; ++j) hit |= ok[i] && ok[j] && ((x[i] ^ x[j]) >> CK_FPSH) == 0;
    if (hit) {  // rare: confirm on the ids themselves
      for (uint32_t i = 0; i < CK_S; ++i)
        for (uint32_t j = i + 1; j < CK_S; ++j)
          if (ok[i] && ok[j] && ((x[i] ^ x[j]) >> CK_FPSH) == 0)
            dup |= src[x[i] & ((1u << CK_FPSH) - 1)] == src[x[j] & ((1u << CK_FPSH) - 1)];
    }
  }
  // overflow ids: against their (full) bucket's words and the later overflow ids
  const uint32_t no = min(novf, CK_OVF);
  for (uint32_t o = threadIdx.x; o < no; o += CCT) {
    const uint64_t v = ovf[o];
    const uint32_t b = (uint32_t)v & (CK_NB - 1), f = ck_fp(v);
    for (uint32_t j = 0; j < CK_S; ++j) {
      const uint32_t w = bkt[b * CK_S + j];
      if ((w >> CK_FPSH) == f) dup |= src[w & ((1u << CK_FPSH) - 1)] == v;
    }
    for (uint32_t t = o + 1; t < no; ++t) dup |= ovf[t] == v;
  }
  if (dup) atomicOr(&counters[C_CERT], CERT_DUP);
  if (lost) atomicOr(&counters[C_CERT], CERT_OVF);
}
#else
__global__ void __launch_bounds__(CCT) k_cert_check(const unsigned long long *__restrict__ pool, uint32_t cap,
                                                   const unsigned int *__restrict__ cur, uint32_t cur_stride,
                                                   unsigned int *__restrict__ counters) {
  __shared__ ulonglong2 bkt2[CK_NB * CK_S / 2];
  __shared__ uint32_t bcnt[CK_NB];
  __shared__ unsigned long long ovf[CK_OVF];
  __shared__ uint32_t novf;
  unsigned long long *bkt = reinterpret_cast<unsigned long long *>(bkt2);
  const uint32_t sb = blockIdx.x;
  const uint32_t m = min(cur[(uint64_t)sb * cur_stride], cap);
  if (m == 0) return;
  const unsigned long long *src = pool + (uint64_t)sb * cap;
  uint64_t h[CK_PER];
#pragma unroll
  for (int q = 0; q < CK_PER; ++q) {  // every load in flight while the counters are cleared
    const uint32_t e = q * CCT + threadIdx.x;
    h[q] = e < m ? src[e] : 0;
  }
  for (uint32_t k = threadIdx.x; k < CK_NB; k += CCT) bcnt[k] = 0;
  if (threadIdx.x == 0) novf = 0;
  __syncthreads();
  bool lost = false;
#pragma unroll
  for (int q = 0; q < CK_PER; ++q) {
    if (h[q] == 0) continue;  // padding (and cert_hash(0) == 0: span id 0, reported as F_ZERO_ID)
    const uint32_t b = (uint32_t)h[q] & (CK_NB - 1);
    const uint32_t slot = atomicAdd(&bcnt[b], 1u);
    if (slot < CK_S) {
      // slot s of bucket b at position s ^ ((b >> 1) & 7): a bucket's 64 B
      // cover 16 of the 32 banks a ds_write_b64 group sees, so without the
      // swizzle the first slots of all buckets land on the same few banks
      bkt[b * CK_S + (slot ^ ((b >> 1) & 7))] = h[q];
    } else {
      const uint32_t o = atomicAdd(&novf, 1u);
      if (o < CK_OVF) ovf[o] = h[q];
      else lost = true;
    }
  }
  __syncthreads();
  bool dup = false;
  // pairs within each bucket's slots
  for (uint32_t b = threadIdx.x; b < CK_NB; b += CCT) {
    const uint32_t c = min(bcnt[b], CK_S);
    if (c < 2) continue;
    uint64_t x[CK_S];
    // a bucket is 64 B (16 banks): read in lane order, lanes b, b+4, b+8,
    // b+12 of a 16-lane group would hit the same four banks (4-way conflict on
    // every ds_read_b128); rotating each lane's start by b/4 spreads a group
    // over all 64 banks.  (Slot order does not matter to the pair test.)
    const uint32_t rot = (b >> 2) & 3, sw = (b >> 1) & 7;
#pragma unroll
    for (uint32_t j = 0; j < CK_S; j += 2) {
      const uint32_t jj = (((j >> 1) + rot) & 3) << 1;
      const ulonglong2 v = bkt2[(b * CK_S + jj) / 2];
      x[j] = v.x;
      x[j + 1] = v.y;
    }
    // (x[] holds the positions in rotated order; position p holds slot p ^ sw,
    // valid iff that slot < c)
    bool ok[CK_S];
#pragma unroll
    for (uint32_t j = 0; j < CK_S; ++j) ok[j] = ((((((j >> 1) + rot) & 3) << 1) | (j & 1)) ^ sw) < c;
#pragma unroll
    for (uint32_t i = 0; i < CK_S; ++i)
#pragma unroll
      for (uint32_t j = i + 1; j < CK_S; ++j) dup |= ok[i] && ok[j] && x[i] == x[j];
  }
  // overflow ids: against their bucket's slots and the later overflow ids
  const uint32_t no = min(novf, CK_OVF);
  for (uint32_t o = threadIdx.x; o < no; o += CCT) {
    const uint64_t v = ovf[o];
    const uint32_t b = (uint32_t)v & (CK_NB - 1);
#pragma unroll
    for (uint32_t j = 0; j < CK_S; ++j) dup |= bkt[b * CK_S + j] == v;  // (a full bucket: all 8 slots written)
    for (uint32_t t = o + 1; t < no; ++t) dup |= ovf[t] == v;
  }
  if (dup) atomicOr(&counters[C_CERT], CERT_DUP);
  if (lost) atomicOr(&counters[C_CERT], CERT_OVF);
}
#endif

// ---- MISS parents: semi-join of the missing parent ids against all span ids
__device__ __forceinline__ uint64_t mslot(uint64_t key, uint32_t mcap) { return slot_of(key ^ 0x7F4A7C159E3779B9ull, mcap); }

// The MISS/PEND kernels are launched on every join run without a host round
// trip; they read the join's counters first and return when there is nothing
// to do (or when the miss table is too small: the host grows it and runs
// again).  They run even when the certificate failed, so that cparent is
// always well formed (indices < n, NONE or CYC) for the kernels after them.
__device__ __forceinline__ bool miss_skip(const unsigned int *counters, uint32_t mcap) {
  const uint32_t m = counters[C_MISS];
  if (m == 0) return true;
  if ((uint64_t)m * 2 > mcap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(const_cast<unsigned int *>(counters) + C_FLAGS, F_MISS_OVERFLOW);
    return true;
  }
  return false;
}

__global__ void __launch_bounds__(256) k_miss_insert(const uint64_t *__restrict__ pid, const uint32_t *__restrict__ dp,
                                                     uint32_t n, unsigned long long *__restrict__ mkey, uint32_t mcap,
                                                     const unsigned int *counters) {
  if (miss_skip(counters, mcap)) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (dp[i] != MISSV) continue;
    const uint64_t key = pid[i];
    uint32_t pos = (uint32_t)mslot(key, mcap);
    for (uint32_t z = 0; z < mcap; ++z) {
      unsigned long long c = atomicCAS(&mkey[pos], 0ull, (unsigned long long)key);
      if (c == 0 || c == key) break;
      pos = pos + 1 == mcap ? 0 : pos + 1;
    }
  }
}

__global__ void __launch_bounds__(256) k_miss_probe(const uint64_t *__restrict__ sid, uint32_t n,
                                                    const unsigned long long *__restrict__ mkey,
                                                    uint32_t *__restrict__ mval, uint32_t mcap,
                                                    const unsigned int *counters) {
  if (miss_skip(counters, mcap)) return;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint64_t key = sid[j];
    if (key == 0) continue;
    uint32_t pos = (uint32_t)mslot(key, mcap);
    for (uint32_t z = 0; z < mcap; ++z) {
      const unsigned long long c = mkey[pos];
      if (c == 0) break;
      if (c == key) {
        mval[pos] = j;  // ids are unique (certificate): one writer per slot
        break;
      }
      pos = pos + 1 == mcap ? 0 : pos + 1;
    }
  }
}

__global__ void __launch_bounds__(256) k_miss_fix(const uint64_t *__restrict__ pid, uint32_t *__restrict__ dp,
                                                  uint32_t n, const unsigned long long *__restrict__ mkey,
                                                  const uint32_t *__restrict__ mval, uint32_t mcap,
                                                  const unsigned int *counters) {
  if (miss_skip(counters, mcap)) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (dp[i] != MISSV) continue;
    const uint64_t key = pid[i];
    uint32_t pos = (uint32_t)mslot(key, mcap), r = NONE;
    for (uint32_t z = 0; z < mcap; ++z) {
      const unsigned long long c = mkey[pos];
      if (c == 0) break;
      if (c == key) {
        r = mval[pos];
        break;
      }
      pos = pos + 1 == mcap ? 0 : pos + 1;
    }
    dp[i] = r;
  }
}

// PEND chains over the global dp array
__global__ void __launch_bounds__(256) k_pend(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ dp,
                                              uint32_t n, uint32_t *__restrict__ cparent,
                                              const unsigned int *counters) {
  if (counters[C_PEND] == 0) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (cparent[i] != PEND) continue;
    uint32_t j = dp[i], hops = 0, cp;
    for (;;) {
      if (j >= n) {
        cp = NONE;
        break;
      }
      if (kind[j] != KIND_CLIENT) {
        cp = j;
        break;
      }
      if (++hops > MAX_DEPTH) {
        cp = CYC;
        break;
      }
      j = dp[j];
    }
    cparent[i] = cp;
  }
}

// ---------------------------------------------------------------------------

// (Measured and dropped at 10^9 ids, where this pass 2 takes 8.7 ms against
// 0.51 ms at 10^8: R rounds of 8192 records per workgroup with one
// reservation per (workgroup, sub-bin) -- 8.85 ms, so the 6.7e8 device-scope
// reservations are not what bounds it; a pass 3 that holds a 4x larger
// sub-bin in registers and checks it in 4 phases, so that pass 2 writes runs
// 4x longer -- split 8.9 -> 7.4 ms but check 2.9 -> 5.6 ms, and at 10^8
// split 0.56 -> 0.49, check 0.27 -> 0.50 ms; 8 phases worse still.)
bool cert_plan(uint32_t n, CertPlan *pl, bool wide, bool force_wide) {
  // sub-bins of <= ~3072 ids (4096 with 2^8 bins): a check workgroup holds 6144
  uint32_t B1 = CERT_B1, lim = 3072;
  // (2^8 bins past ~1.0e8 ids and up to 2^29: measured at 5e8 ids, join +
  // split + check 11.55 -> 11.01 ms; at 1e9, 22.0 -> 22.6 ms -- the wider
  // join's 8 ballots and 2048-entry scan cost more than the split's 4x longer
  // runs gain, whose time there is bound by its one-workgroup-per-CU latency)
  if (force_wide || (wide && (uint64_t)n > (3072ull << (CERT_B1 + 9)) && n <= (1u << 29))) {
    B1 = CERT_B1W;
    lim = 4096;
  }
  uint32_t B2 = 0;
  while (B2 < 12 && (uint64_t)n > ((uint64_t)lim << (B1 + B2))) ++B2;
  const double mean2 = (double)n / ((uint64_t)1 << (B1 + B2));
  pl->B1 = B1;
  pl->B2 = B2;
  pl->cap2 = (uint32_t)(mean2 * 1.15) + 256;
  pl->B3 = pl->cap3 = pl->chunks3 = 0;
  const uint32_t tpc = (CERT_PQ * 24) << (B1 - CERT_B1);
  pl->chunks = (join_tiles(n) + tpc - 1) / tpc;
  // runs shorter than ~16 records per (chunk, sub-bin): split in two levels
  if (B2 > 9) {
    const uint32_t b2 = B2 / 2;
    pl->B3 = B2 - b2;
    pl->B2 = b2;
    pl->cap3 = pl->cap2;
    pl->cap2 = (uint32_t)((double)n / ((uint64_t)1 << (B1 + b2)) * 1.02) + 4096;
    pl->chunks3 = (pl->cap2 + CERT_PQ * 1024 - 1) / (CERT_PQ * 1024);
    return pl->cap3 <= CERT_SET * 3 / 4;
  }
  return pl->cap2 <= CERT_SET * 3 / 4;
}

static uint64_t cert_level2_words(const CertPlan &pl) { return ((uint64_t)1 << (pl.B1 + pl.B2)) * pl.cap2; }
uint64_t cert_pool2_bytes(const CertPlan &pl) {
  return (cert_level2_words(pl) + (pl.B3 ? ((uint64_t)1 << (pl.B1 + pl.B2 + pl.B3)) * pl.cap3 : 0)) * 8;
}
uint64_t cert_cur_words(const CertPlan &pl) {
  return ((uint64_t)1 << (pl.B1 + pl.B2)) + (pl.B3 ? ((uint64_t)1 << (pl.B1 + pl.B2 + pl.B3)) : 0);
}

uint64_t cert_pool1_words(uint32_t n) { return (uint64_t)join_tiles(n) * JT; }
uint64_t cert_dir_entries(uint32_t n, const CertPlan &pl) { return (uint64_t)join_tiles(n) << pl.B1; }

void launch_join(hipStream_t s, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind, uint32_t n,
                 uint32_t *cparent, uint32_t *dp, unsigned long long *pool1, uint16_t *jdir, unsigned int *counters,
                 const CertPlan &pl, uint32_t ablate, const JoinRoute &rt) {
  if (!n) return;
  if (pl.B1 == CERT_B1W)
    hipLaunchKernelGGL(k_join_window<CERT_B1W>, dim3(join_tiles(n)), dim3(JTT), 0, s, sid, pid, kind, n, cparent, dp,
                       pool1, jdir, counters, ablate, rt);
  else
    hipLaunchKernelGGL(k_join_window<CERT_B1>, dim3(join_tiles(n)), dim3(JTT), 0, s, sid, pid, kind, n, cparent, dp,
                       pool1, jdir, counters, ablate, rt);
}

void launch_cert_split(hipStream_t s, uint32_t n, const unsigned long long *pool1, const uint16_t *jdir,
                       const CertPlan &pl, unsigned long long *pool2, unsigned int *cur2, unsigned int *counters,
                       const uint16_t *tsz) {
  if (!n) return;
  const size_t lds = CERT_PQ * 1024 * 8 + (size_t)2 * (1u << pl.B2) * 4;
  if (pl.B1 == CERT_B1W)
    hipLaunchKernelGGL((k_cert_split<CERT_PQ, CERT_B1W>), dim3((1u << CERT_B1W) * pl.chunks), dim3(1024), lds, s, pool1,
                       jdir, n, pl.chunks, pl.B2, pool2, pl.cap2, cur2, counters, tsz);
  else
    hipLaunchKernelGGL((k_cert_split<CERT_PQ, CERT_B1>), dim3(CERT_BINS * pl.chunks), dim3(1024), lds, s, pool1, jdir, n,
                       pl.chunks, pl.B2, pool2, pl.cap2, cur2, counters, tsz);
  if (pl.B3) {  // level 3: after level 2 in the same pool and counter block
    const uint32_t n2 = 1u << (pl.B1 + pl.B2);
    const size_t lds3 = CERT_PQ * 1024 * 8 + (size_t)2 * (1u << pl.B3) * 4;
    hipLaunchKernelGGL(k_cert_resplit<CERT_PQ>, dim3(n2 * pl.chunks3), dim3(1024), lds3, s, pool2, pl.cap2, cur2,
                       pl.chunks3, 64 - pl.B1 - pl.B2 - pl.B3, pl.B3, pool2 + cert_level2_words(pl), pl.cap3, cur2 + n2,
                       counters);
  }
}

void launch_cert_check(hipStream_t s, uint32_t n, const CertPlan &pl, const unsigned long long *pool2,
                       const unsigned int *cur2, unsigned int *counters) {
  if (!n) return;
  if (pl.B3)
    hipLaunchKernelGGL(k_cert_check, dim3(1u << (pl.B1 + pl.B2 + pl.B3)), dim3(CCT), 0, s,
                       pool2 + cert_level2_words(pl), pl.cap3, cur2 + (1u << (pl.B1 + pl.B2)), 1u, counters);
  else
    hipLaunchKernelGGL(k_cert_check, dim3(1u << (pl.B1 + pl.B2)), dim3(CCT), 0, s, pool2, pl.cap2, cur2, 1u, counters);
}

void launch_miss(hipStream_t s, const uint64_t *sid, const uint64_t *pid, uint32_t *dp, uint32_t n,
                 unsigned long long *mkey, uint32_t *mval, uint32_t mcap, const unsigned int *counters) {
  if (!n) return;
  const uint32_t g = std::min<uint32_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_miss_insert, dim3(g), dim3(256), 0, s, pid, dp, n, mkey, mcap, counters);
  hipLaunchKernelGGL(k_miss_probe, dim3(g), dim3(256), 0, s, sid, n, mkey, mval, mcap, counters);
  hipLaunchKernelGGL(k_miss_fix, dim3(g), dim3(256), 0, s, pid, dp, n, mkey, mval, mcap, counters);
}

void launch_pend(hipStream_t s, const uint8_t *kind, const uint32_t *dp, uint32_t n, uint32_t *cparent,
                 const unsigned int *counters) {
  if (!n) return;
  const uint32_t g = std::min<uint32_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_pend, dim3(g), dim3(256), 0, s, kind, dp, n, cparent, counters);
}

}  // namespace kmz

extern "C" int kmz__debug_join(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmz::g_join_dbg), sizeof(kmz::g_join_dbg)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(kmz::g_join_dbg), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
