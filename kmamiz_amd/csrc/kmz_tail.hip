// kmz_tail.hip -- the service-level tail over the reduced edge set (SURVEY.md
// 8a row a8; config 5's "service risk/instability/coupling recompute").
//
// The reference derives every service metric from the endpoint rows of
// EndpointDependencies.toServiceDependencies (EndpointDependencies.ts:369-470):
// per service (the rows' uniqueServiceName) it collects the distinct link keys
//
//     linked usn \t method \t labelName \t type \t distance          (419-421)
//
// over the dependingOn (type SERVER) and dependingBy (type CLIENT) entries of
// its rows, then counts them per linked service (the key's first three
// fields) and distance (427-466).  Instability (614-641), ACS / coupling
// (643-657, RiskAnalyzer.ts:145-169), the relying factor (RiskAnalyzer.ts:
// 124-137) and cohesion (565-612) are small functions of those counts.
//
// On the reduced form a row's entries are the run's edge keys
// (anc, desc, distance, on): desc's row has (anc, distance) in dependingBy,
// and anc's row -- when the ancestor occurrence is a SERVER span (on) -- has
// (desc, distance) in dependingOn.  So one pass over the edge keys produces
// every link key of every service:
//
//     (svc[desc], cls[anc], CLIENT, d)              always
//     (svc[anc],  cls[desc], SERVER, d)             if on
//
// where cls = interned (uniqueServiceName, method, labelName) and svc =
// interned uniqueServiceName of an endpoint (host-supplied maps: the label map
// is the host's, as in EndpointDependencies.label()).  The link keys are
// bucketed by hash (k_tail_part) and each bucket deduplicated in LDS
// (k_tail_dedup); a key's first occurrence adds itself to its (svc,
// lsvc(cls), d) detail counters (count, dependingBy, dependingOn).  Cohesion
// needs, per service, the distinct
// (consumer service, consumed endpoint) pairs at distance 1: the pair set
// (desc, usn[anc]) does the same on its own winners.  `hasin` marks rows with
// a non-empty dependingBy (a service with a row without one is a gateway,
// RiskAnalyzer.ts:155-158).
//
// Everything is integer; the fp64 metrics are finished on the host over at
// most services x linked services x distances detail rows.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_kernels.h"

namespace kmz {

constexpr uint32_t TAIL_PROBE_MAX = 1024;
// per-service counters (8 u32 per service, kmz_tail_service_stats)
constexpr uint32_t TS_NBY = 0, TS_NON = 1, TS_AIS = 2, TS_ADS = 3, TS_CONSUMERS = 4, TS_CONSUMES = 5, TS_ROWS = 6,
                   TS_GATEWAY = 7;
static_assert(TS_NON == TS_NBY + 1 && TS_ADS == TS_AIS + 1, "the link type (0 CLIENT, 1 SERVER) selects the counter");

// insert `key` (nonzero) into an open-addressing set; true if this call put it there
__device__ __forceinline__ bool tail_set_put(unsigned long long *__restrict__ set, uint64_t cap, uint64_t key,
                                             uint32_t *flags) {
  uint64_t pos = slot_of(key, cap);
  for (uint32_t z = 0; z < TAIL_PROBE_MAX; ++z) {
    unsigned long long cur = set[pos];
    if (cur == key) return false;
    if (cur == 0) {
      cur = atomicCAS(&set[pos], 0ull, (unsigned long long)key);
      if (cur == 0) return true;
      if (cur == key) return false;
    }
    pos = pos + 1 == cap ? 0 : pos + 1;
  }
  *flags |= F_TRIPLE_OVERFLOW;
  return false;
}

// the slot of `key` in an aggregation table (inserted if new), or cap on overflow
__device__ __forceinline__ uint64_t tail_agg_slot(unsigned long long *__restrict__ akey, uint64_t cap, uint64_t key,
                                                  uint32_t *flags) {
  uint64_t pos = slot_of(key, cap);
  for (uint32_t z = 0; z < TAIL_PROBE_MAX; ++z) {
    unsigned long long cur = akey[pos];
    if (cur == key) return pos;
    if (cur == 0) {
      cur = atomicCAS(&akey[pos], 0ull, (unsigned long long)key);
      if (cur == 0 || cur == key) return pos;
    }
    pos = pos + 1 == cap ? 0 : pos + 1;
  }
  *flags |= F_TRIPLE_OVERFLOW;
  return cap;
}

// Link keys repeat, but not enough for a cache: config 5's 2.7e7 link keys
// per step (1e8 spans) hold a few million distinct ones (1.3e6 of 6.6e6 at
// 4.5e6 spans), and their details (service, linked service, distance) nearly
// as many (9.1e5 there).  The round-3 k_tail_links put every link key in a
// global set behind a per-workgroup LDS cache and added every first
// occurrence into a global detail table: millions of dependent device-scope
// probes and atomics (1.35 ms, waves waiting on memory 78 % of their cycles).
// Here both dedups stay in LDS by partitioning on the (service, linked
// service) pair -- every link key, detail and pair flag of a pair lands in one
// bucket:
//   k_tail_part   per edge key its link keys, minus those its workgroup has
//                 already emitted (a direct-mapped LDS filter: hot keys), into
//                 one of 2^bits buckets by a hash of (service, linked service)
//                 -- an LDS counting sort per 2048 edge keys; every workgroup
//                 owns a slab of each bucket and counts its fill in LDS (one
//                 device atomic per bucket and step on 2^11 shared counters
//                 was 1.2e7 contended atomics per run); cohesion pairs into
//                 the pair set.
//   k_tail_dedup  one 1024-thread workgroup per bucket: its link keys (the
//                 workgroups' slabs, located by a scan of their fills) into an
//                 LDS set; each distinct key into its detail (LDS table:
//                 count, dependingBy, dependingOn) and its pair's flags (a
//                 by / on link at any distance / at distance 1); the details
//                 written out as kmz_tail_detail records (one reservation per
//                 bucket) with their relying-factor sums, each pair's flags
//                 added to its service's counters.
// A bucket whose LDS tables are too small, a full slab or an output that is
// full flags the run and the host repeats the tail with twice the buckets (or
// larger slabs or output): exact either way.
constexpr uint32_t TA_T = 512, TA_U = 4;         // pass A: threads, edge keys per thread and step
constexpr uint32_t TA_STEP = TA_T * TA_U;        // 2048 edge keys, <= 4096 link keys per step
constexpr uint32_t TA_SEEN = 2048;               // pass A: LDS filter of emitted link keys (16 KB)
constexpr uint32_t TAIL_PSEEN = 512;
constexpr uint32_t TAIL_BMAX = 12;               // buckets: 2^11 (2^12 after an overflow)
constexpr uint32_t TB_T = 1024;                  // pass B: one workgroup per CU
constexpr uint32_t TB_LSET = 8192, TB_DSET = 2048, TB_PSET = 2048;  // LDS: 64 + 40 + 24 KB
constexpr uint32_t TA_GRID = 512;                // pass A workgroups (slabs per bucket)
// a link key's (service, linked service) pair and its bucket
__device__ __forceinline__ uint32_t tail_bucket(uint64_t pair, uint32_t bits) {
  return (uint32_t)(mix64(pair ^ 0x2545F4914F6CDD1Dull) >> (64 - bits));
}
// insert k (nonzero) into an LDS open-addressing table of 2^lb slots -> its
// slot, or ~0u when 64 probes find no room
__device__ __forceinline__ uint32_t lds_slot(unsigned long long *tab, uint32_t lb, uint64_t k) {
  uint32_t h = (uint32_t)mix64(k) & ((1u << lb) - 1);
  for (uint32_t z = 0; z < 64; ++z) {
    const unsigned long long cur = tab[h];
    if (cur == k) return h;
    if (cur == 0) {
      const unsigned long long was = atomicCAS(&tab[h], 0ull, (unsigned long long)k);
      if (was == 0 || was == k) return h;
    }
    h = (h + 1) & ((1u << lb) - 1);
  }
  return ~0u;
}

// link key: svc << 40 | cls << 16 | type << 15 | d   (type 1 = SERVER / dependingOn)
// detail key: svc << 40 | lsvc << 16 | d
// pair key: (desc + 1) << 32 | consumer usn;  pair detail key: (svc + 1) << 32 | consumer usn
template <uint32_t BITS>
__global__ void __launch_bounds__(TA_T) k_tail_part(const unsigned long long *__restrict__ keys,
                                                    const unsigned long long *__restrict__ n_keys,
                                                    const uint32_t *__restrict__ svc, const uint32_t *__restrict__ cls,
                                                    const uint32_t *__restrict__ lsvc_of_cls,
                                                    const uint32_t *__restrict__ usn, uint32_t n_ep, uint32_t n_cls,
                                                    unsigned long long *__restrict__ lbkt, uint32_t slab,
                                                    uint32_t *__restrict__ lbn,
                                                    unsigned long long *__restrict__ pset, uint64_t pcap,
                                                    unsigned long long *__restrict__ pkey, uint32_t *__restrict__ pval,
                                                    uint64_t pacap, uint8_t *__restrict__ hasin,
                                                    uint32_t *__restrict__ sstat, unsigned int *__restrict__ counters,
                                                    uint32_t knobs) {
  const uint64_t n = *n_keys;
  constexpr uint32_t nb = 1u << BITS, bits = BITS;
  __shared__ unsigned long long stg[2 * TA_STEP];  // 32 KB
  __shared__ uint32_t hist[nb], fill[nb], wsum[TA_T / 64 + 1];  // this step's offsets; the slabs' fill
  __shared__ unsigned long long pseen[TAIL_PSEEN], lseen[TA_SEEN];
  __shared__ uint16_t bk[2 * TA_STEP];  // each staged key's bucket
  for (uint32_t x = threadIdx.x; x < TAIL_PSEEN; x += TA_T) pseen[x] = 0;
  for (uint32_t x = threadIdx.x; x < TA_SEEN; x += TA_T) lseen[x] = 0;
  for (uint32_t x = threadIdx.x; x < nb; x += TA_T) fill[x] = 0;
  uint32_t flags = 0, won_p = 0;
  // the next step's edge keys are loaded while this step is sorted and written
  uint64_t kn[TA_U];
  auto load = [&](uint64_t s1) {
#pragma unroll
    for (int u = 0; u < (int)TA_U; ++u) {
      const uint64_t i = s1 + u * TA_T + threadIdx.x;
      kn[u] = i < n ? keys[i] : 0;
    }
  };
  load((uint64_t)blockIdx.x * TA_STEP);
  for (uint64_t s0 = (uint64_t)blockIdx.x * TA_STEP; s0 < n; s0 += (uint64_t)gridDim.x * TA_STEP) {
    uint64_t kq[TA_U];
#pragma unroll
    for (int u = 0; u < (int)TA_U; ++u) kq[u] = kn[u];
    load(s0 + (uint64_t)gridDim.x * TA_STEP);
    uint32_t cq_a[TA_U], cq_s[TA_U], sv_a[TA_U], sv_s[TA_U], us_a[TA_U];
#pragma unroll
    for (int u = 0; u < (int)TA_U; ++u) {
      const uint32_t a = (uint32_t)(kq[u] >> 40), s = (uint32_t)(kq[u] >> 16) & 0xFFFFFFu;
      const bool in = a < n_ep && s < n_ep;
      cq_a[u] = in ? cls[a] : NONE;
      cq_s[u] = in ? cls[s] : NONE;
      sv_a[u] = in ? svc[a] : 0;
      sv_s[u] = in ? svc[s] : 0;
      us_a[u] = in ? usn[a] : 0;
    }
    for (uint32_t x = threadIdx.x; x < nb; x += TA_T) hist[x] = 0;
    __syncthreads();
    uint64_t lk[2 * TA_U];
    uint32_t rk[2 * TA_U], lb[2 * TA_U];
#pragma unroll
    for (int u = 0; u < (int)TA_U; ++u) {
      lk[2 * u] = lk[2 * u + 1] = 0;
      if (s0 + u * TA_T + threadIdx.x >= n) continue;
      const uint64_t k = kq[u];
      const uint32_t a = (uint32_t)(k >> 40), s = (uint32_t)(k >> 16) & 0xFFFFFFu, d = (uint32_t)(k >> 1) & 0x7FFFu;
      const bool on = (k & 1) != 0;
      if (a >= n_ep || s >= n_ep || cq_a[u] >= n_cls || cq_s[u] >= n_cls) {
        flags |= F_RANGE;
        continue;
      }
      if (!hasin[s]) hasin[s] = 1;  // (read first: ~10^7 keys share ~10^4 bytes)
      if (!(knobs & 1)) {  // (diagnostic knob 1: no link keys -- timing only, wrong results)
        // desc's row: (anc, d) in dependingBy; anc's row, when on: (desc, d) in dependingOn
        lk[2 * u] = ((uint64_t)sv_s[u] << 40) | ((uint64_t)cq_a[u] << 16) | d;
        if (on) lk[2 * u + 1] = ((uint64_t)sv_a[u] << 40) | ((uint64_t)cq_s[u] << 16) | (1u << 15) | d;
        // emitted by this workgroup already: drop (a lossy filter; pass B dedups exactly)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (!lk[2 * u + t]) continue;
          unsigned long long &e = lseen[(uint32_t)(lk[2 * u + t] * 0x9E3779B97F4A7C15ull >> 52) & (TA_SEEN - 1)];
          if (e == lk[2 * u + t])
            lk[2 * u + t] = 0;
          else
            e = lk[2 * u + t];
        }
      }
      // cohesion: (consumer service, consumed endpoint) at distance 1
      bool pwon = false;
      if (d == 1 && !(knobs & 2)) {
        const uint64_t pk = ((uint64_t)(s + 1) << 32) | us_a[u];
        unsigned long long &pseen_e = pseen[(uint32_t)(pk * 0x9E3779B97F4A7C15ull >> 55) & (TAIL_PSEEN - 1)];
        if (pseen_e != pk) {
          pwon = tail_set_put(pset, pcap, pk, &flags);
          pseen_e = pk;
        }
      }
      if (pwon) {
        ++won_p;
        const uint64_t p = tail_agg_slot(pkey, pacap, ((uint64_t)(sv_s[u] + 1) << 32) | us_a[u], &flags);
        if (p != pacap) {
          atomicAdd(&sstat[8 * sv_s[u] + TS_CONSUMES], 1u);
          if (atomicAdd(&pval[p], 1u) == 0) atomicAdd(&sstat[8 * sv_s[u] + TS_CONSUMERS], 1u);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < (int)(2 * TA_U); ++j) {  // (the bucket: the key's (service, linked service) pair)
      lb[j] = lk[j] ? tail_bucket(((lk[j] >> 40) << 24) | lsvc_of_cls[(uint32_t)(lk[j] >> 16) & 0xFFFFFFu], bits) : 0;
      rk[j] = lk[j] ? atomicAdd(&hist[lb[j]], 1u) : 0;
    }
    __syncthreads();
    {  // exclusive scan of hist (nb / TA_T per thread)
      const uint32_t per = nb / TA_T, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      uint32_t run = 0;
      for (uint32_t j = 0; j < per; ++j) run += hist[per * threadIdx.x + j];
      uint32_t x = run;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
      }
      if (lane == 63) wsum[w] = x;
      __syncthreads();
      uint32_t before = x - run;
      for (uint32_t k = 0; k < w; ++k) before += wsum[k];
      if (threadIdx.x == TA_T - 1) wsum[TA_T / 64] = before + run;  // the step's link keys
      __syncthreads();
      for (uint32_t j = 0; j < per; ++j) {  // hist := offsets
        const uint32_t c = hist[per * threadIdx.x + j];
        hist[per * threadIdx.x + j] = before;
        before += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (int)(2 * TA_U); ++j)
      if (lk[j]) {
        const uint32_t at = hist[lb[j]] + rk[j];
        stg[at] = lk[j];
        bk[at] = (uint16_t)lb[j];
      }
    __syncthreads();
    const uint32_t tot = wsum[TA_T / 64];
    for (uint32_t e = threadIdx.x; e < tot; e += TA_T) {
      const uint32_t b = bk[e];
      const uint32_t pos = fill[b] + e - hist[b];  // (this workgroup's slab of bucket b)
      if (pos < slab)
        lbkt[((uint64_t)b * gridDim.x + blockIdx.x) * slab + pos] = stg[e];
      else
        flags |= F_TRIPLE_OVERFLOW;  // (the host repeats the tail with larger slabs)
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < nb; x += TA_T)  // the slabs' fill after this step
      fill[x] += (x + 1 < nb ? hist[x + 1] : tot) - hist[x];
    __syncthreads();  // (stg and hist are reused by the next step)
  }
  for (uint32_t x = threadIdx.x; x < nb; x += TA_T) lbn[(uint64_t)x * gridDim.x + blockIdx.x] = fill[x];
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) won_p += __shfl_xor(won_p, o, 64);
  if ((threadIdx.x & 63) == 0 && won_p) atomicAdd(&counters[9], won_p);  // (u32 word 9 of the tail's counter block)
}

// pass B: bucket b -> its distinct link keys -> details (written out) and
// pair flags (into the services' counters)
constexpr uint32_t PF_BY = 1, PF_ON = 2, PF_BY1 = 4, PF_ON1 = 8;
__global__ void __launch_bounds__(TB_T) k_tail_dedup(const unsigned long long *__restrict__ lbkt, uint32_t slab,
                                                     const uint32_t *__restrict__ lbn, uint32_t nwg, uint32_t bits,
                                                     const uint32_t *__restrict__ lsvc_of_cls,
                                                     kmz_tail_detail *__restrict__ dout, uint64_t dcap,
                                                     unsigned long long *__restrict__ dcount,
                                                     uint32_t *__restrict__ sstat, uint32_t *__restrict__ rel,
                                                     uint32_t n_dist, unsigned int *__restrict__ counters) {
  __shared__ unsigned long long lset[TB_LSET], dkey[TB_DSET], pkey[TB_PSET];
  __shared__ uint32_t dval[3][TB_DSET], pflag[TB_PSET];
  __shared__ uint32_t s_full, s_nd, s_won;
  __shared__ unsigned long long s_base;
  __shared__ uint32_t soff[TA_GRID + 1], wsum[TB_T / 64];  // the slabs' fills -> their offsets in the bucket
  constexpr uint32_t LB = 13, DB = 11, PB = 11;
  static_assert((1u << LB) == TB_LSET && (1u << DB) == TB_DSET && (1u << PB) == TB_PSET, "LDS table sizes");
  uint32_t flags = 0;
  for (uint32_t b = blockIdx.x; b < (1u << bits); b += gridDim.x) {
    for (uint32_t x = threadIdx.x; x < TB_LSET; x += TB_T) lset[x] = 0;
    for (uint32_t x = threadIdx.x; x < TB_DSET; x += TB_T) {
      dkey[x] = 0;
      dval[0][x] = dval[1][x] = dval[2][x] = 0;
    }
    for (uint32_t x = threadIdx.x; x < TB_PSET; x += TB_T) {
      pkey[x] = 0;
      pflag[x] = 0;
    }
    if (threadIdx.x == 0) s_full = s_nd = s_won = 0;
    {  // exclusive scan of the nwg slab fills (nwg <= TB_T: one per thread)
      const uint32_t c = threadIdx.x < nwg ? min(lbn[(uint64_t)b * nwg + threadIdx.x], slab) : 0;
      const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      uint32_t x = c;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
      }
      if (lane == 63) wsum[w] = x;
      __syncthreads();
      uint32_t before = x - c;
      for (uint32_t k = 0; k < w; ++k) before += wsum[k];
      if (threadIdx.x < nwg) soff[threadIdx.x] = before;
      if (threadIdx.x == TB_T - 1) soff[nwg] = before + c;
    }
    __syncthreads();
    const uint32_t m = soff[nwg];
    const unsigned long long *src = lbkt + (uint64_t)b * nwg * slab;
    // 1. the bucket's link keys into the LDS set (entry e: slab w with
    // soff[w] <= e < soff[w + 1], by a binary search)
    uint64_t xn[4];  // the next chunk's keys load while this chunk's are inserted
    auto load = [&](uint32_t e0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t e = e0 + u * TB_T + threadIdx.x;
        xn[u] = 0;
        if (e < m) {
          uint32_t lo = 0;
#pragma unroll
          for (uint32_t step = TA_GRID / 2; step; step >>= 1)
            if (lo + step < nwg && soff[lo + step] <= e) lo += step;
          xn[u] = src[(uint64_t)lo * slab + (e - soff[lo])];
        }
      }
    };
    load(0);
    for (uint32_t e0 = 0; e0 < m; e0 += 4 * TB_T) {
      uint64_t xq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) xq[u] = xn[u];
      load(e0 + 4 * TB_T);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (xq[u] && lds_slot(lset, LB, xq[u]) == ~0u) s_full = 1;
    }
    __syncthreads();
    // 2. each distinct link key: its detail and its pair's flags
    uint32_t won = 0;
    if (!s_full) {
      for (uint32_t x = threadIdx.x; x < TB_LSET; x += TB_T) {
        const uint64_t lk = lset[x];
        if (!lk) continue;
        ++won;
        const uint32_t c = (uint32_t)(lk >> 16) & 0xFFFFFFu, d = (uint32_t)lk & 0x7FFFu;
        const uint32_t ty = (uint32_t)(lk >> 15) & 1u;  // dependingBy (CLIENT) / dependingOn (SERVER)
        const uint64_t pr = ((lk >> 40) << 24) | lsvc_of_cls[c];
        const uint64_t dk = ((lk >> 40) << 40) | ((uint64_t)lsvc_of_cls[c] << 16) | d;
        const uint32_t q = lds_slot(dkey, DB, dk + 1);  // (+1: the key of svc 0, lsvc 0, d 0 is never 0 in LDS)
        const uint32_t r = lds_slot(pkey, PB, pr + 1);
        if (q == ~0u || r == ~0u) {
          s_full = 1;
          continue;
        }
        atomicAdd(&dval[0][q], 1u);
        atomicAdd(&dval[1 + ty][q], 1u);
        atomicOr(&pflag[r], (ty ? PF_ON : PF_BY) | (d == 1 ? (ty ? PF_ON1 : PF_BY1) : 0u));
      }
    }
    __syncthreads();
    if (s_full) {  // (uniform) a table too small for this bucket: the host redoes the tail with more buckets
      if (threadIdx.x == 0) atomicOr(&counters[10], 1u);
    } else {
      for (int o = 32; o > 0; o >>= 1) won += __shfl_xor(won, o, 64);
      if ((threadIdx.x & 63) == 0 && won) atomicAdd(&s_won, won);
      // 3. the details out (one reservation), the pairs into the services' counters
      uint32_t nd = 0;
      for (uint32_t x = threadIdx.x; x < TB_DSET; x += TB_T) nd += dkey[x] != 0;
      for (int o = 32; o > 0; o >>= 1) nd += __shfl_xor(nd, o, 64);
      if ((threadIdx.x & 63) == 0 && nd) atomicAdd(&s_nd, nd);
      __syncthreads();
      if (threadIdx.x == 0) {
        s_base = s_nd ? atomicAdd(dcount, (unsigned long long)s_nd) : 0;
        if (s_won) atomicAdd(&counters[8], s_won);  // (u32 word 8: distinct link keys)
        s_nd = 0;
      }
      __syncthreads();
      for (uint32_t x = threadIdx.x; x < TB_DSET; x += TB_T) {
        const unsigned long long k = dkey[x];
        if (!k) continue;
        const uint64_t dk = k - 1;
        const uint64_t at = s_base + atomicAdd(&s_nd, 1u);
        const uint32_t sv = (uint32_t)(dk >> 40), d = (uint32_t)dk & 0xFFFFu;
        if (at < dcap) {
          kmz_tail_detail r;
          r.svc = sv;
          r.lsvc = (uint32_t)(dk >> 16) & 0xFFFFFFu;
          r.distance = d;
          r.count = dval[0][x];
          r.depending_by = dval[1][x];
          r.depending_on = dval[2][x];
          dout[at] = r;
        } else {
          flags |= F_TRIPLE_OVERFLOW;
        }
        // RelyingFactor: sum of dependingBy / distance (RiskAnalyzer.ts:124-137),
        // per (service, distance) -- one add per detail, not per link key
        if (dval[1][x]) {
          if (d < n_dist)
            atomicAdd(&rel[(uint64_t)sv * n_dist + d], dval[1][x]);
          else
            atomicMax(&counters[6], d);  // deeper than the dense table: the host uses the details
        }
      }
      // a service's instability counts its linked services with a by / on link
      // (EndpointDependencies.ts:618-628), its ACS those at distance 1
      // (RiskAnalyzer.ts:150-166): every (service, linked service) pair is in
      // this bucket only
      for (uint32_t x = threadIdx.x; x < TB_PSET; x += TB_T) {
        const uint32_t f = pflag[x];
        if (!f) continue;
        const uint32_t sv = (uint32_t)((pkey[x] - 1) >> 24);
        if (f & PF_BY) atomicAdd(&sstat[8 * sv + TS_NBY], 1u);
        if (f & PF_ON) atomicAdd(&sstat[8 * sv + TS_NON], 1u);
        if (f & PF_BY1) atomicAdd(&sstat[8 * sv + TS_AIS], 1u);
        if (f & PF_ON1) atomicAdd(&sstat[8 * sv + TS_ADS], 1u);
      }
    }
    __syncthreads();
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
}

// aggregation tables -> dense kmz_tail_detail (MODE 0) / kmz_tail_pair (MODE 1)
// records.  Each workgroup owns a contiguous range of the table, counts its
// entries, reserves their output range with ONE atomic (a per-wave atomic on
// one counter serialises: ~10^5 of them cost 1.5 ms), then writes them.
constexpr uint32_t TAIL_COMPACT_BLOCKS = 1024;
template <int MODE>
__global__ void __launch_bounds__(256) k_tail_compact(const unsigned long long *__restrict__ akey,
                                                      const uint32_t *__restrict__ aval, uint64_t cap,
                                                      uint32_t *__restrict__ out,
                                                      unsigned long long *__restrict__ count,
                                                      uint32_t *__restrict__ rel, uint32_t n_dist,
                                                      unsigned int *__restrict__ counters) {
  constexpr uint32_t W = MODE == 0 ? 6 : 3;  // record words
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long base;
  const uint64_t per = (cap + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = min(cap, b0 + per);
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t c = 0;
  for (uint64_t p = b0 + threadIdx.x; p < b1; p += 256) c += akey[p] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) wsum[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    base = t ? atomicAdd(count, (unsigned long long)t) : 0;
  }
  __syncthreads();
  unsigned long long run = base;
  for (uint64_t p0 = b0; p0 < b1; p0 += 256) {
    const uint64_t p = p0 + threadIdx.x;
    const unsigned long long k = p < b1 ? akey[p] : 0;
    const uint64_t m = __ballot(k != 0);
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t v = 0; v < 4; ++v) {
      before += v < w ? wsum[v] : 0;
      tot += wsum[v];
    }
    if (k) {
      uint32_t *r = out + (uint64_t)W * (run + before + __popcll(m & ((1ull << lane) - 1)));
      if (MODE == 0) {  // detail key svc << 40 | lsvc << 16 | d
        r[0] = (uint32_t)(k >> 40);
        r[1] = (uint32_t)(k >> 16) & 0xFFFFFFu;
        r[2] = (uint32_t)k & 0xFFFFu;
        r[3] = aval[4 * p + 0];
        r[4] = aval[4 * p + 1];
        r[5] = aval[4 * p + 2];
        // RelyingFactor: sum of dependingBy / distance (RiskAnalyzer.ts:124-137),
        // per (service, distance) -- one add per detail, not per link key
        const uint32_t d = (uint32_t)k & 0xFFFFu;
        if (r[4]) {
          if (d < n_dist)
            atomicAdd(&rel[(uint64_t)r[0] * n_dist + d], r[4]);
          else
            atomicMax(&counters[6], d);  // deeper than the dense table: the host uses the details
        }
      } else {  // pair detail key (svc + 1) << 32 | consumer
        r[0] = (uint32_t)(k >> 32) - 1;
        r[1] = (uint32_t)k;
        r[2] = aval[p];
      }
    }
    run += tot;
    __syncthreads();
  }
}

// per service, from the dependency endpoints' merged rows (what
// toServiceDependencies groups by uniqueServiceName, EndpointDependencies.ts:
// 372-384): rows (endpoints with a row), gateway (some row without a
// dependingBy, RiskAnalyzer.ts:155-158) and the first row's global index
// (the services' output order).  `epf` is the endpoint partial of the first
// row: (first row << 1 | not external), UINT64_MAX for none.  Integer
// atomics: the result does not depend on their order.
__global__ void __launch_bounds__(256) k_tail_service_rows(const unsigned long long *__restrict__ epf,
                                                           const uint32_t *__restrict__ svc,
                                                           const uint8_t *__restrict__ hasin, uint32_t n_ep,
                                                           uint32_t *__restrict__ sstat,
                                                           unsigned long long *__restrict__ sfirst) {
  for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < n_ep; e += gridDim.x * 256) {
    const unsigned long long f = epf[e];
    if (f == ~0ull) continue;
    const uint32_t v = svc[e];
    atomicAdd(&sstat[8 * v + TS_ROWS], 1u);
    if (!hasin[e]) atomicOr(&sstat[8 * v + TS_GATEWAY], 1u);
    atomicMin(&sfirst[v], f >> 1);
  }
}

void launch_tail_service_rows(hipStream_t s, const unsigned long long *epf, const uint32_t *svc, const uint8_t *hasin,
                              uint32_t n_ep, uint32_t *sstat, unsigned long long *sfirst) {
  if (!n_ep) return;
  hipLaunchKernelGGL(k_tail_service_rows, dim3(std::min<uint32_t>((n_ep + 255) / 256, 1024)), dim3(256), 0, s, epf, svc,
                     hasin, n_ep, sstat, sfirst);
}

// RiskAnalyzer.RealtimeRisk's per-service sums over the combined groups
// (RiskAnalyzer.ts:18, 228-248): for the groups with combined > 0 of the
// service's endpoints, sum(cv * combined), sum(combined), sum(combined of 5xx
// statuses) and the smallest first index (the services' output order).  One
// wave per service walks its groups in ascending group index -- the order in
// which the host's per-row sums (np.bincount over the rows) add them -- and
// lane 0 adds the products in that order, so the fp64 sum is the host's bit
// for bit (no contraction: -ffp-contract=off).  `off` / `eps`: the services'
// endpoints in ascending order (CSR).
__global__ void __launch_bounds__(256) k_service_sums(const kmz_group *__restrict__ grp, uint32_t n_status,
                                                      const uint32_t *__restrict__ off, const uint32_t *__restrict__ eps,
                                                      const uint8_t *__restrict__ is5, uint32_t n_sid,
                                                      kmz_service_sum *__restrict__ out) {
  __shared__ double prod[4][64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t sid = blockIdx.x * 4 + w;
  if (sid >= n_sid) return;  // (whole waves; no workgroup barrier below)
  const uint32_t a = off[sid], m = (off[sid + 1] - a) * n_status;
  double ws = 0.0;
  unsigned long long cnt = 0, err = 0, first = ~0ull;
  for (uint32_t j0 = 0; j0 < m; j0 += 64) {
    const uint32_t j = j0 + lane;
    double p = 0.0;
    bool used = false;
    if (j < m) {
      const uint32_t st = j % n_status;
      const kmz_group &x = grp[(uint64_t)eps[a + j / n_status] * n_status + st];
      const unsigned long long c = x.combined;
      if (c) {
        used = true;
        p = x.cv * (double)c;
        cnt += c;
        if (is5[st]) err += c;
        first = min(first, (unsigned long long)x.first);
      }
    }
    prod[w][lane] = p;
    const uint64_t um = __ballot(used);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane == 0)
      for (uint64_t b = um; b; b &= b - 1) ws += prod[w][__builtin_ctzll(b)];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    err += __shfl_xor(err, o, 64);
    first = min(first, (unsigned long long)__shfl_xor(first, o, 64));
  }
  if (lane == 0) {
    kmz_service_sum r;
    r.wsum = ws;
    r.count = (double)cnt;
    r.err = (double)err;
    r.first = first;
    out[sid] = r;
  }
}

void launch_service_sums(hipStream_t s, const kmz_group *grp, uint32_t n_status, const uint32_t *off, const uint32_t *eps,
                         const uint8_t *is5, uint32_t n_sid, kmz_service_sum *out) {
  if (!n_sid) return;
  hipLaunchKernelGGL(k_service_sums, dim3((n_sid + 3) / 4), dim3(256), 0, s, grp, n_status, off, eps, is5, n_sid, out);
}

uint32_t tail_bucket_bits_max() { return TAIL_BMAX; }
uint32_t tail_part_grid(uint64_t n_max) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_max + TA_STEP - 1) / TA_STEP, TA_GRID));
}

void launch_tail(hipStream_t s, const unsigned long long *keys, const unsigned long long *n_keys, uint64_t n_max,
                 const uint32_t *svc, const uint32_t *cls, const uint32_t *lsvc_of_cls, const uint32_t *usn,
                 uint32_t n_ep, uint32_t n_cls, uint32_t bits, unsigned long long *lbkt, uint32_t slab, uint32_t *lbn,
                 unsigned long long *pset, uint64_t pcap, unsigned long long *pkey, uint32_t *pval, uint64_t pacap,
                 uint8_t *hasin, uint32_t *sstat, uint32_t *rel, uint32_t n_dist, unsigned int *counters,
                 kmz_tail_detail *links_out, uint64_t dcap, uint32_t *pairs_out, unsigned long long *out_counts,
                 uint32_t knobs) {
  // (a few workgroups per CU, each over many steps: the LDS filter sees more
  // of the hot keys; lbkt / lbn are sized for tail_part_grid(n_max) slabs)
  const uint32_t g = tail_part_grid(n_max);
  if (bits == TAIL_BMAX)
    hipLaunchKernelGGL(k_tail_part<TAIL_BMAX>, dim3(g), dim3(TA_T), 0, s, keys, n_keys, svc, cls, lsvc_of_cls, usn, n_ep,
                       n_cls, lbkt, slab, lbn, pset, pcap, pkey, pval, pacap, hasin, sstat, counters, knobs);
  else
    hipLaunchKernelGGL(k_tail_part<TAIL_BMAX - 1>, dim3(g), dim3(TA_T), 0, s, keys, n_keys, svc, cls, lsvc_of_cls, usn,
                       n_ep, n_cls, lbkt, slab, lbn, pset, pcap, pkey, pval, pacap, hasin, sstat, counters, knobs);
  hipLaunchKernelGGL(k_tail_dedup, dim3(1u << bits), dim3(TB_T), 0, s, lbkt, slab, lbn, g, bits, lsvc_of_cls, links_out,
                     dcap, out_counts, sstat, rel, n_dist, counters);
  const uint32_t gp = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((pacap + 255) / 256, TAIL_COMPACT_BLOCKS));
  hipLaunchKernelGGL(k_tail_compact<1>, dim3(gp), dim3(256), 0, s, pkey, pval, pacap, pairs_out, out_counts + 1, rel,
                     n_dist, counters);
}

}  // namespace kmz
