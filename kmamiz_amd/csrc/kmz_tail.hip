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

// add (count, dependingBy, dependingOn) to the detail dk in the global table;
// the first link of a type there also counts into the service's ACS
// (distance 1, RiskAnalyzer.ts:150-166) and instability (any distance,
// EndpointDependencies.ts:618-628) counters
__device__ __forceinline__ void detail_add(uint64_t dk, uint32_t cnt, uint32_t by, uint32_t on,
                                           unsigned long long *__restrict__ akey, uint32_t *__restrict__ aval,
                                           uint64_t acap, unsigned long long *__restrict__ fkey,
                                           uint32_t *__restrict__ fval, uint64_t fcap, uint32_t *__restrict__ sstat,
                                           uint32_t *flags) {
  const uint64_t p = tail_agg_slot(akey, acap, dk, flags);
  if (p == acap) return;
  const uint32_t sv = (uint32_t)(dk >> 40), d = (uint32_t)dk & 0xFFFFu;
  atomicAdd(&aval[4 * p + 0], cnt);
  for (uint32_t ty = 0; ty < 2; ++ty) {
    const uint32_t v = ty ? on : by;
    if (!v || atomicAdd(&aval[4 * p + 1 + ty], v)) continue;
    if (d == 1) atomicAdd(&sstat[8 * sv + TS_AIS + ty], 1u);
    const uint64_t q = tail_agg_slot(fkey, fcap, (dk >> 16) + 1, flags);  // (svc, lsvc)
    if (q == fcap) continue;
    const uint32_t was = atomicOr(&fval[q], 1u << ty);
    if (!(was & (1u << ty))) atomicAdd(&sstat[8 * sv + TS_NBY + ty], 1u);
  }
}

constexpr uint32_t TAIL_LAGG = 1024;  // per-workgroup LDS detail slots (20 KB)
// Link keys repeat: config 5's 2.7e7 link keys per step hold ~5e4 distinct
// ones, spread so evenly over the edge keys that a per-workgroup LDS cache of
// 2048 keys caught few of them (every miss a probe of the global link set:
// 1.0 of the tail's 1.35 ms).  So the link keys are partitioned first: pass A
// (k_tail_part) derives them from the edge keys and writes each into one of
// TAIL_P buckets by its hash (an LDS counting sort per 2048 edge keys, one
// reservation per bucket and step); pass B (k_tail_dedup) takes one bucket
// per workgroup, where every occurrence of a link key lands, and dedups it in
// an LDS set -- a key that wins there is a first occurrence of the run.
// Cohesion pairs stay in pass A (a direct-mapped LDS cache in front of the
// global pair set: they are few).
constexpr uint32_t TAIL_P = 1024;               // link-key buckets
constexpr uint32_t TAIL_PSEEN = 512;
constexpr uint32_t TA_T = 256, TA_U = 8;         // pass A: threads, edge keys per thread and step
constexpr uint32_t TA_STEP = TA_T * TA_U;        // 2048 edge keys, <= 4096 link keys per step
constexpr uint32_t TB_T = 256, TB_SET = 4096;    // pass B: threads, LDS set slots (32 KB)
__device__ __forceinline__ uint32_t tail_bucket(uint64_t lk) { return (uint32_t)(mix64(lk) >> 54); }  // 10 bits
static_assert(TAIL_P == 1024, "tail_bucket takes 10 bits");

// link key: svc << 40 | cls << 16 | type << 15 | d   (type 1 = SERVER / dependingOn)
// detail key: svc << 40 | lsvc << 16 | d
// pair key: (desc + 1) << 32 | consumer usn;  pair detail key: (svc + 1) << 32 | consumer usn
__global__ void __launch_bounds__(TA_T) k_tail_part(const unsigned long long *__restrict__ keys,
                                                    const unsigned long long *__restrict__ n_keys,
                                                    const uint32_t *__restrict__ svc, const uint32_t *__restrict__ cls,
                                                    const uint32_t *__restrict__ usn, uint32_t n_ep, uint32_t n_cls,
                                                    unsigned long long *__restrict__ lbkt, uint32_t bcap,
                                                    uint32_t *__restrict__ lbn, unsigned long long *__restrict__ pset,
                                                    uint64_t pcap, unsigned long long *__restrict__ pkey,
                                                    uint32_t *__restrict__ pval, uint64_t pacap,
                                                    uint8_t *__restrict__ hasin, uint32_t *__restrict__ sstat,
                                                    unsigned int *__restrict__ counters, uint32_t knobs) {
  const uint64_t n = *n_keys;
  __shared__ unsigned long long stg[2 * TA_STEP];  // 32 KB
  __shared__ uint32_t hist[TAIL_P], base[TAIL_P], wsum[TA_T / 64 + 1];
  __shared__ unsigned long long pseen[TAIL_PSEEN];
  for (uint32_t x = threadIdx.x; x < TAIL_PSEEN; x += TA_T) pseen[x] = 0;
  uint32_t flags = 0, won_p = 0;
  for (uint64_t s0 = (uint64_t)blockIdx.x * TA_STEP; s0 < n; s0 += (uint64_t)gridDim.x * TA_STEP) {
    uint64_t kq[TA_U];
#pragma unroll
    for (int u = 0; u < (int)TA_U; ++u) {
      const uint64_t i = s0 + u * TA_T + threadIdx.x;
      kq[u] = i < n ? keys[i] : 0;
    }
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
    for (uint32_t x = threadIdx.x; x < TAIL_P; x += TA_T) hist[x] = 0;
    __syncthreads();
    uint64_t lk[2 * TA_U];
    uint32_t rk[2 * TA_U];
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
    for (int j = 0; j < (int)(2 * TA_U); ++j) rk[j] = lk[j] ? atomicAdd(&hist[tail_bucket(lk[j])], 1u) : 0;
    __syncthreads();
    // each bucket's run of this step: one reservation, the local offsets by a scan
    for (uint32_t x = threadIdx.x; x < TAIL_P; x += TA_T) {
      const uint32_t h = hist[x];
      base[x] = h ? atomicAdd(&lbn[x], h) : 0;
    }
    {  // exclusive scan of hist (TAIL_P = 4 per thread)
      const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      uint32_t v[4], run = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = run;
        run += hist[4 * threadIdx.x + j];
      }
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
#pragma unroll
      for (int j = 0; j < 4; ++j) hist[4 * threadIdx.x + j] = before + v[j];  // hist := offsets
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (int)(2 * TA_U); ++j)
      if (lk[j]) stg[hist[tail_bucket(lk[j])] + rk[j]] = lk[j];
    __syncthreads();
    const uint32_t tot = wsum[TA_T / 64];
    for (uint32_t e = threadIdx.x; e < tot; e += TA_T) {
      const uint64_t x = stg[e];
      const uint32_t b = tail_bucket(x);
      const uint32_t pos = base[b] + e - hist[b];
      if (pos < bcap)
        lbkt[(uint64_t)b * bcap + pos] = x;
      else
        flags |= F_TRIPLE_OVERFLOW;  // (the host repeats the tail with larger buckets)
    }
    __syncthreads();  // (stg, hist and base are reused by the next step)
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) won_p += __shfl_xor(won_p, o, 64);
  if ((threadIdx.x & 63) == 0 && won_p) atomicAdd(&counters[9], won_p);  // (u32 word 9 of the tail's counter block)
}

// pass B: bucket b's link keys -> first occurrences -> details.  A key that
// finds no LDS slot in 64 probes (more than ~3000 distinct keys in one bucket)
// goes to the global link set, which decides for it exactly.
__global__ void __launch_bounds__(TB_T) k_tail_dedup(const unsigned long long *__restrict__ lbkt, uint32_t bcap,
                                                     const uint32_t *__restrict__ lbn,
                                                     const uint32_t *__restrict__ lsvc_of_cls,
                                                     unsigned long long *__restrict__ lset, uint64_t lcap,
                                                     unsigned long long *__restrict__ akey, uint32_t *__restrict__ aval,
                                                     uint64_t acap, unsigned long long *__restrict__ fkey,
                                                     uint32_t *__restrict__ fval, uint64_t fcap,
                                                     uint32_t *__restrict__ sstat, unsigned int *__restrict__ counters) {
  __shared__ unsigned long long set[TB_SET];
  __shared__ unsigned long long lkey[TAIL_LAGG];
  __shared__ uint32_t lval[TAIL_LAGG][3];
  uint32_t flags = 0, won_l = 0;
  for (uint32_t b = blockIdx.x; b < TAIL_P; b += gridDim.x) {
    for (uint32_t x = threadIdx.x; x < TB_SET; x += TB_T) set[x] = 0;
    for (uint32_t x = threadIdx.x; x < TAIL_LAGG; x += TB_T) {
      lkey[x] = 0;
      lval[x][0] = lval[x][1] = lval[x][2] = 0;
    }
    __syncthreads();
    const uint32_t m = min(lbn[b], bcap);
    const unsigned long long *src = lbkt + (uint64_t)b * bcap;
    for (uint32_t e0 = 0; e0 < m; e0 += 4 * TB_T) {
      uint64_t xq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t e = e0 + u * TB_T + threadIdx.x;
        xq[u] = e < m ? src[e] : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t lk = xq[u];
        if (!lk) continue;
        uint32_t h = (uint32_t)mix64(lk) & (TB_SET - 1);  // (the bucket took the top bits)
        int won = -1;  // -1: undecided in LDS
        for (uint32_t z = 0; z < 64; ++z) {
          const unsigned long long cur = set[h];
          if (cur == lk) {
            won = 0;
            break;
          }
          if (cur == 0) {
            const unsigned long long was = atomicCAS(&set[h], 0ull, (unsigned long long)lk);
            if (was == 0) {
              won = 1;
              break;
            }
            if (was == lk) {
              won = 0;
              break;
            }
          }
          h = (h + 1) & (TB_SET - 1);
        }
        if (won < 0) won = tail_set_put(lset, lcap, lk, &flags) ? 1 : 0;
        if (!won) continue;
        ++won_l;
        const uint32_t c = (uint32_t)(lk >> 16) & 0xFFFFFFu, d = (uint32_t)lk & 0x7FFFu;
        const uint64_t dk = (lk & ~((1ull << 40) - 1)) | ((uint64_t)lsvc_of_cls[c] << 16) | d;
        const uint32_t ty = (uint32_t)(lk >> 15) & 1u;  // dependingBy (CLIENT) / dependingOn (SERVER)
        uint32_t q = (uint32_t)(mix64(dk) & (TAIL_LAGG - 1));
        bool done = false;
        for (uint32_t z = 0; z < 16; ++z) {
          const unsigned long long cur = atomicCAS(&lkey[q], 0ull, (unsigned long long)dk);
          if (cur == 0 || cur == dk) {
            atomicAdd(&lval[q][0], 1u);
            atomicAdd(&lval[q][1 + ty], 1u);
            done = true;
            break;
          }
          q = (q + 1) & (TAIL_LAGG - 1);
        }
        if (!done) detail_add(dk, 1u, ty == 0, ty == 1, akey, aval, acap, fkey, fval, fcap, sstat, &flags);
      }
    }
    __syncthreads();  // this bucket's details -> the global table
    for (uint32_t x = threadIdx.x; x < TAIL_LAGG; x += TB_T)
      if (lkey[x]) detail_add(lkey[x], lval[x][0], lval[x][1], lval[x][2], akey, aval, acap, fkey, fval, fcap, sstat,
                              &flags);
    __syncthreads();
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) won_l += __shfl_xor(won_l, o, 64);
  if ((threadIdx.x & 63) == 0 && won_l) atomicAdd(&counters[8], won_l);  // (u32 word 8 of the tail's counter block)
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

uint32_t tail_buckets() { return TAIL_P; }

void launch_tail(hipStream_t s, const unsigned long long *keys, const unsigned long long *n_keys, uint64_t n_max,
                 const uint32_t *svc, const uint32_t *cls, const uint32_t *lsvc_of_cls, const uint32_t *usn,
                 uint32_t n_ep, uint32_t n_cls, unsigned long long *lbkt, uint32_t bcap, uint32_t *lbn,
                 unsigned long long *lset, uint64_t lcap, unsigned long long *akey, uint32_t *aval, uint64_t acap,
                 unsigned long long *pset, uint64_t pcap, unsigned long long *pkey, uint32_t *pval, uint64_t pacap,
                 uint8_t *hasin, unsigned long long *fkey, uint32_t *fval, uint64_t fcap, uint32_t *sstat,
                 uint32_t *rel, uint32_t n_dist, unsigned int *counters, uint32_t *links_out, uint32_t *pairs_out,
                 unsigned long long *out_counts, uint32_t knobs) {
  const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_max + TA_STEP - 1) / TA_STEP, 2048));
  hipLaunchKernelGGL(k_tail_part, dim3(g), dim3(TA_T), 0, s, keys, n_keys, svc, cls, usn, n_ep, n_cls, lbkt, bcap, lbn,
                     pset, pcap, pkey, pval, pacap, hasin, sstat, counters, knobs);
  hipLaunchKernelGGL(k_tail_dedup, dim3(TAIL_P), dim3(TB_T), 0, s, lbkt, bcap, lbn, lsvc_of_cls, lset, lcap, akey, aval,
                     acap, fkey, fval, fcap, sstat, counters);
  const uint32_t ga = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((acap + 255) / 256, TAIL_COMPACT_BLOCKS));
  hipLaunchKernelGGL(k_tail_compact<0>, dim3(ga), dim3(256), 0, s, akey, aval, acap, links_out, out_counts, rel, n_dist,
                     counters);
  const uint32_t gp = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((pacap + 255) / 256, TAIL_COMPACT_BLOCKS));
  hipLaunchKernelGGL(k_tail_compact<1>, dim3(gp), dim3(256), 0, s, pkey, pval, pacap, pairs_out, out_counts + 1, rel,
                     n_dist, counters);
}

}  // namespace kmz
