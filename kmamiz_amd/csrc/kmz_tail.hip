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
// is the host's, as in EndpointDependencies.label()).  A link key that wins its
// slot in the link set adds itself to its (svc, lsvc(cls), d) detail counters
// in the same step (count, dependingBy, dependingOn), so duplicates cost one
// probe and no second pass runs.  Cohesion needs, per service, the distinct
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
// ones.  A workgroup remembers the link / pair keys it has already put in the
// global sets (direct-mapped LDS caches); a key found there is in its set, so
// it is not a first occurrence and needs no global probe.  (A slot overwritten
// by another key only costs a probe.)
constexpr uint32_t TAIL_LSEEN = 2048, TAIL_PSEEN = 512;
#ifndef KMZ_TAIL_U
#define KMZ_TAIL_U 4
#endif
constexpr int TAIL_U = KMZ_TAIL_U;  // edge keys per thread and step

// link key: svc << 40 | cls << 16 | type << 15 | d   (type 1 = SERVER / dependingOn)
// detail key: svc << 40 | lsvc << 16 | d
// pair key: (desc + 1) << 32 | consumer usn;  pair detail key: (svc + 1) << 32 | consumer usn
__global__ void __launch_bounds__(256) k_tail_links(const unsigned long long *__restrict__ keys,
                                                    const unsigned long long *__restrict__ n_keys,
                                                    const uint32_t *__restrict__ svc, const uint32_t *__restrict__ cls,
                                                    const uint32_t *__restrict__ lsvc_of_cls,
                                                    const uint32_t *__restrict__ usn, uint32_t n_ep, uint32_t n_cls,
                                                    unsigned long long *__restrict__ lset, uint64_t lcap,
                                                    unsigned long long *__restrict__ akey, uint32_t *__restrict__ aval,
                                                    uint64_t acap, unsigned long long *__restrict__ pset,
                                                    uint64_t pcap, unsigned long long *__restrict__ pkey,
                                                    uint32_t *__restrict__ pval, uint64_t pacap,
                                                    uint8_t *__restrict__ hasin, unsigned long long *__restrict__ fkey,
                                                    uint32_t *__restrict__ fval, uint64_t fcap,
                                                    uint32_t *__restrict__ sstat, uint32_t *__restrict__ rel,
                                                    uint32_t n_dist, unsigned int *__restrict__ counters,
                                                    uint32_t knobs) {
  const uint64_t n = *n_keys;
  uint32_t flags = 0, won_l = 0, won_p = 0;  // first occurrences in the link / pair sets (sizes the next run's sets)
  // winners' details are summed in LDS first (hot (service, linked service,
  // distance) entries see one global update per workgroup, not one per link)
  __shared__ unsigned long long lkey[TAIL_LAGG];
  __shared__ uint32_t lval[TAIL_LAGG][3];
  __shared__ unsigned long long lseen[TAIL_LSEEN], pseen[TAIL_PSEEN];
  for (uint32_t x = threadIdx.x; x < TAIL_LSEEN; x += blockDim.x) lseen[x] = 0;
  for (uint32_t x = threadIdx.x; x < TAIL_PSEEN; x += blockDim.x) pseen[x] = 0;
  for (uint32_t x = threadIdx.x; x < TAIL_LAGG; x += blockDim.x) {
    lkey[x] = 0;
    lval[x][0] = lval[x][1] = lval[x][2] = 0;
  }
  __syncthreads();
  // TAIL_U keys per thread and step: their loads and table gathers are issued
  // together (the per-key chain of dependent loads is what bounds this kernel)
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += TAIL_U * stride) {
    uint64_t kq[TAIL_U];
#pragma unroll
    for (int u = 0; u < TAIL_U; ++u) {
      const uint64_t i = i0 + u * stride;
      kq[u] = i < n ? keys[i] : 0;
    }
    uint32_t cq_a[TAIL_U], cq_s[TAIL_U], sv_a[TAIL_U], sv_s[TAIL_U], us_a[TAIL_U];
    bool okq[TAIL_U];
#pragma unroll
    for (int u = 0; u < TAIL_U; ++u) {
      const uint32_t a = (uint32_t)(kq[u] >> 40), s = (uint32_t)(kq[u] >> 16) & 0xFFFFFFu;
      okq[u] = i0 + u * stride < n;
      const bool in = a < n_ep && s < n_ep;
      cq_a[u] = in ? cls[a] : NONE;
      cq_s[u] = in ? cls[s] : NONE;
      sv_a[u] = in ? svc[a] : 0;
      sv_s[u] = in ? svc[s] : 0;
      us_a[u] = in ? usn[a] : 0;
    }
#pragma unroll
    for (int u = 0; u < TAIL_U; ++u) {
      if (!okq[u]) continue;
      const uint64_t k = kq[u];
      const uint32_t a = (uint32_t)(k >> 40), s = (uint32_t)(k >> 16) & 0xFFFFFFu, d = (uint32_t)(k >> 1) & 0x7FFFu;
      const bool on = (k & 1) != 0;
      if (a >= n_ep || s >= n_ep || cq_a[u] >= n_cls || cq_s[u] >= n_cls) {
        flags |= F_RANGE;
        continue;
      }
      if (!hasin[s]) hasin[s] = 1;  // (read first: ~10^7 keys share ~10^4 bytes)
      // desc's row: (anc, d) in dependingBy
      uint32_t side = 0;
      uint64_t lk[2];
      lk[side++] = ((uint64_t)sv_s[u] << 40) | ((uint64_t)cq_a[u] << 16) | d;
      if (on) lk[side++] = ((uint64_t)sv_a[u] << 40) | ((uint64_t)cq_s[u] << 16) | (1u << 15) | d;
      if (knobs & 1) side = 0;  // (diagnostic knob: no link keys -- timing only, wrong results)
      for (uint32_t t = 0; t < side; ++t) {
        unsigned long long &seen = lseen[(uint32_t)(lk[t] * 0x9E3779B97F4A7C15ull >> 53) & (TAIL_LSEEN - 1)];
        if (seen == lk[t]) continue;  // put in the set by this workgroup already
        const bool won = tail_set_put(lset, lcap, lk[t], &flags);
        seen = lk[t];  // (in the set now, whoever won)
        if (!won) continue;
        ++won_l;
        const uint32_t c = (uint32_t)(lk[t] >> 16) & 0xFFFFFFu;
        const uint64_t dk = (lk[t] & ~((1ull << 40) - 1)) | ((uint64_t)lsvc_of_cls[c] << 16) | d;
        const uint32_t ty = (uint32_t)(lk[t] >> 15) & 1u;  // dependingBy (CLIENT) / dependingOn (SERVER)
        uint32_t h = (uint32_t)(mix64(dk) & (TAIL_LAGG - 1));
        bool done = false;
        for (uint32_t z = 0; z < 16; ++z) {
          const unsigned long long cur = atomicCAS(&lkey[h], 0ull, (unsigned long long)dk);
          if (cur == 0 || cur == dk) {
            atomicAdd(&lval[h][0], 1u);
            atomicAdd(&lval[h][1 + ty], 1u);
            done = true;
            break;
          }
          h = (h + 1) & (TAIL_LAGG - 1);
        }
        if (!done) detail_add(dk, 1u, ty == 0, ty == 1, akey, aval, acap, fkey, fval, fcap, sstat, &flags);
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
  }
  __syncthreads();  // this workgroup's details -> the global table
  for (uint32_t x = threadIdx.x; x < TAIL_LAGG; x += blockDim.x)
    if (lkey[x]) detail_add(lkey[x], lval[x][0], lval[x][1], lval[x][2], akey, aval, acap, fkey, fval, fcap, sstat,
                            &flags);
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) {
    won_l += __shfl_xor(won_l, o, 64);
    won_p += __shfl_xor(won_p, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && (won_l | won_p)) {
    atomicAdd(&counters[8], won_l);  // (u32 words 8 and 9 of the tail's counter block)
    atomicAdd(&counters[9], won_p);
  }
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

void launch_tail(hipStream_t s, const unsigned long long *keys, const unsigned long long *n_keys, uint64_t n_max,
                 const uint32_t *svc, const uint32_t *cls, const uint32_t *lsvc_of_cls, const uint32_t *usn,
                 uint32_t n_ep, uint32_t n_cls, unsigned long long *lset, uint64_t lcap, unsigned long long *akey,
                 uint32_t *aval, uint64_t acap, unsigned long long *pset, uint64_t pcap, unsigned long long *pkey,
                 uint32_t *pval, uint64_t pacap, uint8_t *hasin, unsigned long long *fkey, uint32_t *fval,
                 uint64_t fcap, uint32_t *sstat, uint32_t *rel, uint32_t n_dist, unsigned int *counters,
                 uint32_t *links_out, uint32_t *pairs_out, unsigned long long *out_counts, uint32_t knobs) {
  const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_max + 255) / 256, 1024));
  hipLaunchKernelGGL(k_tail_links, dim3(g), dim3(256), 0, s, keys, n_keys, svc, cls, lsvc_of_cls, usn, n_ep, n_cls,
                     lset, lcap, akey, aval, acap, pset, pcap, pkey, pval, pacap, hasin, fkey, fval, fcap, sstat, rel,
                     n_dist, counters, knobs);
  const uint32_t ga = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((acap + 255) / 256, TAIL_COMPACT_BLOCKS));
  hipLaunchKernelGGL(k_tail_compact<0>, dim3(ga), dim3(256), 0, s, akey, aval, acap, links_out, out_counts, rel, n_dist,
                     counters);
  const uint32_t gp = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((pacap + 255) / 256, TAIL_COMPACT_BLOCKS));
  hipLaunchKernelGGL(k_tail_compact<1>, dim3(gp), dim3(256), 0, s, pkey, pval, pacap, pairs_out, out_counts + 1, rel,
                     n_dist, counters);
}

}  // namespace kmz
