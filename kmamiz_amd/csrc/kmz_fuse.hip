// kmz_fuse.hip -- K2 + K4 over one LDS window: the parent join, the CLIENT
// contraction and the chain walk of chain interning in one kernel.
//
// Separately, k_join_window (kmz_join.hip) stages a 2048-span tile and its
// 256-span halos to resolve parents (Traces.ts:117-137), and k4_chain
// (kmz_chain.hip) then reads the contracted parents, kinds and shapes of every
// 1024-span tile and its halos back from HBM to walk each row's ancestry
// (Traces.ts:138-208).  Here one workgroup does both over the join's window:
//
//   1. the join as k_join_window: ids into the LDS two-choice hash, every
//      window span's parent looked up (halo spans too: the walk passes
//      through them), CLIENT chains contracted for every non-CLIENT span of
//      the window; the tile's cparent / dp / counters exactly as the join
//      writes them, and its hashed ids binned for the certificate;
//   2. the walk as k4_chain<false>: the window rebuilt as 16-byte records
//      {element hash, endpoint, window-local contracted parent | kind} in the
//      LDS the join's hash used; the tile's non-CLIENT spans compacted, walked,
//      hashed, probed against the chain table; one leader per new chain stages
//      its keys and claims the slot.
//
// Saved against the two kernels: the walk's window loads (cparent, kind,
// shape with their halo, ~11 B/span), its endpoint gather's second round trip
// and a launch.  Ancestries that leave the window -- a parent outside it
// (MISS), a CLIENT chain leaving it (PEND), or a contracted parent beyond it --
// go to the pending list, which k4_chain_pend finishes over the global
// cparent after the MISS / PEND fix-ups, as for k4_chain.  The lists k4_chain
// keeps per persistent workgroup (staged keys, deferred checks, claimed
// chain-table slots) are global here, reserved by one atomic per new chain.
// Direct enumeration (config 5) keeps the two kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "kmz_joinw.h"
#include "kmz_walkw.h"

namespace kmz {

constexpr int FPW = JW / JTT;  // window slots per thread
constexpr int FPT = JT / JTT;  // tile slots per thread
constexpr int FTW = 2;         // walkers per thread and round

__device__ unsigned long long g_fuse_dbg[16];  // diagnostic phase clocks (KMZ_ABLATE bit 22 only)
#define KMZ_FSTAMP(k)                                           \
  if (dbg_t) {                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0 && tprev) tacc[k] += t_ - tprev;       \
    tprev = t_;                                                 \
  }
static_assert(JW * 16 == JW * 8 + JB * 16 + JB * 4, "the walk's records reuse the join's ids, buckets and counts");

__global__ void __launch_bounds__(JTT, 4) k_join_chain(
    const uint64_t *__restrict__ sid, const uint64_t *__restrict__ pid, const uint8_t *__restrict__ kind,
    const uint32_t *__restrict__ shape, const int64_t *__restrict__ ts, uint32_t n, const uint4 *__restrict__ etab,
    uint32_t n_shapes, uint32_t n_ep, uint64_t index_base, uint64_t seed, uint32_t *__restrict__ cparent,
    uint32_t *__restrict__ dp, unsigned long long *__restrict__ pool1, uint16_t *__restrict__ jdir,
    unsigned int *__restrict__ counters, unsigned long long *__restrict__ ctab, uint64_t ccap,
    unsigned long long *__restrict__ trip, uint64_t tcap, unsigned long long *__restrict__ ep_ts,
    unsigned long long *__restrict__ rowpos_out, uint32_t *__restrict__ plist, uint32_t pcap,
    uint32_t *__restrict__ tile_stats, unsigned long long *__restrict__ stage, uint32_t scap,
    unsigned long long *__restrict__ defer, uint32_t dcap, uint32_t *__restrict__ gpos, uint32_t gcap,
    uint32_t ablate) {
  constexpr uint32_t NW = JTT / 64;
  // 40 KB: the join's ids [JW] u64, buckets [JB] x 16 B and bucket counts [JB]
  // u32; after the certificate's pass 1 the walk's records [JW] x 16 B
  __shared__ uint4 lrec[JW];
  uint64_t *const lsid = reinterpret_cast<uint64_t *>(lrec);
  uint4 *const lbkt = lrec + JW / 2;
  uint32_t *const lcnt = reinterpret_cast<uint32_t *>(lrec + JW / 2 + JB);
  __shared__ uint16_t ldp[JW], lcp[JW];
  __shared__ uint8_t lkind[JW];
  __shared__ uint32_t wcnt[CERT_BINS * NW], wsum[NW];
  __shared__ uint16_t stash[JSTASH];
  __shared__ uint32_t nstash, wcount;
  __shared__ ChainLds L;  // the walk's leader map and list reservations
  __shared__ uint16_t wlist[JT];
  __shared__ uint32_t red[NW][4];
  const bool dbg_t = (ablate & (1u << 22)) != 0;
  unsigned long long tprev = 0, tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // (stamps 0-6)
  KMZ_FSTAMP(0);
  const uint32_t t0 = blockIdx.x * JT, t1 = min(n, t0 + JT);
  const uint32_t w0 = t0 > JH ? t0 - JH : 0, w1 = min(n, t1 + JH);
  const uint32_t toff = t0 - w0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t flags = 0;
  for (uint32_t k = threadIdx.x; k < JB; k += JTT) {
    lbkt[k] = make_uint4(0, 0, 0, 0);
    lcnt[k] = 0;
  }
  chain_lds_init(L);
  if (threadIdx.x == 0) nstash = wcount = 0;
  // ---- 1. the join --------------------------------------------------------
  uint64_t s[FPW], p[FPW];
  uint8_t k[FPW];
  uint32_t sh[FPW];
#pragma unroll
  for (int q = 0; q < FPW; ++q) {  // clamped and unconditional: every load in flight together
    const uint32_t jj = min(w0 + q * JTT + threadIdx.x, n - 1);
    s[q] = sid[jj];
    p[q] = pid[jj];
    k[q] = kind[jj];
    sh[q] = shape[jj];
  }
  uint32_t hs[FPW];
#pragma unroll
  for (int q = 0; q < FPW; ++q) {
    const uint32_t jl = q * JTT + threadIdx.x;
    if (w0 + jl >= w1) {
      s[q] = p[q] = 0;
      k[q] = 0;
    }
    hs[q] = jfold(s[q]);
    if (w0 + jl < w1) {
      lsid[jl] = s[q];
      lkind[jl] = k[q];
    }
  }
  // the endpoint gather of the walk's records, in flight through the join
  // (used after the certificate's pass 1)
  uint4 e[FPW];
#pragma unroll
  for (int q = 0; q < FPW; ++q) e[q] = etab[sh[q] < n_shapes ? sh[q] : 0];
  __syncthreads();
  KMZ_FSTAMP(0);
  bool ovf = false;
  {  // insert: the emptier of the two buckets, else the other, else the stash (k_join_window)
    uint32_t bq[FPW], sq[FPW];
    bool iq[FPW];
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      iq[q] = w0 + q * JTT + threadIdx.x < w1 && s[q] != 0;
      const uint32_t b1 = jb1(hs[q]), b2 = jb2(hs[q]);
      bq[q] = lcnt[b1] <= lcnt[b2] ? b1 : b2;
    }
#pragma unroll
    for (int q = 0; q < FPW; ++q) sq[q] = iq[q] ? atomicAdd(&lcnt[bq[q]], 1u) : 0u;
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t jl = q * JTT + threadIdx.x;
      if (!iq[q]) continue;
      uint32_t b = bq[q], slot = sq[q];
      if (slot >= 8) {
        b = b ^ jb1(hs[q]) ^ jb2(hs[q]);
        slot = atomicAdd(&lcnt[b], 1u);
      }
      const uint16_t e = (uint16_t)((jfp(hs[q]) << 12) | (jl + 1));
      if (slot < 8) {
        reinterpret_cast<uint16_t *>(&lbkt[b])[slot] = e;
      } else {
        const uint32_t t = atomicAdd(&nstash, 1u);
        if (t < JSTASH)
          stash[t] = e;
        else
          ovf = true;
      }
    }
  }
  __syncthreads();
  KMZ_FSTAMP(1);
  {  // every window span's parent (the halo's too: the walk passes through them)
    const uint32_t ns = min(nstash, JSTASH);
    uint32_t cq[FPW], hq[FPW], eq[FPW];
    bool nq[FPW];
    uint16_t rq[FPW];
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t jl = q * JTT + threadIdx.x;
      nq[q] = w0 + jl < w1 && p[q] != 0 && !(ablate & 512);
      rq[q] = nq[q] ? L_MISS : L_NONE;
      hq[q] = jfold(p[q]);
      const uint32_t f = jfp(hq[q]);
      const uint4 x = lbkt[nq[q] ? jb1(hq[q]) : 0], y = lbkt[nq[q] ? jb2(hq[q]) : 0];
      const uint32_t c[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
      const uint32_t pat = (f << 12) | (f << 28);
      uint32_t cand = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t v = c[t], z = v ^ pat;
        cand |= ((z & 0xF000u) == 0 ? 1u : 0u) << (2 * t);
        cand |= ((z & 0xF0000000u) == 0 ? 1u : 0u) << (2 * t + 1);
      }
      cq[q] = nq[q] ? cand : 0;
    }
    const uint16_t *lbkt16 = reinterpret_cast<const uint16_t *>(lbkt);
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t t = __builtin_ctz(cq[q] | 0x10000u);
      const uint32_t b = t < 8 ? jb1(hq[q]) : jb2(hq[q]);
      eq[q] = cq[q] ? lbkt16[b * 8 + (t & 7)] & 0xFFF : 0;
    }
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const bool hit = eq[q] && lsid[eq[q] ? eq[q] - 1 : 0] == p[q];
      if (hit) rq[q] = (uint16_t)(eq[q] - 1);
      if (!hit) cq[q] &= cq[q] - 1;
      else cq[q] = 0;
    }
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t jl = q * JTT + threadIdx.x;
      if (w0 + jl >= w1) continue;
      uint32_t r = rq[q];
      uint32_t cand = cq[q];
      while (cand) {  // (rare) further candidates
        const uint32_t t = __builtin_ctz(cand);
        cand &= cand - 1;
        const uint32_t en = lbkt16[(t < 8 ? jb1(hq[q]) : jb2(hq[q])) * 8 + (t & 7)] & 0xFFF;
        if (lsid[en - 1] == p[q]) {
          r = en - 1;
          break;
        }
      }
      if (nq[q] && r == L_MISS) {
        const uint32_t f = jfp(hq[q]);
        for (uint32_t t = 0; t < ns; ++t) {
          const uint32_t en = stash[t];
          if ((en >> 12) == f && lsid[(en & 4095) - 1] == p[q]) r = (en & 4095) - 1;
        }
      }
      ldp[jl] = (uint16_t)r;
    }
  }
  if (ovf) atomicOr(&counters[C_CERT], CERT_OVF);
  __syncthreads();
  KMZ_FSTAMP(2);
  // CLIENT contraction of every non-CLIENT window span, in lockstep: the
  // window-local contracted parent, or W_NONE (root) / W_OUT (MISS or PEND:
  // outside the window) / W_CYC
  {
    uint32_t j[FPW], hops[FPW], cpl[FPW];
    bool act[FPW];
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t jl = q * JTT + threadIdx.x;
      const bool ok = w0 + jl < w1;
      act[q] = ok && k[q] != KIND_CLIENT;
      j[q] = ok ? ldp[jl] : L_NONE;
      cpl[q] = W_NONE;
      hops[q] = 0;
    }
    for (;;) {
      bool any = false;
      uint8_t kj[FPW];
#pragma unroll
      for (int q = 0; q < FPW; ++q) kj[q] = (act[q] && j[q] < JW) ? lkind[j[q]] : 0;
#pragma unroll
      for (int q = 0; q < FPW; ++q) {
        if (!act[q]) continue;
        if (j[q] >= JW) {
          cpl[q] = j[q] == L_NONE ? W_NONE : W_OUT;
          act[q] = false;
        } else if (kj[q] != KIND_CLIENT) {
          cpl[q] = j[q];
          act[q] = false;
        } else if (++hops[q] > MAX_DEPTH) {
          cpl[q] = W_CYC;
          act[q] = false;
        } else {
          j[q] = ldp[j[q]];
          any = true;
        }
      }
      if (!any) break;
    }
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t jl = q * JTT + threadIdx.x;
      if (w0 + jl < w1) lcp[jl] = (uint16_t)cpl[q];
    }
  }
  __syncthreads();
  // the tile's outputs, exactly as k_join_window writes them
  uint32_t miss = 0, pend = 0, zero = 0;
  uint64_t hv[FPT];
#pragma unroll
  for (int q = 0; q < FPT; ++q) {
    const uint32_t i = t0 + q * JTT + threadIdx.x, il = i - w0;
    hv[q] = 0;
    if (i >= t1) continue;
    const uint32_t d0 = ldp[il], cl = lcp[il];
    const uint32_t cp = cl < JW ? w0 + cl : (cl == W_NONE ? NONE : (cl == W_CYC ? CYC : PEND));
    cparent[i] = cp;
    dp[i] = d0 == L_NONE ? NONE : (d0 == L_MISS ? MISSV : w0 + d0);
    miss += d0 == L_MISS;
    pend += cp == PEND;
    const uint64_t key = lsid[il];
    zero += key == 0;
    hv[q] = cert_hash(key);
  }
  for (int o = 32; o > 0; o >>= 1) {
    miss += __shfl_xor(miss, o, 64);
    pend += __shfl_xor(pend, o, 64);
    zero += __shfl_xor(zero, o, 64);
  }
  if (lane == 0) {
    if (miss) atomicAdd(&counters[C_MISS], miss);
    if (pend) atomicAdd(&counters[C_PEND], pend);
    if (zero) atomicOr(&counters[C_FLAGS], F_ZERO_ID);
  }
  // certificate pass 1 (k_join_window): the tile's hashed ids into 64 bins,
  // staged in the bucket region
  for (uint32_t x = threadIdx.x; x < CERT_BINS * NW; x += JTT) wcnt[x] = 0;
  __syncthreads();
  KMZ_FSTAMP(3);
  {
    uint64_t *stg = reinterpret_cast<uint64_t *>(lbkt);
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t rk[FPT];
#if KMZ_RANK_ATOMIC
    // ranks from wave-major LDS bin counters in the dead bucket counts
    // (k_join_window), transposed to bin-major for the scan
    uint32_t *const wmaj = lcnt;
    static_assert(CERT_BINS * NW <= JB, "the wave-major counters live in the bucket counts");
    for (uint32_t x = threadIdx.x; x < CERT_BINS * NW; x += JTT) wmaj[x] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < FPT; ++q)
      rk[q] = t0 + q * JTT + threadIdx.x < t1
                  ? atomicAdd(&wmaj[wv * CERT_BINS + (uint32_t)(hv[q] >> (64 - CERT_B1))], 1u)
                  : 0u;
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < CERT_BINS * NW; x += JTT) wcnt[x] = wmaj[(x % NW) * CERT_BINS + x / NW];
    (void)lt;
#else
#pragma unroll
    for (int q = 0; q < FPT; ++q) {
      const bool ok = t0 + q * JTT + threadIdx.x < t1;
      const uint32_t bin = (uint32_t)(hv[q] >> (64 - CERT_B1));
      const uint64_t peers = match6(bin, __ballot(ok));
      uint32_t prior = 0;
      if (ok) prior = wcnt[bin * NW + wv];
      rk[q] = prior + __popcll(peers & lt);
      if (ok && (peers & lt) == 0) wcnt[bin * NW + wv] = prior + __popcll(peers);
    }
#endif
    __syncthreads();
    block_scan_lds(wcnt, CERT_BINS * NW, wsum);
    if (threadIdx.x < CERT_BINS) jdir[(uint64_t)blockIdx.x * CERT_BINS + threadIdx.x] = (uint16_t)wcnt[threadIdx.x * NW];
#pragma unroll
    for (int q = 0; q < FPT; ++q)
      if (t0 + q * JTT + threadIdx.x < t1) stg[wcnt[(uint32_t)(hv[q] >> (64 - CERT_B1)) * NW + wv] + rk[q]] = hv[q];
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < t1 - t0; x += JTT) pool1[(uint64_t)t0 + x] = stg[x];
  }
  __syncthreads();  // the ids, buckets and staging are dead: the region becomes the walk's records
  KMZ_FSTAMP(4);
  // ---- 2. the walk (k4_chain<false>) --------------------------------------
  bool other = false;  // a span neither SERVER nor CLIENT in the window (rows' lastUsage path)
#pragma unroll
  for (int q = 0; q < FPW; ++q) {
    const uint32_t jl = q * JTT + threadIdx.x;
    const bool in = w0 + jl < w1;
    const bool client = k[q] == KIND_CLIENT;
    const uint32_t ep = (client || sh[q] >= n_shapes) ? NONE : e[q].x;
    uint64_t el = ((uint64_t)e[q].z << 32) | e[q].y;  // SERVER
    if (client) el = 0;
    else if ((k[q] & 3) != KIND_SERVER || sh[q] >= n_shapes) el = sig_elem(ep, k[q] == KIND_SERVER, seed);  // (rare)
    if (in) lrec[jl] = make_uint4((uint32_t)el, (uint32_t)(el >> 32), ep, lcp[jl] | ((uint32_t)(k[q] & 3) << 16));
    other |= in && (k[q] & 3) != KIND_SERVER && !client;
  }
  // the tile's non-CLIENT spans (rows and other kinds) into wlist
#pragma unroll
  for (int q = 0; q < FPT; ++q) {
    const uint32_t jl = toff + q * JTT + threadIdx.x;
    const bool in = w0 + jl < t1;
    const bool isw = in && lkind[jl] != KIND_CLIENT;
    if (rowpos_out && in && !isw) rowpos_out[w0 + jl] = NONE64;
    const uint64_t mk = __ballot(isw);
    uint32_t b = 0;
    if (lane == 0 && mk) b = atomicAdd(&wcount, (uint32_t)__popcll(mk));
    b = __shfl(b, 0, 64);
    if (isw) wlist[b + __popcll(mk & ((1ull << lane) - 1))] = (uint16_t)(jl - toff);
  }
  const bool any_other = __syncthreads_or(other);
  KMZ_FSTAMP(5);
  uint32_t rows = 0, rel = 0, maxd = 0, fresh_n = 0;
  {
    ChainRun a;
    a.ts = ts;
    a.ctab = ctab;
    a.ccap = ccap;
    a.trip = trip;
    a.tcap = tcap;
    a.ep_ts = ep_ts;
    a.rowpos_out = rowpos_out;
    a.plist = plist;
    a.pcap = pcap;
    a.counters = counters;
    a.stage = stage;
    a.scap = scap;
    a.defer = defer;
    a.dcap = dcap;
    a.gpos = gpos;
    a.gcap = gcap;
    a.n_ep = n_ep;
    a.index_base = index_base;
    a.seed = seed;
    a.ablate = ablate;
    chain_walk_rounds<JW, JTT, FTW>(lrec, wlist, wcount, w0, toff, any_other, L, a, rows, rel, maxd, fresh_n, flags);
  }
  KMZ_FSTAMP(6);
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  chain_tile_stats<JTT>(rows, rel, maxd, fresh_n, red, tile_stats);
  if (dbg_t && threadIdx.x == 0)
    for (int kk = 0; kk < 10; ++kk) atomicAdd(&g_fuse_dbg[kk], tacc[kk]);
}

// the staged keys and deferred chain checks of the fused kernel (one global
// list each): keys -> the edge set, checks joined or inserted (every entry the
// tile kernel claimed is published by now)
__global__ void __launch_bounds__(256) k_chain_settle_list(const unsigned long long *__restrict__ stage, uint32_t scap,
                                                           const unsigned long long *__restrict__ defer, uint32_t dcap,
                                                           unsigned long long *__restrict__ trip, uint64_t tcap,
                                                           unsigned long long *__restrict__ ctab, uint64_t ccap,
                                                           unsigned int *__restrict__ counters,
                                                           unsigned long long *__restrict__ stats64,
                                                           uint32_t *__restrict__ gpos, uint32_t gcap, uint32_t spin,
                                                           const uint32_t *__restrict__ id_ep, uint32_t n_ids) {
  const uint32_t m = min(counters[C_FSTAGE], scap), md = min(counters[C_FDEFER], dcap);
  const uint32_t t0 = blockIdx.x * 256 + threadIdx.x, ts = gridDim.x * 256;
  uint32_t flags = 0, fresh = 0;
  // (id_ep: k4_tile8 staged its keys over shape ids; here they become
  // endpoint keys -- the gathers the walk left out)
  for (uint32_t x = t0; x < m; x += ts)
    edge_insert(id_ep ? key_ids_to_eps(stage[x], id_ep, n_ids) : stage[x], trip, tcap, &flags);
  for (uint32_t x = t0; x < md; x += ts) {
    const unsigned long long *r = defer + 2 * (uint64_t)x;
    int rr = 0;
    for (uint32_t t = 0; t < spin && rr == 0; ++t) rr = chain_put(ctab, ccap, r[0], r[1], &flags, gpos, gcap, counters);
    if (rr == 0) flags |= F_SPIN;
    fresh += rr == 1;
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) fresh += __shfl_xor(fresh, o, 64);
  if ((threadIdx.x & 63) == 0 && fresh) atomicAdd(&stats64[S_CHAINS], (unsigned long long)fresh);
}

void launch_join_chain(hipStream_t s, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind,
                       const uint32_t *shape, const int64_t *ts, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes,
                       uint32_t n_ep, uint64_t index_base, uint64_t seed, uint32_t *cparent, uint32_t *dp,
                       unsigned long long *pool1, uint16_t *jdir, unsigned int *counters, void *ctab, uint64_t ccap,
                       unsigned long long *trip, uint64_t tcap, unsigned long long *ep_ts, unsigned long long *rowpos,
                       uint32_t *plist, uint32_t pcap, uint32_t *tile_stats, unsigned long long *stage, uint32_t scap,
                       unsigned long long *defer, uint32_t dcap, uint32_t *gpos, uint32_t gcap, uint4 *etab,
                       uint32_t ablate, bool etab_ok) {
  if (!n) return;
  if (!etab_ok) launch_chain_etab(s, dep_ep, n_shapes, seed, etab);  // (etab_ok: this shape table's, this seed's)
  hipLaunchKernelGGL(k_join_chain, dim3(join_tiles(n)), dim3(JTT), 0, s, sid, pid, kind, shape, ts, n, etab, n_shapes,
                     n_ep, index_base, seed, cparent, dp, pool1, jdir, counters,
                     reinterpret_cast<unsigned long long *>(ctab), ccap, trip, tcap, ep_ts, rowpos, plist, pcap,
                     tile_stats, stage, scap, defer, dcap, gpos, gcap, ablate);
}

void launch_chain_settle_list(hipStream_t s, uint32_t nt, void *ctab, uint64_t ccap, unsigned long long *trip,
                              uint64_t tcap, unsigned int *counters, const uint32_t *tile_stats,
                              unsigned long long *stats64, const unsigned long long *stage, uint32_t scap,
                              const unsigned long long *defer, uint32_t dcap, uint32_t *gpos, uint32_t gcap,
                              uint32_t ablate, const uint32_t *id_ep, uint32_t n_ids) {
  if (!nt) return;
  // (2048 workgroups at any size: the lists' lengths are on the device, and a
  // small batch's keys taken ~8 per thread, each insert a round trip, made
  // this a serial latency chain: 28 / 65 us of the mesh / config 5 ticks)
  hipLaunchKernelGGL(k_chain_settle_list, dim3(2048), dim3(256), 0, s,
                     stage, scap, defer, dcap, trip, tcap, reinterpret_cast<unsigned long long *>(ctab), ccap, counters,
                     stats64, gpos, gcap, spin_bound(ablate), id_ep, n_ids);
  launch_tile_sum(s, tile_stats, nt, 4u, 4u, stats64 + S_ROWS, 2u);  // rows, rel, maxd, chains
}

}  // namespace kmz

extern "C" int kmz__debug_fuse(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmz::g_fuse_dbg), sizeof(kmz::g_fuse_dbg)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(kmz::g_fuse_dbg), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
