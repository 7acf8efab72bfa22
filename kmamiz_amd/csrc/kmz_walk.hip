// kmz_walk.hip -- K4 by chain interning, one workgroup per tile.
//
// The reference walks every SERVER row up its non-CLIENT ancestors
// (Traces.ts:138-208); chain interning (kmz_chain.hip) emits each distinct
// ancestry's edge keys once.  k4_chain<false> does that with persistent
// workgroups that prefetch the next tile into registers; its per-tile chain of
// round trips (window loads, the endpoint gather, the walk, the chain-table
// probe, the leaders' claims) is hidden only by the 4 workgroups a CU holds at
// its 123 VGPRs.  Measured on config 3 (10^8 spans): 1.07 ms, of which the
// window loads and LDS fill alone take 0.51 ms (KMZ_ABLATE bit 16) and the
// probes 0.4 ms.
//
// k4_tile keeps no state across tiles: one 256-thread workgroup per 1024-span
// tile (+ 128-span halos), no prefetch registers, so that more workgroups
// fit a CU and their round trips overlap each other.  The window is loaded,
// its endpoints gathered (per-shape table, L2-resident), built as 16-byte LDS
// records, and walked / probed / settled by the rounds shared with the fused
// kernel (kmz_walkw.h).  The staged keys, claimed slots and deferred checks go
// to the run's global lists (k_chain_settle_list), as the fused kernel's.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_walkw.h"

namespace kmz {

#ifndef KMZ_TILE_T
#define KMZ_TILE_T 960  // spans per tile: a tile's ~T/2 non-CLIENT spans fit one round of 2 x 256 walkers
#endif
#ifndef KMZ_TILE_TW
#define KMZ_TILE_TW 2  // walkers per thread and round
#endif
constexpr uint32_t WT = KMZ_TILE_T, WH = 128, WW = WT + 2 * WH;
constexpr int WTT = 256, WTW = KMZ_TILE_TW;
constexpr int WPW = (WW + WTT - 1) / WTT;  // window slots per thread
constexpr int WPT = (WT + WTT - 1) / WTT;  // tile slots per thread
static_assert(WW <= 0xFFFD, "window-local indices below the W_* markers");
#ifndef KMZ_TILE_WAVES
#define KMZ_TILE_WAVES 5
#endif

__global__ void __launch_bounds__(WTT, KMZ_TILE_WAVES) k4_tile(const uint8_t *__restrict__ kind,
                                                               const uint32_t *__restrict__ shape,
                                                               const uint32_t *__restrict__ cparent, uint32_t n,
                                                               const uint4 *__restrict__ etab, uint32_t n_shapes,
                                                               uint32_t *__restrict__ tile_stats, ChainRun a) {
  __shared__ uint4 lrec[WW];
  __shared__ uint16_t wlist[WT];
  __shared__ ChainLds L;
  __shared__ uint32_t wcount;
  __shared__ uint32_t red[WTT / 64][4];
  const uint32_t t0 = blockIdx.x * WT, t1 = min(n, t0 + WT);
  const uint32_t w0 = t0 > WH ? t0 - WH : 0, w1 = min(n, t1 + WH), wn = w1 - w0, toff = t0 - w0;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t flags = 0;
  // the window's columns, every load in flight together (clamped, unconditional)
  uint32_t c[WPW], sh[WPW];
  uint8_t k[WPW];
#pragma unroll
  for (int q = 0; q < WPW; ++q) {
    const uint32_t j = min(w0 + q * WTT + threadIdx.x, n - 1);
    c[q] = cparent[j];
    k[q] = kind[j];
    sh[q] = shape[j];
  }
  chain_lds_init(L);
  if (threadIdx.x == 0) wcount = 0;
  // each non-CLIENT slot's endpoint and SERVER element hash (k_chain_etab;
  // a CLIENT slot's record holds neither, so half the window skips the gather)
  uint3 e[WPW];
#pragma unroll
  for (int q = 0; q < WPW; ++q)  // (unconditional: a CLIENT slot gathers entry 0, unused; see k4_chain)
    e[q] = *reinterpret_cast<const uint3 *>(etab + ((k[q] != KIND_CLIENT && sh[q] < n_shapes) ? sh[q] : 0));
  // window -> LDS records {element hash, endpoint, local contracted parent | kind << 16}
  bool other = false;  // a span neither SERVER nor CLIENT in the window (rows' lastUsage path)
#pragma unroll
  for (int q = 0; q < WPW; ++q) {
    const uint32_t jl = q * WTT + threadIdx.x;
    if (jl >= wn) continue;
    const bool client = k[q] == KIND_CLIENT;
    const uint32_t ep = (client || sh[q] >= n_shapes) ? NONE : e[q].x;
    const uint32_t cp =
        c[q] == NONE ? W_NONE : (c[q] == CYC ? W_CYC : ((c[q] >= w0 && c[q] < w1) ? c[q] - w0 : W_OUT));
    uint64_t el = ((uint64_t)e[q].z << 32) | e[q].y;  // SERVER
    if (client) el = 0;
    else if ((k[q] & 3) != KIND_SERVER || sh[q] >= n_shapes) el = sig_elem(ep, k[q] == KIND_SERVER, a.seed);  // (rare)
    lrec[jl] = make_uint4((uint32_t)el, (uint32_t)(el >> 32), ep, cp | ((uint32_t)(k[q] & 3) << 16));
    other |= (k[q] & 3) != KIND_SERVER && !client;
  }
  // the tile's non-CLIENT spans into wlist (one LDS add per wave and slot),
  // from the kinds still in registers (tile slot jl = toff + q * WTT + t is
  // window slot jl, i.e. register (jl / WTT, jl % WTT) of its thread: read
  // back from LDS instead)
  const bool any_other = __syncthreads_or(other);
#pragma unroll
  for (int q = 0; q < WPT; ++q) {
    const uint32_t jl = toff + q * WTT + threadIdx.x;
    const bool in = w0 + jl < t1 && q * WTT + threadIdx.x < WT;
    const bool isw = in && ((lrec[min(jl, WW - 1)].w >> 16) & 3) != KIND_CLIENT;
    if (a.rowpos_out && in && !isw) a.rowpos_out[w0 + jl] = NONE64;
    const uint64_t mk = __ballot(isw);
    uint32_t b = 0;
    if (lane == 0 && mk) b = atomicAdd(&wcount, (uint32_t)__popcll(mk));
    b = __shfl(b, 0, 64);
    if (isw) wlist[b + __popcll(mk & ((1ull << lane) - 1))] = (uint16_t)(jl - toff);
  }
  __syncthreads();
  uint32_t rows = 0, rel = 0, maxd = 0, fresh_n = 0;
  chain_walk_rounds<WW, WTT, WTW>(lrec, wlist, wcount, w0, toff, any_other, L, a, rows, rel, maxd, fresh_n, flags);
  if (flags) atomicOr(&a.counters[C_FLAGS], flags);
  chain_tile_stats<WTT>(rows, rel, maxd, fresh_n, red, tile_stats);
}

// k4_tile8 (round 5): the same tiles and rounds over 8-byte window records
// (Rec8: the packed kind | element id word and the window parent).  The
// element ids are shapes whenever the dependency table maps every shape into
// range (a.id_ep set, BY_SHAPE): a window slot is then three plain loads
// (contracted parent, kind, shape) and one 8-byte LDS store, with no dependent
// shape -> endpoint gather before the window can be built; only a leader
// staging a new chain's keys (and the rare non-SERVER ancestor) maps shapes
// to endpoints.  A chain of shapes determines its chain of endpoints, so
// interning by shape is exact; it only interns less where several shapes
// share an endpoint (one shape per endpoint on the synthetic meshes).
// Otherwise the endpoints are gathered per slot (!BY_SHAPE).  Half the LDS of
// k4_tile and fewer registers: KMZ_TILE8_WAVES workgroups per CU.
#ifndef KMZ_TILE8_WAVES
#define KMZ_TILE8_WAVES 7
#endif
template <bool BY_SHAPE>
__global__ void __launch_bounds__(WTT, KMZ_TILE8_WAVES) k4_tile8(const uint8_t *__restrict__ kind,
                                                                 const uint32_t *__restrict__ shape,
                                                                 const uint32_t *__restrict__ cparent, uint32_t n,
                                                                 const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                                 uint32_t *__restrict__ tile_stats, ChainRun a) {
  __shared__ uint2 lrec[WW];
  __shared__ uint16_t wlist[WT];
  __shared__ ChainLds L;
  __shared__ uint32_t wcount;
  __shared__ uint32_t red[WTT / 64][4];
  const uint32_t t0 = blockIdx.x * WT, t1 = min(n, t0 + WT);
  const uint32_t w0 = t0 > WH ? t0 - WH : 0, w1 = min(n, t1 + WH), wn = w1 - w0, toff = t0 - w0;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t flags = 0;
  uint32_t c[WPW], e[WPW];
  uint8_t k[WPW];
  // (the window's columns from workgroup-uniform bases, so that every load
  // takes a 32-bit lane offset: no 64-bit address arithmetic per slot)
  const uint32_t *__restrict__ cpw = cparent + w0;
  const uint8_t *__restrict__ kw = kind + w0;
  const uint32_t *__restrict__ sw = shape + w0;
  const uint32_t last = n - 1 - w0;
#pragma unroll
  for (int q = 0; q < WPW; ++q) {  // clamped, unconditional: every load in flight together
    const uint32_t j = min((uint32_t)(q * WTT) + threadIdx.x, last);
    c[q] = cpw[j];
    k[q] = kw[j];
    e[q] = sw[j];
  }
#pragma unroll
  for (int q = 0; q < WPW; ++q) {
    const bool none = k[q] == KIND_CLIENT || e[q] >= n_shapes;
    if constexpr (BY_SHAPE)
      e[q] = epk_pack(k[q], none ? NONE : e[q]);
    else
      e[q] = epk_pack(k[q], none ? NONE : dep_ep[e[q]]);
  }
  chain_lds_init(L);
  if (threadIdx.x == 0) wcount = 0;
  bool other = false;  // a span neither SERVER nor CLIENT in the window (rows' lastUsage path)
#pragma unroll
  for (int q = 0; q < WPW; ++q) {
    const uint32_t jl = q * WTT + threadIdx.x;
    if (jl >= wn) continue;
    // (branch-free: in-window offset, else W_OUT; NONE and CYC on top)
    const uint32_t rel = c[q] - w0;
    uint32_t cp = rel < wn ? rel : (uint32_t)W_OUT;
    cp = c[q] == NONE ? (uint32_t)W_NONE : cp;
    cp = c[q] == CYC ? (uint32_t)W_CYC : cp;
    lrec[jl] = make_uint2(e[q], cp | ((uint32_t)(k[q] & 3) << 16));
    other |= (k[q] & 3) != KIND_SERVER && k[q] != KIND_CLIENT;
  }
  const bool any_other = __syncthreads_or(other);
#pragma unroll
  for (int q = 0; q < WPT; ++q) {
    const uint32_t jl = toff + q * WTT + threadIdx.x;
    const bool in = w0 + jl < t1 && q * WTT + threadIdx.x < WT;
    const bool isw = in && Rec8::kind(lrec[min(jl, WW - 1)]) != KIND_CLIENT;
    if (a.rowpos_out && in && !isw) a.rowpos_out[w0 + jl] = NONE64;
    const uint64_t mk = __ballot(isw);
    uint32_t b = 0;
    if (lane == 0 && mk) b = atomicAdd(&wcount, (uint32_t)__popcll(mk));
    b = __shfl(b, 0, 64);
    if (isw) wlist[b + __popcll(mk & ((1ull << lane) - 1))] = (uint16_t)(jl - toff);
  }
  __syncthreads();
  uint32_t rows = 0, rel = 0, maxd = 0, fresh_n = 0;
  chain_walk_rounds<WW, WTT, WTW, Rec8>(lrec, wlist, wcount, w0, toff, any_other, L, a, rows, rel, maxd, fresh_n,
                                        flags);
  if (flags) atomicOr(&a.counters[C_FLAGS], flags);
  chain_tile_stats<WTT>(rows, rel, maxd, fresh_n, red, tile_stats);
}

// k4_tile9 (round 6): k4_tile8's tiles and chains, built to issue fewer VALU
// instructions (k4_tile8: ~1030 per wave, VALU busy 79 % of its SIMD cycles):
// * each window slot's element hash is computed once, when the window is
//   built, and kept in LDS beside a 4-byte record {window parent (11 bits),
//   kind (2), id (19)}: a walk step is two LDS reads, a rotate and an xor,
//   with no multiply (k4_tile8 recomputed sig_elem, a 32 x 64-bit product, at
//   every step of every walker);
// * the walk ends on three sentinel slots (root, CLIENT loop, outside the
//   window) whose parent is themselves and whose element is 0, so a finished
//   walker needs no select: it keeps rotating its fold, which is rotated back
//   once at the end by the steps it idled; the depth is a count of active steps;
// * the tile's non-CLIENT spans are compacted by wave ballots and one table
//   of per-wave counts (no LDS atomic per wave and slot).
// The sigs, the probe, the leaders and the row counts are k4_tile8's
// (chain_round_tail): same chains, same sigs, same lists.  Ids (shapes, or
// endpoints when gathered) must be < ID9_NONE (checked on the host).
constexpr uint32_t S9_ROOT = WW, S9_CYC = WW + 1, S9_OUT = WW + 2, W9 = WW + 3;
constexpr uint32_t P9_BITS = 11, ID9_NONE = (1u << 19) - 1;
static_assert(W9 <= (1u << P9_BITS), "window slots and sentinels in 11 bits");
__device__ __forceinline__ uint32_t p9_parent(uint32_t pk) { return pk & ((1u << P9_BITS) - 1); }
__device__ __forceinline__ uint32_t p9_kind(uint32_t pk) { return (pk >> P9_BITS) & 3; }
__device__ __forceinline__ uint32_t p9_id(uint32_t pk) {
  const uint32_t id = pk >> (P9_BITS + 2);
  return id == ID9_NONE ? NONE : id;
}
#ifndef KMZ_TILE9_WAVES
#define KMZ_TILE9_WAVES 7
#endif
#ifndef KMZ_TILE9_MAP
#define KMZ_TILE9_MAP 128  // leader-map entries (16 B each); 256 spilled 2 VGPRs, walk 0.955 -> 0.946 ms at 128
#endif
template <bool BY_SHAPE>
__global__ void __launch_bounds__(WTT, KMZ_TILE9_WAVES) k4_tile9(const uint8_t *__restrict__ kind,
                                                                 const uint32_t *__restrict__ shape,
                                                                 const uint32_t *__restrict__ cparent, uint32_t n,
                                                                 const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                                 uint32_t *__restrict__ tile_stats, ChainRun a) {
  constexpr int NW = WTT / 64;
  __shared__ uint64_t lel[W9];  // element hash (0 on the sentinels)
  __shared__ uint32_t lpk[W9];  // window parent | kind << 11 | id << 13
  __shared__ uint16_t wlist[WT];
  __shared__ ChainLdsT<KMZ_TILE9_MAP> L;
  __shared__ uint32_t wcnt[WPT][NW];
  __shared__ uint32_t red[NW][4];
  const uint32_t t0 = blockIdx.x * WT, t1 = min(n, t0 + WT);
  const uint32_t w0 = t0 > WH ? t0 - WH : 0, w1 = min(n, t1 + WH), wn = w1 - w0, toff = t0 - w0;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t flags = 0;
  uint32_t c[WPW], e[WPW];
  uint8_t k[WPW];
  const uint32_t *__restrict__ cpw = cparent + w0;
  const uint8_t *__restrict__ kw = kind + w0;
  const uint32_t *__restrict__ sw = shape + w0;
  const uint32_t last = n - 1 - w0;
#pragma unroll
  for (int q = 0; q < WPW; ++q) {  // clamped, unconditional: every load in flight together
    const uint32_t j = min((uint32_t)(q * WTT) + threadIdx.x, last);
    c[q] = cpw[j];
    k[q] = kw[j];
    e[q] = sw[j];
  }
  chain_lds_init(L);
  if (threadIdx.x < 3) {
    lpk[WW + threadIdx.x] = (WW + threadIdx.x) | ((uint32_t)KIND_CLIENT << P9_BITS) | (ID9_NONE << (P9_BITS + 2));
    lel[WW + threadIdx.x] = 0;
  }
  bool other = false;  // a span neither SERVER nor CLIENT in the window (rows' lastUsage path)
#pragma unroll
  for (int q = 0; q < WPW; ++q) {
    const uint32_t jl = q * WTT + threadIdx.x;
    const uint32_t kk = k[q] & 3;
    const bool none = kk == KIND_CLIENT || e[q] >= n_shapes;
    uint32_t id;
    if constexpr (BY_SHAPE)
      id = none ? NONE : e[q];
    else
      id = none ? NONE : dep_ep[e[q]];
    const uint32_t rel = c[q] - w0;
    uint32_t cp = rel < wn ? rel : S9_OUT;
    cp = c[q] == NONE ? S9_ROOT : cp;
    cp = c[q] == CYC ? S9_CYC : cp;
    if (jl < wn) {
      lpk[jl] = cp | (kk << P9_BITS) | (min(id, ID9_NONE) << (P9_BITS + 2));
      lel[jl] = sig_elem(id, kk == KIND_SERVER, a.seed);
    }
    other |= jl < wn && kk != KIND_SERVER && kk != KIND_CLIENT;
  }
  const bool any_other = __syncthreads_or(other);
  // the tile's non-CLIENT spans -> wlist: a ballot per slot row, per-wave
  // counts in LDS, each lane's place from them and its rank in the ballot
  uint64_t mk[WPT];
#pragma unroll
  for (int q = 0; q < WPT; ++q) {
    const uint32_t jl = toff + q * WTT + threadIdx.x;
    const bool in = w0 + jl < t1 && q * WTT + threadIdx.x < WT;
    const bool isw = in && p9_kind(lpk[min(jl, WW - 1)]) != KIND_CLIENT;
    if (a.rowpos_out && in && !isw) a.rowpos_out[w0 + jl] = NONE64;
    mk[q] = __ballot(isw);
    if (lane == 0) wcnt[q][wave] = (uint32_t)__popcll(mk[q]);
  }
  __syncthreads();
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < WPT; ++q) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t x = wcnt[q][w];
      before += w < (int)wave ? x : 0;
      all += x;
    }
    const uint32_t jl = toff + q * WTT + threadIdx.x;
    if ((mk[q] >> lane) & 1) wlist[m + before + __popcll(mk[q] & ((1ull << lane) - 1))] = (uint16_t)(jl - toff);
    m += all;
  }
  __syncthreads();
  uint32_t rows = 0, rel = 0, maxd = 0, fresh_n = 0;
  const bool hash_on = !(a.ablate & (1u << 16));  // diagnostic knob: no hashing / probing / inserting
  constexpr int TW = WTW;
  for (uint32_t r0 = 0; r0 < m; r0 += TW * WTT) {
    uint64_t sg[TW], ps[TW], acc[TW];
    uint32_t dd[TW], wa[TW], myep[TW], jq[TW];
    uint8_t st[TW], kq[TW];
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      const uint32_t idx = r0 + q * WTT + threadIdx.x;
      const bool on = idx < m;
      const uint32_t jl = on ? toff + wlist[idx] : S9_ROOT;  // (the root sentinel: a CLIENT, no walker)
      jq[q] = jl;
      const uint32_t pk = lpk[jl];
      kq[q] = (uint8_t)p9_kind(pk);
      myep[q] = p9_id(pk);
      sg[q] = lel[jl];  // the element hash until the walk is done
      acc[q] = 0;
      dd[q] = 0;
      st[q] = on ? S_DONE : S_NONE;
      wa[q] = (on && hash_on) ? p9_parent(pk) : S9_ROOT;
      // (ids that are shapes are in range whenever they are not NONE)
      if (on && hash_on && kq[q] == KIND_SERVER && (BY_SHAPE ? myep[q] == NONE : myep[q] >= a.n_ep)) flags |= F_RANGE;
    }
    // the TW walks of a thread step together; a finished walk sits on its
    // sentinel (parent itself, element 0) and only rotates its fold
    uint32_t steps = 0;
    auto walk = [&](auto other_tag) {
      constexpr bool OTHER = decltype(other_tag)::value;
      for (; steps < WIN_DEPTH; ++steps) {
        bool go = false;
#pragma unroll
        for (int q = 0; q < TW; ++q) go |= wa[q] < WW;
        if (__ballot(go) == 0) break;
        uint32_t pk[TW];
        uint64_t el[TW];
#pragma unroll
        for (int q = 0; q < TW; ++q) {
          pk[q] = lpk[wa[q]];
          el[q] = lel[wa[q]];
        }
#pragma unroll
        for (int q = 0; q < TW; ++q) {
          const bool act = wa[q] < WW;
          if (OTHER && act && kq[q] == KIND_SERVER && p9_kind(pk[q]) != KIND_SERVER) {
            // (rare) a non-SERVER ancestor of a row: its lastUsage
            const uint32_t x = run_ep(a, p9_id(pk[q]));
            if (x < a.n_ep)
              atomicMax(&a.ep_ts[x], (unsigned long long)((uint64_t)a.ts[w0 + wa[q]] ^ TS_BIAS));
            else
              flags |= F_RANGE;
          }
          dd[q] += act ? 1u : 0u;
          acc[q] = sig_step(acc[q], el[q]);
          wa[q] = p9_parent(pk[q]);
        }
      }
    };
    if (any_other)
      walk(std::true_type{});
    else
      walk(std::false_type{});
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      if (st[q] != S_DONE || !hash_on) {
        sg[q] = 0;
        continue;
      }
      if (wa[q] != S9_ROOT) {  // S9_OUT: leaves the window (or deeper than WIN_DEPTH); S9_CYC: CLIENT loop
        if (wa[q] == S9_CYC) flags |= F_CYCLE;
        st[q] = S_PEND;
        sg[q] = 0;
        continue;
      }
      const uint32_t d = dd[q];
      const uint64_t f = rotl64(acc[q], (64u - (SIG_R * (steps - d)) % 64u) % 64u);  // the idle steps' rotations undone
      ps[q] = d ? sig_final(f, d - 1, a.seed, &flags) : ROOT_SIG;
      sg[q] = sig_final(rotl64(sg[q], SIG_R * d) ^ f, d, a.seed, &flags);
      if (a.ablate & (1u << 24)) {  // test knob: 4-bit sigs, i.e. collisions (F_SIG, then a retry with another seed)
        sg[q] = (sg[q] & 0xF) + 2;
        ps[q] = d ? (ps[q] & 0xF) + 2 : ROOT_SIG;
      }
      if (!(a.ablate & (1u << 17))) st[q] = S_PUT;  // diagnostic knob: hash only
    }
    chain_round_tail<WTT, TW>(sg, ps, st, kq, dd, jq, myep, w0, [&](uint32_t x) {
      const uint32_t pk = lpk[x];
      return AncRec{p9_id(pk), p9_kind(pk), p9_parent(pk)};
    }, L, a, rows, rel, maxd, fresh_n, flags);
    __syncthreads();  // (wlist / imap reads of this round before the next round's leaders)
  }
  if (flags) atomicOr(&a.counters[C_FLAGS], flags);
  chain_tile_stats<WTT>(rows, rel, maxd, fresh_n, red, tile_stats);
}

bool chain_tile9_fits(uint32_t n_ids) { return n_ids < ID9_NONE; }

void launch_chain_tile9(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint32_t *cparent, uint32_t n,
                        const uint32_t *dep_ep, uint32_t n_shapes, uint32_t *tile_stats, const ChainRun &a) {
  if (!n) return;
  if (a.id_ep)
    hipLaunchKernelGGL(k4_tile9<true>, dim3(walk_tiles(n)), dim3(WTT), 0, s, kind, shape, cparent, n, dep_ep,
                       n_shapes, tile_stats, a);
  else
    hipLaunchKernelGGL(k4_tile9<false>, dim3(walk_tiles(n)), dim3(WTT), 0, s, kind, shape, cparent, n, dep_ep,
                       n_shapes, tile_stats, a);
}

uint32_t walk_tiles(uint32_t n) { return (n + WT - 1) / WT; }

void launch_chain_tile8(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint32_t *cparent, uint32_t n,
                        const uint32_t *dep_ep, uint32_t n_shapes, uint32_t *tile_stats, const ChainRun &a) {
  if (!n) return;
  if (a.id_ep)
    hipLaunchKernelGGL(k4_tile8<true>, dim3(walk_tiles(n)), dim3(WTT), 0, s, kind, shape, cparent, n, dep_ep,
                       n_shapes, tile_stats, a);
  else
    hipLaunchKernelGGL(k4_tile8<false>, dim3(walk_tiles(n)), dim3(WTT), 0, s, kind, shape, cparent, n, dep_ep,
                       n_shapes, tile_stats, a);
}

void launch_chain_tile(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint32_t *cparent, uint32_t n,
                       const uint32_t *dep_ep, uint32_t n_shapes, uint4 *etab, uint32_t *tile_stats, const ChainRun &a) {
  if (!n) return;
  launch_chain_etab(s, dep_ep, n_shapes, a.seed, etab);
  hipLaunchKernelGGL(k4_tile, dim3(walk_tiles(n)), dim3(WTT), 0, s, kind, shape, cparent, n, etab, n_shapes,
                     tile_stats, a);
}

}  // namespace kmz
