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
// diagnostic phase clocks of k4_tile9 (a -DKMZ_T9_CLOCKS=1 build only):
// s_memtime deltas seen by thread 0, summed over workgroups (kmz__debug_walk9)
#ifndef KMZ_T9_TAIL
#define KMZ_T9_TAIL 1  // 0 (A/B build): k4_tile8's round tail (chain_round_tail) in k4_tile9
#endif
#ifndef KMZ_T9_X
#define KMZ_T9_X 0  // (timing-only A/B builds, wrong results) 1: no list writes, 2: no claims, 4: no probes
#endif
#ifndef KMZ_WG_REGIONS
#define KMZ_WG_REGIONS 1  // 0 (A/B build): k4_tile9's list entries all in the global lists
#endif
constexpr uint32_t R_STAGE = KMZ_WG_REGIONS ? WG_STAGE : 0, R_POS = KMZ_WG_REGIONS ? WG_POS : 0,
                   R_DEFER = KMZ_WG_REGIONS ? WG_DEFER : 0;
#ifndef KMZ_T9_BAR
#define KMZ_T9_BAR 0  // 1 (A/B build): workgroup barriers after the probes and after the claims, as k4_tile8's tail
#endif
#ifndef KMZ_T9_LDSPAD
#define KMZ_T9_LDSPAD 0
#endif
#ifndef KMZ_T9_CLOCKS
#define KMZ_T9_CLOCKS 0
#endif
__device__ unsigned long long g_walk9_dbg[12];
#if KMZ_T9_CLOCKS
#define T9_STAMP(k)                                             \
  {                                                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0 && t9prev) t9acc[k] += t_ - t9prev;    \
    t9prev = t_;                                                \
  }
#else
#define T9_STAMP(k)
#endif

// k4_tile9's probe / claim / lists (against chain_round_tail: fewer dependent
// round trips per workgroup).  A walker whose probe finds its chain checks
// the parent sig; one that finds the home slot empty claims it with one CAS
// (no LDS leader map: two walkers of a workgroup with the same new chain,
// 0.4 % of them, both CAS and the second defers); the winner publishes its
// parent sig and stages its keys.  Its list entries are placed by an LDS add
// in the workgroup's own region of each list (WG_STAGE keys, WG_POS claimed
// slots: no device atomic and no barrier between the claim and the writes);
// past the region a device atomic reserves them in the global list.  A claim
// that lost the slot, or a chain found unpublished, goes to the deferred
// checks (global list, as before).  need[0] / need[1]: the workgroup's key /
// claim counts so far; need[2]: where the first key reservation that did not
// fit the region started (its keys, and every later one's, went to the global
// list), so the region's valid keys are the first min(need[0], need[2]);
// need[3]: deferred checks (the first WG_DEFER in the workgroup's region).
template <int NT, int TW, class Anc>
__device__ __forceinline__ void chain_round_tail9(uint64_t (&sg)[TW], const uint64_t (&ps)[TW], uint8_t (&st)[TW],
                                                  const uint8_t (&kq)[TW], const uint32_t (&dd)[TW],
                                                  const uint32_t (&jq)[TW], const uint32_t (&myep)[TW], uint32_t w0,
                                                  Anc anc, uint32_t *need, ChainLds &L, uint32_t (&hf)[TW],
                                                  const ChainRun &a, uint32_t &rows, uint32_t &rel, uint32_t &maxd,
                                                  uint32_t &fresh_n, uint32_t &flags, unsigned long long *t9acc,
                                                  unsigned long long &t9prev) {
  const uint32_t spin = spin_bound(a.ablate);
  ulonglong2 w01[TW];  // (sig, parent sig) of the probed slot
  uint64_t pos[TW];
  // (unconditional loads, slot 0 for a walker that does not probe: the
  // branchy form let the compiler wait for the first probe before issuing
  // the second -- two round trips instead of one, walk 0.95 -> 1.35 ms)
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    pos[q] = st[q] == S_PUT ? cslot(sg[q], a.ccap) : 0;
    w01[q] = (KMZ_T9_X & 4) ? make_ulonglong2(sg[q], ps[q]) : *reinterpret_cast<const ulonglong2 *>(a.ctab + 2 * pos[q]);
  }
#pragma unroll
  for (int q = 0; q < TW; ++q)
    if (st[q] != S_PUT) w01[q] = make_ulonglong2(0, 0);
  bool lead[TW], dfr[TW];
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    lead[q] = dfr[q] = false;
    if (st[q] != S_PUT) continue;
    for (uint32_t z = 0; w01[q].x != sg[q] && w01[q].x != 0 && z < PROBE_MAX; ++z) {  // another chain's slot
      pos[q] = pos[q] + 1 == a.ccap ? 0 : pos[q] + 1;
      w01[q] = *reinterpret_cast<const ulonglong2 *>(a.ctab + 2 * pos[q]);
    }
    st[q] = S_DONE;
    if (w01[q].x == sg[q] && w01[q].y != 0) {  // found and published: check it
      if (w01[q].y != ps[q]) flags |= F_SIG;
      continue;
    }
    if (a.ablate & (1u << 18)) continue;  // diagnostic knob: probe but no inserts
    // not found, or found unpublished: one leader per distinct sig in the
    // workgroup (LDS map; a hot new chain repeats within a tile, and every
    // repeat's CAS on one address, from every workgroup at once, serialised
    // the walk, 0.95 -> 1.35 ms); a follower checks the leader's parent sig
    // after the round's barrier (hf)
    uint32_t h = (uint32_t)(sig_place(sg[q]) >> 32) & (IMAP - 1);
    lead[q] = true;  // (a leader without a map slot when the map is full)
    for (uint32_t t = 0; t < 8; ++t) {
      const unsigned long long kk = atomicCAS(&L.imap_sig[h], 0ull, (unsigned long long)sg[q]);
      if (kk == 0) {
        L.imap_psig[h] = ps[q];
        break;
      }
      if (kk == sg[q]) {
        lead[q] = false;
        hf[q] = h;
        break;
      }
      h = (h + 1) & (IMAP - 1);
    }
    // a leader finding its chain unpublished defers the check (its CAS
    // returns the sig: joined); one finding the slot empty claims it
  }
  T9_STAMP(4);
#if KMZ_T9_BAR
  __syncthreads();
#endif
  // the claims, all in flight together; a winner publishes at once
  unsigned long long cvq[TW];
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    cvq[q] = 0;
    if (!lead[q]) continue;
    unsigned long long *en = a.ctab + 2 * pos[q];
    if (KMZ_T9_X & 2) continue;
    cvq[q] = atomicCAS(&en[0], 0ull, (unsigned long long)sg[q]);
    if (cvq[q] == 0) atomicExch(&en[1], (unsigned long long)ps[q]);
  }
#if KMZ_T9_CLOCKS
  if (__ballot(cvq[0] == 1234567 || cvq[TW - 1] == 1234567)) flags |= 0;  // (waits for the claims)
#endif
  T9_STAMP(5);
#if KMZ_T9_BAR
  __syncthreads();
#endif
  const uint32_t blk = blockIdx.x, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1;  // (the lanes below this one)
  // The list entries, reserved per wave: one LDS add for the wave's entries in
  // the workgroup's region, and -- for a wave whose entries do not fit it --
  // one device atomic for all of them in the global list.  (The workgroups
  // that run first find nearly every chain new, ~480 claims and ~2000 keys
  // each: a device atomic per walker on one counter serialised them, walk
  // 0.67 -> 1.33 ms on the mesh.)  Every lane takes part in the ballots and
  // shuffles; the per-walker work is predicated.
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    if (KMZ_T9_X & 1) break;
    const uint32_t d = dd[q];
    const bool won = lead[q] && cvq[q] == 0;
    fresh_n += won;
    // claimed slots (cleared after the run)
    {
      const uint64_t mk = __ballot(won);
      if (mk) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&need[1], (uint32_t)__popcll(mk));
        base = __shfl(base, 0, 64);
        const uint32_t o = base + (uint32_t)__popcll(mk & lt);
        const uint64_t mo = __ballot(won && o >= R_POS);
        uint32_t gb = 0;
        if (mo && lane == 0) gb = atomicAdd(&a.counters[C_WPOS], (uint32_t)__popcll(mo));
        gb = __shfl(gb, 0, 64);
        if (won) {
          if (o < R_POS) {
            a.wgpos[(uint64_t)blk * WG_POS + o] = (uint32_t)pos[q];
          } else {
            const uint32_t x = gb + (uint32_t)__popcll(mo & lt);
            if (x < a.gcap)
              a.gpos[x] = (uint32_t)pos[q];
            else
              flags |= F_CTAB_DIRTY;
          }
        }
      }
    }
    // a row whose chain this walker inserted (or lost to another chain: the
    // deferred check may insert it) stages its keys (ancestor k, row id, k,
    // ancestor is SERVER); one that joined the same chain leaves them to the
    // winner (knob 19: diagnostic, none)
    const bool stg = lead[q] && kq[q] == KIND_SERVER && d && cvq[q] != sg[q] && !(a.ablate & (1u << 19));
    if (__ballot(stg)) {
      const uint32_t nd = stg ? d : 0u;
      uint32_t incl = nd;  // the wave's inclusive scan of the key counts
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += y;
      }
      const uint32_t tot = __shfl(incl, 63, 64), pre = incl - nd;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&need[0], tot);
      base = __shfl(base, 0, 64);
      unsigned long long *dst;
      uint64_t cap;
      if (base + tot <= R_STAGE) {  // (wave-uniform)
        dst = a.wstage + (uint64_t)blk * WG_STAGE + base + pre;
        cap = nd;
      } else {  // (the region's valid keys end where the first reservation past it starts: need[2])
        uint32_t gb = 0;
        if (lane == 0) {
          atomicMin(&need[2], base);
          gb = atomicAdd(&a.counters[C_FSTAGE], tot);
        }
        gb = __shfl(gb, 0, 64);
        dst = a.stage + gb + pre;
        cap = gb + pre < a.scap ? a.scap - (gb + pre) : 0;
      }
      if (stg) {
        uint32_t an = anc(jq[q]).parent;
        for (uint32_t kk = 1; kk <= d; ++kk) {
          const AncRec r = anc(an);
          const uint64_t key = edge_key(r.ep, myep[q], kk, r.kind == KIND_SERVER);
          if (kk - 1 < cap) {
            dst[kk - 1] = key;
          } else {
            edge_insert(a.id_ep ? key_ids_to_eps(key, a.id_ep, a.n_ids) : key, a.trip, a.tcap, &flags);
            flags |= F_STAGE_FULL;
          }
          an = r.parent;
        }
      }
    }
    // deferred checks: found unpublished, joined an unpublished claim, or
    // lost the slot to another chain
    const bool dq = dfr[q] || cvq[q] != 0;
    const uint64_t md = __ballot(dq);
    if (md) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&need[3], (uint32_t)__popcll(md));
      base = __shfl(base, 0, 64);
      const uint32_t o = base + (uint32_t)__popcll(md & lt);
      const uint64_t mo = __ballot(dq && o >= R_DEFER);
      uint32_t gb = 0;
      if (mo && lane == 0) gb = atomicAdd(&a.counters[C_FDEFER], (uint32_t)__popcll(mo));
      gb = __shfl(gb, 0, 64);
      if (dq) {
        const uint32_t x = gb + (uint32_t)__popcll(mo & lt);
        if (o < R_DEFER) {
          *reinterpret_cast<ulonglong2 *>(a.wdefer + 2 * ((uint64_t)blk * WG_DEFER + o)) =
              make_ulonglong2(sg[q], ps[q]);
        } else if (x < a.dcap) {
          *reinterpret_cast<ulonglong2 *>(a.defer + 2 * (uint64_t)x) = make_ulonglong2(sg[q], ps[q]);
        } else {
          int rr = 0;
          for (uint32_t t = 0; t < spin && rr == 0; ++t)
            rr = chain_put(a.ctab, a.ccap, sg[q], ps[q], &flags, a.gpos, a.gcap, a.counters);
          if (rr == 0) flags |= F_SPIN;  // unchecked: the run is redone on the exact walk
          fresh_n += rr == 1;
        }
      }
    }
  }
  T9_STAMP(6);
  // per walker: row counts, pending list, rowpos
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    if (kq[q] == KIND_CLIENT) continue;  // (an empty walker slot)
    const uint32_t i = w0 + jq[q];
    const bool pending = st[q] == S_PEND;
    uint64_t rp = NONE64;
    if (kq[q] == KIND_SERVER) {
      rp = a.index_base + i;
      if (!pending) {
        ++rows;
        rel += dd[q];
        maxd = max(maxd, dd[q]);
      }
    }
    if (pending) {
      const uint32_t x = atomicAdd(&a.counters[C_PLIST], 1u);
      if (x < a.pcap) a.plist[x] = i;
    }
    if (a.rowpos_out) a.rowpos_out[i] = rp;
  }
  T9_STAMP(7);
}
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
  __shared__ uint32_t need[4];  // the workgroup's staged keys, claimed slots and deferred checks (chain_round_tail9)
  __shared__ ChainLds L;  // (the leader map)
#if KMZ_T9_LDSPAD  // (A/B builds: LDS held back to cap the workgroups per CU)
  __shared__ uint32_t ldspad[KMZ_T9_LDSPAD / 4];
  if (threadIdx.x == 0) ldspad[(blockIdx.x * 7u) % (KMZ_T9_LDSPAD / 4)] = blockIdx.x;
#endif
  __shared__ uint32_t wcnt[WPT][NW];
  __shared__ uint32_t red[NW][4];
  const uint32_t t0 = blockIdx.x * WT, t1 = min(n, t0 + WT);
  const uint32_t w0 = t0 > WH ? t0 - WH : 0, w1 = min(n, t1 + WH), wn = w1 - w0, toff = t0 - w0;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t flags = 0;
  unsigned long long t9acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, t9prev = 0;
  T9_STAMP(0);
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
  if (threadIdx.x < 4) need[threadIdx.x] = threadIdx.x == 2 ? ~0u : 0u;
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
  T9_STAMP(0);
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
  T9_STAMP(1);
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
    T9_STAMP(2);
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
    T9_STAMP(3);
#if KMZ_T9_TAIL
    uint32_t hf[TW];  // a follower's leader-map slot (IMAP + 1: none)
#pragma unroll
    for (int q = 0; q < TW; ++q) hf[q] = IMAP + 1;
    chain_round_tail9<WTT, TW>(sg, ps, st, kq, dd, jq, myep, w0, [&](uint32_t x) {
      const uint32_t pk = lpk[x];
      return AncRec{p9_id(pk), p9_kind(pk), p9_parent(pk)};
    }, need, L, hf, a, rows, rel, maxd, fresh_n, flags, t9acc, t9prev);
    __syncthreads();  // (the leaders' parent sigs are in the map; it stays for a next round, as k4_tile8's)
#pragma unroll
    for (int q = 0; q < TW; ++q)
      if (hf[q] <= IMAP && L.imap_psig[hf[q]] != ps[q]) flags |= F_SIG;
#else  // (A/B: k4_tile8's tail -- LDS leader map, lists reserved per workgroup with device atomics)
    chain_round_tail<WTT, TW>(sg, ps, st, kq, dd, jq, myep, w0, [&](uint32_t x) {
      const uint32_t pk = lpk[x];
      return AncRec{p9_id(pk), p9_kind(pk), p9_parent(pk)};
    }, L, a, rows, rel, maxd, fresh_n, flags);
    __syncthreads();
#endif
  }
  __syncthreads();  // (the workgroup's list counts are final)
  if (threadIdx.x == 0) {
    a.wn[blockIdx.x] = min(need[0], need[2]);  // (the region's valid keys)
    a.wn[a.ntiles + blockIdx.x] = min(need[1], R_POS);
    a.wn[2 * a.ntiles + blockIdx.x] = min(need[3], R_DEFER);
  }
  if (flags) atomicOr(&a.counters[C_FLAGS], flags);
  T9_STAMP(8);
  chain_tile_stats<WTT>(rows, rel, maxd, fresh_n, red, tile_stats);
  T9_STAMP(9);
#if KMZ_T9_CLOCKS
  if (threadIdx.x == 0)
    for (int kk = 0; kk < 10; ++kk) atomicAdd(&g_walk9_dbg[kk], t9acc[kk]);
#endif
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

extern "C" int kmz__debug_walk9(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmz::g_walk9_dbg), sizeof(kmz::g_walk9_dbg)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[12] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(kmz::g_walk9_dbg), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
