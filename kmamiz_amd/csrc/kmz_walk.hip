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
  for (int q = 0; q < WPW; ++q)
    e[q] = k[q] == KIND_CLIENT ? make_uint3(0, 0, 0)
                               : *reinterpret_cast<const uint3 *>(etab + (sh[q] < n_shapes ? sh[q] : 0));
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
