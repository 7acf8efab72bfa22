// kmz_chain.hip -- K4: the dependency graph by ancestor-chain interning.
//
// The reference walks every SERVER row up its non-CLIENT ancestors and records
// one (ancestor, descendant, distance) entry per step (Traces.ts:128-180); the
// deduplicated union of those entries is the edge set that EndpointDependencies
// combineWith/trim keep (EndpointDependencies.ts:499-563).  A row's entries are
// a function of its endpoint and of the (endpoint, kind) sequence of its
// ancestors only.  That sequence -- the row's *chain* -- is interned in a
// global open-addressing table of 32-byte entries
//
//     { sig(chain), sig(parent chain) (ROOT_SIG at a root) }
//
// Rows that share a chain (most of them: the 100M-span mesh has ~0.5M distinct
// chains) produce identical edge keys, so only the workgroup that inserts a new
// chain emits its keys; nothing per relation is written to HBM.
//
// `sig` is a 64-bit hash of the whole ancestry (a rotate-xor fold of the
// ancestors' mix64 element hashes, finished by an xor with a depth constant),
// computed by walking the ancestors in LDS, so every span probes the table once, in one
// round, with no dependency on its parent's probe or insert.  Exactness does
// not rest on the hash: every span checks the entry it found or joined against
// its own parent sig.  The table holds one entry per sig, so by induction from
// the roots a checked parent sig names one exact parent chain; for that parent
// the fold, the finish and the element hash are all bijective in the span's
// own (endpoint, kind), so an equal sig is an equal chain.  (The two values the
// finish may not produce, 0 and ROOT_SIG, raise F_SIG like a failed check: the
// run is repeated with another hash seed.)  An entry is 16 bytes.
//
//   k4_chain       persistent workgroups over 1024-span tiles + a 128-span halo
//                  per side in LDS (contracted parent, kind, endpoint, element
//                  hash).  Per tile: hash every non-CLIENT ancestry in the
//                  window (a Horner walk over the LDS element hashes), probe
//                  the tile's, check what the probes found, elect one leader
//                  per distinct unknown chain in the workgroup; a leader
//                  stages its chain's keys and claims the probed slot with one
//                  CAS, publishing if it won and deferring a check to
//                  k_chain_settle otherwise -- nothing waits on another
//                  workgroup.  Ancestries that leave the window (or are deeper
//                  than WIN_DEPTH inside it) go to a pending list.  The next
//                  tile's window is loaded into registers while a tile computes.
//   k_chain_settle the staged keys -> the global edge set; the deferred chain
//                  checks (join + verify, or insert).
//   k4_chain_pend  the pending spans, one pass, hashing over the global
//                  contracted parents (rare).
//
// Per-endpoint lastUsage / first row / external of rows come from the K3
// shape-level partials (kmz_api.hip, k_collapse_endpoints); non-SERVER
// ancestors (not rows) add their timestamps here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "kmz_chainw.h"

namespace kmz {

#ifndef KMZ_CHAIN_CT
#define KMZ_CHAIN_CT 1024  // (768 -> 1024: less halo per span, mesh walk 1.20 -> 1.10 ms)
#endif
#ifndef KMZ_CHAIN_CH
#define KMZ_CHAIN_CH 128
#endif
constexpr uint32_t CT = KMZ_CHAIN_CT, CH = KMZ_CHAIN_CH, CW = CT + 2 * CH;
constexpr int CTT = 256;
constexpr int CPW = CW / CTT;  // window slots per thread (slot jl = q * CTT + thread)
constexpr int TPW = CT / CTT;  // tile slots per thread
// walker slots per thread and round: the tile's non-CLIENT spans (the only
// ones that walk, probe and count) are compacted into a list first, so a
// thread works on TW of them per round instead of TPW slots of which about
// half are CLIENT spans
#ifndef KMZ_CHAIN_TW
#define KMZ_CHAIN_TW 2
#endif
constexpr int TW = KMZ_CHAIN_TW;
static_assert(TW <= TPW, "walker slots per thread");
static_assert(CT % CTT == 0, "tile slots must split evenly over the threads");
static_assert(CW % CTT == 0, "window slots must split evenly over the threads");
// staged keys are binned by the edge set's slices: 2^lb1 coarse bins per tile
// workgroup (k4_chain), each split into 2^lb2 slices by k_key_part
constexpr uint32_t KB1_MAX = 8, KB2_MAX = 8;
// direct enumeration: a workgroup drops keys it staged recently (a direct-mapped
// LDS cache of KCACHE keys).  Hot edge keys repeat ~10^5 times per run; without
// the cache they overfill their slice's bucket.
// (4096 keys measured on config 5: k_key_part + k_key_slice 2.61 -> 2.49 ms,
// but the direct walk 2.00 -> 2.85 ms)
#ifndef KMZ_KCACHE
#define KMZ_KCACHE 1024
#endif
constexpr uint32_t KCACHE = KMZ_KCACHE;
// where the next tile's endpoint gather is issued: 0 after the probes' check
// (round 3: mesh walk 1.11 -> 1.08 ms, two A/B runs, tools/r03_var.sh), 1
// before the probes (round 2's choice), 2 at the tile's end (1.09-1.11)
#ifndef KMZ_GATHER_EARLY
#define KMZ_GATHER_EARLY 0
#endif
#ifndef KMZ_CAS_EARLY  // 1: the leaders' claim CAS issued before the tile's row counts (variant)
#define KMZ_CAS_EARLY 0
#endif
#ifndef KMZ_CHAIN_WAVES
#define KMZ_CHAIN_WAVES 4
#endif
constexpr int CHAIN_WAVES = KMZ_CHAIN_WAVES;  // waves per SIMD: 4 -> 2 workgroups per CU (<= 128 VGPRs), 6 -> 3
constexpr uint32_t CHAIN_WG = 256 * CHAIN_WAVES * 4 / (CTT / 64);  // persistent workgroups (fill the CUs)
__device__ unsigned long long g_chain_dbg[8];  // diagnostic phase clocks (KMZ_ABLATE bit 22 only)

template <bool DIRECT>
__global__ void __launch_bounds__(CTT, CHAIN_WAVES) k4_chain(
    const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape, const int64_t *__restrict__ ts,
    const uint32_t *__restrict__ cparent, uint32_t n, const uint4 *__restrict__ etab, uint32_t n_shapes,
    uint32_t n_ep, uint64_t index_base, uint64_t seed, unsigned long long *__restrict__ ctab, uint64_t ccap,
    unsigned long long *__restrict__ trip, uint64_t tcap, unsigned long long *__restrict__ ep_ts,
    unsigned long long *__restrict__ rowpos_out, uint32_t *__restrict__ plist, uint32_t pcap,
    unsigned int *__restrict__ counters, uint32_t *__restrict__ wg_stats, unsigned long long *__restrict__ stage,
    uint32_t scap, uint32_t *__restrict__ stage_n, unsigned long long *__restrict__ defer, uint32_t dcap,
    uint32_t *__restrict__ defer_n, uint32_t *__restrict__ wpos, uint32_t wcap, uint32_t *__restrict__ wpos_n,
    uint32_t nt, uint32_t lb1, uint32_t lb2, uint32_t ablate, uint32_t cmode) {
  // one 16-byte record per window slot: element hash (x, y), endpoint (z),
  // contracted parent | kind << 16 (w) -- a walk step is one LDS read
  __shared__ uint4 lrec[CW];
  __shared__ unsigned long long imap_sig[DIRECT ? 1 : IMAP], imap_psig[DIRECT ? 1 : IMAP];
  __shared__ uint32_t lbin[1u << KB1_MAX];  // keys staged per coarse bin (k_key_part), deferred records
  __shared__ unsigned long long kcache[DIRECT ? KCACHE : 1];
  // direct: per-wave ring of keys waiting to be staged (the walk's active
  // lanes append; 64 at a time are staged by all lanes together)
  __shared__ unsigned long long squeue[DIRECT ? CTT / 64 : 1][DIRECT ? 256 : 1];
  __shared__ uint32_t dcnt;
  __shared__ uint16_t wlist[CT];  // this tile's non-CLIENT spans (tile-local), compacted
  __shared__ uint32_t wcount;
  __shared__ uint32_t wcnt;        // chain-table slots this workgroup claimed (cleared after the run)
  __shared__ uint32_t red[CTT / 64][4];
  // diagnostic phase clock (KMZ_ABLATE bit 22 only): s_memtime deltas by thread 0
  const bool dbg_t = (ablate & (1u << 22)) != 0;
  const uint32_t spin = spin_bound(ablate);
  unsigned long long tprev = 0, tacc[6] = {0, 0, 0, 0, 0, 0};
#define KMZ_STAMP(k)                                         \
  if (dbg_t) {                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0 && tprev) tacc[k] += t_ - tprev;       \
    tprev = t_;                                                 \
  }
  // persistent: this workgroup walks tiles blockIdx.x, +gridDim.x, ...; the
  // next tile's window is loaded into registers while the current one computes
  uint32_t c[CPW], sh[CPW];
  uint4 e[CPW];  // the slot's shape: endpoint, SERVER element hash (k_chain_etab)
  uint8_t k[CPW];
  auto fetch = [&](uint32_t tl) {
    const uint32_t tb = tl * CT, wb = tb > CH ? tb - CH : 0;
#pragma unroll
    for (int q = 0; q < CPW; ++q) {  // clamped, unconditional: every load in flight together
      const uint32_t j = min(wb + q * CTT + threadIdx.x, n - 1);
      c[q] = cparent[j];
      k[q] = kind[j];
      sh[q] = shape[j];
    }
  };
  auto gather_ep = [&]() {
    // (every slot gathers -- a CLIENT slot entry 0, unused -- so that the
    // loads carry no branch: a load under a branch made the compiler wait for
    // it at the merge, which serialised the CPW gathers and the prefetch of the
    // next tile behind them)
#pragma unroll
    for (int q = 0; q < CPW; ++q) e[q] = etab[(k[q] != KIND_CLIENT && sh[q] < n_shapes) ? sh[q] : 0];
  };
  if (threadIdx.x == 0) dcnt = wcnt = wcount = 0;
  if (threadIdx.x < (1u << KB1_MAX)) lbin[threadIdx.x] = 0;
  if (DIRECT)
    for (uint32_t x = threadIdx.x; x < KCACHE; x += CTT) kcache[x] = 0;
  if (blockIdx.x < nt) {
    fetch(blockIdx.x);
    gather_ep();
  }
  uint32_t rows = 0, rel = 0, maxd = 0, fresh_n = 0, flags = 0;
  // staged keys: this workgroup's region holds 2^lb1 runs of `sub` keys, one
  // per coarse bin of the edge set's slices (k_key_part takes them from there)
  const uint32_t sub = scap >> lb1;
  const uint32_t tshift = 64u - (uint32_t)__builtin_ctzll(tcap);  // (tcap is ESLICE * 2^k: key_bins)
  // compact staging (cmode: endpoints < 2^16, >= 64 coarse bins): a compact
  // key is staged as the low 38 - lb1 <= 32 bits of its x38 (kmz_common.h),
  // its coarse bin being the top lb1; other keys are inserted in place (rare:
  // distances >= 32)
  uint32_t *const stage32 = reinterpret_cast<uint32_t *>(stage);
  auto stage_key = [&](uint64_t key) {
    if (ablate & (1u << 21)) return;  // diagnostic knob: walk only
    const uint64_t h = ekey_hash(key);
    const uint64_t pos = h >> tshift;  // eslot(key, tcap): tcap = 2^(64 - tshift)
    unsigned long long &ce = kcache[DIRECT ? (uint32_t)pos & (KCACHE - 1) : 0];
    if (ce == key) return;  // staged recently by this workgroup (races only let a duplicate through)
    ce = key;
    if ((ablate & (1u << 31)) || (cmode && !ekey_compact(key))) {  // (knob 31, diagnostic: insert in place)
      edge_insert(key, trip, tcap, &flags);
      return;
    }
    const uint32_t b = (uint32_t)((pos / ESLICE) >> lb2);
    const uint32_t x = atomicAdd(&lbin[b], 1u);
    const uint64_t at = (((uint64_t)blockIdx.x << lb1) + b) * sub + x;
    if (x < sub) {
      if (cmode)
        stage32[at] = (uint32_t)((h >> 26) & ((1ull << (38 - lb1)) - 1));
      else
        stage[at] = key;
    } else {  // this run is full: insert here (slow: one lane per key); more staging next run
      edge_insert(key, trip, tcap, &flags);
      flags |= F_STAGE_FULL;
    }
  };
  // chain interning (one run per workgroup, lb1 = 0): the keys of the row in
  // window slot jl, (ancestor k, row endpoint es, k, ancestor is SERVER),
  // under one reservation
  auto stage_row = [&](uint32_t jl, uint32_t es, uint32_t d) {
    const uint32_t base = atomicAdd(&lbin[0], d);
    uint32_t a = lrec[jl].w & 0xFFFF;
    for (uint32_t kk = 1; kk <= d; ++kk) {
      const uint4 r = lrec[a];
      const uint64_t key = edge_key(r.z, es, kk, ((r.w >> 16) & 3) == KIND_SERVER);
      if (base + kk - 1 < sub) {
        stage[(uint64_t)blockIdx.x * sub + base + kk - 1] = key;
      } else {
        edge_insert(key, trip, tcap, &flags);
        flags |= F_STAGE_FULL;
      }
      a = r.w & 0xFFFF;
    }
  };
  for (uint32_t tile = blockIdx.x; tile < nt; tile += gridDim.x) {
    KMZ_STAMP(0);
    const uint32_t t0 = tile * CT, t1 = min(n, t0 + CT);
    const uint32_t w0 = t0 > CH ? t0 - CH : 0, w1 = min(n, t1 + CH), wn = w1 - w0;
    if (threadIdx.x == 0) wcount = 0;  // (read by every thread before the last barrier of the previous tile)
    // window -> LDS, with every non-CLIENT slot's element hash
    bool other = false;  // a span neither SERVER nor CLIENT in the window (rows' lastUsage path)
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const uint32_t jl = q * CTT + threadIdx.x;
      const bool client = k[q] == KIND_CLIENT;
      const uint32_t ep = (client || sh[q] >= n_shapes) ? NONE : e[q].x;
      const uint32_t cp =
          c[q] == NONE ? W_NONE : (c[q] == CYC ? W_CYC : ((c[q] >= w0 && c[q] < w1) ? c[q] - w0 : W_OUT));
      uint64_t el = ((uint64_t)e[q].z << 32) | e[q].y;  // SERVER
      if (client) el = 0;
      else if ((k[q] & 3) != KIND_SERVER || sh[q] >= n_shapes) el = sig_elem(ep, k[q] == KIND_SERVER, seed);  // (rare)
      if (jl < wn) lrec[jl] = make_uint4((uint32_t)el, (uint32_t)(el >> 32), ep, cp | ((uint32_t)(k[q] & 3) << 16));
      other |= jl < wn && (k[q] & 3) != KIND_SERVER && !client;
    }
    if (!DIRECT)
      for (uint32_t x = threadIdx.x; x < IMAP; x += CTT) imap_sig[x] = 0;
    const bool any_other = __syncthreads_or(other);
    KMZ_STAMP(1);
    const bool more = tile + gridDim.x < nt;
    if (more) fetch(tile + gridDim.x);  // lands while this tile computes
    const uint32_t toff = t0 - w0;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // compact the tile's non-CLIENT spans into wlist (one LDS add per wave and
    // slot); CLIENT spans are not rows
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
      const uint32_t jl = toff + q * CTT + threadIdx.x;
      const bool in = w0 + jl < t1;
      const bool isw = in && ((lrec[min(jl, CW - 1)].w >> 16) & 3) != KIND_CLIENT;
      if (rowpos_out && in && !isw) rowpos_out[w0 + jl] = NONE64;
      const uint64_t mk = __ballot(isw);
      uint32_t b = 0;
      if (lane == 0 && mk) b = atomicAdd(&wcount, (uint32_t)__popcll(mk));
      b = __shfl(b, 0, 64);
      if (isw) wlist[b + __popcll(mk & ((1ull << lane) - 1))] = (uint16_t)(jl - toff);
    }
    __syncthreads();
    const uint32_t m = wcount;
    // rounds of TW walkers per thread (uniform); the first always runs and
    // issues the next tile's endpoint gather at one fixed point (so the
    // gathered registers are dead before it)
    auto round = [&](const uint32_t r0, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    // hash the ancestry of every non-CLIENT span of the tile by a fold walk
    // over the LDS element hashes of its ancestors a1..aD:
    //   pacc = rotl^(D-1)(elem(a1)) ^ ... ^ elem(aD)
    //   sig  = final(rotl^D(elem(s)) ^ pacc, D),  parent sig = final(pacc, D-1)
    // (the parent's own sig, so halo spans need no walk), and issue the probes
    // at once.  A row's walk also gives its non-SERVER ancestors (not rows)
    // their lastUsage.
    uint64_t sg[TW], ps[TW], acc[TW];
    uint32_t dd[TW], wa[TW], myep[TW], jq[TW];
    uint8_t st[TW], kq[TW];
    const bool hash_on = !(ablate & (1u << 16));  // diagnostic knob: no hashing / probing / inserting
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      const uint32_t idx = r0 + q * CTT + threadIdx.x;
      const bool on = idx < m;
      const uint32_t jl = on ? toff + wlist[idx] : CW - 1;
      jq[q] = jl;
      const uint4 r = lrec[jl];
      kq[q] = (r.w >> 16) & 3;
      myep[q] = r.z;
      sg[q] = (uint64_t)r.y << 32 | r.x;  // the element hash until the walk is done
      acc[q] = 0;
      dd[q] = 0;
      wa[q] = W_NONE;
      st[q] = S_NONE;
      if (!on) {  // (no walker in this slot)
        kq[q] = KIND_CLIENT;
        continue;
      }
      st[q] = S_DONE;
      if (!hash_on) continue;
      if (kq[q] == KIND_SERVER && r.z >= n_ep) flags |= F_RANGE;
      if (DIRECT && kq[q] != KIND_SERVER) continue;  // direct: only rows walk (no chains to intern)
      wa[q] = r.w & 0xFFFF;
    }
    // the TW walks of a thread step together: TW independent LDS reads in
    // flight per step.  Direct: the loop runs while any lane of the wave walks
    // (wave-uniform), the keys go through the wave's ring.
    uint32_t qh = 0, qt = 0;  // ring head / tail (wave-uniform)
    auto drain = [&](bool all) {
      while (qt - qh >= 64 || (all && qt != qh)) {
        const uint32_t m = min(qt - qh, 64u);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (lane < m) stage_key(squeue[DIRECT ? wv : 0][(qh + lane) & 255]);
        qh += m;
        __builtin_amdgcn_wave_barrier();  // the slots are rewritten by the next appends
      }
    };
    // (two copies of the loop: the non-SERVER-ancestor branch is compiled out
    // of the usual all-SERVER/CLIENT window)
    auto walk = [&](auto other_tag) {
    constexpr bool OTHER = decltype(other_tag)::value;
    // every walk starts at step 0 and advances once per step while it is in
    // the window, so a walk's depth is the step count: the depth bound is the
    // (wave-uniform) loop bound, and the loop runs while any lane walks
    for (uint32_t it = 0; it < WIN_DEPTH; ++it) {
      bool go = false;
#pragma unroll
      for (int q = 0; q < TW; ++q) go |= wa[q] < CW;
      if (__ballot(go) == 0) break;
      // all TW reads first, then branch-free updates (selects), so the reads
      // stay in flight together
      uint4 r[TW];
#pragma unroll
      for (int q = 0; q < TW; ++q) r[q] = lrec[wa[q] < CW ? wa[q] : 0];
#pragma unroll
      for (int q = 0; q < TW; ++q) {
        const bool act = wa[q] < CW;
        const uint64_t nacc = sig_step(acc[q], (uint64_t)r[q].y << 32 | r[q].x);
        if (OTHER && act && kq[q] == KIND_SERVER && ((r[q].w >> 16) & 3) != KIND_SERVER) {
          // (rare) a non-SERVER ancestor of a row
          if (r[q].z < n_ep)
            atomicMax(&ep_ts[r[q].z], (unsigned long long)((uint64_t)ts[w0 + wa[q]] ^ TS_BIAS));
          else
            flags |= F_RANGE;
        }
        // direct: a row stages each key as its walk reaches the ancestor (a
        // row that turns out pending stages them all again in k4_chain_pend:
        // duplicates are harmless in the edge set)
        if (DIRECT) {
          const uint64_t mk = __ballot(act);
          if (act)
            squeue[DIRECT ? wv : 0][(qt + __popcll(mk & ((1ull << lane) - 1))) & 255] =
                edge_key(r[q].z, myep[q], dd[q] + 1, ((r[q].w >> 16) & 3) == KIND_SERVER);
          qt += __popcll(mk);
        }
        acc[q] = act ? nacc : acc[q];
        dd[q] = act ? it + 1 : dd[q];
        wa[q] = act ? (r[q].w & 0xFFFF) : wa[q];
      }
      if (DIRECT) drain(false);
    }
    };
    if (any_other)
      walk(std::true_type{});
    else
      walk(std::false_type{});
    // per span of the tile: row counts, pending list, rowpos (reads the walk's
    // state only: with KMZ_CAS_EARLY it runs while the leaders' claims are in flight)
    auto tile_stats = [&]() {
#pragma unroll
      for (int q = 0; q < TW; ++q) {
        const uint32_t jl = jq[q], i = w0 + jl;
        if (kq[q] == KIND_CLIENT) continue;  // (an empty walker slot)
        const uint8_t kj = kq[q];
        uint64_t rp = NONE64;
        const bool pending = st[q] == S_PEND;
        if (kj == KIND_SERVER) {
          rp = index_base + i;
          if (!pending) {
            ++rows;
            rel += dd[q];
            maxd = max(maxd, dd[q]);
          }
        }
        if (pending) {
          const uint32_t x = atomicAdd(&counters[C_PLIST], 1u);
          if (x < pcap) plist[x] = i;
        }
        if (rowpos_out) rowpos_out[i] = rp;
      }
    };
    if (DIRECT) drain(true);
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      if (st[q] != S_DONE || !hash_on) {
        sg[q] = 0;
        continue;
      }
      if (wa[q] != W_NONE) {  // W_OUT: leaves the window or deeper than WIN_DEPTH; W_CYC: CLIENT loop
        if (wa[q] == W_CYC) flags |= F_CYCLE;
        st[q] = S_PEND;
        sg[q] = 0;
        continue;
      }
      if (DIRECT) continue;  // every row stages its keys: no chain sig
      const uint32_t d = dd[q];
      ps[q] = d ? sig_final(acc[q], d - 1, seed, &flags) : ROOT_SIG;
      sg[q] = sig_final(rotl64(sg[q], SIG_R * d) ^ acc[q], d, seed, &flags);
      if (ablate & (1u << 24)) {  // test knob: 4-bit sigs, i.e. collisions (F_SIG, then a retry with another seed)
        sg[q] = (sg[q] & 0xF) + 2;
        ps[q] = d ? (ps[q] & 0xF) + 2 : ROOT_SIG;
      }
      if (!(ablate & (1u << 17))) st[q] = S_PUT;  // diagnostic knob: hash only
    }
    if (DIRECT) {  // (the rows staged their keys during the walk)
      if (more && FIRST) gather_ep();
    } else {
#if KMZ_GATHER_EARLY == 1
      // the next tile's endpoints (variant): the gather's round trip overlaps
      // the probes' below, but the shapes may not have landed yet
      if (more && FIRST) gather_ep();
#endif
      ulonglong2 w01[TW];  // (sig, parent sig) of the probed slot
      uint64_t pos[TW];
#pragma unroll
      for (int q = 0; q < TW; ++q) {
        const bool pr = st[q] == S_PUT;
        pos[q] = pr ? cslot(sg[q], ccap) : 0;
        const unsigned long long *en = ctab + 2 * pos[q];
        w01[q] = pr ? *reinterpret_cast<const ulonglong2 *>(en) : make_ulonglong2(0, 0);
      }
      KMZ_STAMP(2);
      // check what the probes found against (parent sig, endpoint, kind); a
      // chain not found (or not yet published) elects one leader per distinct
      // sig in this workgroup
      uint32_t hslot[TW];
#pragma unroll
      for (int q = 0; q < TW; ++q) {
        hslot[q] = IMAP + 1;  // not an insert
        if (st[q] != S_PUT) continue;
        for (uint32_t z = 0; w01[q].x != sg[q] && w01[q].x != 0 && z < PROBE_MAX; ++z) {  // another chain's slot
          pos[q] = pos[q] + 1 == ccap ? 0 : pos[q] + 1;
          w01[q] = *reinterpret_cast<const ulonglong2 *>(ctab + 2 * pos[q]);
        }
        st[q] = S_DONE;
        if (w01[q].x == sg[q] && w01[q].y != 0) {
          if (w01[q].y != ps[q]) flags |= F_SIG;
          continue;
        }
        uint32_t h = (uint32_t)(sig_place(sg[q]) >> 32) & (IMAP - 1);
        hslot[q] = IMAP;  // a leader without a map slot (map full)
        for (uint32_t t = 0; t < 8; ++t) {
          const unsigned long long kk = atomicCAS(&imap_sig[h], 0ull, (unsigned long long)sg[q]);
          if (kk == 0) {  // leader: publish what the followers compare against
            imap_psig[h] = ps[q];
            hslot[q] = h;
            break;
          }
          if (kk == sg[q]) {  // follower
            hslot[q] = h | 0x80000000u;
            break;
          }
          h = (h + 1) & (IMAP - 1);
        }
      }
#if KMZ_GATHER_EARLY == 0
      // the next tile's endpoints: its shapes have landed by now, and the
      // gather's round trip overlaps the leaders and the row counts
      if (more && FIRST) gather_ep();
#endif
      if (ablate & (1u << 18))  // diagnostic knob: probe but no inserts
#pragma unroll
        for (int q = 0; q < TW; ++q) hslot[q] = IMAP + 1;
      __syncthreads();
      KMZ_STAMP(3);
      // followers compare with their leader; leaders claim the slot the probe
      // ended on (one CAS), publish if they won, and defer a final check to
      // k_chain_settle otherwise.  Keys of a leader's chain are staged whether
      // or not it is new (duplicates are harmless in the edge set), so nothing
      // here waits on another workgroup.
#if KMZ_CAS_EARLY
      // the leaders' claims in flight while the tile's row counts are taken
      unsigned long long cvq[TW];
#pragma unroll
      for (int q = 0; q < TW; ++q)
        cvq[q] = hslot[q] <= IMAP ? atomicCAS(ctab + 2 * pos[q], 0ull, (unsigned long long)sg[q]) : 0ull;
      tile_stats();
#endif
#pragma unroll
      for (int q = 0; q < TW; ++q) {
        if (hslot[q] > IMAP) {
          if (hslot[q] != IMAP + 1) {  // follower
            const uint32_t h = hslot[q] & (IMAP - 1);
            if (imap_psig[h] != ps[q]) flags |= F_SIG;
          }
          continue;
        }
        const uint32_t jl = jq[q];
        unsigned long long *en = ctab + 2 * pos[q];
#if KMZ_CAS_EARLY
        const unsigned long long cv = cvq[q];
#else
        const unsigned long long cv = atomicCAS(&en[0], 0ull, (unsigned long long)sg[q]);
#endif
        const uint32_t d = dd[q];
        // a row whose chain this leader inserted (or lost to another chain: the
        // deferred check may insert it) stages its keys; one that joined the
        // same chain leaves them to the winner (knob 19: diagnostic, none)
        // publish before anything below can wait: a lane that spins on another
        // workgroup's unpublished entry (chain_put) must never hold back, in
        // its own wave, the publish of an entry that workgroup may spin on
        if (cv == 0) atomicExch(&en[1], (unsigned long long)ps[q]);
        __builtin_amdgcn_wave_barrier();
        if (kq[q] == KIND_SERVER && d && cv != sg[q] && !(ablate & (1u << 19))) stage_row(jl, myep[q], d);
        if (cv == 0) {  // won the slot (published above)
          ++fresh_n;
          const uint32_t x = atomicAdd(&wcnt, 1u);
          if (x < wcap)
            wpos[(uint64_t)blockIdx.x * wcap + x] = (uint32_t)pos[q];
          else
            flags |= F_CTAB_DIRTY;
        } else {  // joined an unpublished entry, or lost the slot to another chain
          const uint32_t x = atomicAdd(&dcnt, 1u);
          if (x < dcap) {
            *reinterpret_cast<ulonglong2 *>(defer + 2 * ((uint64_t)blockIdx.x * dcap + x)) = make_ulonglong2(sg[q], ps[q]);
          } else {
            int rr = 0;
            for (uint32_t t = 0; t < spin && rr == 0; ++t)
              rr = chain_put(ctab, ccap, sg[q], ps[q], &flags, wpos + (uint64_t)gridDim.x * wcap, wcap,
                             counters);  // (the run's global written list follows the per-workgroup ones)
            if (rr == 0) flags |= F_SPIN;  // unchecked: the run is redone on the exact walk
            fresh_n += rr == 1;
          }
        }
      }
    }
    KMZ_STAMP(4);
    if (DIRECT || !KMZ_CAS_EARLY) tile_stats();
    __syncthreads();  // LDS is rewritten by the next round / tile
    KMZ_STAMP(5);
    };
    round(0u, std::true_type{});
    for (uint32_t r0 = TW * CTT; r0 < m; r0 += TW * CTT) round(r0, std::false_type{});
#if KMZ_GATHER_EARLY == 2
    if (!DIRECT && more) gather_ep();  // (diagnostic variant: at the tile's end, a full tile after the shapes' loads)
#endif
  }
  // per workgroup: rows, relations, max depth, new chains
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) {
    fresh_n += __shfl_xor(fresh_n, o, 64);
    rows += __shfl_xor(rows, o, 64);
    rel += __shfl_xor(rel, o, 64);
    maxd = max(maxd, (uint32_t)__shfl_xor(maxd, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6][0] = rows;
    red[threadIdx.x >> 6][1] = rel;
    red[threadIdx.x >> 6][2] = maxd;
    red[threadIdx.x >> 6][3] = fresh_n;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    uint32_t a = 0;
    for (int w = 0; w < CTT / 64; ++w) a = threadIdx.x == 2 ? max(a, red[w][2]) : a + red[w][threadIdx.x];
    wg_stats[(uint64_t)blockIdx.x * 4 + threadIdx.x] = a;
  }
  for (uint32_t b = threadIdx.x; b < (1u << lb1); b += CTT) stage_n[((uint64_t)blockIdx.x << lb1) + b] = min(lbin[b], sub);
  if (threadIdx.x == 0) {
    defer_n[blockIdx.x] = min(dcnt, dcap);
    wpos_n[blockIdx.x] = min(wcnt, wcap);
  }
  if (dbg_t && threadIdx.x == 0)
    for (int kk = 0; kk < 6; ++kk) atomicAdd(&g_chain_dbg[kk], tacc[kk]);
#undef KMZ_STAMP
}

// Direct enumeration stages every relation's key (~450M at config 5's 1e8
// spans, ~30 per distinct key): they reach the edge set in two passes that
// keep every HBM access streaming and every probe in LDS:
//   k_key_part   one (workgroup, coarse bin) run at a time, 4096 keys per
//                step: ranks within the run's 2^lb2 slices from an LDS
//                histogram, one global reservation per (step, slice), the
//                keys counting-sorted by slice in LDS and written out as one
//                contiguous piece per slice (~64 keys at config 5)
//   k_key_slice  one slice per workgroup: its ESLICE slots of the edge set
//                into LDS, its bucket's keys inserted there (the slice is a
//                self-contained table, eset_next), the slice written back
// A full bucket inserts in place (edge_insert) and asks for more staging.
// Chain interning stages few keys (new chains only): k_chain_settle inserts
// them in place, which is cheaper at that volume.
constexpr uint32_t KP_T = 256, KP_PER = 16, KP_STEP = KP_T * KP_PER;  // 4096 keys per step
// a direct-mapped LDS cache of the keys this workgroup already wrote out
// (its runs are all of one coarse bin: the grid is a multiple of 2^lb1), so a
// key that recurs across its runs -- config 5's power-law head -- is written
// once: the edge set is a set, and a key found in the cache was written by the
// thread that put it there
// 16 KB: 4096 32-bit residuals (compact staging), else 2048 whole keys
// (2048 whole keys measured against 1024 and 4096: 7.50 against 7.67 / 7.74
// ms on config 5, the larger cache costing occupancy)
#ifndef KMZ_KP_CACHE_BYTES
#define KMZ_KP_CACHE_BYTES 16384
#endif
// (Measured and dropped: each step's keys first put in an 8192-slot LDS set
// and the repeats dropped before the slice sort -- k_key_part + k_key_slice
// 2.63 -> 3.10 ms on config 5: few repeats fall inside one 4096-key step.)

// exclusive prefix sum of v[0..m) in LDS (m <= 4 * KP_T), by the whole workgroup
__device__ __forceinline__ void kp_scan(uint32_t *__restrict__ v, uint32_t m, uint32_t *__restrict__ wsum) {
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t loc[4], run = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t i = 4 * t + j;
    loc[j] = run;
    run += i < m ? v[i] : 0;
  }
  uint32_t x = run;  // inclusive scan of the per-thread totals over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = x - run;
  for (uint32_t k = 0; k < w; ++k) before += wsum[k];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t i = 4 * t + j;
    if (i < m) v[i] = before + loc[j];
  }
  __syncthreads();
}

// C (compact staging): the runs hold 32-bit x38 residuals below their coarse
// bin's lb1 bits, and the buckets 32-bit residuals below the slice's
// lb1 + lb2 bits (kmz_common.h); else whole 64-bit keys
template <bool C>
__global__ void __launch_bounds__(KP_T) k_key_part(const void *__restrict__ stage_v, uint32_t sub,
                                                   const uint32_t *__restrict__ stage_n, uint32_t nruns, uint32_t lb1,
                                                   uint32_t lb2, void *__restrict__ bucket_v,
                                                   uint64_t bcap, uint32_t *__restrict__ bucket_n,
                                                   unsigned long long *__restrict__ trip, uint64_t tcap,
                                                   unsigned int *__restrict__ counters, bool dedup) {
  using KT = typename std::conditional<C, uint32_t, unsigned long long>::type;
  const KT *__restrict__ stage = static_cast<const KT *>(stage_v);
  KT *__restrict__ bucket = static_cast<KT *>(bucket_v);
  __shared__ KT sorted[KP_STEP];  // 32 KB (16 KB compact)
  // the cache: residuals of this workgroup's coarse bin, or whole keys; all ones = empty
  constexpr uint32_t KP_CACHE = KMZ_KP_CACHE_BYTES / sizeof(KT);
  __shared__ KT kcache[KP_CACHE];
  for (uint32_t x = threadIdx.x; x < KP_CACHE; x += KP_T) kcache[x] = (KT)~0ull;
  __shared__ uint32_t hist[1u << KB2_MAX], off[1u << KB2_MAX], base[1u << KB2_MAX], wsum[KP_T / 64];
  static_assert((1u << KB2_MAX) <= 4 * KP_T, "kp_scan covers the slices of a coarse bin");
  const uint32_t nf = 1u << lb2;
  const uint32_t ls = lb1 + lb2;  // slices = 2^ls
  uint32_t flags = 0;
  // fine slice of a staged entry of coarse bin c, and the entry as a bucket entry
  auto fine = [&](KT v) -> uint32_t {
    if (C) return (uint32_t)((uint64_t)v >> (38 - ls)) & (nf - 1);  // (v: below the coarse bits)
    return (uint32_t)(eslot((uint64_t)v, tcap) / ESLICE) & (nf - 1);
  };
  auto to_bucket = [&](KT v) -> KT {
    if (C) return (KT)((uint64_t)v & ((1ull << (38 - ls)) - 1));
    return v;
  };
  auto whole = [&](KT v, uint32_t c) -> uint64_t {
    if (C) return ekey_from_x38(((uint64_t)c << (38 - lb1)) | (uint64_t)v);
    return (uint64_t)v;
  };
  // this workgroup's steps: runs blockIdx.x, +gridDim.x, ..., 4096 keys at a
  // time; the next step's keys are loaded while this one is sorted
  uint32_t r = blockIdx.x, c0 = 0, m = 0;
  auto seek = [&]() {
    while (r < nruns && c0 >= (m = stage_n[r])) {
      r += gridDim.x;
      c0 = 0;
    }
  };
  KT kn[KP_PER];
  uint32_t nn = 0;  // valid entries of the loaded step
  auto load = [&]() {
    const KT *src = stage + (uint64_t)min(r, nruns - 1) * sub;
    nn = r < nruns ? min(m - c0, KP_STEP) : 0;
#pragma unroll
    for (int j = 0; j < (int)KP_PER; ++j) {
      const uint32_t i = c0 + j * KP_T + threadIdx.x;
      kn[j] = (r < nruns && i < m) ? src[i] : (KT)0;
    }
  };
  seek();
  load();
  while (r < nruns) {
    const uint32_t c = r & ((1u << lb1) - 1);  // this step's coarse bin
    KT k[KP_PER];
    const uint32_t nv = nn;
#pragma unroll
    for (int j = 0; j < (int)KP_PER; ++j) k[j] = kn[j];
    c0 += KP_STEP;
    seek();
    load();  // (in flight during the LDS work below)
    for (uint32_t x = threadIdx.x; x < nf; x += KP_T) hist[x] = 0;
    __syncthreads();
    uint32_t f[KP_PER], rk[KP_PER];
    bool keep[KP_PER];
#pragma unroll
    for (int j = 0; j < (int)KP_PER; ++j) {
      keep[j] = j * KP_T + threadIdx.x < nv;
      if (dedup && keep[j] && k[j] != (KT)~0ull) {  // (one coarse bin per workgroup: the residual is the key)
        const uint64_t e = (uint64_t)k[j];
        const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
        const uint32_t slot = (lo ^ (lo >> 12) ^ (lo >> 24) ^ hi ^ (hi >> 12)) & (KP_CACHE - 1);
        if (kcache[slot] == k[j])
          keep[j] = false;
        else
          kcache[slot] = k[j];
      }
      f[j] = fine(k[j]);
      rk[j] = keep[j] ? atomicAdd(&hist[f[j]], 1u) : 0;  // rank within its slice
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < nf; x += KP_T) {
      const uint32_t h = hist[x];
      base[x] = h ? atomicAdd(&bucket_n[(c << lb2) + x], h) : 0;
      off[x] = h;
    }
    __syncthreads();
    kp_scan(off, nf, wsum);
#pragma unroll
    for (int j = 0; j < (int)KP_PER; ++j)
      if (keep[j]) sorted[off[f[j]] + rk[j]] = k[j];
    __syncthreads();
    // consecutive threads -> consecutive slots of one slice's bucket
    const uint32_t nz = off[nf - 1] + hist[nf - 1];
    for (uint32_t i = threadIdx.x; i < nz; i += KP_T) {
      const KT key = sorted[i];
      const uint32_t fb = fine(key);
      const uint64_t p = (uint64_t)base[fb] + (i - off[fb]);
      if (p < bcap) {
        bucket[(uint64_t)((c << lb2) + fb) * bcap + p] = to_bucket(key);
      } else {
        edge_insert(whole(key, c), trip, tcap, &flags);
        flags |= F_STAGE_FULL;
      }
    }
    __syncthreads();
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
}

constexpr uint32_t KS_T = 1024, KS_PER = 8;  // 16 waves per slice, 8 keys per thread in flight
template <bool C>
__global__ void __launch_bounds__(KS_T) k_key_slice(const void *__restrict__ bucket_v, uint64_t bcap,
                                                    const uint32_t *__restrict__ bucket_n, uint32_t nsl, uint32_t ls,
                                                    unsigned long long *__restrict__ trip, uint64_t tcap,
                                                    unsigned int *__restrict__ counters) {
  using KT = typename std::conditional<C, uint32_t, unsigned long long>::type;
  const KT *__restrict__ bucket = static_cast<const KT *>(bucket_v);
  __shared__ unsigned long long tab[ESLICE];  // 64 KB
  uint32_t flags = 0;
  for (uint32_t b = blockIdx.x; b < nsl; b += gridDim.x) {
    const uint32_t m = (uint32_t)min((uint64_t)bucket_n[b], bcap);
    if (!m) continue;  // (uniform over the workgroup) the slice keeps what it holds
    ulonglong2 *g = reinterpret_cast<ulonglong2 *>(trip + (uint64_t)b * ESLICE);
    ulonglong2 *l = reinterpret_cast<ulonglong2 *>(tab);
    for (uint32_t x = threadIdx.x; x < ESLICE / 2; x += KS_T) l[x] = g[x];
    __syncthreads();
    const KT *src = bucket + (uint64_t)b * bcap;
    // the next chunk's keys load while this chunk's are inserted
    KT kn[KS_PER];
    auto load = [&](uint32_t x1) {
#pragma unroll
      for (int j = 0; j < (int)KS_PER; ++j) {
        const uint32_t i = x1 + j * KS_T + threadIdx.x;
        kn[j] = i < m ? src[i] : (KT)0;
      }
    };
    load(0);
    for (uint32_t x0 = 0; x0 < m; x0 += KS_T * KS_PER) {
      KT k[KS_PER];
#pragma unroll
      for (int j = 0; j < (int)KS_PER; ++j) k[j] = kn[j];
      load(x0 + KS_T * KS_PER);
#pragma unroll
      for (int j = 0; j < (int)KS_PER; ++j) {
        if (x0 + j * KS_T + threadIdx.x >= m || (flags & F_TRIPLE_OVERFLOW)) continue;  // (a full slice: the run is repeated larger)
        const uint64_t key = C ? ekey_from_x38(((uint64_t)b << (38 - ls)) | (uint64_t)k[j]) : (uint64_t)k[j];
        uint32_t p = (uint32_t)(eslot(key, tcap) & (ESLICE - 1));
        uint32_t z = 0;
        for (; z < PROBE_MAX; ++z) {
          unsigned long long cur = tab[p];
          if (cur == key) break;
          if (cur == 0) {
            cur = atomicCAS(&tab[p], 0ull, (unsigned long long)key);
            if (cur == 0 || cur == key) break;
          }
          p = (p + 1) & (uint32_t)(ESLICE - 1);
        }
        if (z == PROBE_MAX) flags |= F_TRIPLE_OVERFLOW;
      }
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < ESLICE / 2; x += KS_T) g[x] = l[x];
    __syncthreads();
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
}

// chain interning: the keys the tile kernel staged (workgroup w's runs) ->
// the edge set in place; and the deferred chain checks: every entry the tile
// kernel claimed is published by now, so each deferred (sig, parent sig) is
// joined and checked, or inserted if its slot was lost to another chain
__global__ void __launch_bounds__(256) k_chain_settle(const unsigned long long *__restrict__ stage, uint32_t sub,
                                                      const uint32_t *__restrict__ stage_n, uint32_t lb1,
                                                      unsigned long long *__restrict__ trip, uint64_t tcap,
                                                      const unsigned long long *__restrict__ defer, uint32_t dcap,
                                                      const uint32_t *__restrict__ defer_n, uint32_t nwg,
                                                      unsigned long long *__restrict__ ctab, uint64_t ccap,
                                                      unsigned int *__restrict__ counters,
                                                      unsigned long long *__restrict__ stats64,
                                                      uint32_t *__restrict__ gpos, uint32_t gcap, uint32_t spin) {
  uint32_t flags = 0, fresh = 0;
  // parts workgroups per tile workgroup's runs (gridDim.y): the inserts are
  // latency-bound device-scope CASes, so small batches (few tile workgroups,
  // every chain new) want more threads than one workgroup per run
  const uint32_t parts = gridDim.y, t0 = blockIdx.y * blockDim.x + threadIdx.x, ts = parts * blockDim.x;
  for (uint32_t w = blockIdx.x; w < nwg; w += gridDim.x) {
    for (uint32_t b = 0; b < (1u << lb1); ++b) {
      const uint64_t r = ((uint64_t)w << lb1) + b;
      const uint32_t m = stage_n[r];
      for (uint32_t x = t0; x < m; x += ts) edge_insert(stage[r * sub + x], trip, tcap, &flags);
    }
    const uint32_t md = defer_n[w];
    for (uint32_t x = t0; x < md; x += ts) {
      const unsigned long long *r = defer + 2 * ((uint64_t)w * dcap + x);
      int rr = 0;
      for (uint32_t t = 0; t < spin && rr == 0; ++t)
        rr = chain_put(ctab, ccap, r[0], r[1], &flags, gpos, gcap, counters);
      if (rr == 0) flags |= F_SPIN;
      fresh += rr == 1;
    }
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
  for (int o = 32; o > 0; o >>= 1) fresh += __shfl_xor(fresh, o, 64);
  if ((threadIdx.x & 63) == 0 && fresh) atomicAdd(&stats64[S_CHAINS], (unsigned long long)fresh);
}

// The pending spans (ancestry outside their LDS window), one pass: each hashes
// its own and its parent's ancestry over the global contracted parents, then
// joins or inserts its chain exactly like the tile kernel (no ordering needed).
// The first PB ancestors of the walk stay in registers, so that a row's keys
// are formed without walking again and their edge-set probes and claims go
// out together (one round trip each instead of one per ancestor, in turn:
// the pending spans are the deepest ancestries, and this kernel is a serial
// latency chain on small batches -- 62 us of config 5's 2 500-trace tick).
#ifndef KMZ_PEND_PB
#define KMZ_PEND_PB 16
#endif
constexpr int PB = KMZ_PEND_PB;
// edge_insert from the slot after `pos` (its home slot was taken by another key)
__device__ __forceinline__ void edge_insert_after(uint64_t key, uint64_t pos, unsigned long long *__restrict__ trip,
                                                  uint64_t tcap, uint32_t *flags) {
  for (uint32_t z = 1; z < PROBE_MAX; ++z) {
    pos = eset_next(pos, tcap);
    uint64_t cur = trip[pos];
    if (cur == key) return;
    if (cur == 0) {
      cur = atomicCAS(&trip[pos], 0ull, (unsigned long long)key);
      if (cur == 0 || cur == key) return;
    }
  }
  *flags |= F_TRIPLE_OVERFLOW;
}

__global__ void __launch_bounds__(256) k4_chain_pend(const uint32_t *__restrict__ plist, uint32_t pcap,
                                                     const uint8_t *__restrict__ kind,
                                                     const uint32_t *__restrict__ shape,
                                                     const int64_t *__restrict__ ts,
                                                     const uint32_t *__restrict__ cparent, uint32_t n,
                                                     const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                     uint32_t n_ep, uint64_t seed,
                                                     unsigned long long *__restrict__ ctab, uint64_t ccap,
                                                     unsigned long long *__restrict__ trip, uint64_t tcap,
                                                     unsigned long long *__restrict__ ep_ts,
                                                     unsigned int *__restrict__ counters,
                                                     unsigned long long *__restrict__ stats64,
                                                     uint32_t *__restrict__ gpos, uint32_t gcap, bool direct,
                                                     uint32_t spin, bool by_shape) {
  // by_shape: the run's chain elements are shapes (k4_tile8 on a dependency
  // table that maps every shape into range), as the tile kernel's
  const uint32_t m = min(counters[C_PLIST], pcap);
  uint32_t flags = 0;
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < m; x += gridDim.x * blockDim.x) {
    const uint32_t i = plist[x];
    const uint8_t ki = kind[i];
    const uint32_t sh = shape[i];
    const uint32_t es = sh < n_shapes ? dep_ep[sh] : NONE;
    const bool on = ki == KIND_SERVER;
    if (es >= n_ep && on) flags |= F_RANGE;
    // fold hashes of the span's ancestry and of its parent's (suffix) ancestry
    uint64_t acc = sig_elem(by_shape ? (sh < n_shapes ? sh : NONE) : es, on, seed), pacc = 0;
    uint32_t d = 0;
    bool bad = false;
    const uint32_t a = cparent[i];
    uint32_t aid[PB], ash[PB];  // the first PB ancestors: index, shape, SERVER or not
    bool asrv[PB];
    uint32_t cur = a;
    auto hop = [&](uint32_t c, uint32_t &sa, bool &srv) -> bool {  // one ancestor into the folds
      if (c >= n) {  // CYC (a CLIENT loop); never another value (k_pend/k_resolve leave indices < n)
        flags |= c == CYC ? F_CYCLE : F_RANGE;
        return false;
      }
      if (++d > MAX_DEPTH) {
        flags |= F_CYCLE;
        return false;
      }
      sa = shape[c];
      srv = kind[c] == KIND_SERVER;
      const uint32_t ea = sa < n_shapes ? (by_shape ? sa : dep_ep[sa]) : NONE;
      const uint64_t el = sig_elem(ea, srv, seed);
      acc = sig_step(acc, el);
      pacc = d == 1 ? el : sig_step(pacc, el);
      return true;
    };
#pragma unroll
    for (int k = 0; k < PB; ++k) {
      aid[k] = 0;
      ash[k] = NONE;
      asrv[k] = false;
      if (bad || cur == NONE) continue;
      aid[k] = cur;
      if (!hop(cur, ash[k], asrv[k])) {
        bad = true;
        continue;
      }
      cur = cparent[cur];
    }
    for (; !bad && cur != NONE; cur = cparent[cur]) {  // deeper than PB: folded, not kept
      uint32_t sa;
      bool srv;
      if (!hop(cur, sa, srv)) bad = true;
    }
    if (bad) continue;
    const uint64_t sg = sig_final(acc, d, seed, &flags), psig = a == NONE ? ROOT_SIG : sig_final(pacc, d - 1, seed, &flags);
    int r = direct ? 3 : 0;  // direct: no chain table, every row inserts its keys
    for (uint32_t t = 0; t < spin && r == 0; ++t)
      r = chain_put(ctab, ccap, sg, psig, &flags, gpos, gcap, counters);
    if (r == 0) flags |= F_SPIN;  // (the row is not counted: the run is redone on the exact walk)
    if (r <= 0) continue;         // (-1: F_CHAIN_OVERFLOW, redone with a larger table)
    if (on) {  // a row: its relations, keys (new chain) and non-SERVER ancestors
      const uint32_t dk = min(d, (uint32_t)PB);
      // every load of the kept ancestors issued before any is used
      uint32_t eak[PB];
      int64_t tk[PB];
#pragma unroll
      for (int k = 0; k < PB; ++k) {
        eak[k] = n_shapes ? dep_ep[(uint32_t)k < dk && ash[k] < n_shapes ? ash[k] : 0] : NONE;
        tk[k] = ts[aid[k]];
      }
      uint64_t key[PB], pos[PB], cv[PB];
      bool ins[PB], ok = true;
#pragma unroll
      for (int k = 0; k < PB; ++k) {
        ins[k] = false;
        if ((uint32_t)k >= dk || !ok) continue;
        const uint32_t ea = ash[k] < n_shapes ? eak[k] : NONE;
        if (ea >= n_ep) {  // (as the walk: the keys stop at the first unmapped ancestor)
          flags |= F_RANGE;
          ok = false;
          continue;
        }
        key[k] = edge_key(ea, es, k + 1, asrv[k]);
        ins[k] = r != 2 && !(flags & F_TRIPLE_OVERFLOW);
        if (!asrv[k]) atomicMax(&ep_ts[ea], (unsigned long long)((uint64_t)tk[k] ^ TS_BIAS));
      }
#pragma unroll
      for (int k = 0; k < PB; ++k) {  // home slots: loads, then claims, in flight together
        pos[k] = ins[k] ? eslot(key[k], tcap) : 0;
        cv[k] = ins[k] ? trip[pos[k]] : 0;
      }
#pragma unroll
      for (int k = 0; k < PB; ++k)
        if (ins[k] && cv[k] == 0) cv[k] = atomicCAS(&trip[pos[k]], 0ull, (unsigned long long)key[k]);
#pragma unroll
      for (int k = 0; k < PB; ++k)  // (rare: the home slot held another key)
        if (ins[k] && cv[k] != 0 && cv[k] != key[k]) edge_insert_after(key[k], pos[k], trip, tcap, &flags);
      if (d > PB && ok) {  // deeper ancestors, one at a time
        uint32_t kk = PB;
        for (uint32_t c = cparent[aid[PB - 1]]; c != NONE; c = cparent[c]) {
          ++kk;
          const uint8_t ka = kind[c];
          const uint32_t sa = shape[c];
          const uint32_t ea = sa < n_shapes ? dep_ep[sa] : NONE;
          if (ea >= n_ep) {
            flags |= F_RANGE;
            break;
          }
          if (r != 2) edge_insert(edge_key(ea, es, kk, ka == KIND_SERVER), trip, tcap, &flags);
          if (ka != KIND_SERVER) atomicMax(&ep_ts[ea], (unsigned long long)((uint64_t)ts[c] ^ TS_BIAS));
        }
      }
      atomicAdd(&stats64[S_ROWS], 1ull);
      atomicAdd(&stats64[S_REL], (unsigned long long)d);
      atomicMax(&stats64[S_MAXD], (unsigned long long)d);
    }
    if (r == 1) atomicAdd(&stats64[S_CHAINS], 1ull);
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
}

// multi-GPU union of edge-key sets: other ranks' keys into this context's set
__global__ void __launch_bounds__(256) k_key_insert(const unsigned long long *__restrict__ keys, uint64_t n,
                                                    unsigned long long *__restrict__ trip, uint64_t tcap,
                                                    unsigned int *__restrict__ counters) {
  uint32_t flags = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const unsigned long long k = keys[i];
    if (k) edge_insert(k, trip, tcap, &flags);  // 0: padding
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
}

void launch_key_insert(hipStream_t s, const unsigned long long *keys, uint64_t n, unsigned long long *trip,
                       uint64_t tcap, unsigned int *counters) {
  if (!n) return;
  const uint32_t g = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_key_insert, dim3(g), dim3(256), 0, s, keys, n, trip, tcap, counters);
}

uint32_t chain_tiles(uint32_t n) { return (n + CT - 1) / CT; }
}  // namespace kmz
extern "C" int kmz__debug_chain(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kmz::g_chain_dbg), sizeof(kmz::g_chain_dbg)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(kmz::g_chain_dbg), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
namespace kmz {

// persistent workgroups of k4_chain: what the device keeps resident at once
// (CUs x the occupancy of the larger of the two instances), so a workgroup
// only ever waits on workgroups that are running.  Queried once per device;
// CHAIN_WG (the 256-CU figure at CHAIN_WAVES) if the query fails.
static uint32_t chain_resident() {
  static std::mutex mu;
  static uint32_t cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return CHAIN_WG;
  std::lock_guard<std::mutex> lk(mu);
  if (!cached[dev]) {
    int cus = 0, o0 = 0, o1 = 0;
    uint32_t g = CHAIN_WG;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&o0, k4_chain<false>, CTT, 0) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&o1, k4_chain<true>, CTT, 0) == hipSuccess && std::min(o0, o1) > 0)
      g = (uint32_t)cus * (uint32_t)std::min(o0, o1);
    cached[dev] = g;
  }
  return cached[dev];
}
uint32_t chain_grid(uint32_t n) { return std::min<uint32_t>(chain_tiles(n), chain_resident()); }

// per shape: its dependency endpoint and the element hash of a SERVER span of
// it under this run's seed (the walk's per-slot hash is then one gather)
__global__ void __launch_bounds__(256) k_chain_etab(const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                    uint64_t seed, uint4 *__restrict__ etab) {
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n_shapes; s += gridDim.x * 256) {
    const uint32_t ep = dep_ep[s];
    const uint64_t el = sig_elem(ep, true, seed);
    etab[s] = make_uint4(ep, (uint32_t)el, (uint32_t)(el >> 32), 0);
  }
}

void launch_chain_etab(hipStream_t s, const uint32_t *dep_ep, uint32_t n_shapes, uint64_t seed, uint4 *etab) {
  hipLaunchKernelGGL(k_chain_etab, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n_shapes + 255) / 256, 1024))),
                     dim3(256), 0, s, dep_ep, n_shapes, seed, etab);
}

void launch_chain(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                  const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                  uint64_t index_base, uint64_t seed, void *ctab, uint64_t ccap, unsigned long long *trip,
                  uint64_t tcap, unsigned long long *ep_ts, unsigned long long *rowpos, uint32_t *plist,
                  uint32_t pcap, unsigned int *counters, uint32_t *wg_stats, unsigned long long *stats64,
                  unsigned long long *stage, uint32_t scap, uint32_t *stage_n, unsigned long long *defer,
                  uint32_t dcap, uint32_t *defer_n, uint32_t *wpos, uint32_t wcap, uint32_t *wpos_n,
                  uint4 *etab, bool direct, uint32_t ablate, bool cmode, bool etab_ok) {
  const uint32_t nt = chain_tiles(n);
  if (!nt) return;
  uint32_t lb1, lb2;
  key_bins(tcap, &lb1, &lb2);
  if (!direct) {  // chain interning stages few keys: one run per workgroup, inserted in place
    lb2 += lb1;
    lb1 = 0;
  }
  const uint32_t g = chain_grid(n);
  unsigned long long *tab = reinterpret_cast<unsigned long long *>(ctab);
  if (!etab_ok) launch_chain_etab(s, dep_ep, n_shapes, seed, etab);  // (etab_ok: this shape table's, this seed's)
  if (direct)
    hipLaunchKernelGGL(k4_chain<true>, dim3(g), dim3(CTT), 0, s, kind, shape, ts, cparent, n, etab, n_shapes, n_ep,
                       index_base, seed, tab, ccap, trip, tcap, ep_ts, rowpos, plist, pcap, counters, wg_stats, stage,
                       scap, stage_n, defer, dcap, defer_n, wpos, wcap, wpos_n, nt, lb1, lb2, ablate, cmode ? 1u : 0u);
  else
    hipLaunchKernelGGL(k4_chain<false>, dim3(g), dim3(CTT), 0, s, kind, shape, ts, cparent, n, etab, n_shapes, n_ep,
                       index_base, seed, tab, ccap, trip, tcap, ep_ts, rowpos, plist, pcap, counters, wg_stats, stage,
                       scap, stage_n, defer, dcap, defer_n, wpos, wcap, wpos_n, nt, lb1, lb2, ablate, 0u);
}

bool compact_staging(uint64_t tcap, uint32_t n_ep) {
  uint32_t lb1, lb2;
  return key_bins(tcap, &lb1, &lb2) && lb1 >= 6 && n_ep <= 65536;  // (x38 residuals below >= 6 coarse bits: <= 32 bits)
}

bool key_bins(uint64_t tcap, uint32_t *lb1, uint32_t *lb2) {
  // slices of the edge set: tcap / ESLICE (tcap a power of two >= ESLICE)
  uint32_t ls = 0;
  while ((ESLICE << ls) < tcap) ++ls;
  *lb1 = std::min<uint32_t>(ls, 6);  // 64 coarse bins, more when the slices outnumber 64 x 2^KB2_MAX
  if (ls - *lb1 > KB2_MAX) *lb1 = std::min<uint32_t>(ls - KB2_MAX, KB1_MAX);
  *lb2 = ls - *lb1;
  return (ESLICE << ls) == tcap && *lb2 <= KB2_MAX;
}

void launch_chain_settle(hipStream_t s, uint32_t n, bool direct, void *ctab, uint64_t ccap, unsigned long long *trip,
                         uint64_t tcap, unsigned int *counters, const uint32_t *wg_stats, unsigned long long *stats64,
                         const unsigned long long *stage, uint32_t scap, const uint32_t *stage_n,
                         unsigned long long *bucket, uint64_t bcap, uint32_t *bucket_n,
                         const unsigned long long *defer, uint32_t dcap, const uint32_t *defer_n, uint32_t *gpos,
                         uint32_t gcap, uint32_t ablate, bool cmode, uint32_t ablate2) {
  if (!chain_tiles(n)) return;
  const uint32_t g = chain_grid(n);
  uint32_t lb1, lb2;
  key_bins(tcap, &lb1, &lb2);
  if (!direct) {  // (as launch_chain)
    lb2 += lb1;
    lb1 = 0;
  }
  const uint32_t nsl = (uint32_t)(tcap / ESLICE), nruns = g << lb1;
  if (direct) {
    const uint32_t gp = std::min<uint32_t>(nruns, 8192), gs = std::min<uint32_t>(nsl, 8192);
    // the key cache needs one coarse bin per workgroup (KMZ_ABLATE2 bit 16: off, for comparison)
    const bool dedup = !(ablate2 & 65536u) && gp % (1u << lb1) == 0;
    if (cmode) {
      hipLaunchKernelGGL(k_key_part<true>, dim3(gp), dim3(KP_T), 0, s, (const void *)stage, scap >> lb1, stage_n,
                         nruns, lb1, lb2, (void *)bucket, bcap, bucket_n, trip, tcap, counters, dedup);
      hipLaunchKernelGGL(k_key_slice<true>, dim3(gs), dim3(KS_T), 0, s, (const void *)bucket, bcap, bucket_n, nsl,
                         lb1 + lb2, trip, tcap, counters);
    } else {
      hipLaunchKernelGGL(k_key_part<false>, dim3(gp), dim3(KP_T), 0, s, (const void *)stage, scap >> lb1, stage_n,
                         nruns, lb1, lb2, (void *)bucket, bcap, bucket_n, trip, tcap, counters, dedup);
      hipLaunchKernelGGL(k_key_slice<false>, dim3(gs), dim3(KS_T), 0, s, (const void *)bucket, bcap, bucket_n, nsl,
                         lb1 + lb2, trip, tcap, counters);
    }
  } else {
    const uint32_t parts = std::max<uint32_t>(1, std::min<uint32_t>(16, 2048 / g));
    hipLaunchKernelGGL(k_chain_settle, dim3(g, parts), dim3(256), 0, s, stage, scap >> lb1, stage_n, lb1, trip, tcap, defer,
                       dcap, defer_n, g, reinterpret_cast<unsigned long long *>(ctab), ccap, counters, stats64, gpos,
                       gcap, spin_bound(ablate));
  }
  launch_tile_sum(s, wg_stats, g, 4u, 4u, stats64 + S_ROWS, 2u);  // rows, rel, maxd, chains
}

// zero the chain-table entries this run wrote: the per-workgroup lists of the
// tile kernel and the run's global list (settle / pending / inline inserts)
__global__ void __launch_bounds__(256) k_chain_clear(unsigned long long *__restrict__ ctab,
                                                     const uint32_t *__restrict__ wpos, uint32_t wcap,
                                                     const uint32_t *__restrict__ wpos_n, uint32_t nwg,
                                                     const uint32_t *__restrict__ gpos, uint32_t gcap,
                                                     const unsigned int *__restrict__ counters) {
  auto clear = [&](uint32_t p) { *reinterpret_cast<ulonglong2 *>(ctab + 2 * (uint64_t)p) = make_ulonglong2(0, 0); };
  for (uint32_t w = blockIdx.x; w < nwg; w += gridDim.x) {
    const uint32_t m = min(wpos_n[w], wcap);
    for (uint32_t x = threadIdx.x; x < m; x += 256) clear(wpos[(uint64_t)w * wcap + x]);
  }
  const uint32_t mg = min(counters[C_WPOS], gcap);
  for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < mg; x += gridDim.x * 256) clear(gpos[x]);
}

void launch_chain_clear(hipStream_t s, uint32_t n, void *ctab, const uint32_t *wpos, uint32_t wcap,
                        const uint32_t *wpos_n, const uint32_t *gpos, uint32_t gcap, const unsigned int *counters) {
  if (!chain_tiles(n)) return;
  const uint32_t g = chain_grid(n);
  hipLaunchKernelGGL(k_chain_clear, dim3(g), dim3(256), 0, s, reinterpret_cast<unsigned long long *>(ctab), wpos,
                     wcap, wpos_n, g, gpos, gcap, counters);
}

void launch_chain_clear_list(hipStream_t s, void *ctab, const uint32_t *gpos, uint32_t gcap, const unsigned int *counters) {
  hipLaunchKernelGGL(k_chain_clear, dim3(1024), dim3(256), 0, s, reinterpret_cast<unsigned long long *>(ctab), gpos, 0u,
                     gpos, 0u, gpos, gcap, counters);
}

void launch_chain_pend(hipStream_t s, const uint32_t *plist, uint32_t pcap, const uint8_t *kind,
                       const uint32_t *shape, const int64_t *ts, const uint32_t *cparent, uint32_t n,
                       const uint32_t *dep_ep,
                       uint32_t n_shapes, uint32_t n_ep, uint64_t seed, void *ctab, uint64_t ccap,
                       unsigned long long *trip, uint64_t tcap, unsigned long long *ep_ts, unsigned int *counters,
                       unsigned long long *stats64, uint32_t *gpos, uint32_t gcap, bool direct, uint32_t ablate,
                       bool by_shape) {
  hipLaunchKernelGGL(k4_chain_pend, dim3(1024), dim3(256), 0, s, plist, pcap, kind, shape, ts, cparent, n, dep_ep,
                     n_shapes, n_ep, seed, reinterpret_cast<unsigned long long *>(ctab), ccap, trip, tcap, ep_ts,
                     counters, stats64, gpos, gcap, direct, spin_bound(ablate), by_shape);
}

}  // namespace kmz
