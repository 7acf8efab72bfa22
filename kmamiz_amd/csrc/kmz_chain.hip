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
//     { sig(chain), sig(parent chain) (0 at a root), endpoint, kind == SERVER }
//
// Rows that share a chain (most of them: the 100M-span mesh has ~0.5M distinct
// chains) produce identical edge keys, so only the workgroup that inserts a new
// chain emits its keys; nothing per relation is written to HBM.
//
// `sig` is a 64-bit polynomial hash of the whole ancestry, computed by walking
// the ancestors in LDS, so every span probes the table once, in one round, with
// no dependency on its parent's probe or insert.  Exactness does not rest on
// the hash: an entry records the exact recursive definition (parent chain,
// endpoint, kind) and every span checks the entry it found or joined against
// its own.  The table holds one entry per sig, so by induction from the roots
// (parent sig 0) equal sigs are equal chains; a failed check (a 64-bit
// collision) raises F_SIG and the run is repeated with another hash seed.
//
//   k4_chain       2048-span tile + 512-span halo per side in LDS (contracted
//                  parent, kind, endpoint).  Marks the tile's spans and their
//                  in-window ancestors, hashes the ancestries (a Horner walk
//                  over LDS element hashes), probes, inserts
//                  the new chains (one leader per distinct chain per
//                  workgroup), then emits the new chains' keys with the whole
//                  workgroup.  Ancestries that leave the window (or are deeper
//                  than WIN_DEPTH inside it) go to a pending list.
//   k4_chain_pend  the pending spans, one pass, hashing over the global
//                  contracted parents (rare).
//
// Per-endpoint lastUsage / first row / external of rows come from the K3
// shape-level partials (kmz_api.hip, k_collapse_endpoints); non-SERVER
// ancestors (not rows) add their timestamps here.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_kernels.h"

namespace kmz {

constexpr uint32_t CT = 2048, CH = 512, CW = CT + 2 * CH;
constexpr int CTT = 512;
constexpr int CPT = CT / CTT;  // tile spans per thread
constexpr int CPW = CW / CTT;  // window spans per thread
static_assert(CW % CTT == 0 && CT % CTT == 0 && CH % CTT == 0, "window slots must map to fixed threads");
constexpr uint16_t W_NONE = 0xFFFF, W_CYC = 0xFFFE, W_OUT = 0xFFFD;
constexpr uint32_t WIN_DEPTH = 255;  // deeper in-window ancestries take the pending path
constexpr uint32_t PROBE_MAX = 512;
constexpr uint32_t IMAP = 512;  // LDS map: one inserting leader per distinct new chain
constexpr uint32_t WAIT_ROUNDS = 256;
constexpr uint32_t FMAX = CT;   // new SERVER chains per tile whose keys the workgroup emits
constexpr uint64_t SIG_M = 0xD6E8FEB86659FD93ull;
// lst: per window slot
constexpr uint8_t S_NONE = 0, S_DONE = 1, S_PUT = 2, S_PEND = 3;

__device__ __forceinline__ uint64_t sig_elem(uint32_t ep, bool on, uint64_t seed) {
  return mix64((((uint64_t)ep << 1) | (on ? 1ull : 0ull)) ^ seed);
}
constexpr uint64_t ROOT_SIG = ~0ull;  // the "parent sig" of a root
__device__ __forceinline__ uint64_t sig_final(uint64_t acc, uint32_t d, uint64_t seed) {
  const uint64_t z = mix64(acc ^ ((uint64_t)d * 0x632BE59BD9B4E019ull) ^ (seed << 1));
  return (z == 0 || z == ROOT_SIG) ? 1 : z;  // 0 marks an unwritten word, ROOT_SIG a root's parent
}
__device__ __forceinline__ uint64_t epon_of(uint32_t ep, bool on) {
  return (1ull << 63) | ((uint64_t)ep << 1) | (on ? 1ull : 0ull);  // never 0 (0 = unpublished)
}

__device__ __forceinline__ uint64_t edge_key(uint32_t ea, uint32_t es, uint32_t d, bool on) {
  return ((uint64_t)ea << 40) | ((uint64_t)es << 16) | ((uint64_t)d << 1) | (on ? 1ull : 0ull);
}

// the global edge-key set (one insert per key of a NEW chain only); its size
// is counted by the compaction
__device__ __forceinline__ void edge_insert(uint64_t key, unsigned long long *__restrict__ trip, uint64_t tcap,
                                           uint32_t *flags) {
  uint64_t pos = slot_of(key, tcap);
  for (uint32_t z = 0; z < PROBE_MAX; ++z) {
    uint64_t cur = trip[pos];
    if (cur == key) return;
    if (cur == 0) {
      cur = atomicCAS(&trip[pos], 0ull, (unsigned long long)key);
      if (cur == 0 || cur == key) return;
    }
    pos = pos + 1 == tcap ? 0 : pos + 1;
  }
  *flags |= F_TRIPLE_OVERFLOW;
}

// Chain table entry words: [0] sig, [1] parent sig (ROOT_SIG at a root),
// [2] endpoint/kind, [3] unused.  Every word is written once with a nonzero
// value, so a reader needs no ordering between them: an entry is published
// once all three are nonzero.
// Insert (or join) the chain `sig`.  Returns 1 inserted, 2 found (and
// checked), 0 not yet decidable (the winner has not published), -1 probe bound.
__device__ __forceinline__ int chain_put(unsigned long long *__restrict__ ctab, uint64_t ccap, uint64_t sig,
                                         uint64_t psig, uint64_t epon, uint32_t *flags) {
  uint64_t pos = slot_of(sig, ccap);
  for (uint32_t z = 0; z < PROBE_MAX; ++z) {
    unsigned long long *e = ctab + 4 * pos;
    const unsigned long long c = atomicCAS(&e[0], 0ull, (unsigned long long)sig);
    if (c == 0) {
      atomicExch(&e[1], (unsigned long long)psig);
      atomicExch(&e[2], (unsigned long long)epon);
      return 1;
    }
    if (c == sig) {
      const unsigned long long ps = atomicAdd(&e[1], 0ull), w = atomicAdd(&e[2], 0ull);  // memory-side reads
      if (w == 0 || ps == 0) return 0;
      if (w != epon || ps != psig) *flags |= F_SIG;
      return 2;
    }
    pos = pos + 1 == ccap ? 0 : pos + 1;
  }
  *flags |= F_CHAIN_OVERFLOW;
  return -1;
}

__device__ unsigned long long g_chain_dbg[8];  // diagnostic counters (KMZ_ABLATE bit 21 only)

__global__ void __launch_bounds__(CTT, 4) k4_chain(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                   const int64_t *__restrict__ ts,
                                                   const uint32_t *__restrict__ cparent, uint32_t n,
                                                   const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                   uint32_t n_ep, uint64_t index_base, uint64_t seed,
                                                   unsigned long long *__restrict__ ctab, uint64_t ccap,
                                                   unsigned long long *__restrict__ trip, uint64_t tcap,
                                                   unsigned long long *__restrict__ ep_ts,
                                                   unsigned long long *__restrict__ rowpos_out,
                                                   uint32_t *__restrict__ plist, uint32_t pcap,
                                                   unsigned int *__restrict__ counters,
                                                   uint32_t *__restrict__ tile_stats, uint32_t ablate) {
  __shared__ unsigned long long lsig[CW];
  __shared__ uint32_t lep[CW];
  __shared__ uint16_t lcp[CW], ldep[CW];
  __shared__ uint8_t lkind[CW], lneed[CW], lanc[CW], lst[CW];
  __shared__ unsigned long long imap_sig[IMAP];
  __shared__ uint32_t imap_state[IMAP];  // 0 open, 1 leader working, 2 leader done
  __shared__ uint16_t fresh[FMAX];
  __shared__ uint32_t foff[FMAX + 1];
  __shared__ uint32_t nfresh;
  __shared__ uint32_t red[CTT / 64][4];
  const uint32_t tile = blockIdx.x, t0 = tile * CT, t1 = min(n, t0 + CT);
  const uint32_t w0 = t0 > CH ? t0 - CH : 0, w1 = min(n, t1 + CH), wn = w1 - w0;
  {  // window -> LDS; every global load of a thread in flight together
    uint32_t c[CPW], sh[CPW];
    uint8_t k[CPW];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {  // clamped, unconditional: no branch between the loads
      const uint32_t j = min(w0 + q * CTT + threadIdx.x, n - 1);
      c[q] = cparent[j];
      k[q] = kind[j];
      sh[q] = shape[j];
    }
    uint32_t e[CPW];
#pragma unroll
    for (int q = 0; q < CPW; ++q) e[q] = dep_ep[sh[q] < n_shapes ? sh[q] : 0];
#pragma unroll
    for (int q = 0; q < CPW; ++q)
      if (k[q] == KIND_CLIENT || sh[q] >= n_shapes || !n_shapes) e[q] = NONE;
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const uint32_t jl = q * CTT + threadIdx.x;
      if (jl < wn) {
        lkind[jl] = k[q];
        lep[jl] = e[q];
        lcp[jl] = c[q] == NONE ? W_NONE
                               : (c[q] == CYC ? W_CYC : ((c[q] >= w0 && c[q] < w1) ? (uint16_t)(c[q] - w0) : W_OUT));
      }
      lneed[jl] = 0;
      lanc[jl] = 0;
      lst[jl] = S_NONE;
    }
    for (uint32_t x = threadIdx.x; x < IMAP; x += CTT) {
      imap_sig[x] = 0;
      imap_state[x] = 0;
    }
    if (threadIdx.x == 0) nfresh = 0;
  }
  __syncthreads();
  // mark: the tile's non-CLIENT spans need their chain, and so do their
  // in-window ancestors (lanc: ancestor of a tile row, for non-SERVER
  // lastUsage).  Every store writes 1, so concurrent marking loses nothing.
  uint32_t flags = 0;
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const uint32_t i = t0 + q * CTT + threadIdx.x;
    if (i >= t1) continue;
    const uint32_t jl = i - w0;
    const uint8_t kj = lkind[jl];
    if (kj == KIND_CLIENT) continue;
    const bool row = kj == KIND_SERVER;
    lneed[jl] = 1;
    for (uint32_t a = lcp[jl], steps = 0; a < CW && steps < CW; ++steps) {
      if (lneed[a] && (!row || lanc[a])) break;  // marked from here up already
      lneed[a] = 1;
      if (row) lanc[a] = 1;
      a = lcp[a];
    }
  }
  __syncthreads();
  // hash every needed ancestry (Horner over s, a1, ..., aD, walked in LDS):
  //   acc = ((elem(s) M + elem(a1)) M + ...) M + elem(aD),  sig = final(acc, D)
  // lsig first holds every slot's element hash, then the finished sigs.
  const bool hash_on = !(ablate & (1u << 16));  // diagnostic knob: no hashing / probing / inserting
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const uint32_t jl = q * CTT + threadIdx.x;
    if (jl < wn && lneed[jl]) lsig[jl] = sig_elem(lep[jl], lkind[jl] == KIND_SERVER, seed);
  }
  __syncthreads();
  {
    uint64_t sg[CPW];
    uint32_t dd[CPW];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const uint32_t jl = q * CTT + threadIdx.x;
      sg[q] = 0;
      dd[q] = 0;
      if (jl >= wn || !lneed[jl]) continue;
      if (!hash_on) {
        lst[jl] = S_DONE;
        continue;
      }
      if (lep[jl] >= n_ep && (lkind[jl] == KIND_SERVER || lanc[jl])) flags |= F_RANGE;
      uint64_t acc = lsig[jl];
      uint32_t d = 0, a = lcp[jl];
      while (a < CW && d < WIN_DEPTH) {
        acc = acc * SIG_M + lsig[a];
        ++d;
        a = lcp[a];
      }
      if (a != W_NONE) {  // W_OUT: leaves the window or deeper than WIN_DEPTH; W_CYC: CLIENT loop
        if (a == W_CYC) flags |= F_CYCLE;
        lst[jl] = S_PEND;
        continue;
      }
      sg[q] = sig_final(acc, d, seed);
      dd[q] = d;
      lst[jl] = (ablate & (1u << 17)) ? S_DONE : S_PUT;  // diagnostic knob: hash only
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const uint32_t jl = q * CTT + threadIdx.x;
      if (jl < wn && lneed[jl] && lst[jl] != S_PEND) {
        lsig[jl] = sg[q];
        ldep[jl] = (uint16_t)dd[q];
      }
    }
  }
  __syncthreads();
  // one round of probes, all in flight; a found entry is checked against the
  // span's own (parent sig, endpoint, kind)
  {
    ulonglong2 w01[CPW], w23[CPW];  // (sig, parent sig), (endpoint/kind, -)
    uint64_t pos[CPW], sgq[CPW];
    bool pr[CPW];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const uint32_t jl = q * CTT + threadIdx.x;
      pr[q] = jl < wn && lst[jl] == S_PUT;
      sgq[q] = pr[q] ? lsig[jl] : 0;
      pos[q] = pr[q] ? slot_of(sgq[q], ccap) : 0;
      const ulonglong2 *e = reinterpret_cast<const ulonglong2 *>(ctab + 4 * pos[q]);
      w01[q] = pr[q] ? e[0] : make_ulonglong2(0, 0);
      w23[q] = pr[q] ? e[1] : make_ulonglong2(0, 0);
    }
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      if (!pr[q]) continue;
      const uint32_t jl = q * CTT + threadIdx.x;
      const uint64_t sg = sgq[q];
      for (uint32_t z = 0; w01[q].x != sg && w01[q].x != 0 && z < PROBE_MAX; ++z) {  // another chain's slot
        pos[q] = pos[q] + 1 == ccap ? 0 : pos[q] + 1;
        const ulonglong2 *e = reinterpret_cast<const ulonglong2 *>(ctab + 4 * pos[q]);
        w01[q] = e[0];
        w23[q] = e[1];
      }
      if (w01[q].x == sg && w01[q].y != 0 && w23[q].x != 0) {
        const uint32_t p = lcp[jl];
        const uint64_t psig = p == W_NONE ? ROOT_SIG : lsig[p];
        if (w23[q].x != epon_of(lep[jl], lkind[jl] == KIND_SERVER) || w01[q].y != psig) flags |= F_SIG;
        lst[jl] = S_DONE;
      }
    }
  }
  // chains not in the table: insert (no ordering among them: an entry names
  // its parent by sig), one leader per distinct chain in this workgroup
  uint32_t fresh_n = 0, dbg_put = 0, dbg_r[3] = {0, 0, 0}, dbg_rounds = 0;
  if (ablate & (1u << 21))
    for (uint32_t jl = threadIdx.x; jl < wn; jl += CTT) dbg_put += lst[jl] == S_PUT;
  if (ablate & (1u << 18))  // diagnostic knob: probe but no inserts
    for (uint32_t jl = threadIdx.x; jl < wn; jl += CTT)
      if (lst[jl] == S_PUT) lst[jl] = S_DONE;
  __syncthreads();
  for (uint32_t round = 0;; ++round) {
    bool prog = false, waiting = false;
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const uint32_t jl = q * CTT + threadIdx.x;
      if (jl >= wn || lst[jl] != S_PUT) continue;
      const uint64_t sg = lsig[jl];
      const uint32_t p = lcp[jl];
      const uint64_t psig = p == W_NONE ? ROOT_SIG : lsig[p];
      const bool on = lkind[jl] == KIND_SERVER;
      const uint64_t epon = epon_of(lep[jl], on);
      uint32_t h = (uint32_t)(sg >> 32) & (IMAP - 1), slot = IMAP;
      bool leader = true;
      for (uint32_t t = 0; t < 8; ++t) {
        unsigned long long k = imap_sig[h];
        if (k == 0) k = atomicCAS(&imap_sig[h], 0ull, (unsigned long long)sg);
        if (k == 0 || k == sg) {  // this sig's slot: lead it if nobody does
          slot = h;
          leader = atomicCAS(&imap_state[h], 0u, 1u) == 0u;
          break;
        }
        h = (h + 1) & (IMAP - 1);
      }
      if (!leader) {  // the leader's check covers this span too: same sig => same entry
        if (imap_state[slot] == 2) {
          lst[jl] = S_DONE;
          prog = true;
        } else {
          waiting = true;
        }
        continue;
      }
      const int r = chain_put(ctab, ccap, sg, psig, epon, &flags);
      if (r >= 0) ++dbg_r[r];
      if (r == 0) {  // another workgroup inserted it and has not published yet
        if (slot < IMAP) imap_state[slot] = 0;  // reopen the leadership for the next round
        waiting = true;
        continue;
      }
      prog = true;
      lst[jl] = r < 0 ? S_PEND : S_DONE;
      if (slot < IMAP) imap_state[slot] = r < 0 ? 0u : 2u;
      if (r == 1) {
        ++fresh_n;
        if (on && ldep[jl]) {  // a new chain: its keys are emitted below
          const uint32_t f = atomicAdd(&nfresh, 1u);
          if (f < FMAX)
            fresh[f] = (uint16_t)jl;
          else
            flags |= F_TRIPLE_OVERFLOW;  // cannot happen: FMAX covers every tile span
        }
      }
    }
    ++dbg_rounds;
    if (!__syncthreads_or(prog || (waiting && round < ((ablate & (1u << 20)) ? 0u : WAIT_ROUNDS)))) break;
  }
  if (ablate & (1u << 21)) {
    atomicAdd(&g_chain_dbg[0], (unsigned long long)dbg_put);
    atomicAdd(&g_chain_dbg[1], (unsigned long long)dbg_r[0]);
    atomicAdd(&g_chain_dbg[2], (unsigned long long)dbg_r[1]);
    atomicAdd(&g_chain_dbg[3], (unsigned long long)dbg_r[2]);
    if (threadIdx.x == 0) {
      atomicAdd(&g_chain_dbg[4], (unsigned long long)dbg_rounds);
      atomicAdd(&g_chain_dbg[5], 1ull);
    }
  }
  // the new chains' keys: (ancestor k, chain, k) work items over the workgroup
  const uint32_t nf = (ablate & (1u << 19)) ? 0 : min(nfresh, FMAX);  // diagnostic knob: no emission
  if (nf) {
    if (threadIdx.x == 0) {
      uint32_t acc = 0;
      for (uint32_t f = 0; f < nf; ++f) {
        foff[f] = acc;
        acc += ldep[fresh[f]];
      }
      foff[nf] = acc;
    }
    __syncthreads();
    const uint32_t total = foff[nf];
    for (uint32_t it = threadIdx.x; it < total; it += CTT) {
      uint32_t lo = 0, hi = nf;  // last f with foff[f] <= it
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (foff[mid] <= it)
          lo = mid;
        else
          hi = mid;
      }
      const uint32_t jl = fresh[lo], k = it - foff[lo] + 1;
      uint32_t a = lcp[jl];
      for (uint32_t t = 1; t < k; ++t) a = lcp[a];
      edge_insert(edge_key(lep[a], lep[jl], k, lkind[a] == KIND_SERVER), trip, tcap, &flags);
    }
  }
  // per tile: rows, relations, max depth; pending spans
  uint32_t rows = 0, rel = 0, maxd = 0;
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const uint32_t i = t0 + q * CTT + threadIdx.x;
    if (i >= t1) continue;
    const uint32_t jl = i - w0;
    const uint8_t kj = lkind[jl];
    uint64_t rp = NONE64;
    if (kj != KIND_CLIENT) {
      const bool pending = lst[jl] != S_DONE;  // S_PUT left over: a starved wait
      if (kj == KIND_SERVER) {
        rp = index_base + i;
        if (!pending) {
          const uint32_t d = ldep[jl];
          ++rows;
          rel += d;
          maxd = max(maxd, d);
        }
      }
      if (pending) {
        const uint32_t x = atomicAdd(&counters[C_PLIST], 1u);
        if (x < pcap) plist[x] = i;
      }
    }
    if (rowpos_out) rowpos_out[i] = rp;
  }
  // non-SERVER ancestors of rows are not rows: their use counts for lastUsage
#pragma unroll
  for (int q = 0; q < CPW; ++q) {
    const uint32_t jl = q * CTT + threadIdx.x;
    if (jl < wn && lanc[jl] && lkind[jl] != KIND_SERVER && lep[jl] < n_ep)
      atomicMax(&ep_ts[lep[jl]], (unsigned long long)((uint64_t)ts[w0 + jl] ^ TS_BIAS));
  }
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
    tile_stats[(uint64_t)tile * 4 + threadIdx.x] = a;
  }
}

// The pending spans (ancestry outside their LDS window), one pass: each hashes
// its own and its parent's ancestry over the global contracted parents, then
// joins or inserts its chain exactly like the tile kernel (no ordering needed).
__global__ void __launch_bounds__(256) k4_chain_pend(const uint32_t *__restrict__ plist, uint32_t pcap,
                                                     const uint8_t *__restrict__ kind,
                                                     const uint32_t *__restrict__ shape,
                                                     const int64_t *__restrict__ ts,
                                                     const uint32_t *__restrict__ cparent,
                                                     const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                     uint32_t n_ep, uint64_t seed,
                                                     unsigned long long *__restrict__ ctab, uint64_t ccap,
                                                     unsigned long long *__restrict__ trip, uint64_t tcap,
                                                     unsigned long long *__restrict__ ep_ts,
                                                     unsigned int *__restrict__ counters,
                                                     unsigned long long *__restrict__ stats64) {
  const uint32_t m = min(counters[C_PLIST], pcap);
  uint32_t flags = 0;
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < m; x += gridDim.x * blockDim.x) {
    const uint32_t i = plist[x];
    const uint8_t ki = kind[i];
    const uint32_t sh = shape[i];
    const uint32_t es = sh < n_shapes ? dep_ep[sh] : NONE;
    const bool on = ki == KIND_SERVER;
    if (es >= n_ep && on) flags |= F_RANGE;
    // Horner hashes of the span's ancestry and of its parent's (suffix) ancestry
    uint64_t acc = sig_elem(es, on, seed), pacc = 0;
    uint32_t d = 0;
    bool bad = false;
    const uint32_t a = cparent[i];
    for (uint32_t cur = a; cur != NONE; cur = cparent[cur]) {
      if (cur == CYC || ++d > MAX_DEPTH) {
        flags |= F_CYCLE;
        bad = true;
        break;
      }
      const uint32_t sa = shape[cur];
      const uint32_t ea = sa < n_shapes ? dep_ep[sa] : NONE;
      const uint64_t el = sig_elem(ea, kind[cur] == KIND_SERVER, seed);
      acc = acc * SIG_M + el;
      pacc = d == 1 ? el : pacc * SIG_M + el;
    }
    if (bad) continue;
    const uint64_t sg = sig_final(acc, d, seed), psig = a == NONE ? ROOT_SIG : sig_final(pacc, d - 1, seed);
    int r = 0;
    for (uint32_t t = 0; t < 1u << 20 && r == 0; ++t) r = chain_put(ctab, ccap, sg, psig, epon_of(es, on), &flags);
    if (r <= 0) continue;
    if (on) {  // a row: its relations, keys (new chain) and non-SERVER ancestors
      uint32_t k = 0;
      for (uint32_t cur = a; cur != NONE; cur = cparent[cur]) {
        ++k;
        const uint8_t ka = kind[cur];
        const uint32_t sa = shape[cur];
        const uint32_t ea = sa < n_shapes ? dep_ep[sa] : NONE;
        if (ea >= n_ep) {
          flags |= F_RANGE;
          break;
        }
        if (r == 1) edge_insert(edge_key(ea, es, k, ka == KIND_SERVER), trip, tcap, &flags);
        if (ka != KIND_SERVER) atomicMax(&ep_ts[ea], (unsigned long long)((uint64_t)ts[cur] ^ TS_BIAS));
      }
      atomicAdd(&stats64[S_ROWS], 1ull);
      atomicAdd(&stats64[S_REL], (unsigned long long)d);
      atomicMax(&stats64[S_MAXD], (unsigned long long)d);
    }
    if (r == 1) atomicAdd(&stats64[S_CHAINS], 1ull);
  }
  if (flags) atomicOr(&counters[C_FLAGS], flags);
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

void launch_chain(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                  const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                  uint64_t index_base, uint64_t seed, void *ctab, uint64_t ccap, unsigned long long *trip,
                  uint64_t tcap, unsigned long long *ep_ts, unsigned long long *rowpos, uint32_t *plist,
                  uint32_t pcap, unsigned int *counters, uint32_t *tile_stats, unsigned long long *stats64,
                  uint32_t ablate) {
  const uint32_t nt = chain_tiles(n);
  if (!nt) return;
  hipLaunchKernelGGL(k4_chain, dim3(nt), dim3(CTT), 0, s, kind, shape, ts, cparent, n, dep_ep, n_shapes, n_ep,
                     index_base, seed, reinterpret_cast<unsigned long long *>(ctab), ccap, trip, tcap, ep_ts, rowpos,
                     plist, pcap, counters, tile_stats, ablate);
  launch_tile_sum(s, tile_stats, nt, 4u, 4u, stats64 + S_ROWS, 2u);  // rows, rel, maxd, chains
}

void launch_chain_pend(hipStream_t s, const uint32_t *plist, uint32_t pcap, const uint8_t *kind,
                       const uint32_t *shape, const int64_t *ts, const uint32_t *cparent, const uint32_t *dep_ep,
                       uint32_t n_shapes, uint32_t n_ep, uint64_t seed, void *ctab, uint64_t ccap,
                       unsigned long long *trip, uint64_t tcap, unsigned long long *ep_ts, unsigned int *counters,
                       unsigned long long *stats64) {
  hipLaunchKernelGGL(k4_chain_pend, dim3(1024), dim3(256), 0, s, plist, pcap, kind, shape, ts, cparent, dep_ep,
                     n_shapes, n_ep, seed, reinterpret_cast<unsigned long long *>(ctab), ccap, trip, tcap, ep_ts,
                     counters, stats64);
}

}  // namespace kmz
