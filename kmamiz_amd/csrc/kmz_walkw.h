// kmz_walkw.h -- the chain walk of chain interning over one LDS window: the
// rounds that hash, probe and settle a tile's non-CLIENT spans, shared by the
// fused join + walk (k_join_chain, kmz_fuse.hip) and the per-tile walk
// (k4_tile, kmz_walk.hip).  See kmz_chain.hip for the chain table and its
// exactness argument; the reference walk is Traces.ts:138-208.
//
// Input: the window as LDS records (Rec16 / Rec8 below: element hash or
// endpoint, window-local contracted parent | kind << 16; W_NONE root, W_OUT
// outside the window, W_CYC a CLIENT loop) and the tile's non-CLIENT spans compacted into
// `wlist` (tile-local indices).  Per round every thread takes TW of them:
//   walk     a Horner fold over the LDS element hashes of the ancestors (the
//            depth is the step count; the loop runs while any lane walks);
//   probe    one read of the chain table at the sig's home slot;
//   check    a found chain's parent sig against the walk's; a chain not found
//            elects one leader per distinct sig in the workgroup (LDS map);
//   leaders  claim the probed slot (one CAS, published at once), stage the
//            row's keys, and record the claimed slot or a deferred check in the
//            global lists, reserved by one device atomic per list and
//            workgroup (k_chain_settle_list settles them);
//   rows     counts, the pending list (ancestries leaving the window), rowpos.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kmz_chainw.h"

namespace kmz {

// the tables and global lists of one chain-interning run
struct ChainRun {
  const int64_t *ts;
  unsigned long long *ctab;
  uint64_t ccap;
  unsigned long long *trip;
  uint64_t tcap;
  unsigned long long *ep_ts;
  unsigned long long *rowpos_out;  // (null unless the run keeps span links)
  uint32_t *plist;
  uint32_t pcap;
  unsigned int *counters;
  unsigned long long *stage;  // staged keys (C_FSTAGE)
  uint32_t scap;
  unsigned long long *defer;  // deferred chain checks (C_FDEFER)
  uint32_t dcap;
  uint32_t *gpos;  // claimed chain-table slots (C_WPOS)
  uint32_t gcap;
  uint32_t n_ep;
  uint64_t index_base, seed;
  uint32_t ablate;
  // the records' element ids are shapes (k4_tile8 on a dependency table that
  // maps every shape into range): id_ep maps one to its endpoint where a key
  // or an endpoint update needs it; null: the ids are endpoints
  const uint32_t *id_ep = nullptr;
  uint32_t n_ids = 0;  // (shape ids: n_shapes; an id past it is NONE)
};

// an edge key over shape ids -> the same key over their dependency endpoints
// (an id past n_ids -- NONE's 24 bits -- stays as it is, as NONE did)
__device__ __forceinline__ uint64_t key_ids_to_eps(uint64_t key, const uint32_t *__restrict__ id_ep, uint32_t n_ids) {
  const uint32_t ia = (uint32_t)(key >> 40), id = (uint32_t)(key >> 16) & 0xFFFFFFu;
  const uint64_t ea = ia < n_ids ? id_ep[ia] : ia, ed = id < n_ids ? id_ep[id] : id;
  return (ea << 40) | (ed << 16) | (key & 0xFFFFull);
}

// a record id's dependency endpoint (NONE stays NONE)
__device__ __forceinline__ uint32_t run_ep(const ChainRun &a, uint32_t id) {
  return (a.id_ep && id != NONE) ? a.id_ep[id] : id;
}

// per-round LDS of the walk: the leader map (M entries, a power of two) and
// the list reservations
template <uint32_t M>
struct ChainLdsT {
  static constexpr uint32_t MAP = M;
  unsigned long long imap_sig[M], imap_psig[M];
  uint32_t l_need[3], l_base[3];  // a round's reservations in the global lists (stage, claimed, deferred)
};
using ChainLds = ChainLdsT<IMAP>;

template <uint32_t M>
__device__ __forceinline__ void chain_lds_init(ChainLdsT<M> &L) {
  for (uint32_t x = threadIdx.x; x < M; x += blockDim.x) L.imap_sig[x] = 0;
  if (threadIdx.x < 3) L.l_need[threadIdx.x] = 0;
}

// Window records.  Rec16 (the fused join + walk): {element lo, element hi,
// endpoint, window parent | kind << 16}.  Rec8 (k4_tile, round 5): {epk
// (kind << 30 | endpoint), window parent | kind << 16}; the element is
// computed per step from the endpoint (sig_elem: one multiply), so the record
// is half the LDS and one ds_read_b64.  Both give the same elements.
struct Rec16 {
  using T = uint4;
  static __device__ __forceinline__ uint32_t kind(const T &r) { return (r.w >> 16) & 3; }
  static __device__ __forceinline__ uint32_t ep(const T &r) { return r.z; }
  static __device__ __forceinline__ uint32_t parent(const T &r) { return r.w & 0xFFFF; }
  static __device__ __forceinline__ uint64_t elem(const T &r, uint64_t) { return (uint64_t)r.y << 32 | r.x; }
};
struct Rec8 {  // (the id: a shape, or an endpoint)
  using T = uint2;
  static __device__ __forceinline__ uint32_t kind(const T &r) { return (r.y >> 16) & 3; }
  static __device__ __forceinline__ uint32_t ep(const T &r) { return epk_ep(r.x); }
  static __device__ __forceinline__ uint32_t parent(const T &r) { return r.y & 0xFFFF; }
  static __device__ __forceinline__ uint64_t elem(const T &r, uint64_t seed) {
    return sig_elem(r.x & EPK_NONE, ((r.y >> 16) & 3) == KIND_SERVER, seed);
  }
};

// a window slot as the leaders' key staging reads it: its id (endpoint or
// shape; NONE for none), kind and window parent
struct AncRec {
  uint32_t ep, kind, parent;
};

// The probe, check, leaders and row counts of one round, after the walk
// (shared by the walk kernels).  Per walker slot q: st (S_PUT: probe the chain
// sg with parent sig ps; S_PEND: its ancestry leaves the window; S_DONE:
// nothing to probe), kq (KIND_CLIENT: an empty walker slot), the depth dd, the
// window slot jq and the id myep; anc(x) gives window slot x's AncRec.
template <int NT, int TW, class Anc, uint32_t M>
__device__ __forceinline__ void chain_round_tail(uint64_t (&sg)[TW], const uint64_t (&ps)[TW], uint8_t (&st)[TW],
                                                 const uint8_t (&kq)[TW], const uint32_t (&dd)[TW],
                                                 const uint32_t (&jq)[TW], const uint32_t (&myep)[TW], uint32_t w0,
                                                 Anc anc, ChainLdsT<M> &L, const ChainRun &a, uint32_t &rows,
                                                 uint32_t &rel, uint32_t &maxd, uint32_t &fresh_n, uint32_t &flags) {
  const uint32_t spin = spin_bound(a.ablate);
  ulonglong2 w01[TW];  // (sig, parent sig) of the probed slot
  uint64_t pos[TW];
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    const bool pr = st[q] == S_PUT;
    pos[q] = pr ? cslot(sg[q], a.ccap) : 0;
    w01[q] = pr ? *reinterpret_cast<const ulonglong2 *>(a.ctab + 2 * pos[q]) : make_ulonglong2(0, 0);
  }
  // check what the probes found; one leader per distinct unknown sig
  uint32_t hslot[TW];
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    hslot[q] = M + 1;  // not an insert
    if (st[q] != S_PUT) continue;
    for (uint32_t z = 0; w01[q].x != sg[q] && w01[q].x != 0 && z < PROBE_MAX; ++z) {  // another chain's slot
      pos[q] = pos[q] + 1 == a.ccap ? 0 : pos[q] + 1;
      w01[q] = *reinterpret_cast<const ulonglong2 *>(a.ctab + 2 * pos[q]);
    }
    st[q] = S_DONE;
    if (w01[q].x == sg[q] && w01[q].y != 0) {
      if (w01[q].y != ps[q]) flags |= F_SIG;
      continue;
    }
    uint32_t h = (uint32_t)(sig_place(sg[q]) >> 32) & (M - 1);
    hslot[q] = M;  // a leader without a map slot (map full)
    for (uint32_t t = 0; t < 8; ++t) {
      const unsigned long long kk = atomicCAS(&L.imap_sig[h], 0ull, (unsigned long long)sg[q]);
      if (kk == 0) {
        L.imap_psig[h] = ps[q];
        hslot[q] = h;
        break;
      }
      if (kk == sg[q]) {
        hslot[q] = h | 0x80000000u;
        break;
      }
      h = (h + 1) & (M - 1);
    }
  }
  if (a.ablate & (1u << 18))  // diagnostic knob: probe but no inserts
#pragma unroll
    for (int q = 0; q < TW; ++q) hslot[q] = M + 1;
  __syncthreads();
  // followers compare with their leader; leaders claim the probed slot (one
  // CAS) and publish at once (a lane that waits on another workgroup's
  // unpublished entry must never hold back, in its own wave, a publish that
  // workgroup may wait on).  Their list entries are reserved in LDS, then in
  // the global lists with one atomic per list and workgroup.
  unsigned long long cvq[TW];
  uint32_t os[TW], ol[TW];
  bool lead[TW];
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    lead[q] = false;
    os[q] = ol[q] = 0;
    cvq[q] = 0;
    if (hslot[q] > M) {
      if (hslot[q] != M + 1) {
        const uint32_t h = hslot[q] & (M - 1);
        if (L.imap_psig[h] != ps[q]) flags |= F_SIG;
      }
      continue;
    }
    lead[q] = true;
    unsigned long long *en = a.ctab + 2 * pos[q];
    cvq[q] = atomicCAS(&en[0], 0ull, (unsigned long long)sg[q]);
    if (cvq[q] == 0) atomicExch(&en[1], (unsigned long long)ps[q]);
  }
  __builtin_amdgcn_wave_barrier();
  bool anyl = false;
#pragma unroll
  for (int q = 0; q < TW; ++q) {
    if (!lead[q]) continue;
    anyl = true;
    // a row whose chain this leader inserted (or lost to another chain: the
    // deferred check may insert it) stages its keys; one that joined the
    // same chain leaves them to the winner (knob 19: diagnostic, none)
    if (kq[q] == KIND_SERVER && dd[q] && cvq[q] != sg[q] && !(a.ablate & (1u << 19)))
      os[q] = atomicAdd(&L.l_need[0], dd[q]) + 1;
    ol[q] = atomicAdd(&L.l_need[cvq[q] == 0 ? 1 : 2], 1u);
  }
  if (__syncthreads_or(anyl)) {
    if (threadIdx.x < 3) {
      const uint32_t need = L.l_need[threadIdx.x];
      L.l_base[threadIdx.x] =
          need ? atomicAdd(&a.counters[threadIdx.x == 0 ? C_FSTAGE : (threadIdx.x == 1 ? C_WPOS : C_FDEFER)], need)
               : 0;
      L.l_need[threadIdx.x] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      if (!lead[q]) continue;
      const uint32_t d = dd[q];
      if (os[q]) {  // the row's keys (ancestor k, row endpoint, k, ancestor is SERVER)
        const uint64_t base = (uint64_t)L.l_base[0] + os[q] - 1;
        // (shape ids: the keys are staged over shapes and mapped to
        // endpoints by k_chain_settle_list -- no gather in the walk)
        uint32_t an = anc(jq[q]).parent;
        for (uint32_t kk = 1; kk <= d; ++kk) {
          const AncRec r = anc(an);
          const uint64_t key = edge_key(r.ep, myep[q], kk, r.kind == KIND_SERVER);
          if (base + kk - 1 < a.scap) {
            a.stage[base + kk - 1] = key;
          } else {
            edge_insert(a.id_ep ? key_ids_to_eps(key, a.id_ep, a.n_ids) : key, a.trip, a.tcap, &flags);
            flags |= F_STAGE_FULL;
          }
          an = r.parent;
        }
      }
      if (cvq[q] == 0) {  // won the slot (published above)
        ++fresh_n;
        const uint64_t x = (uint64_t)L.l_base[1] + ol[q];
        if (x < a.gcap)
          a.gpos[x] = (uint32_t)pos[q];
        else
          flags |= F_CTAB_DIRTY;
      } else {  // joined an unpublished entry, or lost the slot to another chain
        const uint64_t x = (uint64_t)L.l_base[2] + ol[q];
        if (x < a.dcap) {
          *reinterpret_cast<ulonglong2 *>(a.defer + 2 * x) = make_ulonglong2(sg[q], ps[q]);
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
}

// All rounds of one tile.  W: window slots (an index >= W is not a window
// slot); NT: threads of the workgroup; TW: walkers per thread and round; R:
// the record layout.  The caller has published lrec / wlist / m with a
// barrier; this returns after a barrier (the window may be rewritten).
template <uint32_t W, int NT, int TW, class R = Rec16>
__device__ __forceinline__ void chain_walk_rounds(const typename R::T *__restrict__ lrec,
                                                  const uint16_t *__restrict__ wlist, uint32_t m, uint32_t w0,
                                                  uint32_t toff, bool any_other, ChainLds &L, const ChainRun a,
                                                  uint32_t &rows, uint32_t &rel, uint32_t &maxd, uint32_t &fresh_n,
                                                  uint32_t &flags) {
  using RT = typename R::T;
  const bool hash_on = !(a.ablate & (1u << 16));  // diagnostic knob: no hashing / probing / inserting
  for (uint32_t r0 = 0; r0 < m; r0 += TW * NT) {
    uint64_t sg[TW], ps[TW], acc[TW];
    uint32_t dd[TW], wa[TW], myep[TW], jq[TW];
    uint8_t st[TW], kq[TW];
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      const uint32_t idx = r0 + q * NT + threadIdx.x;
      const bool on = idx < m;
      const uint32_t jl = on ? toff + wlist[idx] : W - 1;
      jq[q] = jl;
      const RT r = lrec[jl];
      kq[q] = R::kind(r);
      myep[q] = R::ep(r);
      sg[q] = R::elem(r, a.seed);  // the element hash until the walk is done
      acc[q] = 0;
      dd[q] = 0;
      wa[q] = W_NONE;
      st[q] = S_NONE;
      if (!on) {
        kq[q] = KIND_CLIENT;  // (no walker in this slot)
        continue;
      }
      st[q] = S_DONE;
      if (!hash_on) continue;
      // (ids that are shapes are in range whenever they are not NONE)
      if (kq[q] == KIND_SERVER && (a.id_ep ? myep[q] == NONE : myep[q] >= a.n_ep)) flags |= F_RANGE;
      wa[q] = R::parent(r);
    }
    // the TW walks of a thread step together: TW independent LDS reads in
    // flight per step, then branch-free updates (compiled without the
    // non-SERVER-ancestor branch when the window has no such span)
    auto walk = [&](auto other_tag) {
      constexpr bool OTHER = decltype(other_tag)::value;
      for (uint32_t it = 0; it < WIN_DEPTH; ++it) {
        bool go = false;
#pragma unroll
        for (int q = 0; q < TW; ++q) go |= wa[q] < W;
        if (__ballot(go) == 0) break;
        RT r[TW];
#pragma unroll
        for (int q = 0; q < TW; ++q) r[q] = lrec[wa[q] < W ? wa[q] : 0];
#pragma unroll
        for (int q = 0; q < TW; ++q) {
          const bool act = wa[q] < W;
          const uint64_t nacc = sig_step(acc[q], R::elem(r[q], a.seed));
          if (OTHER && act && kq[q] == KIND_SERVER && R::kind(r[q]) != KIND_SERVER) {
            // (rare) a non-SERVER ancestor of a row: its lastUsage
            const uint32_t e = run_ep(a, R::ep(r[q]));
            if (e < a.n_ep)
              atomicMax(&a.ep_ts[e], (unsigned long long)((uint64_t)a.ts[w0 + wa[q]] ^ TS_BIAS));
            else
              flags |= F_RANGE;
          }
          acc[q] = act ? nacc : acc[q];
          dd[q] = act ? it + 1 : dd[q];
          wa[q] = act ? R::parent(r[q]) : wa[q];
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
      if (wa[q] != W_NONE) {  // W_OUT: leaves the window (or deeper than WIN_DEPTH); W_CYC: CLIENT loop
        if (wa[q] == W_CYC) flags |= F_CYCLE;
        st[q] = S_PEND;
        sg[q] = 0;
        continue;
      }
      const uint32_t d = dd[q];
      ps[q] = d ? sig_final(acc[q], d - 1, a.seed, &flags) : ROOT_SIG;
      sg[q] = sig_final(rotl64(sg[q], SIG_R * d) ^ acc[q], d, a.seed, &flags);
      if (a.ablate & (1u << 24)) {  // test knob: 4-bit sigs, i.e. collisions (F_SIG, then a retry with another seed)
        sg[q] = (sg[q] & 0xF) + 2;
        ps[q] = d ? (ps[q] & 0xF) + 2 : ROOT_SIG;
      }
      if (!(a.ablate & (1u << 17))) st[q] = S_PUT;  // diagnostic knob: hash only
    }
    chain_round_tail<NT, TW>(sg, ps, st, kq, dd, jq, myep, w0, [&](uint32_t x) {
      const RT r = lrec[x];
      return AncRec{R::ep(r), R::kind(r), R::parent(r)};
    }, L, a, rows, rel, maxd, fresh_n, flags);
    __syncthreads();  // (wlist / imap reads of this round before the next round's leaders)
  }
}

// the workgroup's row counts (rows, relations, max depth, new chains) -> tile_stats[tile * 4 ..]
template <int NT>
__device__ __forceinline__ void chain_tile_stats(uint32_t rows, uint32_t rel, uint32_t maxd, uint32_t fresh_n,
                                                 uint32_t (*red)[4], uint32_t *__restrict__ tile_stats) {
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
    uint32_t s = 0;
    for (int w = 0; w < NT / 64; ++w) s = threadIdx.x == 2 ? max(s, red[w][2]) : s + red[w][threadIdx.x];
    tile_stats[(uint64_t)blockIdx.x * 4 + threadIdx.x] = s;
  }
}

}  // namespace kmz
