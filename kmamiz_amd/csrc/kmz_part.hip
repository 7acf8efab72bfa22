// kmz_part.hip -- partitioned (atomic-free) variants of K3 and K4 for large
// key spaces (the 20k-endpoint mesh and up).
//
// K3P  (endpoint x status) reduction when G > 1024 groups:
//   produce: each 2048-span tile bins its SERVER records by group partition
//            (1024 groups each) in LDS and writes them contiguously into its
//            own tile region + a dense [partition][tile] directory word;
//   reduce:  slice workgroups of one partition accumulate the records in LDS
//            (direct-indexed, 48 B per group) and write dense slice partials;
//   combine: sum / max / min over slices -> the 6 x G u64 group partials.
//   No global atomics, bit-deterministic.
//
// K4T  ancestor traversal over LDS windows:
//   a 2048-span tile loads the cparent / kind / endpoint of its window (tile
//   +-512 spans) into LDS, so the per-row ancestor chains run in LDS instead
//   of as dependent global loads (a chain leaving the window continues with
//   global loads).  Edge keys are partitioned by DESCENDANT endpoint range:
//   pass 0 counts keys per (partition, tile), an exclusive scan places them,
//   pass 1 writes them, and one workgroup per partition deduplicates its keys
//   in an LDS hash set (all keys of a descendant endpoint land in one
//   partition, so the LDS set is exact).
#include <hip/hip_runtime.h>

#include "kmz_kernels.h"

namespace kmz {

// ---------------------------------------------------------------------------
// block-wide exclusive scan of cnt[0..P) into off[0..P) (P <= 2 * blockDim)
// ---------------------------------------------------------------------------
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan_pairs(const uint32_t *cnt, uint32_t *off, uint32_t P,
                                                          uint32_t *wave_tot) {
  const uint32_t t = threadIdx.x;
  uint32_t a = 2 * t < P ? cnt[2 * t] : 0;
  uint32_t b = 2 * t + 1 < P ? cnt[2 * t + 1] : 0;
  uint32_t s = a + b;
  uint32_t lane = t & 63, wv = t >> 6;
  uint32_t x = s;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wave_tot[wv] = x;
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < THREADS / 64; ++w) {
      uint32_t v = wave_tot[w];
      wave_tot[w] = acc;
      acc += v;
    }
    wave_tot[THREADS / 64] = acc;
  }
  __syncthreads();
  uint32_t excl = wave_tot[wv] + x - s;
  if (2 * t < P) off[2 * t] = excl;
  if (2 * t + 1 < P) off[2 * t + 1] = excl + a;
  return wave_tot[THREADS / 64];  // total
}

// ===========================================================================
// K3P
// ===========================================================================
struct __align__(8) Rec {
  uint64_t tsx;  // timestamp ^ 2^63
  uint32_t i;    // local span index
  uint32_t d;    // duration (us)
  uint32_t kl;   // group within the partition
  uint32_t pad;
};

constexpr uint32_t K3T = 2048;     // spans per tile
constexpr uint32_t K3R = 1024;     // groups per partition
constexpr uint32_t K3PMAX = 1024;  // partitions (G <= 1M)
constexpr int K3PT = 512;          // producer threads

__global__ void __launch_bounds__(K3PT) k3_produce(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                   const uint16_t *__restrict__ status, const uint32_t *__restrict__ dur,
                                                   const int64_t *__restrict__ ts, uint32_t n,
                                                   const uint32_t *__restrict__ ep_of_shape, uint32_t n_shapes,
                                                   uint32_t n_ep, uint32_t n_status, uint32_t P, uint32_t ntiles,
                                                   Rec *__restrict__ pool, uint32_t *__restrict__ dir,
                                                   unsigned int *__restrict__ counters,
                                                   uint32_t *__restrict__ tile_servers) {
  __shared__ uint32_t cnt[K3PMAX], off[K3PMAX];
  __shared__ uint32_t wave_tot[K3PT / 64 + 1];
  __shared__ Rec stage[K3T];
  const uint32_t tile = blockIdx.x, t0 = tile * K3T;
  for (uint32_t p = threadIdx.x; p < P; p += K3PT) cnt[p] = 0;
  __syncthreads();
  constexpr int PER = K3T / K3PT;
  uint32_t pp[PER], rr[PER];
  Rec rec[PER];
  uint32_t servers = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    uint32_t i = t0 + k * K3PT + threadIdx.x;
    pp[k] = NONE;
    if (i < n && kind[i] == KIND_SERVER) {
      ++servers;
      uint32_t sh = shape[i], st = status[i];
      uint32_t ep = sh < n_shapes ? ep_of_shape[sh] : NONE;
      if (ep >= n_ep || st >= n_status) {
        atomicOr(&counters[C_FLAGS], F_RANGE);
        continue;
      }
      uint32_t g = ep * n_status + st;
      pp[k] = g / K3R;
      rec[k].kl = g % K3R;
      rec[k].d = dur[i];
      rec[k].i = i;
      rec[k].tsx = (uint64_t)ts[i] ^ TS_BIAS;
      rec[k].pad = 0;
      rr[k] = atomicAdd(&cnt[pp[k]], 1u);
    }
  }
  __syncthreads();
  uint32_t total = block_excl_scan_pairs<K3PT>(cnt, off, P, wave_tot);
  for (uint32_t p = threadIdx.x; p < P; p += K3PT) dir[(uint64_t)p * ntiles + tile] = (off[p] << 16) | cnt[p];
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (pp[k] != NONE) stage[off[pp[k]] + rr[k]] = rec[k];
  __syncthreads();
  // coalesced copy of the partition-sorted tile into its region
  const uint64_t *src = reinterpret_cast<const uint64_t *>(stage);
  uint64_t *dst = reinterpret_cast<uint64_t *>(pool + (uint64_t)tile * K3T);
  for (uint32_t w = threadIdx.x; w < total * 3; w += K3PT) dst[w] = src[w];
  // realtime-row count: per tile, summed later (no same-address atomics)
  for (int o = 32; o > 0; o >>= 1) servers += __shfl_xor(servers, o, 64);
  if ((threadIdx.x & 63) == 0) wave_tot[threadIdx.x >> 6] = servers;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < K3PT / 64; ++w) t += wave_tot[w];
    tile_servers[tile] = t;
  }
}

// sum of per-tile counters by ONE workgroup (replaces ~1e5 same-address atomics)
__global__ void __launch_bounds__(1024) k_tile_sum(const uint32_t *__restrict__ v, uint32_t ntiles, uint32_t stride,
                                                   uint32_t fields, unsigned long long *__restrict__ out,
                                                   uint32_t max_field) {
  __shared__ unsigned long long red[16][4];
  unsigned long long acc[4] = {0, 0, 0, 0};
  for (uint32_t t = threadIdx.x; t < ntiles; t += 1024)
    for (uint32_t f = 0; f < fields; ++f) {
      uint64_t x = v[(uint64_t)t * stride + f];
      acc[f] = (f == max_field) ? max(acc[f], (unsigned long long)x) : acc[f] + x;
    }
  for (uint32_t f = 0; f < fields; ++f)
    for (int o = 32; o > 0; o >>= 1) {
      unsigned long long y = __shfl_xor(acc[f], o, 64);
      acc[f] = (f == max_field) ? max(acc[f], y) : acc[f] + y;
    }
  if ((threadIdx.x & 63) == 0)
    for (uint32_t f = 0; f < fields; ++f) red[threadIdx.x >> 6][f] = acc[f];
  __syncthreads();
  if (threadIdx.x < fields) {
    unsigned long long r = 0;
    for (int w = 0; w < 16; ++w) r = (threadIdx.x == max_field) ? max(r, red[w][threadIdx.x]) : r + red[w][threadIdx.x];
    if (threadIdx.x == max_field)
      atomicMax(&out[threadIdx.x], r);
    else
      atomicAdd(&out[threadIdx.x], r);
  }
}

// slice s of partition p: tiles s, s+S, ...  -> part[(s*6 + f) * G + g]
__global__ void __launch_bounds__(256) k3_reduce(const Rec *__restrict__ pool, const uint32_t *__restrict__ dir,
                                                 uint32_t ntiles, uint32_t S, uint32_t G, uint64_t index_base,
                                                 unsigned long long *__restrict__ part) {
  __shared__ unsigned long long a_cnt[K3R], a_s1[K3R], a_s2a[K3R], a_s2b[K3R], a_tsx[K3R], a_fst[K3R];
  const uint32_t s = blockIdx.x, p = blockIdx.y;
  for (uint32_t k = threadIdx.x; k < K3R; k += blockDim.x) {
    a_cnt[k] = a_s1[k] = a_s2a[k] = a_s2b[k] = a_tsx[k] = 0;
    a_fst[k] = ~0ull;
  }
  __syncthreads();
  const uint32_t *row = dir + (uint64_t)p * ntiles;
  for (uint64_t k = (uint64_t)s + (uint64_t)threadIdx.x * S; k < ntiles; k += (uint64_t)blockDim.x * S) {
    uint32_t w = row[k];
    uint32_t off = w >> 16, c = w & 0xFFFF;
    const Rec *r = pool + k * K3T + off;
    for (uint32_t q = 0; q < c; ++q) {
      Rec x = r[q];
      uint64_t d = x.d, dd = d * d;
      atomicAdd(&a_cnt[x.kl], 1ull);
      atomicAdd(&a_s1[x.kl], (unsigned long long)d);
      atomicAdd(&a_s2a[x.kl], (unsigned long long)(dd & 0xFFFFFFFFull));
      atomicAdd(&a_s2b[x.kl], (unsigned long long)(dd >> 32));
      atomicMax(&a_tsx[x.kl], (unsigned long long)x.tsx);
      atomicMin(&a_fst[x.kl], (unsigned long long)(index_base + x.i));
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < K3R; k += blockDim.x) {
    uint64_t g = (uint64_t)p * K3R + k;
    if (g >= G) break;
    unsigned long long *b = part + (uint64_t)s * 6 * G + g;
    b[0] = a_cnt[k];
    b[G] = a_s1[k];
    b[2ull * G] = a_s2a[k];
    b[3ull * G] = a_s2b[k];
    b[4ull * G] = a_tsx[k];
    b[5ull * G] = a_fst[k];
  }
}

__global__ void __launch_bounds__(256) k3_combine(const unsigned long long *__restrict__ part, uint32_t S, uint32_t G,
                                                  unsigned long long *__restrict__ grp) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    unsigned long long c = 0, s1 = 0, s2a = 0, s2b = 0, tsx = 0, fst = ~0ull;
    for (uint32_t s = 0; s < S; ++s) {
      const unsigned long long *b = part + (uint64_t)s * 6 * G + g;
      c += b[0];
      s1 += b[G];
      s2a += b[2ull * G];
      s2b += b[3ull * G];
      tsx = max(tsx, b[4ull * G]);
      fst = min(fst, b[5ull * G]);
    }
    grp[g] = c;
    grp[G + g] = s1;
    grp[2ull * G + g] = s2a;
    grp[3ull * G + g] = s2b;
    grp[4ull * G + g] = tsx;
    grp[5ull * G + g] = fst;
  }
}

void launch_k3_partitioned(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                           const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                           uint32_t n_shapes, uint32_t n_ep, uint32_t n_status, uint64_t index_base,
                           unsigned long long *grp, unsigned int *counters, unsigned long long *n_server, void *pool,
                           uint32_t *dir, unsigned long long *part, uint32_t S, uint32_t *tile_tmp) {
  if (!n || !n_ep) return;
  uint32_t G = n_ep * n_status;
  uint32_t P = (G + K3R - 1) / K3R;
  uint32_t ntiles = (n + K3T - 1) / K3T;
  hipLaunchKernelGGL(k3_produce, dim3(ntiles), dim3(K3PT), 0, s, kind, shape, status, dur, ts, n, ep_of_shape,
                     n_shapes, n_ep, n_status, P, ntiles, (Rec *)pool, dir, counters, tile_tmp);
  hipLaunchKernelGGL(k_tile_sum, dim3(1), dim3(1024), 0, s, tile_tmp, ntiles, 1u, 1u, n_server, 99u);
  hipLaunchKernelGGL(k3_reduce, dim3(S, P), dim3(256), 0, s, (const Rec *)pool, dir, ntiles, S, G, index_base, part);
  hipLaunchKernelGGL(k3_combine, dim3((G + 255) / 256 < 2048 ? (G + 255) / 256 : 2048), dim3(256), 0, s, part, S, G,
                     grp);
}

uint32_t k3_partitions(uint32_t G) { return (G + K3R - 1) / K3R; }
uint32_t k3_pmax() { return K3PMAX; }
uint64_t k3_pool_bytes(uint32_t n) { return (uint64_t)((n + K3T - 1) / K3T) * K3T * sizeof(Rec); }
uint32_t k3_tiles(uint32_t n) { return (n + K3T - 1) / K3T; }

// ===========================================================================
// K4T -- two passes over 2048-span tiles with their +-512-span LDS window:
//   count: walk every row in LDS, count keys / endpoint records per edge
//          partition -> dense [partition][tile] counts (+ per-tile stats);
//   (exclusive scans place every (partition, tile) run contiguously)
//   emit:  walk again, write keys / endpoint records at their final place;
//   dedup: one workgroup per partition streams its contiguous keys into an
//          LDS hash set and reduces the endpoint records it owns.
// Partitions are hashed by DESCENDANT endpoint, so a key and its endpoint's
// records always meet in one workgroup: the LDS set is exact, no global
// atomics anywhere.
// ===========================================================================
constexpr uint32_t K4T = 2048, K4H = 512, K4W = K4T + 2 * K4H;
constexpr uint16_t L_NONE = 0xFFFF, L_CYC = 0xFFFE, L_OUT = 0xFFFD;
constexpr uint32_t K4PMAX = 1024;  // edge partitions
constexpr int K4TT = 512;          // walk threads
constexpr int K4PER = K4T / K4TT;  // own spans per thread
constexpr uint32_t K4SET = 8192;   // reducer LDS set slots (64 KiB)
constexpr uint64_t FKEY_MASK = (1ull << 40) - 1;  // first_row<<1|!external, 40 bits
constexpr uint32_t K4EMAP = 1024;  // endpoints per edge partition (LDS map slots)

struct Window {
  const uint16_t *lcp;
  const uint8_t *lkind;
  const uint32_t *lep;
  uint32_t w0, w1;
  const uint32_t *cparent;
  const uint8_t *kind;
  const uint32_t *shape;
  const uint32_t *dep_ep;
  uint32_t n_shapes;
  __device__ __forceinline__ bool in(uint32_t g) const { return g >= w0 && g < w1; }
  __device__ __forceinline__ uint32_t next(uint32_t g) const {
    if (in(g)) {
      // no switch here: hipcc (ROCm 7.2) lowers a switch over these u16
      // markers with a wrong signed range split that sends L_OUT to CYC
      const uint32_t c = lcp[g - w0];
      if (c < K4W) return w0 + c;
      if (c != L_OUT) return 0xFFFF0000u | c;  // L_NONE -> NONE, L_CYC -> CYC
    }
    return cparent[g];
  }
  __device__ __forceinline__ uint8_t kind_of(uint32_t g) const { return in(g) ? lkind[g - w0] : kind[g]; }
  __device__ __forceinline__ uint32_t ep_of(uint32_t g) const {
    if (in(g)) return lep[g - w0];
    uint32_t sh = shape[g];
    return sh < n_shapes ? dep_ep[sh] : NONE;
  }
};

// partition of a descendant endpoint (hashed: deep endpoints with many
// ancestors spread evenly)
__device__ __forceinline__ uint32_t edge_part(uint32_t es, uint32_t P) {
  return (uint32_t)(((uint64_t)(uint32_t)(mix64(es + 0x632BE59BD9B4E019ull) >> 32) * P) >> 32);
}

// window -> LDS with every global load of a thread issued before any is used
__device__ __forceinline__ void load_window(uint32_t w0, uint32_t w1, const uint32_t *__restrict__ cparent,
                                            const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                            const uint32_t *__restrict__ dep_ep, uint32_t n_shapes, uint16_t *lcp,
                                            uint8_t *lkind, uint32_t *lep) {
  constexpr int PERW = (K4W + K4TT - 1) / K4TT;
  uint32_t c[PERW], sh[PERW];
  uint8_t k[PERW];
#pragma unroll
  for (int q = 0; q < PERW; ++q) {
    uint32_t j = w0 + q * K4TT + threadIdx.x;
    bool ok = j < w1;
    c[q] = ok ? cparent[j] : NONE;
    k[q] = ok ? kind[j] : 0;
    sh[q] = ok ? shape[j] : NONE;
  }
  uint32_t e[PERW];
#pragma unroll
  for (int q = 0; q < PERW; ++q) e[q] = (k[q] != KIND_CLIENT && sh[q] < n_shapes) ? dep_ep[sh[q]] : NONE;
#pragma unroll
  for (int q = 0; q < PERW; ++q) {
    uint32_t j = w0 + q * K4TT + threadIdx.x;
    if (j < w1) {
      lkind[j - w0] = k[q];
      lep[j - w0] = e[q];
      lcp[j - w0] =
          c[q] == NONE ? L_NONE : (c[q] == CYC ? L_CYC : ((c[q] >= w0 && c[q] < w1) ? (uint16_t)(c[q] - w0) : L_OUT));
    }
  }
}

__device__ unsigned long long g_k4dbg[64];

template <bool EMIT>
__global__ void __launch_bounds__(K4TT) k4_walk(const uint8_t *__restrict__ kind, const uint32_t *__restrict__ shape,
                                                const int64_t *__restrict__ ts, const uint32_t *__restrict__ cparent,
                                                uint32_t n, const uint32_t *__restrict__ dep_ep, uint32_t n_shapes,
                                                uint32_t n_ep, uint64_t index_base, uint32_t P,
                                                uint32_t *__restrict__ kdir, uint32_t *__restrict__ rdir,
                                                const uint32_t *__restrict__ koff, const uint32_t *__restrict__ roff,
                                                unsigned long long *__restrict__ kpool,
                                                unsigned long long *__restrict__ rpool,
                                                unsigned long long *__restrict__ rowpos_out,
                                                unsigned int *__restrict__ counters,
                                                uint32_t *__restrict__ tile_stats) {
  __shared__ uint16_t lcp[K4W];
  __shared__ uint8_t lkind[K4W];
  __shared__ uint32_t lep[K4W];
  __shared__ uint32_t kcnt[K4PMAX], rcnt[K4PMAX];
  __shared__ uint32_t red[K4TT / 64][3];
  if (EMIT && (counters[C_FLAGS] & (F_CYCLE | F_RANGE))) return;  // the run fails anyway
  const uint32_t tile = blockIdx.x, ntiles = gridDim.x, t0 = tile * K4T, t1 = min(n, t0 + K4T);
  const uint32_t w0 = t0 > K4H ? t0 - K4H : 0, w1 = min(n, t1 + K4H);
  for (uint32_t q = threadIdx.x; q < P; q += K4TT) kcnt[q] = rcnt[q] = 0;
  load_window(w0, w1, cparent, kind, shape, dep_ep, n_shapes, lcp, lkind, lep);
  __syncthreads();
  const Window W{lcp, lkind, lep, w0, w1, cparent, kind, shape, dep_ep, n_shapes};
  uint32_t rows = 0, rel = 0, maxd = 0;
  int64_t tsv[K4PER];
  if (EMIT) {
#pragma unroll
    for (int q = 0; q < K4PER; ++q) {
      uint32_t i = t0 + q * K4TT + threadIdx.x;
      tsv[q] = (i < t1 && lkind[i - w0] == KIND_SERVER) ? ts[i] : 0;
    }
  }
#pragma unroll
  for (int q = 0; q < K4PER; ++q) {
    const uint32_t i = t0 + q * K4TT + threadIdx.x;
    uint64_t rp = NONE64;
    if (i < t1 && lkind[i - w0] == KIND_SERVER) {
      const uint32_t es = lep[i - w0];
      if (es >= n_ep) {
        atomicOr(&counters[C_FLAGS], F_RANGE);
      } else {
        const uint32_t p = edge_part(es, P);
        const uint32_t first = W.next(i);
        uint32_t D = 0;
        bool bad = false;
        for (uint32_t cur = first; cur != NONE; cur = W.next(cur)) {
          if (D >= MAX_DEPTH || cur == CYC) {
            atomicOr(&counters[C_FLAGS], F_CYCLE);
            unsigned long long k = atomicAdd(&g_k4dbg[0], 1ull);
            if (k < 15) {
              g_k4dbg[1 + 4 * k] = i;
              g_k4dbg[2 + 4 * k] = first;
              g_k4dbg[3 + 4 * k] = cur;
              g_k4dbg[4 + 4 * k] = ((uint64_t)lcp[i - w0] << 32) | cparent[i];
            }
            bad = true;
            break;
          }
          uint32_t ea = W.ep_of(cur);
          if (ea >= n_ep) {
            atomicOr(&counters[C_FLAGS], F_RANGE);
            bad = true;
            break;
          }
          if (!EMIT && W.kind_of(cur) != KIND_SERVER) atomicAdd(&rcnt[edge_part(ea, P)], 1u);
          ++D;
        }
        if (!bad) {
          rp = index_base + i;
          if (!EMIT) {
            atomicAdd(&kcnt[p], D);
            atomicAdd(&rcnt[p], 1u);
            ++rows;
            rel += D;
            maxd = max(maxd, D);
          } else {
            uint64_t kb = koff[(uint64_t)p * ntiles + tile] + atomicAdd(&kcnt[p], D);
            uint64_t rb = roff[(uint64_t)p * ntiles + tile] + atomicAdd(&rcnt[p], 1u);
            rpool[2 * rb] = ((uint64_t)es << 40) | (((rp << 1) | (first != NONE ? 1ull : 0ull)) & FKEY_MASK);
            rpool[2 * rb + 1] = (uint64_t)tsv[q] ^ TS_BIAS;
            uint32_t cur = first;
            for (uint32_t d = 1; d <= D; ++d, cur = W.next(cur)) {
              uint8_t ka = W.kind_of(cur);
              uint32_t ea = W.ep_of(cur);
              kpool[kb + d - 1] = ((uint64_t)ea << 40) | ((uint64_t)es << 16) | ((uint64_t)d << 1) |
                                  (ka == KIND_SERVER ? 1ull : 0ull);
              if (ka != KIND_SERVER) {  // non-SERVER ancestors are not rows: their use counts for lastUsage
                uint32_t pa = edge_part(ea, P);
                uint64_t r = roff[(uint64_t)pa * ntiles + tile] + atomicAdd(&rcnt[pa], 1u);
                rpool[2 * r] = ((uint64_t)ea << 40) | FKEY_MASK;
                rpool[2 * r + 1] = (uint64_t)ts[cur] ^ TS_BIAS;
              }
            }
          }
        }
      }
    }
    if (!EMIT && rowpos_out && i < t1) rowpos_out[i] = rp;
  }
  if (!EMIT) {
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < P; q += K4TT) {
      kdir[(uint64_t)q * ntiles + tile] = kcnt[q];
      rdir[(uint64_t)q * ntiles + tile] = rcnt[q];
    }
    for (int o = 32; o > 0; o >>= 1) {
      rel += __shfl_xor(rel, o, 64);
      rows += __shfl_xor(rows, o, 64);
      maxd = max(maxd, (uint32_t)__shfl_xor(maxd, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      red[threadIdx.x >> 6][0] = rows;
      red[threadIdx.x >> 6][1] = rel;
      red[threadIdx.x >> 6][2] = maxd;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
      uint32_t a = 0;
      for (int w = 0; w < K4TT / 64; ++w) a = threadIdx.x == 2 ? max(a, red[w][2]) : a + red[w][threadIdx.x];
      tile_stats[(uint64_t)tile * 4 + threadIdx.x] = a;
    }
  }
}

// one workgroup per edge partition: exact key dedup in an LDS hash set and the
// per-endpoint (max ts, min first row) of the endpoints the partition owns.
// Loads are issued 8 per thread before they are consumed (memory-level
// parallelism: the LDS work in between would otherwise serialise them).
constexpr int K4B = 8;
__global__ void __launch_bounds__(1024) k4_dedup(const unsigned long long *__restrict__ kpool,
                                                 const uint32_t *__restrict__ koff,
                                                 const unsigned long long *__restrict__ rpool,
                                                 const uint32_t *__restrict__ roff, uint32_t ntiles,
                                                 unsigned long long *__restrict__ ep_ts,
                                                 unsigned long long *__restrict__ ep_first,
                                                 unsigned long long *__restrict__ out,
                                                 unsigned long long *__restrict__ stats64,
                                                 unsigned int *__restrict__ counters) {
  __shared__ unsigned long long set[K4SET];
  __shared__ uint32_t mkey[K4EMAP];
  __shared__ unsigned long long mts[K4EMAP], mfirst[K4EMAP];
  __shared__ unsigned int used, cursor;
  __shared__ unsigned long long obase;
  const uint32_t p = blockIdx.x;
  for (uint32_t k = threadIdx.x; k < K4SET; k += blockDim.x) set[k] = 0;
  for (uint32_t k = threadIdx.x; k < K4EMAP; k += blockDim.x) {
    mkey[k] = 0;
    mts[k] = 0;
    mfirst[k] = ~0ull;
  }
  if (threadIdx.x == 0) used = cursor = 0;
  __syncthreads();
  bool full = false;
  {  // endpoint records
    const uint64_t b = roff[(uint64_t)p * ntiles], e = roff[(uint64_t)(p + 1) * ntiles];
    for (uint64_t j0 = b; j0 < e; j0 += (uint64_t)K4B * blockDim.x) {
      uint64_t a[K4B], t[K4B];
#pragma unroll
      for (int q = 0; q < K4B; ++q) {
        uint64_t j = j0 + (uint64_t)q * blockDim.x + threadIdx.x;
        a[q] = j < e ? rpool[2 * j] : ~0ull;
        t[q] = j < e ? rpool[2 * j + 1] : 0;
      }
#pragma unroll
      for (int q = 0; q < K4B; ++q) {
        if (a[q] == ~0ull) continue;
        uint32_t ee = (uint32_t)(a[q] >> 40), f = ee + 1;
        uint32_t h = (uint32_t)(mix64(ee) >> 54);  // 10 bits
        uint32_t z = 0;
        for (; z < K4EMAP; ++z) {
          uint32_t c = mkey[h];
          if (c == 0) c = atomicCAS(&mkey[h], 0u, f);
          if (c == 0 || c == f) break;
          h = (h + 1) & (K4EMAP - 1);
        }
        if (z == K4EMAP) {
          full = true;
          continue;
        }
        atomicMax(&mts[h], (unsigned long long)t[q]);
        if ((a[q] & FKEY_MASK) != FKEY_MASK) atomicMin(&mfirst[h], (unsigned long long)(a[q] & FKEY_MASK));
      }
    }
  }
  {  // edge keys
    const uint64_t b = koff[(uint64_t)p * ntiles], e = koff[(uint64_t)(p + 1) * ntiles];
    for (uint64_t j0 = b; j0 < e; j0 += (uint64_t)K4B * blockDim.x) {
      uint64_t kk[K4B];
#pragma unroll
      for (int q = 0; q < K4B; ++q) {
        uint64_t j = j0 + (uint64_t)q * blockDim.x + threadIdx.x;
        kk[q] = j < e ? kpool[j] : 0;
      }
#pragma unroll
      for (int q = 0; q < K4B; ++q) {
        const uint64_t key = kk[q];
        if (!key) continue;
        uint32_t h = (uint32_t)(mix64(key) >> 51);  // 13 bits
        uint32_t z = 0;
        for (; z < 128; ++z) {
          uint64_t c = set[h];
          if (c == key) break;
          if (c == 0) {
            c = atomicCAS(&set[h], 0ull, (unsigned long long)key);
            if (c == 0) {
              atomicAdd(&used, 1u);
              break;
            }
            if (c == key) break;
          }
          h = (h + 1) & (K4SET - 1);
        }
        if (z == 128) full = true;
      }
    }
  }
  if (full) atomicOr(&counters[C_FLAGS], F_TRIPLE_OVERFLOW);
  __syncthreads();
  if (used * 4 > K4SET * 3) {
    if (threadIdx.x == 0) atomicOr(&counters[C_FLAGS], F_TRIPLE_OVERFLOW);
    return;
  }
  // endpoint outputs: each endpoint belongs to exactly one partition
  for (uint32_t k = threadIdx.x; k < K4EMAP; k += blockDim.x) {
    uint32_t f = mkey[k];
    if (!f) continue;
    ep_ts[f - 1] = mts[k];
    ep_first[f - 1] = mfirst[k];
  }
  // unique keys: one global atomic per workgroup for the output range
  if (threadIdx.x == 0) obase = atomicAdd(&stats64[S_TRIP_OUT], (unsigned long long)used);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < K4SET; k += blockDim.x) {
    uint64_t key = set[k];
    bool have = key != 0;
    uint64_t m = __ballot(have);
    if (!m) continue;
    uint32_t lane = threadIdx.x & 63;
    uint32_t leader = __ffsll((long long)m) - 1;
    unsigned int base = 0;
    if (lane == leader) base = atomicAdd(&cursor, (unsigned int)__popcll(m));
    base = __shfl(base, leader, 64);
    if (have) out[obase + base + __popcll(m & ((1ull << lane) - 1))] = key;
  }
}

}  // namespace kmz
extern "C" int kmz__debug_k4(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(kmz::g_k4dbg), sizeof(kmz::g_k4dbg)) == hipSuccess ? 0 : -1;
}
namespace kmz {
uint32_t k4_tiles(uint32_t n) { return (n + K4T - 1) / K4T; }
uint32_t k4_pmax() { return K4PMAX; }
uint32_t k4_set_cap() { return K4SET * 3 / 4; }

void launch_k4_count(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                     const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                     uint64_t index_base, uint32_t P, uint32_t *kdir, uint32_t *rdir, unsigned long long *rowpos,
                     unsigned int *counters, uint32_t *tile_stats, unsigned long long *stats64) {
  uint32_t nt = k4_tiles(n);
  if (!nt) return;
  hipLaunchKernelGGL((k4_walk<false>), dim3(nt), dim3(K4TT), 0, s, kind, shape, ts, cparent, n, dep_ep, n_shapes, n_ep,
                     index_base, P, kdir, rdir, nullptr, nullptr, nullptr, nullptr, rowpos, counters, tile_stats);
  hipLaunchKernelGGL(k_tile_sum, dim3(1), dim3(1024), 0, s, tile_stats, nt, 4u, 3u, stats64 + S_ROWS, 2u);
}

void launch_k4_emit(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                    const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                    uint64_t index_base, uint32_t P, const uint32_t *koff, unsigned long long *kpool,
                    const uint32_t *roff, unsigned long long *rpool, unsigned int *counters) {
  uint32_t nt = k4_tiles(n);
  if (!nt) return;
  hipLaunchKernelGGL((k4_walk<true>), dim3(nt), dim3(K4TT), 0, s, kind, shape, ts, cparent, n, dep_ep, n_shapes, n_ep,
                     index_base, P, nullptr, nullptr, koff, roff, kpool, rpool, nullptr, counters, nullptr);
}

void launch_k4_dedup(hipStream_t s, const unsigned long long *kpool, const uint32_t *koff,
                     const unsigned long long *rpool, const uint32_t *roff, uint32_t n, uint32_t P,
                     unsigned long long *ep_ts, unsigned long long *ep_first, unsigned long long *out,
                     unsigned long long *stats64, unsigned int *counters) {
  if (!P || !n) return;
  hipLaunchKernelGGL(k4_dedup, dim3(P), dim3(1024), 0, s, kpool, koff, rpool, roff, k4_tiles(n), ep_ts, ep_first, out,
                     stats64, counters);
}

}  // namespace kmz
