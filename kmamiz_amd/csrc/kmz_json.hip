// kmz_json.hip -- K1 on the GPU: Zipkin JSON (Trace[][], Trace.ts:1-38, as
// ZipkinService.getTraceListFromZipkinByServiceName returns it,
// ZipkinService.ts:44-57) -> the kmz_spans columns, in HBM.
//
// The device restatement of the host fast path (kmz_ingest.cpp): same fields,
// same domain (anything outside it -> KMZ_E_UNSUPPORTED and the caller parses
// on the host), same output, shapes interned by the raw JSON text of their
// seven fields in first-occurrence order.
//
//   J1 k_json_sum     per 64-byte chunk: quote parity and the bracket depth
//                     change for both string states at the chunk start
//   J2 scan           exclusive scan of those (an associative 3-tuple): each
//                     chunk's entry state (in a string?, depth)
//   J3 k_json_struct  per chunk again, now exact: the span objects' '{' (depth
//                     2, outside strings) as a bitmask, and the outer grammar
//                     `[ [ {..}, .. ], .. ]` checked token by token
//   J4 k_json_starts  the span starts in byte order (scan of the counts)
//   J5 k_json_span    one thread per span: the object's members, as the host
//                     parser reads them; shape / status hashed and inserted
//                     (first occurrence = min span index)
//   J6 k_json_verify  every span's seven raw slices equal its representative's
//                     (a 64-bit hash collision falls back to the host parser)
//   J7 k_json_reps    the distinct shapes / statuses with their slices
//   J8 k_json_remap   raw interning slots -> the caller's shape / status ids
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kmz_kernels.h"

namespace kmz {

namespace {

constexpr uint32_t NF = 7;  // name + the six identity tags (ingest.py SHAPE_TAGS)
constexpr uint64_t SL_ABSENT = 0xFFFFFFull;

__device__ __forceinline__ bool is_ws(uint8_t ch) { return ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t'; }

uint32_t grid_of(uint64_t n, uint32_t cap = 16384) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, cap));
}

// ---- J1 ----------------------------------------------------------------------
__device__ __forceinline__ bool esc_carry(const uint8_t *__restrict__ b, uint64_t s) {
  uint32_t run = 0;
  while (s > 0 && b[s - 1] == '\\') {
    --s;
    ++run;
  }
  return run & 1;
}

__global__ void __launch_bounds__(256) k_json_sum(const uint8_t *__restrict__ b, uint64_t len, uint64_t nch,
                                                  JElem *__restrict__ elem) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = c * JCHUNK, e = min<uint64_t>(s + JCHUNK, len);
    bool esc = esc_carry(b, s);
    int in = 0, d0 = 0, tot = 0;
    uint32_t p = 0;
    for (uint64_t i = s; i < e; ++i) {
      const uint8_t ch = b[i];
      if (esc) {
        esc = false;
        continue;
      }
      if (ch == '\\') {
        esc = true;
        continue;
      }
      if (ch == '"') {
        in ^= 1;
        p ^= 1;
        continue;
      }
      const int v = (ch == '{' || ch == '[') ? 1 : ((ch == '}' || ch == ']') ? -1 : 0);
      tot += v;
      if (!in) d0 += v;
    }
    elem[c] = JElem{(int)p, d0, tot - d0};
  }
}

// ---- J2: exclusive scans (block-local, block totals, block offsets) ------------
template <class T>
struct SumOp {
  __device__ static T id() { return T(0); }
  __device__ static T op(T a, T b) { return a + b; }
};
struct JOp {
  __device__ static JElem id() { return JElem{0, 0, 0}; }
  __device__ static JElem op(JElem a, JElem b) {
    return JElem{a.p ^ b.p, a.d0 + (a.p ? b.d1 : b.d0), a.d1 + (a.p ? b.d0 : b.d1)};
  }
};

constexpr uint32_t SCAN_T = 256, SCAN_I = 8, SCAN_B = SCAN_T * SCAN_I;

// out[i] = exclusive prefix of in[0..i) within the block + (base ? base[block] : id)
template <class T, class Op>
__global__ void __launch_bounds__(SCAN_T) k_scan_block(const T *__restrict__ in, uint64_t n, T *__restrict__ out,
                                                       T *__restrict__ block_sum, const T *__restrict__ base) {
  __shared__ T sh[SCAN_T];
  const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_B;
  T v[SCAN_I];
  T acc = Op::id();
  for (uint32_t k = 0; k < SCAN_I; ++k) {
    const uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_I + k;
    v[k] = i < n ? in[i] : Op::id();
    acc = Op::op(acc, v[k]);
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t off = 1; off < SCAN_T; off <<= 1) {  // inclusive Hillis-Steele over thread totals
    T x = sh[threadIdx.x];
    if (threadIdx.x >= off) x = Op::op(sh[threadIdx.x - off], x);
    __syncthreads();
    sh[threadIdx.x] = x;
    __syncthreads();
  }
  T run = threadIdx.x ? sh[threadIdx.x - 1] : Op::id();
  if (base) run = Op::op(base[blockIdx.x], run);
  if (out)
    for (uint32_t k = 0; k < SCAN_I; ++k) {
      const uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_I + k;
      if (i < n) out[i] = run;
      run = Op::op(run, v[k]);
    }
  if (block_sum && threadIdx.x == SCAN_T - 1) block_sum[blockIdx.x] = sh[SCAN_T - 1];
}

// exclusive scan of in[n] -> out[n]; *total (device) = the whole reduction.
// scratch: >= 2 * ceil(n / SCAN_B) + 2 * ceil(n / SCAN_B^2) + 2 elements.
template <class T, class Op>
void scan(hipStream_t s, const T *in, uint64_t n, T *out, T *total, T *scratch) {
  const uint64_t nb = (n + SCAN_B - 1) / SCAN_B;
  if (nb <= 1) {
    hipLaunchKernelGGL((k_scan_block<T, Op>), dim3(1), dim3(SCAN_T), 0, s, in, n, out, total, (const T *)nullptr);
    return;
  }
  T *bs = scratch, *bo = scratch + nb;
  hipLaunchKernelGGL((k_scan_block<T, Op>), dim3((uint32_t)nb), dim3(SCAN_T), 0, s, in, n, (T *)nullptr, bs,
                     (const T *)nullptr);
  scan<T, Op>(s, bs, nb, bo, total, scratch + 2 * nb);
  hipLaunchKernelGGL((k_scan_block<T, Op>), dim3((uint32_t)nb), dim3(SCAN_T), 0, s, in, n, out, (T *)nullptr,
                     (const T *)bo);
}

// ---- J3 ------------------------------------------------------------------------
__device__ __forceinline__ int prev_nw(const uint8_t *__restrict__ b, uint64_t i) {
  while (i > 0) {
    const uint8_t ch = b[--i];
    if (!is_ws(ch)) return ch;
  }
  return -1;
}
__device__ __forceinline__ int next_nw(const uint8_t *__restrict__ b, uint64_t i, uint64_t len) {
  while (++i < len) {
    const uint8_t ch = b[i];
    if (!is_ws(ch)) return ch;
  }
  return -1;
}

__global__ void __launch_bounds__(256) k_json_struct(const uint8_t *__restrict__ b, uint64_t len, uint64_t nch,
                                                     const JElem *__restrict__ state,
                                                     unsigned long long *__restrict__ mask,
                                                     uint32_t *__restrict__ cnt, unsigned int *__restrict__ flags) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = c * JCHUNK, e = min<uint64_t>(s + JCHUNK, len);
    bool esc = esc_carry(b, s);
    int in = state[c].p, depth = state[c].d0;
    uint64_t m = 0;
    bool bad = false, top = false;
    for (uint64_t i = s; i < e; ++i) {
      const uint8_t ch = b[i];
      if (esc) {
        esc = false;
        continue;
      }
      if (in) {
        if (ch == '\\')
          esc = true;
        else if (ch == '"')
          in = 0;
        continue;
      }
      if (ch == '"') {
        if (depth <= 2) bad = true;  // a string outside a span
        in = 1;
        continue;
      }
      if (ch == '\\') {
        bad = true;
        continue;
      }
      if (is_ws(ch)) continue;
      if (depth >= 3) {
        if (ch == '{' || ch == '[') ++depth;
        if (ch == '}' || ch == ']') --depth;
        continue;
      }
      const int pv = prev_nw(b, i);
      if (depth == 0) {  // the top-level array, first in the input
        if (ch != '[' || pv != -1) bad = true;
        top = true;
        depth = 1;
      } else if (depth == 1) {  // between traces
        if (ch == '[') {
          if (pv != '[' && pv != ',') bad = true;
          depth = 2;
        } else if (ch == ',') {
          if (pv != ']' || next_nw(b, i, len) != '[') bad = true;
        } else if (ch == ']') {
          if (pv != '[' && pv != ']') bad = true;
          depth = 0;
        } else {
          bad = true;
        }
      } else {  // depth 2: between the spans of a trace
        if (ch == '{') {
          if (pv != '[' && pv != ',') bad = true;
          m |= 1ull << (i - s);
          depth = 3;
        } else if (ch == ',') {
          if (pv != '}' || next_nw(b, i, len) != '{') bad = true;
        } else if (ch == ']') {
          if (pv != '[' && pv != '}') bad = true;
          depth = 1;
        } else {
          bad = true;
        }
      }
    }
    mask[c] = m;
    cnt[c] = (uint32_t)__popcll(m);
    if (bad) atomicOr(&flags[0], JF_BAD);
    if (top) atomicOr(&flags[0], JF_TOP);
  }
}

// ---- J4 ------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_json_starts(const unsigned long long *__restrict__ mask,
                                                     const uint32_t *__restrict__ off, uint64_t nch,
                                                     unsigned long long *__restrict__ starts) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t m = mask[c];
    uint32_t k = off[c];
    while (m) {
      starts[k++] = c * JCHUNK + (uint64_t)__builtin_ctzll(m);
      m &= m - 1;
    }
  }
}

// ---- J5: one span --------------------------------------------------------------
struct Cur {
  const uint8_t *b;
  uint64_t p, e;
  bool bad;
};
__device__ __forceinline__ void ws(Cur &c) {
  while (c.p < c.e && is_ws(c.b[c.p])) ++c.p;
}
__device__ __forceinline__ bool eat(Cur &c, uint8_t ch) {
  ws(c);
  if (c.p < c.e && c.b[c.p] == ch) {
    ++c.p;
    return true;
  }
  return false;
}
// at '"': past the closing quote; *esc: an escape occurred
__device__ __forceinline__ bool skip_string(Cur &c, bool *esc) {
  uint64_t p = c.p + 1;
  while (p < c.e) {
    const uint8_t ch = c.b[p];
    if (ch == '"') {
      c.p = p + 1;
      return true;
    }
    if (ch == '\\') {
      *esc = true;
      p += 2;
      continue;
    }
    ++p;
  }
  return false;
}
__device__ bool skip_value(Cur &c) {
  ws(c);
  if (c.p >= c.e) return false;
  const uint8_t ch = c.b[c.p];
  bool esc = false;
  if (ch == '"') return skip_string(c, &esc);
  if (ch == '{' || ch == '[') {
    int depth = 0;
    while (c.p < c.e) {
      const uint8_t d = c.b[c.p];
      if (d == '"') {
        if (!skip_string(c, &esc)) return false;
        continue;
      }
      ++c.p;
      if (d == '{' || d == '[') {
        ++depth;
      } else if (d == '}' || d == ']') {
        if (--depth == 0) return true;
      }
    }
    return false;
  }
  while (c.p < c.e) {
    const uint8_t d = c.b[c.p];
    if (d == ',' || d == '}' || d == ']' || is_ws(d)) break;
    ++c.p;
  }
  return true;
}
// a key without escapes: [ks, ks + kl)
__device__ __forceinline__ bool key(Cur &c, uint64_t *ks, uint32_t *kl) {
  ws(c);
  if (c.p >= c.e || c.b[c.p] != '"') return false;
  const uint64_t s = c.p + 1;
  bool esc = false;
  if (!skip_string(c, &esc)) return false;
  if (esc) c.bad = true;
  *ks = s;
  *kl = (uint32_t)(c.p - 1 - s);
  return eat(c, ':');
}
template <int N>
__device__ __forceinline__ bool key_is(const Cur &c, uint64_t ks, uint32_t kl, const char (&lit)[N]) {
  if (kl != N - 1) return false;
  for (int i = 0; i < N - 1; ++i)
    if (c.b[ks + i] != (uint8_t)lit[i]) return false;
  return true;
}
// packed slice: offset << 24 | length (SL_ABSENT: property missing)
__device__ __forceinline__ uint64_t value_slice(Cur &c) {
  ws(c);
  const uint64_t s = c.p;
  if (!skip_value(c)) {
    c.bad = true;
    return SL_ABSENT;
  }
  const uint64_t n = c.p - s;
  if (n >= SL_ABSENT || s >= (1ull << 40)) {
    c.bad = true;
    return SL_ABSENT;
  }
  return (s << 24) | n;
}
__device__ __forceinline__ int hexv(uint8_t ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  return -1;
}
__device__ uint64_t hex_id(Cur &c, bool allow_empty) {
  ws(c);
  if (c.p >= c.e) return c.bad = true, 0;
  if (allow_empty && c.b[c.p] == 'n' && c.e - c.p >= 4 && c.b[c.p + 1] == 'u' && c.b[c.p + 2] == 'l' &&
      c.b[c.p + 3] == 'l') {
    c.p += 4;
    return 0;
  }
  if (c.b[c.p] != '"') return c.bad = true, 0;
  const uint64_t s = c.p + 1;
  if (allow_empty && s < c.e && c.b[s] == '"') {
    c.p = s + 1;
    return 0;
  }
  if (c.e - s < 17 || c.b[s + 16] != '"') return c.bad = true, 0;
  uint64_t v = 0;
  for (int i = 0; i < 16; ++i) {
    const int h = hexv(c.b[s + i]);
    if (h < 0) return c.bad = true, 0;
    v = v << 4 | (uint64_t)h;
  }
  if (!v) return c.bad = true, 0;
  c.p = s + 17;
  return v;
}
__device__ int64_t int_value(Cur &c, int64_t lo, int64_t hi) {
  ws(c);
  uint64_t s = c.p;
  bool neg = false;
  if (s < c.e && c.b[s] == '-') {
    neg = true;
    ++s;
  }
  if (s >= c.e || c.b[s] < '0' || c.b[s] > '9') return c.bad = true, 0;
  uint64_t v = 0;
  int nd = 0;
  while (s < c.e && c.b[s] >= '0' && c.b[s] <= '9') {
    v = v * 10 + (uint64_t)(c.b[s] - '0');
    if (++nd > 18) return c.bad = true, 0;
    ++s;
  }
  if (s < c.e && (c.b[s] == '.' || c.b[s] == 'e' || c.b[s] == 'E')) return c.bad = true, 0;
  c.p = s;
  const int64_t x = neg ? -(int64_t)v : (int64_t)v;
  if (x < lo || x > hi) return c.bad = true, 0;
  return x;
}

__device__ __forceinline__ uint64_t hmix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
__device__ uint64_t slices_hash(const uint8_t *__restrict__ b, const uint64_t *sl, int nf) {
  uint64_t h = 0x9E3779B97F4A7C15ull * (uint64_t)(nf + 1);
  for (int f = 0; f < nf; ++f) {
    const uint64_t n = sl[f] & SL_ABSENT;
    if (n == SL_ABSENT) {
      h = hmix(h ^ 0xA5A5A5A5ull);
      continue;
    }
    const uint64_t o = sl[f] >> 24;
    h = hmix(h ^ n);
    uint64_t w = 0;
    uint32_t k = 0;
    for (uint64_t i = 0; i < n; ++i) {
      w |= (uint64_t)b[o + i] << (8 * k);
      if (++k == 8) {
        h = hmix(h + w);
        w = 0;
        k = 0;
      }
    }
    h = hmix(h + (w ^ ((uint64_t)k << 56)));
  }
  return h ? h : 1;  // 0 marks an empty slot
}
// open addressing on the 64-bit hash, {hash, ~rep} slots (a zeroed table is
// empty); rep = the min span index (first occurrence) through atomicMax(~i)
__device__ uint32_t intern(unsigned long long *__restrict__ tab, uint64_t cap, uint64_t h, uint64_t i,
                           unsigned int *__restrict__ flags) {
  uint64_t p = slot_of(h, cap);
  const unsigned long long ni = ~i;
  for (uint64_t t = 0; t < min<uint64_t>(cap, 4096); ++t) {
    unsigned long long k = tab[2 * p];
    if (k == 0) k = atomicCAS(&tab[2 * p], 0ull, (unsigned long long)h);
    if (k == 0 || k == h) {
      if (*(volatile unsigned long long *)&tab[2 * p + 1] < ni) atomicMax(&tab[2 * p + 1], ni);
      return (uint32_t)p;
    }
    p = p + 1 == cap ? 0 : p + 1;
  }
  atomicOr(flags, JF_FULL);  // (the caller grows the table and parses again)
  return 0;
}

__global__ void __launch_bounds__(256) k_json_span(const uint8_t *__restrict__ b, uint64_t len,
                                                   const unsigned long long *__restrict__ starts, uint64_t n,
                                                   uint64_t *__restrict__ sid, uint64_t *__restrict__ pid,
                                                   uint8_t *__restrict__ kind, uint32_t *__restrict__ dur,
                                                   int64_t *__restrict__ ts, unsigned long long *__restrict__ slices,
                                                   uint32_t *__restrict__ shape_slot, uint32_t *__restrict__ status_slot,
                                                   unsigned long long *__restrict__ stab, uint64_t scap,
                                                   unsigned long long *__restrict__ ttab, uint64_t tcap,
                                                   unsigned int *__restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    Cur c{b, starts[i], len, false};
    uint64_t s_id = 0, p_id = 0;
    bool have_id = false, have_dur = false, have_ts = false, ok = true;
    uint8_t kd = KMZ_KIND_OTHER;
    int64_t du = 0, t = 0;
    uint64_t f[NF + 1];
    for (uint32_t k = 0; k <= NF; ++k) f[k] = SL_ABSENT;
    if (!eat(c, '{')) ok = false;
    ws(c);
    if (ok && c.p < c.e && c.b[c.p] == '}') {
      ++c.p;
      c.bad = true;  // a span without id / duration / timestamp
    } else {
      while (ok && !c.bad) {
        uint64_t ks;
        uint32_t kl;
        if (!key(c, &ks, &kl)) {
          ok = false;
          break;
        }
        if (key_is(c, ks, kl, "id")) {
          s_id = hex_id(c, false);
          have_id = true;
        } else if (key_is(c, ks, kl, "parentId")) {
          p_id = hex_id(c, true);
        } else if (key_is(c, ks, kl, "kind")) {
          ws(c);
          if (c.p < c.e && c.b[c.p] == '"') {
            const uint64_t s0 = c.p + 1;
            bool esc = false;
            if (!skip_string(c, &esc)) {
              ok = false;
              break;
            }
            if (esc) c.bad = true;
            const uint32_t vl = (uint32_t)(c.p - 1 - s0);
            kd = key_is(c, s0, vl, "SERVER") ? KMZ_KIND_SERVER
                                              : (key_is(c, s0, vl, "CLIENT") ? KMZ_KIND_CLIENT : KMZ_KIND_OTHER);
          } else {
            if (!skip_value(c)) {
              ok = false;
              break;
            }
            kd = KMZ_KIND_OTHER;
          }
        } else if (key_is(c, ks, kl, "name")) {
          f[0] = value_slice(c);
        } else if (key_is(c, ks, kl, "duration")) {
          du = int_value(c, 0, 0xFFFFFFFFll);
          have_dur = true;
        } else if (key_is(c, ks, kl, "timestamp")) {
          t = int_value(c, -(int64_t)0x7FFFFFFFFFFFFFFFll, 0x7FFFFFFFFFFFFFFFll);
          have_ts = true;
        } else if (key_is(c, ks, kl, "tags")) {
          for (uint32_t k = 1; k <= NF; ++k) f[k] = SL_ABSENT;
          ws(c);
          if (c.p + 4 <= c.e && c.b[c.p] == 'n' && c.b[c.p + 1] == 'u' && c.b[c.p + 2] == 'l' && c.b[c.p + 3] == 'l') {
            c.p += 4;
          } else if (!eat(c, '{')) {
            c.bad = true;
          } else {
            ws(c);
            if (c.p < c.e && c.b[c.p] == '}') {
              ++c.p;
            } else {
              for (;;) {
                uint64_t ts0;
                uint32_t tl;
                if (!key(c, &ts0, &tl)) {
                  ok = false;
                  break;
                }
                int hit = -1;
                if (key_is(c, ts0, tl, "http.method")) hit = 1;
                else if (key_is(c, ts0, tl, "http.url")) hit = 2;
                else if (key_is(c, ts0, tl, "istio.canonical_revision")) hit = 3;
                else if (key_is(c, ts0, tl, "istio.canonical_service")) hit = 4;
                else if (key_is(c, ts0, tl, "istio.namespace")) hit = 5;
                else if (key_is(c, ts0, tl, "istio.mesh_id")) hit = 6;
                else if (key_is(c, ts0, tl, "http.status_code")) hit = NF;
                if (hit >= 0)
                  f[hit] = value_slice(c);
                else if (!skip_value(c)) {
                  ok = false;
                  break;
                }
                if (eat(c, ',')) continue;
                if (eat(c, '}')) break;
                ok = false;
                break;
              }
            }
          }
        } else if (!skip_value(c)) {
          ok = false;
          break;
        }
        if (!ok || c.bad) break;
        if (eat(c, ',')) continue;
        if (eat(c, '}')) break;
        ok = false;
      }
    }
    if (!have_id || !have_dur || !have_ts) c.bad = true;
    if (!ok || c.bad) {
      atomicOr(flags, JF_BAD);
      shape_slot[i] = status_slot[i] = NONE;  // (J6 skips it)
      continue;
    }
    sid[i] = s_id;
    pid[i] = p_id;
    kind[i] = kd;
    dur[i] = (uint32_t)du;
    ts[i] = t;
    for (uint32_t k = 0; k <= NF; ++k) slices[i * (NF + 1) + k] = f[k];
    shape_slot[i] = intern(stab, scap, slices_hash(b, f, NF), i, flags);
    status_slot[i] = intern(ttab, tcap, slices_hash(b, f + NF, 1), i, flags);
  }
}

// ---- J6 --------------------------------------------------------------------------
__device__ __forceinline__ bool slices_equal(const uint8_t *__restrict__ b, const unsigned long long *x,
                                             const unsigned long long *y, int nf) {
  for (int f = 0; f < nf; ++f) {
    const uint64_t nx = x[f] & SL_ABSENT, ny = y[f] & SL_ABSENT;
    if (nx != ny) return false;
    if (nx == SL_ABSENT) continue;
    const uint64_t ox = x[f] >> 24, oy = y[f] >> 24;
    for (uint64_t i = 0; i < nx; ++i)
      if (b[ox + i] != b[oy + i]) return false;
  }
  return true;
}
__global__ void __launch_bounds__(256) k_json_verify(const uint8_t *__restrict__ b, uint64_t n,
                                                     const unsigned long long *__restrict__ slices,
                                                     const uint32_t *__restrict__ shape_slot,
                                                     const uint32_t *__restrict__ status_slot,
                                                     const unsigned long long *__restrict__ stab, uint64_t scap,
                                                     const unsigned long long *__restrict__ ttab, uint64_t tcap,
                                                     unsigned int *__restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long *mine = slices + i * (NF + 1);
    const uint32_t ss = shape_slot[i], ts = status_slot[i];
    if (ss >= scap || ts >= tcap) continue;  // a span outside the fast path (JF_BAD is set)
    const uint64_t rs = ~stab[2 * (uint64_t)ss + 1], rt = ~ttab[2 * (uint64_t)ts + 1];
    if (rs >= n || rt >= n) continue;  // an insert that failed (JF_FULL is set)
    if ((rs != i && !slices_equal(b, mine, slices + rs * (NF + 1), NF)) ||
        (rt != i && !slices_equal(b, mine + NF, slices + rt * (NF + 1) + NF, 1)))
      atomicOr(flags, JF_COLLIDE);
  }
}

// ---- J7 --------------------------------------------------------------------------
// out: per distinct entry {rep, slot, slices[nf]} (2 + nf words)
__global__ void __launch_bounds__(256) k_json_reps(const unsigned long long *__restrict__ tab, uint64_t cap,
                                                   const unsigned long long *__restrict__ slices, uint32_t first,
                                                   uint32_t nf, unsigned long long *__restrict__ out, uint64_t ocap,
                                                   uint64_t nspan, unsigned long long *__restrict__ count) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < cap; p += (uint64_t)gridDim.x * blockDim.x) {
    if (!tab[2 * p]) continue;
    const uint64_t rep = ~tab[2 * p + 1];
    if (rep >= nspan) continue;
    const uint64_t x = atomicAdd(count, 1ull);
    if (x >= ocap) continue;  // (the caller grows the output and runs again)
    unsigned long long *o = out + x * (2 + nf);
    o[0] = rep;
    o[1] = p;
    for (uint32_t k = 0; k < nf; ++k) o[2 + k] = slices[rep * (NF + 1) + first + k];
  }
}

// ---- J8 --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_json_remap(uint64_t n, uint32_t *__restrict__ shape,
                                                    const uint32_t *__restrict__ status_slot,
                                                    uint16_t *__restrict__ status, const uint32_t *__restrict__ smap,
                                                    const uint32_t *__restrict__ tmap) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    shape[i] = smap[shape[i]];
    status[i] = (uint16_t)tmap[status_slot[i]];
  }
}

}  // namespace

uint64_t json_scan_scratch(uint64_t n) {
  uint64_t s = 2, m = n;
  while (m > SCAN_B) {
    m = (m + SCAN_B - 1) / SCAN_B;
    s += 2 * m + 2;
  }
  return s + 2;
}

void launch_json_structure(hipStream_t s, const uint8_t *b, uint64_t len, uint64_t nch, JElem *elem, JElem *state,
                           JElem *jtotal, JElem *jscratch, unsigned long long *mask, uint32_t *cnt, uint32_t *off,
                           uint32_t *ctotal, uint32_t *cscratch, unsigned int *flags) {
  hipLaunchKernelGGL(k_json_sum, dim3(grid_of(nch)), dim3(256), 0, s, b, len, nch, elem);
  scan<JElem, JOp>(s, elem, nch, state, jtotal, jscratch);
  hipLaunchKernelGGL(k_json_struct, dim3(grid_of(nch)), dim3(256), 0, s, b, len, nch, state, mask, cnt, flags);
  scan<uint32_t, SumOp<uint32_t>>(s, cnt, nch, off, ctotal, cscratch);
}

void launch_json_starts(hipStream_t s, const unsigned long long *mask, const uint32_t *off, uint64_t nch,
                        unsigned long long *starts) {
  hipLaunchKernelGGL(k_json_starts, dim3(grid_of(nch)), dim3(256), 0, s, mask, off, nch, starts);
}

void launch_json_spans(hipStream_t s, const uint8_t *b, uint64_t len, const unsigned long long *starts, uint64_t n,
                       uint64_t *sid, uint64_t *pid, uint8_t *kind, uint32_t *dur, int64_t *ts,
                       unsigned long long *slices, uint32_t *shape_slot, uint32_t *status_slot, unsigned long long *stab,
                       uint64_t scap, unsigned long long *ttab, uint64_t tcap, unsigned int *flags) {
  if (!n) return;
  hipLaunchKernelGGL(k_json_span, dim3(grid_of(n)), dim3(256), 0, s, b, len, starts, n, sid, pid, kind, dur, ts,
                     slices, shape_slot, status_slot, stab, scap, ttab, tcap, flags);
  hipLaunchKernelGGL(k_json_verify, dim3(grid_of(n)), dim3(256), 0, s, b, n, slices, shape_slot, status_slot, stab,
                     scap, ttab, tcap, flags);
}

void launch_json_reps(hipStream_t s, const unsigned long long *tab, uint64_t cap, const unsigned long long *slices,
                      uint32_t first, uint32_t nf, unsigned long long *out, uint64_t ocap, uint64_t nspan,
                      unsigned long long *count) {
  hipLaunchKernelGGL(k_json_reps, dim3(grid_of(cap)), dim3(256), 0, s, tab, cap, slices, first, nf, out, ocap, nspan,
                     count);
}

void launch_json_remap(hipStream_t s, uint64_t n, uint32_t *shape, const uint32_t *status_slot, uint16_t *status,
                       const uint32_t *smap, const uint32_t *tmap) {
  if (!n) return;
  hipLaunchKernelGGL(k_json_remap, dim3(grid_of(n)), dim3(256), 0, s, n, shape, status_slot, status, smap, tmap);
}

}  // namespace kmz
