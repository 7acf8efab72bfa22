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

// ---- bit-parallel chunk classification (64 bytes -> 64-bit masks) -------------
// bit j of eq4(w, c) <=> byte j of w equals c (exact zero-byte test)
__device__ __forceinline__ uint32_t eq4(uint32_t w, uint32_t c) {
  const uint32_t t = w ^ (c * 0x01010101u);
  const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}
struct CMasks {
  uint64_t q, bs, open, close, comma, ws, valid;
};
__device__ __forceinline__ CMasks chunk_masks(const uint8_t *__restrict__ b, uint64_t s, uint64_t e) {
  CMasks m{0, 0, 0, 0, 0, 0, 0};
  if (e - s == JCHUNK && (reinterpret_cast<uintptr_t>(b + s) & 15) == 0) {
    const uint4 *v = reinterpret_cast<const uint4 *>(b + s);
    const uint4 w0 = v[0], w1 = v[1], w2 = v[2], w3 = v[3];
    const uint32_t w[16] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w,
                            w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z, w3.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t x = w[k];
      const int sh = 4 * k;
      m.q |= (uint64_t)eq4(x, '"') << sh;
      m.bs |= (uint64_t)eq4(x, '\\') << sh;
      m.open |= (uint64_t)(eq4(x, '{') | eq4(x, '[')) << sh;
      m.close |= (uint64_t)(eq4(x, '}') | eq4(x, ']')) << sh;
      m.comma |= (uint64_t)eq4(x, ',') << sh;
      m.ws |= (uint64_t)(eq4(x, ' ') | eq4(x, '\n') | eq4(x, '\r') | eq4(x, '\t')) << sh;
    }
    m.valid = ~0ull;
  } else {
    for (uint64_t i = s; i < e; ++i) {
      const uint8_t ch = b[i];
      const uint64_t bit = 1ull << (i - s);
      if (ch == '"') m.q |= bit;
      if (ch == '\\') m.bs |= bit;
      if (ch == '{' || ch == '[') m.open |= bit;
      if (ch == '}' || ch == ']') m.close |= bit;
      if (ch == ',') m.comma |= bit;
      if (is_ws(ch)) m.ws |= bit;
    }
    m.valid = e - s == JCHUNK ? ~0ull : ((1ull << (e - s)) - 1);
  }
  return m;
}
// characters escaped by a preceding odd-length backslash run; `carry`: the
// chunk's first character is escaped (a run ending at the previous chunk)
__device__ __forceinline__ uint64_t escaped_mask(uint64_t bs, bool carry) {
  const uint64_t even = 0x5555555555555555ull, odd = ~even;
  if (carry) bs &= ~1ull;  // (an escaped backslash starts no escape)
  const uint64_t starts = bs & ~(bs << 1);
  const uint64_t even_ends = (bs + (starts & even)) & ~bs;
  const uint64_t odd_ends = (bs + (starts & odd)) & ~bs;
  return ((even_ends & odd) | (odd_ends & even)) | (carry ? 1ull : 0ull);
}
// bit i = XOR of bits 0..i
__device__ __forceinline__ uint64_t prefix_xor(uint64_t x) {
  x ^= x << 1;
  x ^= x << 2;
  x ^= x << 4;
  x ^= x << 8;
  x ^= x << 16;
  x ^= x << 32;
  return x;
}

__global__ void __launch_bounds__(256) k_json_sum(const uint8_t *__restrict__ b, uint64_t len, uint64_t nch,
                                                  JElem *__restrict__ elem) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = c * JCHUNK, e = min<uint64_t>(s + JCHUNK, len);
    const CMasks m = chunk_masks(b, s, e);
    const uint64_t esc = escaped_mask(m.bs, esc_carry(b, s)) & m.valid;
    const uint64_t qu = m.q & ~esc, op = m.open & ~esc, cl = m.close & ~esc;
    const uint64_t out0 = ~prefix_xor(qu);  // outside strings if the chunk starts outside one
    const int d0 = __popcll(op & out0) - __popcll(cl & out0);
    const int tot = __popcll(op) - __popcll(cl);
    elem[c] = JElem{(int)(__popcll(qu) & 1), d0, tot - d0};
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

// bits a+1 .. b-1 (a may be -1, b may be 64)
__device__ __forceinline__ uint64_t between(int a, int b) {
  const uint64_t hi = b >= 64 ? ~0ull : ((1ull << b) - 1);
  const uint64_t lo = a + 1 >= 64 ? ~0ull : ((1ull << (a + 1)) - 1);
  return hi & ~lo;
}

__global__ void __launch_bounds__(256) k_json_struct(const uint8_t *__restrict__ b, uint64_t len, uint64_t nch,
                                                     const JElem *__restrict__ state,
                                                     unsigned long long *__restrict__ mask,
                                                     uint32_t *__restrict__ cnt, unsigned int *__restrict__ flags) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = c * JCHUNK, e = min<uint64_t>(s + JCHUNK, len);
    const CMasks m = chunk_masks(b, s, e);
    const uint64_t esc = escaped_mask(m.bs, esc_carry(b, s)) & m.valid;
    const uint64_t qu = m.q & ~esc;
    const uint64_t instr = (prefix_xor(qu) ^ (state[c].p ? ~0ull : 0ull)) & m.valid;  // (opening quotes included)
    const uint64_t outside = ~instr & m.valid;
    bool bad = (m.bs & ~esc & outside) != 0;  // a backslash outside a string
    bool top = false;
    uint64_t starts_m = 0;
    const uint64_t tokens = (m.open | m.close) & ~esc & outside;
    // bytes at depth <= 2 that must be whitespace (depth 0) or whitespace and
    // commas (1, 2); an opening quote there starts a string outside a span
    const uint64_t stray0 = outside & ~m.ws, stray12 = stray0 & ~m.comma, openq = qu & instr;
    int depth = state[c].d0;
    int prev = -1;
    uint64_t t = tokens;
    for (;;) {
      const int pos = t ? __builtin_ctzll(t) : 64;
      if (depth <= 2) {  // the region (prev, pos) at this depth
        const uint64_t r = between(prev, pos) & m.valid;
        if ((r & openq) || (r & (depth == 0 ? stray0 : stray12))) bad = true;
        uint64_t cm = depth == 0 ? 0 : (r & m.comma & outside);
        while (cm) {
          const uint64_t i = s + (uint64_t)__builtin_ctzll(cm);
          cm &= cm - 1;
          const int pv = prev_nw(b, i), nx = next_nw(b, i, len);
          if (depth == 1 ? (pv != ']' || nx != '[') : (pv != '}' || nx != '{')) bad = true;
        }
      }
      if (pos == 64) break;
      t &= t - 1;
      const uint64_t i = s + (uint64_t)pos;
      const uint8_t ch = b[i];
      if (depth >= 3) {
        depth += (ch == '{' || ch == '[') ? 1 : -1;
      } else {
        const int pv = prev_nw(b, i);
        if (depth == 0) {  // the top-level array, first in the input
          if (ch != '[' || pv != -1) bad = true;
          top = true;
          depth = 1;
        } else if (depth == 1) {  // between traces
          if (ch == '[') {
            if (pv != '[' && pv != ',') bad = true;
            depth = 2;
          } else if (ch == ']') {
            if (pv != '[' && pv != ']') bad = true;
            depth = 0;
          } else {
            bad = true;
          }
        } else {  // depth 2: between the spans of a trace
          if (ch == '{') {
            if (pv != '[' && pv != ',') bad = true;
            starts_m |= 1ull << pos;
            depth = 3;
          } else if (ch == ']') {
            if (pv != '[' && pv != '}') bad = true;
            depth = 1;
          } else {
            bad = true;
          }
        }
      }
      prev = pos;
    }
    mask[c] = starts_m;
    cnt[c] = (uint32_t)__popcll(starts_m);
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
// The span parser reads bytes through an accessor: a wave first stages the
// bytes of up to 64 consecutive spans into LDS with 16-byte coalesced loads
// (LBytes); a span too large for the stage is parsed from global memory
// (GBytes).  Either way the parse is the host parser's, byte for byte.
constexpr uint32_t JSPAN_T = 64;           // one wave per workgroup
constexpr uint32_t JSPAN_LDS = 32 * 1024;  // bytes staged per round (5 workgroups per CU)

struct GBytes {
  const uint8_t *__restrict__ g;
  __device__ __forceinline__ uint8_t operator[](uint64_t i) const { return g[i]; }
};
struct LBytes {
  const uint8_t *l;
  uint64_t base;
  __device__ __forceinline__ uint8_t operator[](uint64_t i) const { return l[i - base]; }
};
// the first '"' or '\\' at or after p (< e), or e: eight bytes per LDS read
__device__ __forceinline__ uint64_t find_qb(const GBytes &b, uint64_t p, uint64_t e) {
  while (p < e && b[p] != '"' && b[p] != '\\') ++p;
  return p;
}
__device__ __forceinline__ uint64_t find_qb(const LBytes &b, uint64_t p, uint64_t e) {
  const uint64_t lo = 0x0101010101010101ull, hi = 0x8080808080808080ull;
  while (p < e) {
    const uint64_t rel = p - b.base, al = rel & ~7ull;
    uint64_t w = *reinterpret_cast<const uint64_t *>(b.l + al);
    const uint64_t q = w ^ (lo * '"'), s = w ^ (lo * '\\');
    // exact zero-byte masks (no borrow false positives)
    const uint64_t zq = ~(((q & ~hi) + ~hi) | q | ~hi), zs = ~(((s & ~hi) + ~hi) | s | ~hi);
    const uint64_t m = (zq | zs) & (~0ull << (8 * (rel - al)));
    if (m) return min<uint64_t>(b.base + al + (__builtin_ctzll(m) >> 3), e);
    p = b.base + al + 8;
  }
  return e;
}
template <class B>
struct Cur {
  B b;
  uint64_t p, e;
  bool bad;
};
template <class B>
__device__ __forceinline__ void ws(Cur<B> &c) {
  while (c.p < c.e && is_ws(c.b[c.p])) ++c.p;
}
template <class B>
__device__ __forceinline__ bool eat(Cur<B> &c, uint8_t ch) {
  ws(c);
  if (c.p < c.e && c.b[c.p] == ch) {
    ++c.p;
    return true;
  }
  return false;
}
// at '"': past the closing quote; *esc: an escape occurred
template <class B>
__device__ __forceinline__ bool skip_string(Cur<B> &c, bool *esc) {
  uint64_t p = c.p + 1;
  for (;;) {
    p = find_qb(c.b, p, c.e);
    if (p >= c.e) return false;
    if (c.b[p] == '"') {
      c.p = p + 1;
      return true;
    }
    *esc = true;  // a backslash: skip the escaped character
    p += 2;
  }
}
template <class B>
__device__ bool skip_value(Cur<B> &c) {
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
template <class B>
__device__ __forceinline__ bool key(Cur<B> &c, uint64_t *ks, uint32_t *kl) {
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
template <class B, int N>
__device__ __forceinline__ bool key_is(const Cur<B> &c, uint64_t ks, uint32_t kl, const char (&lit)[N]) {
  if (kl != N - 1) return false;
  for (int i = 0; i < N - 1; ++i)
    if (c.b[ks + i] != (uint8_t)lit[i]) return false;
  return true;
}
// packed slice: offset << 24 | length (SL_ABSENT: property missing)
template <class B>
__device__ __forceinline__ uint64_t value_slice(Cur<B> &c) {
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
template <class B>
__device__ uint64_t hex_id(Cur<B> &c, bool allow_empty) {
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
template <class B>
__device__ int64_t int_value(Cur<B> &c, int64_t lo, int64_t hi) {
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
template <class B>
__device__ uint64_t slices_hash(const B &b, const uint64_t *sl, int nf) {
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

struct SpanOut {
  uint64_t *__restrict__ sid, *__restrict__ pid;
  uint8_t *__restrict__ kind;
  uint32_t *__restrict__ dur;
  int64_t *__restrict__ ts;
  unsigned long long *__restrict__ slices;
  uint32_t *__restrict__ shape_slot, *__restrict__ status_slot;
  unsigned long long *__restrict__ stab, *__restrict__ ttab;
  uint64_t scap, tcap;
  unsigned int *__restrict__ flags;
};

template <class B>
__device__ void parse_one(const B &bytes, uint64_t start, uint64_t end, uint64_t i, const SpanOut &o) {
  Cur<B> c{bytes, start, end, false};
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
    atomicOr(o.flags, JF_BAD);
    o.shape_slot[i] = o.status_slot[i] = NONE;  // (J6 skips it)
    return;
  }
  o.sid[i] = s_id;
  o.pid[i] = p_id;
  o.kind[i] = kd;
  o.dur[i] = (uint32_t)du;
  o.ts[i] = t;
  for (uint32_t k = 0; k <= NF; ++k) o.slices[i * (NF + 1) + k] = f[k];
  o.shape_slot[i] = intern(o.stab, o.scap, slices_hash(bytes, f, NF), i, o.flags);
  o.status_slot[i] = intern(o.ttab, o.tcap, slices_hash(bytes, f + NF, 1), i, o.flags);
}

// Copy bytes [a0, hi) (a0 16-aligned) into lds with 16-byte loads (bytewise
// past the end of the buffer).
__device__ __forceinline__ void stage(const uint8_t *__restrict__ b, uint64_t len, uint64_t a0, uint64_t hi,
                                      uint8_t *lds) {
  const uint64_t nq = (hi - a0 + 15) / 16;
  for (uint64_t q = threadIdx.x; q < nq; q += blockDim.x) {
    const uint64_t g = a0 + 16 * q;
    if (g + 16 <= len) {
      *reinterpret_cast<uint4 *>(lds + 16 * q) = *reinterpret_cast<const uint4 *>(b + g);
    } else {
      for (uint64_t k = 0; k < 16 && g + k < len; ++k) lds[16 * q + k] = b[g + k];
    }
  }
}

// Span groups of 64: each round stages the longest prefix of the remaining
// spans whose bytes fit the stage (starts[n] = len), parses them from LDS,
// and a span alone too large for it is parsed from global memory.
template <class Body>
__device__ __forceinline__ void for_staged_spans(const uint8_t *__restrict__ b, uint64_t len,
                                                 const unsigned long long *__restrict__ starts, uint64_t n,
                                                 uint8_t *lds, Body body) {
  const uint32_t lane = threadIdx.x;
  const bool aligned = (reinterpret_cast<uintptr_t>(b) & 15) == 0;
  for (uint64_t i0 = (uint64_t)blockIdx.x * JSPAN_T; i0 < n; i0 += (uint64_t)gridDim.x * JSPAN_T) {
    const uint64_t iend = min<uint64_t>(n, i0 + JSPAN_T);
    uint64_t cur = i0;
    while (cur < iend) {
      const uint64_t lo = starts[cur], a0 = lo & ~15ull;
      const bool fits = aligned && cur + lane < iend && starts[cur + lane + 1] - a0 <= JSPAN_LDS;
      const uint64_t m = (uint64_t)__popcll(__ballot(fits));  // (a prefix: starts increase)
      if (m == 0) {  // one span larger than the stage: from global memory
        if (lane == 0) body(GBytes{b}, cur, len);
        cur += 1;
        continue;
      }
      const uint64_t hi = starts[cur + m];
      __syncthreads();  // the previous round's readers are done
      stage(b, len, a0, hi, lds);
      __syncthreads();
      if (lane < m) body(LBytes{lds, a0}, cur + lane, hi);
      cur += m;
    }
  }
}

__global__ void __launch_bounds__(JSPAN_T) k_json_span(const uint8_t *__restrict__ b, uint64_t len,
                                                       const unsigned long long *__restrict__ starts, uint64_t n,
                                                       SpanOut o) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[JSPAN_LDS];
  for_staged_spans(b, len, starts, n, lds, [&](const auto &bytes, uint64_t i, uint64_t end) {
    parse_one(bytes, starts[i], end, i, o);
  });
}

// ---- J6 --------------------------------------------------------------------------
template <class B>
__device__ __forceinline__ bool slices_equal(const B &bx, const unsigned long long *x, const uint8_t *__restrict__ g,
                                             const unsigned long long *y, int nf) {
  for (int f = 0; f < nf; ++f) {
    const uint64_t nx = x[f] & SL_ABSENT, ny = y[f] & SL_ABSENT;
    if (nx != ny) return false;
    if (nx == SL_ABSENT) continue;
    const uint64_t ox = x[f] >> 24, oy = y[f] >> 24;
    for (uint64_t i = 0; i < nx; ++i)
      if (bx[ox + i] != g[oy + i]) return false;
  }
  return true;
}
__global__ void __launch_bounds__(JSPAN_T) k_json_verify(const uint8_t *__restrict__ b, uint64_t len,
                                                         const unsigned long long *__restrict__ starts, uint64_t n,
                                                         const unsigned long long *__restrict__ slices,
                                                         const uint32_t *__restrict__ shape_slot,
                                                         const uint32_t *__restrict__ status_slot,
                                                         const unsigned long long *__restrict__ stab, uint64_t scap,
                                                         const unsigned long long *__restrict__ ttab, uint64_t tcap,
                                                         unsigned int *__restrict__ flags) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[JSPAN_LDS];
  for_staged_spans(b, len, starts, n, lds, [&](const auto &bytes, uint64_t i, uint64_t) {
    const unsigned long long *mine = slices + i * (NF + 1);
    const uint32_t ss = shape_slot[i], tsl = status_slot[i];
    if (ss >= scap || tsl >= tcap) return;  // a span outside the fast path (JF_BAD is set)
    const uint64_t rs = ~stab[2 * (uint64_t)ss + 1], rt = ~ttab[2 * (uint64_t)tsl + 1];
    if (rs >= n || rt >= n) return;  // an insert that failed (JF_FULL is set)
    if ((rs != i && !slices_equal(bytes, mine, b, slices + rs * (NF + 1), NF)) ||
        (rt != i && !slices_equal(bytes, mine + NF, b, slices + rt * (NF + 1) + NF, 1)))
      atomicOr(flags, JF_COLLIDE);
  });
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
  const uint32_t groups = (uint32_t)std::min<uint64_t>((n + JSPAN_T - 1) / JSPAN_T, 1u << 16);
  SpanOut o{sid, pid, kind, dur, ts, slices, shape_slot, status_slot, stab, ttab, scap, tcap, flags};
  hipLaunchKernelGGL(k_json_span, dim3(groups), dim3(JSPAN_T), 0, s, b, len, starts, n, o);
  hipLaunchKernelGGL(k_json_verify, dim3(groups), dim3(JSPAN_T), 0, s, b, len, starts, n, slices, shape_slot,
                     status_slot, stab, scap, ttab, tcap, flags);
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
