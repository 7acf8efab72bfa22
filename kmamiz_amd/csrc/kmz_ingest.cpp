// kmz_ingest.cpp -- SURVEY.md 8f row 1: Zipkin JSON (Trace[][], Trace.ts:1-38,
// as ZipkinService.getTraceListFromZipkinByServiceName returns it,
// ZipkinService.ts:44-57) straight into the kmz_spans columns, host side.
//
// The reference parses the whole response with JSON.parse and flattens it
// (Traces.ts:29); the engine only needs, per span, the id / parentId / kind /
// duration / timestamp scalars and the interned (name, identity tags) shape and
// status.  This parser reads exactly those, skips everything else without
// building objects, and interns shapes by the raw JSON text of their fields.
// The caller turns each distinct shape into its identities once (ingest.py),
// so a shape only needs its raw field slices.
//
// Anything outside the fast path's exact domain makes it return
// KMZ_E_UNSUPPORTED, and the caller parses the batch the general way: ids
// that are not 16 lowercase hex digits, a non-integer or out-of-range
// duration/timestamp, escapes in keys or in `kind`, `tags` that is not an
// object.  The batch is then not partially parsed.
//
// Large inputs are split by traces over threads: a structural pre-scan finds
// the top-level trace arrays, every thread parses a contiguous range with its
// own interning tables, and the tables merge in thread order, so shape and
// status ids follow first occurrence exactly as a single pass would number them.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <string_view>
#include <thread>
#include <vector>

#include "../../include/kmz.h"

namespace {

constexpr int NFIELD = 7;  // name + the six identity tags (ingest.py SHAPE_TAGS)
const char *const kTags[NFIELD - 1] = {"http.method",           "http.url",        "istio.canonical_revision",
                                        "istio.canonical_service", "istio.namespace", "istio.mesh_id"};
constexpr uint32_t ABSENT = 0xFFFFFFFFu;

struct Slice {
  uint64_t off = 0;
  uint32_t len = ABSENT;  // ABSENT: property missing (undefined)
};

struct Cursor {
  const char *b, *p, *e;  // buffer start, position, end
  bool bad = false;       // outside the fast path's domain
};

inline void ws(Cursor &c) {
  while (c.p < c.e && (*c.p == ' ' || *c.p == '\n' || *c.p == '\r' || *c.p == '\t')) ++c.p;
}
inline bool eat(Cursor &c, char ch) {
  ws(c);
  if (c.p < c.e && *c.p == ch) {
    ++c.p;
    return true;
  }
  return false;
}
// first byte of w (little endian) equal to '"' or '\\', as a bit mask (0: none)
inline uint64_t quote_or_bs(uint64_t w) {
  const uint64_t lo = 0x0101010101010101ull, hi = 0x8080808080808080ull;
  const uint64_t q = w ^ (lo * '"'), s = w ^ (lo * '\\');
  return ((q - lo) & ~q & hi) | ((s - lo) & ~s & hi);  // lowest set bit exact
}
// at '"': past the closing quote; *esc tells whether an escape occurred.
// Eight bytes at a time: JSON strings here are short, and a libc call per
// string costs more than the scan.
inline bool skip_string(Cursor &c, bool *esc = nullptr) {
  const char *p = c.p + 1, *e = c.e;
  for (;;) {
    while (e - p >= 8) {
      uint64_t w;
      memcpy(&w, p, 8);
      const uint64_t m = quote_or_bs(w);
      if (m) {
        p += __builtin_ctzll(m) >> 3;
        goto found;
      }
      p += 8;
    }
    while (p < e && *p != '"' && *p != '\\') ++p;
    if (p >= e) return false;
  found:
    if (*p == '"') {
      c.p = p + 1;
      return true;
    }
    if (esc) *esc = true;  // a backslash: skip the escaped character
    p += 2;
    if (p > e) return false;
  }
}
bool skip_value(Cursor &c) {
  ws(c);
  if (c.p >= c.e) return false;
  const char ch = *c.p;
  if (ch == '"') return skip_string(c);
  if (ch == '{' || ch == '[') {
    int depth = 0;
    while (c.p < c.e) {
      const char d = *c.p;
      if (d == '"') {
        if (!skip_string(c)) return false;
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
  while (c.p < c.e && *c.p != ',' && *c.p != '}' && *c.p != ']' && *c.p != ' ' && *c.p != '\n' && *c.p != '\r' &&
         *c.p != '\t')
    ++c.p;
  return true;
}
// a JSON string key without escapes -> view of its characters
inline bool key(Cursor &c, std::string_view *k) {
  ws(c);
  if (c.p >= c.e || *c.p != '"') return false;
  const char *s = c.p + 1;
  bool esc = false;
  if (!skip_string(c, &esc)) return false;
  if (esc) c.bad = true;  // JSON.parse would decode it: leave the batch to the general parser
  *k = std::string_view(s, (size_t)(c.p - 1 - s));
  return eat(c, ':');
}
inline Slice value_slice(Cursor &c) {
  ws(c);
  Slice s;
  s.off = (uint64_t)(c.p - c.b);
  if (!skip_value(c)) {
    c.bad = true;
    return s;
  }
  s.len = (uint32_t)(c.p - c.b - s.off);
  return s;
}
inline int hexv(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  return -1;
}
// a Zipkin id: exactly 16 lowercase hex digits, not all zero (ingest.py IdMapper)
inline uint64_t hex_id(Cursor &c, bool allow_empty) {
  ws(c);
  if (c.p >= c.e) return c.bad = true, 0;
  if (*c.p == 'n' && c.e - c.p >= 4 && !memcmp(c.p, "null", 4) && allow_empty) {  // falsy parentId
    c.p += 4;
    return 0;
  }
  if (*c.p != '"') return c.bad = true, 0;
  const char *s = c.p + 1;
  if (allow_empty && s < c.e && *s == '"') {  // "" (falsy parentId)
    c.p = s + 1;
    return 0;
  }
  if (c.e - s < 17 || s[16] != '"') return c.bad = true, 0;
  uint64_t v = 0;
  for (int i = 0; i < 16; ++i) {
    const int h = hexv(s[i]);
    if (h < 0) return c.bad = true, 0;
    v = v << 4 | (uint64_t)h;
  }
  if (!v) return c.bad = true, 0;
  c.p = s + 17;
  return v;
}
inline int64_t int_value(Cursor &c, int64_t lo, int64_t hi) {
  ws(c);
  const char *s = c.p;
  bool neg = false;
  if (s < c.e && *s == '-') {
    neg = true;
    ++s;
  }
  if (s >= c.e || *s < '0' || *s > '9') return c.bad = true, 0;
  uint64_t v = 0;
  int nd = 0;
  while (s < c.e && *s >= '0' && *s <= '9') {
    v = v * 10 + (uint64_t)(*s - '0');
    if (++nd > 18) return c.bad = true, 0;
    ++s;
  }
  if (s < c.e && (*s == '.' || *s == 'e' || *s == 'E')) return c.bad = true, 0;
  c.p = s;
  const int64_t x = neg ? -(int64_t)v : (int64_t)v;
  if (x < lo || x > hi) return c.bad = true, 0;
  return x;
}

// Interning of raw-slice tuples: open addressing on a 64-bit hash of the
// slices; equal hashes are confirmed by comparing the bytes (no allocation per span).
inline uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
uint64_t slices_hash(const char *b, const Slice *f, int nf) {
  uint64_t h = 0x9E3779B97F4A7C15ull * (uint64_t)(nf + 1);
  for (int i = 0; i < nf; ++i) {
    if (f[i].len == ABSENT) {
      h = mix(h ^ 0xA5A5A5A5ull);
      continue;
    }
    const char *p = b + f[i].off;
    uint32_t n = f[i].len;
    h = mix(h ^ n);
    while (n >= 8) {
      uint64_t w;
      memcpy(&w, p, 8);
      h = mix(h + w);
      p += 8;
      n -= 8;
    }
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = mix(h + (w ^ ((uint64_t)n << 56)));
  }
  return h;
}
bool slices_equal(const char *b, const Slice *x, const Slice *y, int nf) {
  for (int i = 0; i < nf; ++i) {
    if (x[i].len != y[i].len) return false;
    if (x[i].len != ABSENT && memcmp(b + x[i].off, b + y[i].off, x[i].len)) return false;
  }
  return true;
}
template <int NF>
struct Interner {
  std::vector<std::array<Slice, NF>> items;  // first-occurrence order
  std::vector<uint64_t> hs;                  // their hashes
  std::vector<uint32_t> tab;                 // open addressing: item index + 1 (0 = empty)
  Interner() : tab(256, 0) {}
  uint32_t put(const char *b, const Slice *f, uint64_t h) {
    if ((items.size() + 1) * 2 > tab.size()) grow();
    const size_t m = tab.size() - 1;
    size_t p = (size_t)h & m;
    for (;;) {
      const uint32_t v = tab[p];
      if (!v) break;
      if (hs[v - 1] == h && slices_equal(b, items[v - 1].data(), f, NF)) return v - 1;
      p = (p + 1) & m;
    }
    std::array<Slice, NF> a;
    for (int i = 0; i < NF; ++i) a[i] = f[i];
    items.push_back(a);
    hs.push_back(h);
    tab[p] = (uint32_t)items.size();
    return (uint32_t)items.size() - 1;
  }
  void grow() {
    std::vector<uint32_t> t(tab.size() * 2, 0);
    const size_t m = t.size() - 1;
    for (size_t i = 0; i < items.size(); ++i) {
      size_t p = (size_t)hs[i] & m;
      while (t[p]) p = (p + 1) & m;
      t[p] = (uint32_t)i + 1;
    }
    tab.swap(t);
  }
};

struct Local {  // one thread's output
  std::vector<uint64_t> sid, pid;
  std::vector<uint8_t> kind;
  std::vector<uint32_t> shape, status;
  std::vector<uint32_t> dur;
  std::vector<int64_t> ts;
  Interner<NFIELD> shapes;
  Interner<1> statuses;
  bool bad = false;
};

bool parse_span(Cursor &c, Local &L) {
  if (!eat(c, '{')) return false;
  uint64_t sid = 0, pid = 0;
  bool have_id = false, have_dur = false, have_ts = false;
  uint8_t kd = KMZ_KIND_OTHER;
  int64_t du = 0, ts = 0;
  std::array<Slice, NFIELD> f{};
  Slice st;
  ws(c);
  if (c.p < c.e && *c.p == '}') {
    ++c.p;
    c.bad = true;  // a span without id / duration / timestamp: the general path reports it
    return true;
  }
  for (;;) {
    std::string_view k;
    if (!key(c, &k)) return false;
    if (k == "id") {
      sid = hex_id(c, false);
      have_id = true;
    } else if (k == "parentId") {
      pid = hex_id(c, true);
    } else if (k == "kind") {
      ws(c);
      if (c.p < c.e && *c.p == '"') {
        const char *s = c.p + 1;
        bool esc = false;
        if (!skip_string(c, &esc)) return false;
        if (esc) c.bad = true;
        const std::string_view v(s, (size_t)(c.p - 1 - s));
        kd = v == "SERVER" ? KMZ_KIND_SERVER : (v == "CLIENT" ? KMZ_KIND_CLIENT : KMZ_KIND_OTHER);
      } else {
        if (!skip_value(c)) return false;
        kd = KMZ_KIND_OTHER;
      }
    } else if (k == "name") {
      f[0] = value_slice(c);
    } else if (k == "duration") {
      du = int_value(c, 0, 0xFFFFFFFFll);
      have_dur = true;
    } else if (k == "timestamp") {
      ts = int_value(c, -(int64_t)0x7FFFFFFFFFFFFFFFll, 0x7FFFFFFFFFFFFFFFll);
      have_ts = true;
    } else if (k == "tags") {
      for (int i = 1; i < NFIELD; ++i) f[i] = Slice{};
      st = Slice{};
      ws(c);
      if (c.p < c.e && *c.p == 'n' && c.e - c.p >= 4 && !memcmp(c.p, "null", 4)) {
        c.p += 4;  // `|| {}` (Traces.ts): no tags
      } else {
        if (!eat(c, '{')) return c.bad = true, skip_value(c);
        ws(c);
        if (c.p < c.e && *c.p == '}') {
          ++c.p;
        } else {
          for (;;) {
            std::string_view tk;
            if (!key(c, &tk)) return false;
            int hit = -1;
            for (int i = 0; i < NFIELD - 1; ++i)
              if (tk == kTags[i]) hit = i;
            if (hit >= 0)
              f[1 + hit] = value_slice(c);
            else if (tk == "http.status_code")
              st = value_slice(c);
            else if (!skip_value(c))
              return false;
            if (eat(c, ',')) continue;
            if (eat(c, '}')) break;
            return false;
          }
        }
      }
    } else if (!skip_value(c)) {
      return false;
    }
    if (eat(c, ',')) continue;
    if (eat(c, '}')) break;
    return false;
  }
  if (!have_id || !have_dur || !have_ts) c.bad = true;
  if (c.bad) return true;
  // intern shape and status (first occurrence order)
  const uint32_t shp = L.shapes.put(c.b, f.data(), slices_hash(c.b, f.data(), NFIELD));
  const uint32_t sti = L.statuses.put(c.b, &st, slices_hash(c.b, &st, 1));
  L.sid.push_back(sid);
  L.pid.push_back(pid);
  L.kind.push_back(kd);
  L.shape.push_back(shp);
  L.status.push_back(sti);
  L.dur.push_back((uint32_t)du);
  L.ts.push_back(ts);
  return true;
}

// Parse the traces from p (at a trace's '[') on.  A range that is not the last
// must end exactly at `stop` (the '[' where the next range starts) after a
// comma; the last one ends at the top-level ']' and only whitespace may
// follow.  Strings may run past `stop`: that is how a split point that fell
// inside a string shows (the parse passes over it and never lands on it).
// Returns false when the split was not a trace boundary; L.bad marks input
// outside the fast path's domain.
bool parse_range(const char *b, const char *p, const char *stop, const char *e, bool last, Local &L) {
  Cursor c{b, p, e};
  for (;;) {
    if (!eat(c, '[')) return L.bad = true, false;
    ws(c);
    if (c.p < c.e && *c.p == ']') {
      ++c.p;
    } else {
      for (;;) {
        if (!parse_span(c, L) || c.bad) return L.bad = true, false;
        if (eat(c, ',')) continue;
        if (eat(c, ']')) break;
        return L.bad = true, false;
      }
    }
    if (eat(c, ',')) {
      ws(c);
      if (!last && c.p >= stop) return c.p == stop;
      continue;
    }
    if (last && eat(c, ']')) {
      ws(c);
      if (c.p != c.e) L.bad = true;
      return true;
    }
    L.bad = true;
    return false;
  }
}

// A candidate trace boundary at or after q: `]`, optional whitespace, `,`,
// optional whitespace, then the '[' returned.  Between spans the byte after a
// comma is '{', inside a span it is '"', so outside strings the pattern only
// occurs between traces; one inside a string is caught by parse_range.
const char *next_boundary(const char *q, const char *e) {
  while (q < e) {
    const char *r = (const char *)memchr(q, ']', (size_t)(e - q));
    if (!r) return nullptr;
    const char *t = r + 1;
    while (t < e && (*t == ' ' || *t == '\n' || *t == '\r' || *t == '\t')) ++t;
    if (t < e && *t == ',') {
      ++t;
      while (t < e && (*t == ' ' || *t == '\n' || *t == '\r' || *t == '\t')) ++t;
      if (t < e && *t == '[') return t;
    }
    q = r + 1;
  }
  return nullptr;
}

template <class T>
T *copy_out(const std::vector<Local> &ls, std::vector<T> Local::*col, uint64_t n) {
  T *o = (T *)malloc(std::max<uint64_t>(1, n) * sizeof(T));
  if (!o) return nullptr;
  uint64_t k = 0;
  for (const Local &l : ls) {
    const std::vector<T> &v = l.*col;
    memcpy(o + k, v.data(), v.size() * sizeof(T));
    k += v.size();
  }
  return o;
}

}  // namespace

extern "C" {

int kmz_parse_zipkin(const char *json, uint64_t len, int threads, kmz_zipkin_batch **out) {
  if (!json || !out) return KMZ_E_ARG;
  *out = nullptr;
  const char *b = json, *e = json + len;
  Cursor c{b, b, e};
  if (!eat(c, '[')) return KMZ_E_UNSUPPORTED;
  ws(c);
  bool empty = false;
  if (c.p < c.e && *c.p == ']') {  // no traces
    empty = true;
    ++c.p;
    ws(c);
    if (c.p != c.e) return KMZ_E_UNSUPPORTED;
  }
  // split by bytes at candidate trace boundaries; each range is parsed by its
  // own thread and the split is confirmed by the range before it landing
  // exactly on it.  An unconfirmed split (a pattern inside a string) reparses
  // the batch on one thread.
  std::vector<const char *> starts{c.p};
  const uint64_t bytes = (uint64_t)(e - c.p);
  int T = threads <= 0 ? std::min(16, (int)std::thread::hardware_concurrency()) : threads;
  T = std::max(1, std::min<int>(T, (int)(bytes >> 20)));  // >= 1 MiB a thread
  if (empty) T = 0;
  for (int t = 1; t < T; ++t) {
    const char *q = next_boundary(c.p + bytes * (uint64_t)t / (uint64_t)T, e);
    if (q && q > starts.back()) starts.push_back(q);
  }
  const int R = T ? (int)starts.size() : 0;
  std::vector<Local> ls((size_t)R);
  std::vector<char> aligned((size_t)R, 1);
  {
    std::vector<std::thread> pool;
    for (int t = 0; t < R; ++t) {
      auto run = [&, t]() {
        aligned[t] = parse_range(b, starts[t], t + 1 < R ? starts[t + 1] : e, e, t + 1 == R, ls[t]);
      };
      if (t + 1 == R)
        run();
      else
        pool.emplace_back(run);
    }
    for (auto &th : pool) th.join();
  }
  bool ok = true;
  for (int t = 0; t < R; ++t) ok = ok && aligned[t];
  if (!ok && R > 1) {  // a split was not a trace boundary: one range
    ls.assign(1, Local{});
    parse_range(b, starts[0], e, e, true, ls[0]);
  }
  for (const Local &l : ls)
    if (l.bad) return KMZ_E_UNSUPPORTED;
  // merge the interning tables in thread order (first occurrence order overall)
  kmz_zipkin_batch *r = (kmz_zipkin_batch *)calloc(1, sizeof(kmz_zipkin_batch));
  if (!r) return KMZ_E_ARG;
  Interner<NFIELD> gs;
  Interner<1> gt;
  uint64_t n = 0;
  for (Local &l : ls) {
    std::vector<uint32_t> rs(l.shapes.items.size()), rt(l.statuses.items.size());
    for (size_t i = 0; i < rs.size(); ++i) rs[i] = gs.put(b, l.shapes.items[i].data(), l.shapes.hs[i]);
    for (size_t i = 0; i < rt.size(); ++i) rt[i] = gt.put(b, l.statuses.items[i].data(), l.statuses.hs[i]);
    for (auto &x : l.shape) x = rs[x];
    for (auto &x : l.status) x = rt[x];
    n += l.sid.size();
  }
  std::vector<Slice> shape_f, status_f;
  for (const auto &a : gs.items) shape_f.insert(shape_f.end(), a.begin(), a.end());
  for (const auto &a : gt.items) status_f.push_back(a[0]);
  r->n = n;
  r->span_id = copy_out(ls, &Local::sid, n);
  r->parent_id = copy_out(ls, &Local::pid, n);
  r->kind = copy_out(ls, &Local::kind, n);
  r->shape = copy_out(ls, &Local::shape, n);
  r->status = copy_out(ls, &Local::status, n);
  r->duration = copy_out(ls, &Local::dur, n);
  r->timestamp = copy_out(ls, &Local::ts, n);
  r->n_shapes = (uint32_t)(shape_f.size() / NFIELD);
  r->n_statuses = (uint32_t)status_f.size();
  r->shape_fields = (uint64_t *)malloc(std::max<size_t>(1, shape_f.size()) * 2 * sizeof(uint64_t));
  r->status_fields = (uint64_t *)malloc(std::max<size_t>(1, status_f.size()) * 2 * sizeof(uint64_t));
  if (!r->span_id || !r->parent_id || !r->kind || !r->shape || !r->status || !r->duration || !r->timestamp ||
      !r->shape_fields || !r->status_fields) {
    kmz_zipkin_free(r);
    return KMZ_E_ARG;
  }
  for (size_t i = 0; i < shape_f.size(); ++i) {
    r->shape_fields[2 * i] = shape_f[i].off;
    r->shape_fields[2 * i + 1] = shape_f[i].len == ABSENT ? KMZ_JSON_ABSENT : shape_f[i].len;
  }
  for (size_t i = 0; i < status_f.size(); ++i) {
    r->status_fields[2 * i] = status_f[i].off;
    r->status_fields[2 * i + 1] = status_f[i].len == ABSENT ? KMZ_JSON_ABSENT : status_f[i].len;
  }
  *out = r;
  return KMZ_OK;
}

void kmz_zipkin_free(kmz_zipkin_batch *r) {
  if (!r) return;
  free(r->span_id);
  free(r->parent_id);
  free(r->kind);
  free(r->shape);
  free(r->status);
  free(r->duration);
  free(r->timestamp);
  free(r->shape_fields);
  free(r->status_fields);
  free(r);
}

}  // extern "C"
