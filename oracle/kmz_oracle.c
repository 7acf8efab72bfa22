/*
 * kmz_oracle.c -- CPU ORACLE (test infrastructure only; never shipped, never
 * on the product path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it (oracle/_build/libkmz_oracle.so).
 *
 * Plain-C, single-threaded restatement of the reference's hot path on the
 * columnar batch (the same kmz_spans layout the engine consumes):
 *
 *   oracle_stats  Traces.toRealTimeData / combineLogsToRealtimeData (rows =
 *                 every SERVER occurrence, Traces.ts:28-31,69-72) followed by
 *                 RealtimeDataList.toCombinedRealtimeData: grouping by endpoint
 *                 then status in first-occurrence order (RealtimeDataList.ts:23-45),
 *                 SEQUENTIAL Welford in row order (RealtimeDataList.ts:100-118),
 *                 ToPrecise (Utils.ts:311-313), latestTimestamp = max (63-64).
 *   oracle_deps   Traces.toEndpointDependencies (Traces.ts:112-211): a global
 *                 span-id Map with first-position/last-value semantics, the
 *                 parent walk skipping CLIENT spans, per-row upper/lower maps
 *                 keyed (endpoint, distance) with first-position/last-value
 *                 dedup, lastUsageTimestamp = max(ts/1000) over row endpoints
 *                 and every deduplicated nested entry (Traces.ts:192-208).
 *                 Reduced outputs: the (anc_ep, desc_ep, distance, on) key set,
 *                 per-endpoint lastUsage / first row / isDependedByExternal of
 *                 that first row (= EndpointDependencies.combineWith on an empty
 *                 list, EndpointDependencies.ts:508-541).
 *
 * Identity strings are resolved upstream into dense endpoint ids per shape
 * (the Python oracle kmz_oracle.py restates ExplodeUrl / ToEndpointInfo and is
 * pinned on the reference's golden vectors; this file is pinned against it).
 * Compiled with -O2 -ffp-contract=off: fp64 as V8 evaluates it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NONE32 0xFFFFFFFFu
#define KIND_SERVER 1
#define KIND_CLIENT 2

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* Math.round (ties toward +inf) and Utils.ToPrecise */
static double js_round(double x) {
  double r = floor(x);
  if (x - r >= 0.5) r += 1.0;
  return r;
}
double oracle_to_precise(double x) { return js_round((x + 2.220446049250313e-16) * 1e14) / 1e14; }

/* ------------------------------------------------------------------------ */
/* stats                                                                     */
/* ------------------------------------------------------------------------ */
/* out arrays are dense [n_ep * n_status]; order_ep[e] / order_g[g] receive the
 * first row index of the endpoint / group (UINT64_MAX when absent). */
int oracle_stats(uint64_t n, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                 const uint32_t *dur, const int64_t *ts, const uint32_t *ep_of_shape, uint32_t n_ep, uint32_t n_status,
                 uint64_t *cnt, double *mean_out, double *cv_out, int64_t *latest, uint64_t *first) {
  uint64_t G = (uint64_t)n_ep * n_status;
  double *mean = (double *)calloc(G ? G : 1, sizeof(double));
  double *m2 = (double *)calloc(G ? G : 1, sizeof(double));
  if (!mean || !m2) return -1;
  for (uint64_t g = 0; g < G; ++g) {
    cnt[g] = 0;
    first[g] = UINT64_MAX;
    latest[g] = INT64_MIN;
  }
  for (uint64_t i = 0; i < n; ++i) {
    if (kind[i] != KIND_SERVER) continue;
    uint64_t g = (uint64_t)ep_of_shape[shape[i]] * n_status + status[i];
    double x = (double)dur[i] / 1000.0; /* latency: t.duration / 1000 (Traces.ts:43) */
    uint64_t k = cnt[g];
    if (k == 0) first[g] = i;
    double old = mean[g];
    mean[g] += (x - mean[g]) / (double)(k + 1);
    m2[g] += (x - mean[g]) * (x - old);
    cnt[g] = k + 1;
    if (k == 0 || ts[i] > latest[g]) latest[g] = ts[i];
  }
  for (uint64_t g = 0; g < G; ++g) {
    if (!cnt[g]) {
      mean_out[g] = cv_out[g] = 0;
      continue;
    }
    double var = m2[g] / (double)cnt[g];
    double sd = sqrt(var);
    double cv = mean[g] != 0 ? sd / mean[g] : 0;
    mean_out[g] = oracle_to_precise(mean[g]);
    cv_out[g] = oracle_to_precise(cv);
  }
  free(mean);
  free(m2);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* a tiny open-addressing u64 -> u64 map (JS Map: first position, last value) */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t *key;
  uint64_t *v0, *v1; /* v0 = first position, v1 = last value */
  uint64_t cap, used;
} u64map;

static int map_init(u64map *m, uint64_t expect) {
  uint64_t cap = 16;
  while (cap < expect * 2 + 16) cap <<= 1;
  m->cap = cap;
  m->used = 0;
  m->key = (uint64_t *)calloc(cap, 8);
  m->v0 = (uint64_t *)malloc(cap * 8);
  m->v1 = (uint64_t *)malloc(cap * 8);
  return (m->key && m->v0 && m->v1) ? 0 : -1;
}
static void map_free(u64map *m) {
  free(m->key);
  free(m->v0);
  free(m->v1);
}
/* keys are stored +1 so that 0 marks an empty slot; key ~0 is not supported */
static uint64_t *map_slot(u64map *m, uint64_t key, int *found) {
  uint64_t k = key + 1, mask = m->cap - 1, p = mix64(k) & mask;
  while (m->key[p] && m->key[p] != k) p = (p + 1) & mask;
  *found = m->key[p] == k;
  return &m->key[p];
}
static uint64_t map_find(u64map *m, uint64_t key) {
  int f;
  uint64_t *s = map_slot(m, key, &f);
  return f ? (uint64_t)(s - m->key) : UINT64_MAX;
}
static int map_grow(u64map *m);
static uint64_t map_set(u64map *m, uint64_t key, uint64_t v, int *was_new) {
  if ((m->used + 1) * 2 > m->cap && map_grow(m)) return UINT64_MAX;
  int f;
  uint64_t *s = map_slot(m, key, &f);
  uint64_t p = (uint64_t)(s - m->key);
  if (!f) {
    *s = key + 1;
    m->v0[p] = v;
    m->used++;
  }
  m->v1[p] = v;
  *was_new = !f;
  return p;
}
static int map_grow(u64map *m) {
  u64map n;
  if (map_init(&n, m->cap)) return -1;
  for (uint64_t p = 0; p < m->cap; ++p)
    if (m->key[p]) {
      int f;
      uint64_t *s = map_slot(&n, m->key[p] - 1, &f);
      uint64_t q = (uint64_t)(s - n.key);
      *s = m->key[p];
      n.v0[q] = m->v0[p];
      n.v1[q] = m->v1[p];
      n.used++;
    }
  map_free(m);
  *m = n;
  return 0;
}

static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

/* ------------------------------------------------------------------------ */
/* dependencies                                                              */
/* ------------------------------------------------------------------------ */
/* Outputs:
 *   keys[*n_keys]      sorted unique anc_ep<<40 | desc_ep<<16 | d<<1 | on
 *   ep_last[e]         max over occurrences of timestamp/1000 (0 if none, as
 *                      endpointLastTimestampMap ?? 0)
 *   ep_first[e]        flatten index of the endpoint's first row (UINT64_MAX)
 *   ep_external[e]     isDependedByExternal of that first row
 *   row_last[r]        lastUsageTimestamp of row r (rows in map order)
 *   counts[0..3]       rows, relations, max depth, unique keys
 * Returns 0, -1 on allocation failure, -3 on a cyclic parent chain. */
int oracle_deps(uint64_t n, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind, const uint32_t *shape,
                const int64_t *ts, const uint32_t *dep_ep, uint32_t n_ep, uint64_t max_keys, uint64_t *keys,
                uint64_t *n_keys, double *ep_last, uint64_t *ep_first, uint8_t *ep_external, uint64_t *counts) {
  u64map ids;
  if (map_init(&ids, n)) return -1;
  int nw;
  for (uint64_t i = 0; i < n; ++i) map_set(&ids, sid[i], i, &nw); /* spanDependencyMap.set (117-123) */
  /* rows in map order = by first position */
  uint64_t nrows = 0;
  uint64_t *rows = (uint64_t *)malloc((n ? n : 1) * 16);
  if (!rows) return -1;
  for (uint64_t p = 0; p < ids.cap; ++p)
    if (ids.key[p] && kind[ids.v1[p]] == KIND_SERVER) {
      rows[2 * nrows] = ids.v0[p]; /* position */
      rows[2 * nrows + 1] = ids.v1[p];
      nrows++;
    }
  /* sort by position (pairs) */
  {
    uint64_t *tmp = (uint64_t *)malloc((nrows ? nrows : 1) * 8);
    uint64_t *val = (uint64_t *)malloc((n ? n : 1) * 8);
    if (!tmp || !val) return -1;
    for (uint64_t r = 0; r < nrows; ++r) {
      tmp[r] = rows[2 * r];
      val[rows[2 * r]] = rows[2 * r + 1];
    }
    qsort(tmp, nrows, 8, cmp_u64);
    for (uint64_t r = 0; r < nrows; ++r) {
      rows[2 * r] = tmp[r];
      rows[2 * r + 1] = val[tmp[r]];
    }
    free(tmp);
    free(val);
  }
  for (uint32_t e = 0; e < n_ep; ++e) {
    ep_last[e] = 0;
    ep_first[e] = UINT64_MAX;
    ep_external[e] = 0;
  }
  /* walk (128-143); per row: upper list (ancestor idx, depth) in walk order,
   * lower maps as (ancestor -> list of (descendant row, depth)) */
  uint64_t rel = 0, maxd = 0, relcap = n + 16;
  uint64_t *ra = (uint64_t *)malloc(relcap * 8), *rd = (uint64_t *)malloc(relcap * 8), *rdep = (uint64_t *)malloc(relcap * 8);
  uint64_t *row_off = (uint64_t *)malloc((nrows + 1) * 8);
  if (!ra || !rd || !rdep || !row_off) return -1;
  for (uint64_t r = 0; r < nrows; ++r) {
    uint64_t s = rows[2 * r + 1];
    row_off[r] = rel;
    uint64_t p = pid[s], depth = 1, steps = 0;
    while (p) {
      if (++steps > (1u << 20)) return -3;
      uint64_t slot = map_find(&ids, p);
      if (slot == UINT64_MAX) break;
      uint64_t q = ids.v1[slot];
      if (kind[q] == KIND_CLIENT) {
        p = pid[q];
        continue;
      }
      if (rel == relcap) {
        relcap *= 2;
        ra = (uint64_t *)realloc(ra, relcap * 8);
        rd = (uint64_t *)realloc(rd, relcap * 8);
        rdep = (uint64_t *)realloc(rdep, relcap * 8);
        if (!ra || !rd || !rdep) return -1;
      }
      ra[rel] = q;
      rd[rel] = s;
      rdep[rel] = depth;
      rel++;
      p = pid[q];
      depth++;
    }
    if (depth - 1 > maxd) maxd = depth - 1;
  }
  row_off[nrows] = rel;

  /* edge keys (upperMap/lowerMap keys carry (endpoint name, distance); the
   * dependingOn side exists only for ancestors that are rows, i.e. SERVER) */
  uint64_t nk = 0;
  uint64_t *kk = (uint64_t *)malloc((rel ? rel : 1) * 8);
  if (!kk) return -1;
  for (uint64_t x = 0; x < rel; ++x) {
    uint64_t q = ra[x], s = rd[x];
    kk[nk++] = ((uint64_t)dep_ep[shape[q]] << 40) | ((uint64_t)dep_ep[shape[s]] << 16) | (rdep[x] << 1) |
               (kind[q] == KIND_SERVER ? 1u : 0u);
  }
  qsort(kk, nk, 8, cmp_u64);
  uint64_t u = 0;
  for (uint64_t x = 0; x < nk; ++x)
    if (u == 0 || kk[x] != kk[u - 1]) kk[u++] = kk[x];
  if (keys) {
    if (u > max_keys) {  /* the caller's key buffer is too small: report the size needed */
      *n_keys = u;
      free(kk);
      return -4;
    }
    memcpy(keys, kk, u * 8);
  }
  *n_keys = u;
  free(kk);

  /* lastUsageTimestamp (192-208): row endpoints, every dependingBy entry,
   * deduplicated dependingOn entries (key (desc endpoint, distance) -> the
   * LAST descendant with that key, in outer-loop order).  The deduplicated
   * value is itself a row endpoint, so its timestamp is covered by the rows;
   * the max over {rows} U {ancestors} is therefore exact. */
  for (uint64_t r = 0; r < nrows; ++r) {
    uint64_t s = rows[2 * r + 1];
    uint32_t e = dep_ep[shape[s]];
    double t = (double)ts[s] / 1000.0;
    if (t > ep_last[e]) ep_last[e] = t;
    if (ep_first[e] == UINT64_MAX) {
      ep_first[e] = rows[2 * r];
      ep_external[e] = row_off[r + 1] == row_off[r];
    }
  }
  for (uint64_t x = 0; x < rel; ++x) {
    uint64_t q = ra[x];
    uint32_t e = dep_ep[shape[q]];
    double t = (double)ts[q] / 1000.0;
    if (t > ep_last[e]) ep_last[e] = t;
  }
  counts[0] = nrows;
  counts[1] = rel;
  counts[2] = maxd;
  counts[3] = u;
  free(ra);
  free(rd);
  free(rdep);
  free(row_off);
  free(rows);
  map_free(&ids);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* entry order of the reduced graph                                          */
/* ------------------------------------------------------------------------ */
/* EndpointDependencies([]).combineWith(traces.toEndpointDependencies()).trim()
 * in columnar form (EndpointDependencies.ts:91-112, 499-542 over the per-row
 * lists of Traces.ts:145-190).  The merged row of endpoint e is e's first row
 * with, appended in row order, every entry of e's later rows whose
 * (endpoint name, distance) it has not seen; within one row:
 *   dependingBy = the walk's ancestors in distance order (upperMap),
 *   dependingOn = the rows whose walk reached it, in row order, deduplicated
 *                 by (name, distance): first position, LAST value (lowerMap).
 * One record per entry of the merged graph (sequential first-seen rules):
 *   key   = anc_ep<<40 | desc_ep<<16 | distance<<1 | side
 *           (side 0: dependingBy entry of desc_ep's row, 1: dependingOn entry
 *            of anc_ep's row)
 *   row   = position of the row that contributed it (the first row of the
 *           merged row's endpoint having that entry)
 *   pos   = side 0: = row; side 1: position of the first descendant row
 *   span  = the span whose ToEndpointInfo the entry carries (side 0: the
 *           ancestor at `distance` in that row's walk; side 1: the last
 *           descendant row with the entry's key in that row's lowerMap)
 *   ts, shape of `span`
 * row_ts[e] / row_shape[e]: the value span of e's first row (INT64_MIN /
 * UINT32_MAX without a row).  Records come out in no particular order
 * (n_out = count; -4 when cap is too small, with the count needed). */
int oracle_dep_entries(uint64_t n, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind,
                       const uint32_t *shape, const int64_t *ts, const uint32_t *dep_ep, uint32_t n_ep, uint64_t cap,
                       uint64_t *out /* [cap][6] */, uint64_t *n_out, int64_t *row_ts, uint32_t *row_shape) {
  u64map ids;
  if (map_init(&ids, n)) return -1;
  int nw;
  for (uint64_t i = 0; i < n; ++i) map_set(&ids, sid[i], i, &nw);
  /* rows in map order: positions sorted, value span per position */
  uint64_t *val = (uint64_t *)malloc((n ? n : 1) * 8);
  uint8_t *isrow = (uint8_t *)calloc(n ? n : 1, 1);
  if (!val || !isrow) return -1;
  for (uint64_t p = 0; p < ids.cap; ++p)
    if (ids.key[p] && kind[ids.v1[p]] == KIND_SERVER) {
      val[ids.v0[p]] = ids.v1[p];
      isrow[ids.v0[p]] = 1;
    }
  for (uint32_t e = 0; e < n_ep; ++e) {
    row_ts[e] = INT64_MIN;
    row_shape[e] = UINT32_MAX;
  }
  u64map ent; /* entry key -> record index */
  if (map_init(&ent, 1024)) return -1;
  uint64_t m = 0;
  int rc = 0;
  for (uint64_t r = 0; r < n && rc == 0; ++r) {
    if (!isrow[r]) continue;
    uint64_t s = val[r];
    uint32_t d = dep_ep[shape[s]];
    if (row_shape[d] == UINT32_MAX) {
      row_ts[d] = ts[s];
      row_shape[d] = shape[s];
    }
    uint64_t p = pid[s], depth = 1, steps = 0;
    while (p) {
      if (++steps > (1u << 20)) {
        rc = -3;
        break;
      }
      uint64_t slot = map_find(&ids, p);
      if (slot == UINT64_MAX) break;
      uint64_t q = ids.v1[slot];
      if (kind[q] == KIND_CLIENT) {
        p = pid[q];
        continue;
      }
      uint64_t base = ((uint64_t)dep_ep[shape[q]] << 40) | ((uint64_t)d << 16) | (depth << 1);
      for (int side = 0; side < 2; ++side) {
        if (side == 1 && kind[q] != KIND_SERVER) break;
        uint64_t key = base | (uint64_t)side;
        uint64_t row = side ? ids.v0[slot] : r; /* the row the entry belongs to */
        uint64_t span = side ? s : q;
        uint64_t es = map_find(&ent, key), x;
        if (es == UINT64_MAX) {
          if (m < cap) {
            x = m;
            out[6 * x + 0] = key;
            out[6 * x + 1] = row;
            out[6 * x + 2] = span;
            out[6 * x + 3] = r; /* side 0: = row (== r); side 1: first descendant */
          }
          map_set(&ent, key, m, &nw);
          m++;
          continue;
        }
        x = ent.v1[es];
        if (x >= cap) continue;
        if (row < out[6 * x + 1]) { /* an earlier row of the same endpoint has it */
          out[6 * x + 1] = row;
          out[6 * x + 2] = span;
          out[6 * x + 3] = r;
        } else if (side && row == out[6 * x + 1]) {
          out[6 * x + 2] = span; /* lowerMap: last value */
        }
      }
      p = pid[q];
      depth++;
    }
  }
  for (uint64_t x = 0; x < m && x < cap; ++x) {
    uint64_t sp = out[6 * x + 2];
    out[6 * x + 4] = (uint64_t)ts[sp];
    out[6 * x + 5] = shape[sp];
  }
  *n_out = m;
  map_free(&ent);
  map_free(&ids);
  free(val);
  free(isrow);
  if (rc) return rc;
  return m > cap ? -4 : 0;
}
