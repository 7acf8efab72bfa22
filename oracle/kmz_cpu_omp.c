/*
 * kmz_cpu_omp.c -- ALL-CORE CPU BASELINE (test / benchmark infrastructure
 * only; never shipped, never on the product path).  bench.py's cpu_baseline
 * leg and tests/ load it (oracle/_build/libkmz_cpu_omp.so).
 *
 * An OpenMP restatement of the same path as kmz_oracle.c on the columnar
 * batch, for batches whose span ids are unique (the synthetic configs; a
 * repeated id returns -2 and the caller uses the sequential oracle):
 *
 *   omp_stats  Traces.combineLogsToRealtimeData + RealtimeDataList.
 *              toCombinedRealtimeData (Traces.ts:55-106, RealtimeDataList.ts:
 *              22-118): per-thread (group) accumulators of exact integer
 *              moments n, sum d, sum d^2 (128-bit), max timestamp, first row;
 *              merged, then mean = S1/(1000 n), cv = sqrt(n S2 - S1^2)/S1,
 *              ToPrecise (Utils.ts:311-313) -- within the north_star's 1e-9
 *              of the reference's sequential Welford.
 *   omp_deps   Traces.toEndpointDependencies reduced by EndpointDependencies
 *              combineWith/trim (Traces.ts:112-211, EndpointDependencies.ts:
 *              91-112,499-542): a concurrent span-id hash table, every span's
 *              first non-CLIENT ancestor, one walk per SERVER row emitting
 *              (ancestor ep, row ep, distance, ancestor is SERVER) keys into
 *              one concurrent hash set (one CAS per new key), per-endpoint lastUsage / first row /
 *              isDependedByExternal merged over threads.  Same outputs as
 *              oracle_deps.
 */
#include <math.h>
#include <omp.h>
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
static double js_round(double x) {
  double r = floor(x);
  if (x - r >= 0.5) r += 1.0;
  return r;
}
static double to_precise(double x) { return js_round((x + 2.220446049250313e-16) * 1e14) / 1e14; }

int omp_threads(void) { return omp_get_max_threads(); }

/* ---- stats ---------------------------------------------------------------- */
typedef struct {
  uint64_t cnt, s1;
  unsigned __int128 s2;
  int64_t latest;
  uint64_t first;
} acc_t;

int omp_stats(uint64_t n, const uint8_t *kind, const uint32_t *shape, const uint16_t *status, const uint32_t *dur,
              const int64_t *ts, const uint32_t *ep_of_shape, uint32_t n_ep, uint32_t n_status, uint64_t *cnt,
              double *mean_out, double *cv_out, int64_t *latest, uint64_t *first) {
  const uint64_t G = (uint64_t)n_ep * n_status;
  const int T = omp_get_max_threads();
  acc_t *a = (acc_t *)malloc((size_t)T * (G ? G : 1) * sizeof(acc_t));
  if (!a) return -1;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    acc_t *my = a + (size_t)t * G;
    for (uint64_t g = 0; g < G; ++g) {
      my[g].cnt = my[g].s1 = 0;
      my[g].s2 = 0;
      my[g].latest = INT64_MIN;
      my[g].first = UINT64_MAX;
    }
#pragma omp for schedule(static)
    for (uint64_t i = 0; i < n; ++i) {
      if (kind[i] != KIND_SERVER) continue;
      const uint64_t g = (uint64_t)ep_of_shape[shape[i]] * n_status + status[i];
      const uint64_t d = dur[i];
      acc_t *x = &my[g];
      if (x->cnt == 0) x->first = i; /* static schedule: a thread's rows ascend */
      x->cnt++;
      x->s1 += d;
      x->s2 += (unsigned __int128)(d * d);
      if (ts[i] > x->latest) x->latest = ts[i];
    }
#pragma omp for schedule(static)
    for (uint64_t g = 0; g < G; ++g) {
      uint64_t c = 0, s1 = 0, f = UINT64_MAX;
      unsigned __int128 s2 = 0;
      int64_t lt = INT64_MIN;
      for (int u = 0; u < T; ++u) {
        const acc_t *x = &a[(size_t)u * G + g];
        c += x->cnt;
        s1 += x->s1;
        s2 += x->s2;
        if (x->latest > lt) lt = x->latest;
        if (x->first < f) f = x->first;
      }
      cnt[g] = c;
      first[g] = f;
      latest[g] = lt;
      if (!c) {
        mean_out[g] = cv_out[g] = 0;
        continue;
      }
      const unsigned __int128 r = (unsigned __int128)c * s2 - (unsigned __int128)s1 * s1;
      const double mean = (double)s1 / ((double)c * 1000.0);
      const double num = (double)(uint64_t)(r >> 64) * 18446744073709551616.0 + (double)(uint64_t)r;
      mean_out[g] = to_precise(mean);
      cv_out[g] = to_precise(s1 ? sqrt(num) / (double)s1 : 0.0);
    }
  }
  free(a);
  return 0;
}

/* ---- dependencies ---------------------------------------------------------- */
static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

int omp_deps(uint64_t n, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind, const uint32_t *shape,
             const int64_t *ts, const uint32_t *dep_ep, uint32_t n_ep, uint64_t max_keys, uint64_t *keys,
             uint64_t *n_keys, double *ep_last, uint64_t *ep_first, uint8_t *ep_external, uint64_t *counts) {
  const int T = omp_get_max_threads();
  uint64_t cap = 1024;
  while (cap < 2 * n + 16) cap <<= 1;
  uint64_t *tk = (uint64_t *)calloc(cap, 8);
  uint32_t *tv = (uint32_t *)malloc(cap * 4);
  uint32_t *cparent = (uint32_t *)malloc((n ? n : 1) * 4);
  int64_t *tlast = (int64_t *)malloc((size_t)T * (n_ep ? n_ep : 1) * 8);
  uint64_t *tfirst = (uint64_t *)malloc((size_t)T * (n_ep ? n_ep : 1) * 8);
  uint64_t *tc = (uint64_t *)calloc((size_t)T * 3, 8);
  if (!tk || !tv || !cparent || !tlast || !tfirst || !tc) return -1;
  int dup = 0, cyc = 0, oom = 0;
  const uint64_t mask = cap - 1;
  /* spanDependencyMap (Traces.ts:117-123): concurrent inserts, ids + 1 (0 = empty) */
#pragma omp parallel for schedule(static) num_threads(T) reduction(| : dup)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t k = sid[i] + 1;
    uint64_t p = mix64(k) & mask;
    for (;;) {
      uint64_t cur = 0;
      if (__atomic_compare_exchange_n(&tk[p], &cur, k, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
        tv[p] = (uint32_t)i;
        break;
      }
      if (cur == k) {
        dup = 1; /* a repeated id: first-position/last-value semantics, sequential oracle */
        break;
      }
      p = (p + 1) & mask;
    }
  }
  if (dup) {
    free(tk), free(tv), free(cparent), free(tlast), free(tfirst), free(tc);
    return -2;
  }
  /* first non-CLIENT ancestor of every span (Traces.ts:131-137) */
#pragma omp parallel for schedule(static) num_threads(T) reduction(| : cyc)
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t p = pid[i];
    uint32_t r = NONE32;
    for (uint32_t hops = 0; p; ++hops) {
      if (hops > (1u << 20)) {
        cyc = 1;
        break;
      }
      const uint64_t k = p + 1;
      uint64_t s = mix64(k) & mask;
      while (tk[s] && tk[s] != k) s = (s + 1) & mask;
      if (!tk[s]) break;
      const uint32_t j = tv[s];
      if (kind[j] != KIND_CLIENT) {
        r = j;
        break;
      }
      p = pid[j];
    }
    cparent[i] = r;
  }
  if (cyc) return -3;
  /* one walk per SERVER row (Traces.ts:128-143) -> keys (145-180), into one
   * concurrent set (a key is inserted by one CAS; most rows find theirs) */
  uint64_t kcap = 1u << 16;
  while (kcap < 4 * n + 16) kcap <<= 1; /* distinct keys <= 2n at load <= 1/2 (config 5: ~n/2) */
  uint64_t *kset_sh = (uint64_t *)calloc(kcap, 8);
  if (!kset_sh) return -1;
  const uint64_t kmask = kcap - 1;
#pragma omp parallel num_threads(T) reduction(| : cyc, oom)
  {
    const int t = omp_get_thread_num();
    int64_t *ml = tlast + (size_t)t * n_ep;
    uint64_t *mf = tfirst + (size_t)t * n_ep;
    for (uint32_t e = 0; e < n_ep; ++e) {
      ml[e] = INT64_MIN;
      mf[e] = UINT64_MAX;
    }
    uint64_t rows = 0, rel = 0, maxd = 0;
#pragma omp for schedule(static)
    for (uint64_t s = 0; s < n; ++s) {
      if (kind[s] != KIND_SERVER) continue;
      const uint32_t es = dep_ep[shape[s]];
      ++rows;
      if (ts[s] > ml[es]) ml[es] = ts[s];
      uint64_t d = 0;
      for (uint32_t cur = cparent[s]; cur != NONE32; cur = cparent[cur]) {
        if (++d > (1u << 20)) {
          cyc = 1;
          break;
        }
        const uint32_t ea = dep_ep[shape[cur]];
        const uint64_t key = ((uint64_t)ea << 40) | ((uint64_t)es << 16) | (d << 1) | (kind[cur] == KIND_SERVER);
        uint64_t p = mix64(key) & kmask, z = 0;
        for (; z < kcap; ++z, p = (p + 1) & kmask) {
          uint64_t c = __atomic_load_n(&kset_sh[p], __ATOMIC_RELAXED);
          if (c == key) break;
          if (c == 0) {
            if (__atomic_compare_exchange_n(&kset_sh[p], &c, key, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED) || c == key)
              break;
          }
        }
        if (z == kcap) oom = 1;
        if (ts[cur] > ml[ea]) ml[ea] = ts[cur];
      }
      rel += d;
      if (d > maxd) maxd = d;
      const uint64_t fr = (s << 1) | (cparent[s] != NONE32); /* first row, !external */
      if (fr < mf[es]) mf[es] = fr;
    }
    tc[3 * t] = rows;
    tc[3 * t + 1] = rel;
    tc[3 * t + 2] = maxd;
  }
  if (cyc) return -3;
  if (oom) return -1;
  /* compact + sort */
  uint64_t nk = 0;
  for (uint64_t p = 0; p < kcap; ++p) nk += kset_sh[p] != 0;
  uint64_t *kk = (uint64_t *)malloc(nk * 8 + 8);
  if (!kk) return -1;
  nk = 0;
  for (uint64_t p = 0; p < kcap; ++p)
    if (kset_sh[p]) kk[nk++] = kset_sh[p];
  free(kset_sh);
  qsort(kk, nk, 8, cmp_u64);
  const uint64_t u = nk;
  *n_keys = u;
  int rc = 0;
  if (keys) {
    if (u > max_keys)
      rc = -4;
    else
      memcpy(keys, kk, u * 8);
  }
#pragma omp parallel for schedule(static) num_threads(T)
  for (uint32_t e = 0; e < n_ep; ++e) {
    int64_t l = INT64_MIN;
    uint64_t f = UINT64_MAX;
    for (int t = 0; t < T; ++t) {
      if (tlast[(size_t)t * n_ep + e] > l) l = tlast[(size_t)t * n_ep + e];
      if (tfirst[(size_t)t * n_ep + e] < f) f = tfirst[(size_t)t * n_ep + e];
    }
    const double ms = l == INT64_MIN ? 0.0 : (double)l / 1000.0;
    ep_last[e] = ms > 0 ? ms : 0.0; /* Math.max(map ?? 0, ts / 1000) */
    ep_first[e] = f == UINT64_MAX ? UINT64_MAX : f >> 1;
    ep_external[e] = f == UINT64_MAX ? 0 : (uint8_t)((f & 1) == 0);
  }
  counts[0] = counts[1] = counts[2] = 0;
  for (int t = 0; t < T; ++t) {
    counts[0] += tc[3 * t];
    counts[1] += tc[3 * t + 1];
    if (tc[3 * t + 2] > counts[2]) counts[2] = tc[3 * t + 2];
  }
  counts[3] = u;
  free(kk), free(tk), free(tv), free(cparent), free(tlast), free(tfirst), free(tc);
  return rc;
}
