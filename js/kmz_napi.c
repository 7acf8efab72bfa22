/*
 * kmz_napi.c -- thin, context-aware Node N-API addon over the C ABI
 * (include/kmz.h).  This is the binding a KMamiz deployment loads from its
 * realtime worker thread (src/services/worker/RealtimeWorkerImpl.ts:37-72):
 * typed arrays in, typed arrays out, no per-span JS objects cross the seam.
 *
 * NAPI_MODULE_INIT makes the addon context aware, which Node requires for
 * worker_threads (SURVEY.md 8b "Threading").  No global state: every kmz_ctx
 * lives in a JS external with a finalizer.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/kmz.h"

#define CHECK(call)                                                      \
  do {                                                                   \
    if ((call) != napi_ok) {                                             \
      napi_throw_error(env, "KMZ_NAPI", "N-API call failed: " #call);    \
      return NULL;                                                       \
    }                                                                    \
  } while (0)

static const char *code_name(int rc) {
  switch (rc) {
    case KMZ_E_ARG: return "KMZ_E_ARG";
    case KMZ_E_HIP: return "KMZ_E_HIP";
    case KMZ_E_CYCLE: return "KMZ_E_CYCLE";
    case KMZ_E_ZERO_ID: return "KMZ_E_ZERO_ID";
    case KMZ_E_RANGE: return "KMZ_E_RANGE";
    case KMZ_E_OVERFLOW: return "KMZ_E_OVERFLOW";
    case KMZ_E_STATE: return "KMZ_E_STATE";
    case KMZ_E_UNSUPPORTED: return "KMZ_E_UNSUPPORTED";
    default: return "KMZ_E";
  }
}

static napi_value throw_rc(napi_env env, kmz_ctx *c, int rc) {
  napi_throw_error(env, code_name(rc), kmz_last_error(c));
  return NULL;
}

static void ctx_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  kmz_destroy((kmz_ctx *)data);
}

static kmz_ctx *get_ctx(napi_env env, napi_value v) {
  void *p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, "KMZ_E_ARG", "expected a kmz context");
    return NULL;
  }
  return (kmz_ctx *)p;
}

/* typed array property -> data pointer + element count (checks the type) */
static int typed_prop(napi_env env, napi_value obj, const char *name, napi_typedarray_type want, void **data,
                      size_t *len) {
  napi_value v;
  bool is_ta = false;
  napi_typedarray_type t;
  napi_value ab;
  size_t off;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return -1;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return -1;
  if (napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok) return -1;
  return t == want ? 0 : -1;
}

static uint32_t u32_prop(napi_env env, napi_value obj, const char *name) {
  napi_value v;
  uint32_t x = 0;
  if (napi_get_named_property(env, obj, name, &v) == napi_ok) napi_get_value_uint32(env, v, &x);
  return x;
}

/* create(device) -> context */
static napi_value js_create(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  int32_t dev = 0;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc > 0) napi_get_value_int32(env, argv[0], &dev);
  kmz_ctx *c = kmz_create(dev, NULL);
  if (!c) {
    napi_throw_error(env, "KMZ_E_HIP", "kmz_create failed: no HIP device (the engine has no CPU path)");
    return NULL;
  }
  CHECK(napi_create_external(env, c, ctx_finalize, NULL, &out));
  return out;
}

/* load(ctx, spans, shapes) -- spans: {span_id: BigUint64Array, parent_id:
 * BigUint64Array, kind: Uint8Array, shape: Uint32Array, status: Uint16Array,
 * duration: Uint32Array, timestamp: BigInt64Array, index_base: number};
 * shapes: {rt_ep, tag_ep, dep_ep: Uint32Array, n_rt_ep, n_tag_ep, n_dep_ep, n_status} */
static napi_value js_load(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  kmz_spans s;
  kmz_shapes sh;
  size_t n = 0, m;
  memset(&s, 0, sizeof s);
  memset(&sh, 0, sizeof sh);
  if (typed_prop(env, argv[1], "span_id", napi_biguint64_array, (void **)&s.span_id, &n) ||
      typed_prop(env, argv[1], "parent_id", napi_biguint64_array, (void **)&s.parent_id, &m) || m != n ||
      typed_prop(env, argv[1], "kind", napi_uint8_array, (void **)&s.kind, &m) || m != n ||
      typed_prop(env, argv[1], "shape", napi_uint32_array, (void **)&s.shape, &m) || m != n ||
      typed_prop(env, argv[1], "status", napi_uint16_array, (void **)&s.status, &m) || m != n ||
      typed_prop(env, argv[1], "duration", napi_uint32_array, (void **)&s.duration, &m) || m != n ||
      typed_prop(env, argv[1], "timestamp", napi_bigint64_array, (void **)&s.timestamp, &m) || m != n) {
    napi_throw_type_error(env, "KMZ_E_ARG", "spans: bad or mismatched typed-array columns");
    return NULL;
  }
  s.n = n;
  {
    napi_value v;
    double b = 0;
    if (napi_get_named_property(env, argv[1], "index_base", &v) == napi_ok) napi_get_value_double(env, v, &b);
    s.index_base = (uint64_t)b;
  }
  size_t k1, k2, k3;
  if (typed_prop(env, argv[2], "rt_ep", napi_uint32_array, (void **)&sh.rt_ep, &k1) ||
      typed_prop(env, argv[2], "tag_ep", napi_uint32_array, (void **)&sh.tag_ep, &k2) ||
      typed_prop(env, argv[2], "dep_ep", napi_uint32_array, (void **)&sh.dep_ep, &k3) || k1 != k2 || k1 != k3) {
    napi_throw_type_error(env, "KMZ_E_ARG", "shapes: bad identity tables");
    return NULL;
  }
  sh.n_shapes = (uint32_t)k1;
  sh.n_rt_ep = u32_prop(env, argv[2], "n_rt_ep");
  sh.n_tag_ep = u32_prop(env, argv[2], "n_tag_ep");
  sh.n_dep_ep = u32_prop(env, argv[2], "n_dep_ep");
  sh.n_status = u32_prop(env, argv[2], "n_status");
  int rc = kmz_load(c, &s, &sh, KMZ_MEM_HOST);
  if (rc) return throw_rc(env, c, rc);
  return NULL;
}

static napi_value js_run(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  uint32_t flags = 0;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  napi_get_value_uint32(env, argv[1], &flags);
  int rc = kmz_run(c, flags);
  if (rc) return throw_rc(env, c, rc);
  return NULL;
}

static napi_value set_u64(napi_env env, napi_value obj, const char *name, uint64_t v) {
  napi_value x;
  if (napi_create_double(env, (double)v, &x) != napi_ok) return NULL;
  napi_set_named_property(env, obj, name, x);
  return obj;
}

static napi_value js_info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  kmz_info i;
  int rc = kmz_get_info(c, &i);
  if (rc) return throw_rc(env, c, rc);
  CHECK(napi_create_object(env, &out));
  set_u64(env, out, "n_spans", i.n_spans);
  set_u64(env, out, "n_server", i.n_server);
  set_u64(env, out, "n_rows", i.n_rows);
  set_u64(env, out, "n_relations", i.n_relations);
  set_u64(env, out, "n_triples", i.n_triples);
  set_u64(env, out, "n_dups", i.n_dups);
  set_u64(env, out, "max_depth", i.max_depth);
  set_u64(env, out, "n_groups", i.n_groups);
  set_u64(env, out, "n_chains", i.n_chains);
  return out;
}

/* fresh ArrayBuffer of `bytes`, returns its data pointer */
static napi_value new_buffer(napi_env env, size_t bytes, void **data) {
  napi_value ab;
  if (napi_create_arraybuffer(env, bytes ? bytes : 8, data, &ab) != napi_ok) return NULL;
  return ab;
}

/* groups(ctx) -> ArrayBuffer of kmz_group[n_groups] (40-byte records) */
static napi_value js_groups(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  kmz_info i;
  int rc = kmz_get_info(c, &i);
  if (rc) return throw_rc(env, c, rc);
  void *d;
  napi_value ab = new_buffer(env, i.n_groups * sizeof(kmz_group), &d);
  if (!ab) return NULL;
  rc = kmz_get_groups(c, (kmz_group *)d, i.n_groups);
  if (rc) return throw_rc(env, c, rc);
  return ab;
}

/* endpoints(ctx, n_ep) -> ArrayBuffer of kmz_endpoint[n_ep] (24-byte records) */
static napi_value js_endpoints(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  uint32_t n_ep = 0;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  napi_get_value_uint32(env, argv[1], &n_ep);
  void *d;
  napi_value ab = new_buffer(env, (size_t)n_ep * sizeof(kmz_endpoint), &d);
  if (!ab) return NULL;
  int rc = kmz_get_endpoints(c, (kmz_endpoint *)d, n_ep);
  if (rc) return throw_rc(env, c, rc);
  return ab;
}

/* triples(ctx) -> BigUint64Array of unique edge keys (unordered) */
static napi_value js_triples(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  uint64_t n = 0;
  int rc = kmz_get_triples(c, NULL, 0, &n);
  if (rc) return throw_rc(env, c, rc);
  void *d;
  napi_value ab = new_buffer(env, n * 8, &d);
  if (!ab) return NULL;
  rc = kmz_get_triples(c, (uint64_t *)d, n, &n);
  if (rc) return throw_rc(env, c, rc);
  CHECK(napi_create_typedarray(env, napi_biguint64_array, n, ab, 0, &out));
  return out;
}

/* depEntries(ctx, n_dep) -> {entries: ArrayBuffer of kmz_dep_entry[m] (48-byte
 * records), rowTs: BigInt64Array(n_dep), rowShape: Uint32Array(n_dep)}: the
 * reduced graph of the last KMZ_RUN_DEPS | KMZ_RUN_DEP_ORDER run in its exact
 * entry order (kmz_get_dep_entries), i.e. EndpointDependencies([]).combineWith(
 * traces.toEndpointDependencies()).trim() without a per-row object */
static napi_value js_dep_entries(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out, v;
  uint32_t n_dep = 0;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  napi_get_value_uint32(env, argv[1], &n_dep);
  uint64_t m = 0;
  int rc = kmz_get_dep_entries(c, NULL, 0, &m, NULL, NULL, 0);
  if (rc) return throw_rc(env, c, rc);
  void *de, *dt, *ds;
  napi_value abe = new_buffer(env, m * sizeof(kmz_dep_entry), &de), abt = new_buffer(env, (size_t)n_dep * 8, &dt),
             abs = new_buffer(env, (size_t)n_dep * 4, &ds);
  if (!abe || !abt || !abs) return NULL;
  rc = kmz_get_dep_entries(c, (kmz_dep_entry *)de, m, &m, (int64_t *)dt, (uint32_t *)ds, n_dep);
  if (rc) return throw_rc(env, c, rc);
  CHECK(napi_create_object(env, &out));
  CHECK(napi_set_named_property(env, out, "entries", abe));
  CHECK(napi_create_typedarray(env, napi_bigint64_array, n_dep, abt, 0, &v));
  CHECK(napi_set_named_property(env, out, "rowTs", v));
  CHECK(napi_create_typedarray(env, napi_uint32_array, n_dep, abs, 0, &v));
  CHECK(napi_set_named_property(env, out, "rowShape", v));
  CHECK(napi_create_double(env, (double)m, &v));
  CHECK(napi_set_named_property(env, out, "n", v));
  return out;
}

/* serviceTail(ctx, {svc: Uint32Array, cls: Uint32Array, lsvc: Uint32Array,
 * n_svc, n_lsvc}) -> {stats: Uint32Array(n_svc * 8), byDist: Uint32Array,
 * nDist, hasIn: Uint8Array(n_ep)}: kmz_tail_map_set + kmz_tail_run +
 * kmz_tail_service_stats (the counters behind EndpointDependencies.
 * toServiceInstability / toServiceCoupling / toServiceEndpointCohesion and
 * RiskAnalyzer's relying factor, include/kmz.h) */
static napi_value js_service_tail(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out, v;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  void *svc, *cls, *lsvc;
  size_t n_ep, n_ep2, n_cls;
  if (argc < 2 || typed_prop(env, argv[1], "svc", napi_uint32_array, &svc, &n_ep) ||
      typed_prop(env, argv[1], "cls", napi_uint32_array, &cls, &n_ep2) ||
      typed_prop(env, argv[1], "lsvc", napi_uint32_array, &lsvc, &n_cls) || n_ep != n_ep2) {
    napi_throw_type_error(env, "KMZ_E_ARG", "serviceTail: {svc, cls, lsvc} Uint32Arrays expected");
    return NULL;
  }
  kmz_tail_map m = {(const uint32_t *)svc, (const uint32_t *)cls, (const uint32_t *)lsvc, (uint32_t)n_ep,
                    u32_prop(env, argv[1], "n_svc"), (uint32_t)n_cls, u32_prop(env, argv[1], "n_lsvc")};
  int rc = kmz_tail_map_set(c, &m);
  if (!rc) rc = kmz_tail_run(c, NULL, NULL);
  uint32_t nd = 0;
  if (!rc) rc = kmz_tail_service_stats(c, NULL, 0, NULL, 0, &nd);
  if (rc) return throw_rc(env, c, rc);
  void *ds, *dd, *dh;
  napi_value abs = new_buffer(env, (size_t)m.n_svc * 32, &ds), abd = new_buffer(env, (size_t)m.n_svc * nd * 4, &dd),
             abh = new_buffer(env, n_ep, &dh);
  if (!abs || !abd || !abh) return NULL;
  rc = kmz_tail_service_stats(c, (uint32_t *)ds, (uint64_t)m.n_svc * 8, (uint32_t *)dd, (uint64_t)m.n_svc * nd, &nd);
  if (!rc) rc = kmz_tail_get(c, NULL, 0, NULL, 0, (uint8_t *)dh, n_ep);
  if (rc) return throw_rc(env, c, rc);
  CHECK(napi_create_object(env, &out));
  CHECK(napi_create_typedarray(env, napi_uint32_array, (size_t)m.n_svc * 8, abs, 0, &v));
  CHECK(napi_set_named_property(env, out, "stats", v));
  CHECK(napi_create_typedarray(env, napi_uint32_array, (size_t)m.n_svc * nd, abd, 0, &v));
  CHECK(napi_set_named_property(env, out, "byDist", v));
  CHECK(napi_create_typedarray(env, napi_uint8_array, n_ep, abh, 0, &v));
  CHECK(napi_set_named_property(env, out, "hasIn", v));
  CHECK(napi_create_uint32(env, nd, &v));
  CHECK(napi_set_named_property(env, out, "nDist", v));
  return out;
}

/* spanLinks(ctx, n) -> {cparent: Uint32Array, rowpos: BigUint64Array} */
static napi_value js_span_links(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out, a, b;
  uint32_t n = 0;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  kmz_ctx *c = get_ctx(env, argv[0]);
  if (!c) return NULL;
  napi_get_value_uint32(env, argv[1], &n);
  void *d1, *d2;
  napi_value ab1 = new_buffer(env, (size_t)n * 4, &d1), ab2 = new_buffer(env, (size_t)n * 8, &d2);
  if (!ab1 || !ab2) return NULL;
  int rc = kmz_get_span_links(c, (uint32_t *)d1, (uint64_t *)d2, n);
  if (rc) return throw_rc(env, c, rc);
  CHECK(napi_create_typedarray(env, napi_uint32_array, n, ab1, 0, &a));
  CHECK(napi_create_typedarray(env, napi_biguint64_array, n, ab2, 0, &b));
  CHECK(napi_create_object(env, &out));
  napi_set_named_property(env, out, "cparent", a);
  napi_set_named_property(env, out, "rowpos", b);
  return out;
}

/* copy n elements of `bytes` each into a fresh typed array */
static napi_value copy_typed(napi_env env, napi_typedarray_type t, const void *src, size_t n, size_t bytes) {
  void *d;
  napi_value ab, out;
  if (!(ab = new_buffer(env, n * bytes, &d))) return NULL;
  if (n) memcpy(d, src, n * bytes);
  if (napi_create_typedarray(env, t, n, ab, 0, &out) != napi_ok) return NULL;
  return out;
}

/* (offset, length) pairs -> Float64Array, an absent property as length -1 */
static napi_value field_pairs(napi_env env, const uint64_t *f, size_t pairs) {
  void *d;
  napi_value ab, out;
  if (!(ab = new_buffer(env, pairs * 16, &d))) return NULL;
  double *x = (double *)d;
  for (size_t i = 0; i < pairs; ++i) {
    x[2 * i] = (double)f[2 * i];
    x[2 * i + 1] = f[2 * i + 1] == KMZ_JSON_ABSENT ? -1.0 : (double)f[2 * i + 1];
  }
  if (napi_create_typedarray(env, napi_float64_array, pairs * 2, ab, 0, &out) != napi_ok) return NULL;
  return out;
}

/* parseZipkin(buffer, threads) -> null (outside the fast path: parse it the
 * general way) or {n, span_id, parent_id, kind, shape, status, duration,
 * timestamp, shapeFields, statusFields}: kmz_parse_zipkin's columns, shape and
 * status indices into the raw-slice tables (7 and 1 (offset, length) pairs). */
static napi_value js_parse_zipkin(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out, v;
  int32_t threads = 0;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  void *data = NULL;
  size_t len = 0;
  bool is_buf = false;
  if (argc < 1 || napi_is_buffer(env, argv[0], &is_buf) != napi_ok || !is_buf ||
      napi_get_buffer_info(env, argv[0], &data, &len) != napi_ok) {
    napi_throw_type_error(env, "KMZ_E_ARG", "parseZipkin: expected a Buffer");
    return NULL;
  }
  if (argc > 1) napi_get_value_int32(env, argv[1], &threads);
  kmz_zipkin_batch *b = NULL;
  int rc = kmz_parse_zipkin((const char *)data, len, threads, &b);
  if (rc == KMZ_E_UNSUPPORTED) {
    CHECK(napi_get_null(env, &out));
    return out;
  }
  if (rc) {
    napi_throw_error(env, code_name(rc), "kmz_parse_zipkin failed (allocation)");
    return NULL;
  }
  const size_t n = b->n;
  napi_value cols[9];
  cols[0] = copy_typed(env, napi_biguint64_array, b->span_id, n, 8);
  cols[1] = copy_typed(env, napi_biguint64_array, b->parent_id, n, 8);
  cols[2] = copy_typed(env, napi_uint8_array, b->kind, n, 1);
  cols[3] = copy_typed(env, napi_uint32_array, b->shape, n, 4);
  cols[4] = copy_typed(env, napi_uint32_array, b->status, n, 4);
  cols[5] = copy_typed(env, napi_uint32_array, b->duration, n, 4);
  cols[6] = copy_typed(env, napi_bigint64_array, b->timestamp, n, 8);
  cols[7] = field_pairs(env, b->shape_fields, (size_t)b->n_shapes * 7);
  cols[8] = field_pairs(env, b->status_fields, b->n_statuses);
  kmz_zipkin_free(b);
  static const char *names[9] = {"span_id", "parent_id", "kind",     "shape",       "status",
                                 "duration", "timestamp", "shapeFields", "statusFields"};
  CHECK(napi_create_object(env, &out));
  for (int i = 0; i < 9; ++i) {
    if (!cols[i]) {
      napi_throw_error(env, "KMZ_NAPI", "parseZipkin: allocation failed");
      return NULL;
    }
    napi_set_named_property(env, out, names[i], cols[i]);
  }
  CHECK(napi_create_double(env, (double)n, &v));
  napi_set_named_property(env, out, "n", v);
  return out;
}

static void export_fn(napi_env env, napi_value exports, const char *name, napi_callback fn) {
  napi_value f;
  napi_create_function(env, name, NAPI_AUTO_LENGTH, fn, NULL, &f);
  napi_set_named_property(env, exports, name, f);
}

static void export_u32(napi_env env, napi_value exports, const char *name, uint32_t v) {
  napi_value x;
  napi_create_uint32(env, v, &x);
  napi_set_named_property(env, exports, name, x);
}

NAPI_MODULE_INIT() {
  export_fn(env, exports, "create", js_create);
  export_fn(env, exports, "load", js_load);
  export_fn(env, exports, "run", js_run);
  export_fn(env, exports, "info", js_info);
  export_fn(env, exports, "groups", js_groups);
  export_fn(env, exports, "endpoints", js_endpoints);
  export_fn(env, exports, "triples", js_triples);
  export_fn(env, exports, "spanLinks", js_span_links);
  export_fn(env, exports, "parseZipkin", js_parse_zipkin);
  export_fn(env, exports, "serviceTail", js_service_tail);
  export_fn(env, exports, "depEntries", js_dep_entries);
  export_u32(env, exports, "RUN_DEP_ORDER", KMZ_RUN_DEP_ORDER);
  export_u32(env, exports, "RUN_STATS_RT", KMZ_RUN_STATS_RT);
  export_u32(env, exports, "RUN_STATS_TAG", KMZ_RUN_STATS_TAG);
  export_u32(env, exports, "RUN_DEPS", KMZ_RUN_DEPS);
  export_u32(env, exports, "RUN_SPAN_LINKS", KMZ_RUN_SPAN_LINKS);
  export_u32(env, exports, "ABI_VERSION", (uint32_t)kmz_abi_version());
  return exports;
}
