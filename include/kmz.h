/*
 * kmz.h -- C ABI of the MI355X trace-processing engine (libkmz.so).
 *
 * Drop-in boundary for KMamiz's hot path (Zipkin span -> realtime data ->
 * combined stats + endpoint dependency graph).  Every entry point is plain C:
 * pointers and sizes only, no torch / HIP types in the signatures (streams are
 * passed as opaque `void*` = hipStream_t).
 *
 * What each call replaces in the reference (TypeScript, /root/reference):
 *
 *   kmz_load          new Traces(Trace[][])                  src/classes/Traces.ts:17-21
 *                     (the columnar form of Trace.ts:1-38, produced by the host
 *                      ingest: ids hex->u64, strings interned into "shapes")
 *   kmz_run(STATS_*)  Traces.toRealTimeData / combineLogsToRealtimeData
 *                     + RealtimeDataList.toCombinedRealtimeData
 *                                                            Traces.ts:27-106,
 *                                                            RealtimeDataList.ts:22-118
 *   kmz_run(DEPS)     Traces.toEndpointDependencies          Traces.ts:112-211
 *                     reduced through EndpointDependencies.combineWith/trim
 *                                                            EndpointDependencies.ts:91-112,499-563
 *   kmz_get_groups    CombinedRealtimeDataList rows (count, latestTimestamp,
 *                     latency.mean, latency.cv)              RealtimeDataList.ts:71-89
 *   kmz_get_endpoints per-endpoint lastUsageTimestamp, first row,
 *                     isDependedByExternal of the merged row Traces.ts:182-208,
 *                                                            EndpointDependencies.ts:508-541
 *   kmz_get_triples   the deduplicated (ancestor, descendant, distance) edge set
 *                     behind dependingBy / dependingOn       Traces.ts:128-180
 *   kmz_get_span_links per-span first-non-CLIENT ancestor + row position, from
 *                     which the host materialises the exact per-row JSON
 *                     (Traces.ts:145-190) at small batch sizes
 *
 * Ownership: the context owns its device buffers; results are copied into
 * caller buffers (host or device, as each call states).  Calls on one context
 * are not thread safe; contexts are independent (no global state besides the
 * HIP runtime).  Every call returns 0 on success or a negative KMZ_E* code;
 * kmz_last_error() gives a message.  (The reference's own failure modes:
 * a TypeError from ExplodeUrl on malformed names is raised by the host ingest;
 * the endless loop on cyclic parent chains, Traces.ts:131-142, becomes
 * KMZ_E_CYCLE.)
 */
#ifndef KMZ_H
#define KMZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMZ_ABI_VERSION 1

/* span kinds (Trace.kind) */
#define KMZ_KIND_OTHER 0u
#define KMZ_KIND_SERVER 1u
#define KMZ_KIND_CLIENT 2u

#define KMZ_NONE 0xFFFFFFFFu

/* error codes */
#define KMZ_OK 0
#define KMZ_E_ARG -1      /* bad argument / shape mismatch */
#define KMZ_E_HIP -2      /* HIP runtime error */
#define KMZ_E_CYCLE -3    /* cyclic parentId chain (reference would not terminate) */
#define KMZ_E_ZERO_ID -4  /* span_id 0 is reserved ("absent") */
#define KMZ_E_RANGE -5    /* shape / status / endpoint id out of range */
#define KMZ_E_OVERFLOW -6 /* internal table overflow (retried internally; surfaced if persistent) */
#define KMZ_E_STATE -7    /* call order (e.g. kmz_get_* before kmz_run) */
#define KMZ_E_RCCL -8     /* collective failed */
#define KMZ_E_UNSUPPORTED -9 /* input outside a fast path's domain: the caller takes the general path */

/* kmz_run flags */
#define KMZ_RUN_STATS_RT 1u  /* group by toRealTimeData identity (Traces.ts:32-46) */
#define KMZ_RUN_STATS_TAG 2u /* group by combineLogsToRealtimeData identity (Traces.ts:73-99) */
#define KMZ_RUN_DEPS 4u      /* dependency graph (Traces.ts:112-211) */
#define KMZ_RUN_SPAN_LINKS 8u/* keep per-span links for kmz_get_span_links */
#define KMZ_RUN_DEP_ORDER 16u /* with DEPS: the entry order of the reduced graph (kmz_get_dep_entries) */
/* with DEPS: no uniqueness certificate in the run (the window-join path,
 * whatever the ids).  Only for a caller that checks this batch's span ids for
 * repeats itself, over a superset of them -- the multi-GPU guard routes every
 * span id of every shard, its own included, to an owner that checks them
 * (kmz_route_ids_fixed + kmz_id_repeats_seg_begin): a repeat inside the shard
 * makes this run's dependency results wrong, and the guard's verdict sends
 * the merge to the exact unsharded pass (dist.merge_all). */
#define KMZ_RUN_NO_CERT 32u

/* where a kmz_load buffer lives */
#define KMZ_MEM_HOST 0
#define KMZ_MEM_DEVICE 1

typedef struct kmz_ctx kmz_ctx;

/* A batch of spans in flatten order (this._traces.flat(), Traces.ts:29). */
typedef struct kmz_spans {
  uint64_t n;
  const uint64_t *span_id;   /* Trace.id as u64, never 0 (host remaps)        */
  const uint64_t *parent_id; /* Trace.parentId, 0 = absent or "" (falsy)      */
  const uint8_t *kind;       /* KMZ_KIND_*                                    */
  const uint32_t *shape;     /* interned (name, tags) tuple                   */
  const uint16_t *status;    /* interned tags["http.status_code"]             */
  const uint32_t *duration;  /* Trace.duration, microseconds                  */
  const int64_t *timestamp;  /* Trace.timestamp, microseconds                 */
  uint64_t index_base;       /* global flatten index of span 0 (sharding)     */
} kmz_spans;

/* Per-shape identities, computed once per distinct shape on the host. */
typedef struct kmz_shapes {
  uint32_t n_shapes;
  const uint32_t *rt_ep;  /* shape -> toRealTimeData uniqueEndpointName id          */
  const uint32_t *tag_ep; /* shape -> combineLogsToRealtimeData uniqueEndpointName id */
  const uint32_t *dep_ep; /* shape -> ToEndpointInfo uniqueEndpointName id          */
  uint32_t n_rt_ep, n_tag_ep, n_dep_ep;
  uint32_t n_status;
} kmz_shapes;

/* One (endpoint x status) group of toCombinedRealtimeData, finalised. */
typedef struct kmz_group {
  uint64_t combined;        /* subGroup.length                                  */
  uint64_t first;           /* global index of the first span of the group      */
  int64_t latest_timestamp; /* max Trace.timestamp (us)                         */
  double mean;              /* ToPrecise(mean latency, ms)                      */
  double cv;                /* ToPrecise(coefficient of variation)              */
} kmz_group;

/* Per dependency endpoint (ToEndpointInfo uniqueEndpointName). */
typedef struct kmz_endpoint {
  int64_t last_ts;    /* max timestamp (us) over its occurrences, INT64_MIN if none */
  uint64_t first_row; /* global index of its first row, UINT64_MAX if no row      */
  uint32_t external;  /* isDependedByExternal of that first row                   */
  uint32_t has_row;
} kmz_endpoint;

typedef struct kmz_info {
  uint64_t n_spans;
  uint64_t n_server;    /* realtime rows                                  */
  uint64_t n_rows;      /* dependency rows (unique ids whose last value is SERVER) */
  uint64_t n_relations; /* (row, non-CLIENT ancestor) pairs = A            */
  uint64_t n_triples;   /* unique (anc_ep, desc_ep, distance, on) keys     */
  uint64_t n_dups;      /* span occurrences whose id was seen before       */
  uint64_t max_depth;
  uint64_t n_groups;    /* group slots = n_ep * n_status                    */
  uint32_t flags;       /* internal error bits                             */
  uint32_t path;        /* last dependency run: bit 0 window join (else global span table),
                           bit 1 chain walk k4_chain (else per-relation global walk k_walk),
                           bit 2 direct enumeration (else chain interning),
                           bit 3 k_walk redo after a chain-table wait ran out (F_SPIN),
                           bit 4 join and chain walk fused in one kernel (k_join_chain),
                           bit 5 chain interning by one workgroup per tile (k4_tile; else
                           the persistent k4_chain), bit 6 that tile kernel is k4_tile9 */
  uint64_t n_chains;    /* distinct interned ancestor chains (chain-interning path) */
} kmz_info;

/* With KMZ_HIPGRAPH=1 in the environment at kmz_create, runs of batches
 * below 2^23 spans are replayed from hipGraphs (a run whose launch sequence
 * repeats is captured once; off by default: slower than direct launches at a
 * 2 500-trace tick on MI355X).  How many runs were replayed so far on this
 * context, and how many graphs it holds (diagnostic). */
int kmz_get_graph_stats(kmz_ctx *ctx, uint64_t *launches, uint32_t *cached);

/* ---- host ingest: Zipkin JSON -> kmz_spans columns ---- */
/* Parses the Trace[][] JSON that ZipkinService.getTraceListFromZipkinByServiceName
 * returns (ZipkinService.ts:44-57; span shape Trace.ts:1-38) in flatten order
 * (Traces.ts:29).  Shapes are interned by the raw JSON text of `name` and the
 * six identity tags, statuses by that of tags["http.status_code"]; each comes
 * back as (byte offset, length) slices into `json` (length KMZ_JSON_ABSENT:
 * the property is missing), for the caller's once-per-shape identity rules.
 * Returns KMZ_E_UNSUPPORTED (nothing parsed) for input outside the fast path:
 * ids that are not 16 lowercase hex digits, non-integer or out-of-range
 * duration/timestamp, escaped keys or kinds, non-object tags.  threads <= 0:
 * the hardware threads, at most 16. */
#define KMZ_JSON_ABSENT 0xFFFFFFFFFFFFFFFFull
typedef struct kmz_zipkin_batch {
  uint64_t n;
  uint64_t *span_id, *parent_id; /* parent 0: absent, "" or null (falsy)        */
  uint8_t *kind;
  uint32_t *shape, *status;      /* ids into shape_fields / status_fields       */
  uint32_t *duration;
  int64_t *timestamp;
  uint32_t n_shapes, n_statuses;
  uint64_t *shape_fields;  /* [n_shapes][7][offset, length]: name, http.method, http.url,
                              istio.canonical_revision, istio.canonical_service,
                              istio.namespace, istio.mesh_id */
  uint64_t *status_fields; /* [n_statuses][offset, length] */
} kmz_zipkin_batch;
int kmz_parse_zipkin(const char *json, uint64_t len, int threads, kmz_zipkin_batch **out);
void kmz_zipkin_free(kmz_zipkin_batch *batch);

/* ---- device ingest: Zipkin JSON -> columns on the GPU ---- */
/* The same fast path as kmz_parse_zipkin, on the device: the JSON bytes
 * (host memory: copied to HBM; device memory: read in place, kept valid until
 * kmz_json_load) are scanned for the span objects and every span is parsed by
 * its own thread; span ids, parent ids, kinds, durations and timestamps land
 * in the context's columns.  Shapes and statuses are interned by the raw text
 * of their fields (hash + byte verification) in first-occurrence order, exactly
 * as kmz_parse_zipkin numbers them.  KMZ_E_UNSUPPORTED (nothing loaded) for
 * input outside the fast path, as kmz_parse_zipkin, or on a hash collision
 * between two distinct shapes: the caller then parses on the host. */
int kmz_json_parse(kmz_ctx *ctx, const char *json, uint64_t len, int mem, uint64_t *n_spans, uint32_t *n_shapes,
                   uint32_t *n_statuses);
/* the distinct raw shapes / statuses of the last kmz_json_parse, in the
 * kmz_zipkin_batch layout: [n_shapes][7][offset, length], [n_statuses][offset,
 * length] (length KMZ_JSON_ABSENT: property missing) */
int kmz_json_fields(kmz_ctx *ctx, uint64_t *shape_fields, uint64_t *status_fields);
/* make the parsed spans the loaded batch (as kmz_load): raw shape k becomes
 * shape_of_raw[k], raw status k status_of_raw[k] (< 65536); the identity
 * tables as kmz_load takes them.  The context remembers these ids by the raw
 * JSON text of each shape / status (kmz_json_known). */
int kmz_json_load(kmz_ctx *ctx, const uint32_t *shape_of_raw, const uint32_t *status_of_raw, const kmz_shapes *shapes,
                  uint64_t index_base);
/* Identities across batches (a realtime worker sees the same endpoints every
 * window): after kmz_json_parse, the id given in an earlier kmz_json_load to
 * the same raw text, per raw shape / status of this batch, or KMZ_NONE (new:
 * the caller runs the identity rules for those only).  Exact: keyed by the
 * raw bytes, not a hash.  kmz_json_forget drops what was remembered (the
 * caller's dictionary was reset). */
int kmz_json_known(kmz_ctx *ctx, uint32_t *shape_of_raw, uint32_t *status_of_raw);
int kmz_json_forget(kmz_ctx *ctx);

/* ---- lifecycle ---------------------------------------------------------- */
int kmz_abi_version(void);
/* stream: hipStream_t to launch on (NULL = the context creates its own). */
kmz_ctx *kmz_create(int device, void *stream);
void kmz_destroy(kmz_ctx *ctx);
const char *kmz_last_error(kmz_ctx *ctx);
int kmz_sync(kmz_ctx *ctx);

/* ---- input --------------------------------------------------------------- */
/* where: KMZ_MEM_HOST copies the arrays to HBM; KMZ_MEM_DEVICE borrows device
 * pointers (must stay valid until the next kmz_load / kmz_destroy). The shape
 * table is always host memory. */
int kmz_load(kmz_ctx *ctx, const kmz_spans *spans, const kmz_shapes *shapes, int where);

/* ---- compute (asynchronous on the context stream) ------------------------ */
int kmz_run(kmz_ctx *ctx, uint32_t flags);
/* kmz_run in two halves: _begin validates and enqueues the run (with its
 * read-back) and returns at once; _end waits for it, repeats it where a table
 * must grow or a seed change, and publishes its results.  Between the two the
 * caller may do host work (e.g. the previous batch's service-tail finish);
 * every other call on the context fails with KMZ_E_STATE until _end. */
int kmz_run_begin(kmz_ctx *ctx, uint32_t flags);
int kmz_run_end(kmz_ctx *ctx);

/* ---- results (synchronise the stream) ------------------------------------- */
int kmz_get_info(kmz_ctx *ctx, kmz_info *out);
/* finalised groups, dense [n_ep * n_status] (ep-major), of the last STATS run */
int kmz_get_groups(kmz_ctx *ctx, kmz_group *out, uint64_t cap);
int kmz_get_endpoints(kmz_ctx *ctx, kmz_endpoint *out, uint64_t cap);
/* unique edge keys, unordered: key = anc_ep<<40 | desc_ep<<16 | distance<<1 | on */
int kmz_get_triples(kmz_ctx *ctx, uint64_t *out, uint64_t cap, uint64_t *n_out);
/* the loaded batch's columns back in host memory (any pointer may be NULL);
 * e.g. after kmz_json_load, for the per-span host work of small batches */
int kmz_get_spans(kmz_ctx *ctx, uint64_t *span_id, uint64_t *parent_id, uint8_t *kind, uint32_t *shape,
                  uint16_t *status, uint32_t *duration, int64_t *timestamp, uint64_t cap);
/* per span: first non-CLIENT ancestor (KMZ_NONE if none) and, for rows, the
 * row's global first-occurrence index (KMZ_NONE if the span is not a row) */
int kmz_get_span_links(kmz_ctx *ctx, uint32_t *cparent, uint64_t *rowpos, uint64_t cap);
/* The three result sets of the last run in one call (one stream
 * synchronisation): what a binding returns from Traces.toRealTimeData()
 * .toCombinedRealtimeData() (Traces.ts:27-106, RealtimeDataList.ts:22-97) and
 * Traces.toEndpointDependencies() (Traces.ts:112-211).  Any pointer may be
 * NULL to skip that set; *n_triples receives the edge-key count either way.
 * Pinned (page-locked) output buffers copy fastest. */
int kmz_fetch(kmz_ctx *ctx, kmz_group *groups, uint64_t groups_cap, uint64_t *triples, uint64_t triples_cap,
              uint64_t *n_triples, kmz_endpoint *endpoints, uint64_t endpoints_cap);
/* kmz_fetch with only the USED groups (combined > 0), in ascending group id:
 * ids[k] is group k's index in the dense array, groups[k] its value.  The
 * toCombinedRealtimeData entries are exactly these (RealtimeDataList.ts:22-45
 * emits a group per (endpoint, status) that occurs); a small batch touches a
 * few percent of the (endpoint x status) space, so the dense copy was most of
 * a 2 500-trace tick's fetch.  *n_used receives the count (groups_cap 0 and
 * no other set: the count alone).  KMZ_E_UNSUPPORTED past 2^22 groups (use
 * kmz_fetch). */
int kmz_fetch_used(kmz_ctx *ctx, uint32_t *ids, kmz_group *groups, uint64_t groups_cap, uint64_t *n_used,
                   uint64_t *triples, uint64_t triples_cap, uint64_t *n_triples, kmz_endpoint *endpoints,
                   uint64_t endpoints_cap);
/* kmz_fetch in two halves, for a loop over consecutive batches: _begin takes
 * a device copy of the run's three result sets (on the run's stream, so the
 * next kmz_run may overwrite its own buffers at once) and queues their copies
 * to the host on a transfer stream of the context; _end waits for them and
 * fills `endpoints`.  The next batch's kernels run while the results of this
 * one cross PCIe.  The output buffers must stay valid and untouched until
 * _end; a _begin while one is open ends that one first.  *n_triples is set
 * by _begin. */
int kmz_fetch_begin(kmz_ctx *ctx, kmz_group *groups, uint64_t groups_cap, uint64_t *triples, uint64_t triples_cap,
                    uint64_t *n_triples, kmz_endpoint *endpoints, uint64_t endpoints_cap);
int kmz_fetch_end(kmz_ctx *ctx);

/* ---- reduced graph in exact order ------------------- */
/* The cache layer holds EndpointDependencies reduced to one merged row per
 * endpoint: EndpointDependencies([]).combineWith(traces.toEndpointDependencies())
 * .trim() (EndpointDependencies.ts:91-112, 499-542; Initializer.ts:92,
 * RealtimeWorkerImpl.ts:68-70, Cacheable/CEndpointDependencies.ts:46-48).
 * After kmz_run(KMZ_RUN_DEPS | KMZ_RUN_DEP_ORDER), one record per entry of it:
 *   key   anc_ep<<40 | desc_ep<<16 | distance<<1 | side
 *         side 0: a dependingBy entry of desc_ep's merged row (type CLIENT),
 *         side 1: a dependingOn entry of anc_ep's merged row (type SERVER)
 *   row   global first-occurrence index of the row that brought the entry
 *         into the merged row (the endpoint's first row having it)
 *   pos   its place in that row's list: side 1 the first descendant row's
 *         index (lowerMap insertion order); side 0 = row (upperMap is in
 *         distance order)
 *   span  global index of the span whose ToEndpointInfo the entry carries
 *         (side 0: the ancestor; side 1: the LAST descendant with the key)
 *   ts / shape of that span
 * A merged row lists its entries by (row, pos) for side 1 and (row, distance)
 * for side 0.  row_ts / row_shape[e]: the span of endpoint e's first row
 * (the merged row's `endpoint`; INT64_MIN / KMZ_NONE without a row).
 * out == NULL: *n_out only.  Records come in no particular order. */
typedef struct kmz_dep_entry {
  uint64_t key, row, span, pos;
  int64_t ts;
  uint32_t shape, pad;
} kmz_dep_entry;
int kmz_get_dep_entries(kmz_ctx *ctx, kmz_dep_entry *out, uint64_t cap, uint64_t *n_out, int64_t *row_ts,
                        uint32_t *row_shape, uint64_t row_cap);

/* ---- multi-GPU partials (traceId-sharded batches) ------------------------ */
/* Raw group partials: 6 arrays of n_groups u64, in this order:
 *   [0] count, [1] sum(dur), [2] sum(lo32(dur^2)), [3] sum(hi32(dur^2))  (SUM)
 *   [4] max(timestamp ^ 1<<63)                                           (MAX)
 *   [5] min(first global index)                                          (MIN)
 * Endpoint partials: 2 arrays of n_dep_ep u64:
 *   [0] max(timestamp ^ 1<<63)  (MAX), [1] min(first_row<<1 | !external) (MIN) */
int kmz_group_partials(kmz_ctx *ctx, void **dev_ptr, uint64_t *n_groups);
int kmz_endpoint_partials(kmz_ctx *ctx, void **dev_ptr, uint64_t *n_ep);
/* Copy partials between the context and a caller buffer (host or device
 * memory of the same GPU), for reductions done by the caller (e.g. RCCL via
 * torch.distributed).  which: KMZ_PART_*; direction 0 = export (ctx -> buf),
 * 1 = import (buf -> ctx; not for triples).  kmz_partials_size gives the word
 * count (u64) of each. */
#define KMZ_PART_GROUPS 0
#define KMZ_PART_ENDPOINTS 1
#define KMZ_PART_TRIPLES 2
int kmz_partials_size(kmz_ctx *ctx, int which, uint64_t *words);
int kmz_partials_copy(kmz_ctx *ctx, int which, void *buf, uint64_t words, int mem, int direction);
/* Union of edge-key sets across traceId shards (the dependency half of
 * EndpointDependencies.combineWith, EndpointDependencies.ts:91-112, over the
 * reduced form): inserts n keys (0 = padding, skipped; host or device memory
 * per `mem`) into this context's edge set after a KMZ_RUN_DEPS run;
 * kmz_get_triples / kmz_fetch / KMZ_PART_TRIPLES then return the union. */
int kmz_merge_triples(kmz_ctx *ctx, const uint64_t *keys, uint64_t n, int mem);
/* The same with the given keys REPLACING this context's edge set: the merge of
 * traceId shards whose span-id map crosses shards, where one rank re-ran the
 * dependency pass over the whole batch (dist.merge_all's exact fallback). */
int kmz_set_triples(kmz_ctx *ctx, const uint64_t *keys, uint64_t n, int mem);
/* re-finalise the groups after the partials were reduced in place */
int kmz_finalize(kmz_ctx *ctx);
/* host-side finalisation of one partial (same arithmetic as the device) */
void kmz_finalize_host(const uint64_t *partials, uint64_t n_groups, kmz_group *out);
/* out[i] = exp(in[i]) by the C library's exp, element by element: the host
 * finish of RiskAnalyzer's SigmoidAdj (Normalizer.ts:32-41) over the services
 * in one call instead of one interpreter call per service (the same libm exp
 * Python's math.exp calls, so the results are bit-identical) */
void kmz_host_exp(const double *in, double *out, uint64_t n);

/* ---- multi-GPU sharding guard ---------------------------- */
/* Sharding by whole traces equals the reference's global span map
 * (Traces.ts:117-123) only if no parent link crosses shards.  After a
 * KMZ_RUN_DEPS run on the window-join path: the parent ids of this batch's
 * spans whose parent is not in the batch (ids == NULL: count only; `mem`
 * says where ids lives).  KMZ_E_UNSUPPORTED on the span-table path (repeated
 * ids: sharding is not exact there anyway). */
int kmz_unresolved_parents(kmz_ctx *ctx, uint64_t *ids, uint64_t cap, uint64_t *n_out, int mem);
/* how many of the given ids (0 = padding) are span ids of the loaded batch */
int kmz_count_ids(kmz_ctx *ctx, const uint64_t *ids, uint64_t n, int mem, uint64_t *found);
/* The other half of the global span map (Traces.ts:117-123: a span id seen
 * twice collapses to one row, last value at the first position): ids that
 * repeat ACROSS shards.  kmz_route_ids writes the loaded batch's span ids,
 * each hashed by the certificate's bijection, grouped by owner rank
 * r = (hash >> 32) * world >> 32: rank r's values are out[o_r, o_r + counts[r]),
 * o_r = counts[0] + .. + counts[r-1] (out: n_spans values, host or device
 * memory per `mem`; counts: host, `world` entries, 1 <= world <= 1024).
 * After an all-to-all of those segments, kmz_id_repeats on what a rank
 * received sets *repeated = 1 if any value occurs twice, i.e. some span id
 * is in two shards (the uniqueness certificate over the values; exact).
 * KMZ_E_UNSUPPORTED when it cannot decide (more values than the certificate
 * plans for, or a bucket overflow): the caller checks another way. */
int kmz_route_ids(kmz_ctx *ctx, uint32_t world, uint64_t *out, uint64_t cap, int mem, uint64_t *counts);
int kmz_id_repeats(kmz_ctx *ctx, const uint64_t *vals, uint64_t n, int mem, uint32_t *repeated);
/* kmz_route_ids into fixed segments, with no host round trip: out holds
 * `world` segments of `seg` words; segment r's word 0 is the number of values
 * routed to rank r and its words 1 .. min(count, seg - 1) those values (a
 * count >= seg means the segment overflowed: the caller exchanges exactly).
 * With device memory the routing is only enqueued on the context's stream,
 * so an all-to-all of equal segments can be posted behind it at once
 * (dist.IdGuard; Traces.ts:117-123 is the semantics the check protects). */
int kmz_route_ids_fixed(kmz_ctx *ctx, uint32_t world, uint64_t seg, uint64_t *out, int mem);
/* kmz_route_ids_fixed folded into the next run (kmz_run / kmz_run_begin):
 * arms it, nothing is enqueued here.  The run writes the same fixed segments
 * into `out` (device memory, `world` * `seg` words) from its join's first
 * certificate pass when the run has no certificate of its own
 * (KMZ_RUN_NO_CERT) and world <= the pass's bins (64; 256 past ~10^8 spans),
 * otherwise by kmz_route_ids_fixed's own pass inside the run; either way it
 * records an event once the segments are complete (after the join, before
 * the walk), so the exchange can start while the rest of the run executes.
 * One-shot: the next run consumes it (a run repeated inside kmz_run_end does
 * not route again).  Replaces the separate routing pass the guard ran before
 * the run (the id_hash bins already computed there, Traces.ts:117-123). */
int kmz_route_ids_join(kmz_ctx *ctx, uint32_t world, uint64_t seg, uint64_t *out);
/* After kmz_run_begin of a run armed by kmz_route_ids_join: make `stream` (a
 * hipStream_t; NULL: the context's) wait for its routing.  *in_join (may be
 * NULL) = 1 when the join wrote the segments, 0 when the fallback pass did.
 * KMZ_E_STATE when the last run routed nothing. */
int kmz_route_wait(kmz_ctx *ctx, void *stream, int *in_join);
/* kmz_id_repeats over the fixed segments an all-to-all of
 * kmz_route_ids_fixed outputs delivered (device memory, `world` segments of
 * `seg` words as received), without compacting them first, ENQUEUED on
 * `stream` (a hipStream_t; NULL: the context's stream) -- the stream that
 * waits for the exchange, so that the check runs beside this rank's own run.
 * The segments stay untouched until kmz_id_repeats_seg_end, which waits for
 * it: *max_count = the largest count any source sent (>= seg: a segment
 * overflowed, *repeated is then 0 and meaningless: exchange exactly), else
 * *repeated as kmz_id_repeats.  One open check per context; kmz_id_repeats
 * is refused while it is open. */
int kmz_id_repeats_seg_begin(kmz_ctx *ctx, const uint64_t *segs, uint32_t world, uint64_t seg, void *stream);
int kmz_id_repeats_seg_end(kmz_ctx *ctx, uint32_t *repeated, uint64_t *max_count);

/* ---- traceId sharding (shard = h(traceId) mod G) ------------ */
/* The shard of a trace, from its traceId string (the reference dedups and
 * groups traces by t[0].traceId, RealtimeWorkerImpl.ts:17-27): canonical
 * 16/32-digit lowercase hex ids hash by value, any other string by its bytes. */
uint32_t kmz_trace_shard(const char *trace_id, uint64_t len, uint32_t world);
/* A shard that is not one contiguous range of the global flatten order
 * (Traces.ts:29): after kmz_load, give the runs of the local batch, local
 * index local_start[k] being global index global_start[k] (local_start
 * non-decreasing, local_start[0] = 0; an index maps through the last run
 * whose start is <= it, so empty runs may repeat a start).  Every index a
 * result reports (kmz_group.first, kmz_endpoint.first_row, the partials,
 * span links) is then global; index_base is ignored.  n_runs = 0: contiguous
 * again.  kmz_load resets it. */
int kmz_set_index_map(kmz_ctx *ctx, const uint64_t *local_start, const uint64_t *global_start, uint64_t n_runs);
/* the global flatten index of every loaded span (index_base + i, or through
 * the index map; n_spans values, host or device memory per `mem`) */
int kmz_get_global_index(kmz_ctx *ctx, uint64_t *out, uint64_t cap, int mem);

/* ---- service-level tail over the reduced edge set ---- */
/* Replaces the per-row scans of EndpointDependencies.toServiceDependencies
 * (EndpointDependencies.ts:369-470), whose link counts feed toServiceInstability
 * (614-641), toServiceCoupling / RiskAnalyzer.AbsoluteCriticalityOfServices
 * (643-657, RiskAnalyzer.ts:145-169), RiskAnalyzer.RelyingFactor (124-137) and
 * toServiceEndpointCohesion (565-612).  The host interns the strings:
 *   svc[e]   uniqueServiceName of dependency endpoint e (rows are grouped by it;
 *            also the consumer service of cohesion)
 *   cls[e]   the link identity of e: uniqueServiceName, method, labelName
 *            (EndpointDependencies.ts:419-421; labels from the host's label map)
 *   lsvc[c]  the linked service of link class c (the key's first three fields)
 * All ids < 2^24. */
typedef struct kmz_tail_map {
  const uint32_t *svc;  /* [n_ep] */
  const uint32_t *cls;  /* [n_ep] */
  const uint32_t *lsvc; /* [n_cls] */
  uint32_t n_ep, n_svc, n_cls, n_lsvc;
} kmz_tail_map;
/* one link detail of toServiceDependencies: service svc, linked service lsvc,
 * distance -> count / dependingBy / dependingOn (EndpointDependencies.ts:427-447) */
typedef struct kmz_tail_detail {
  uint32_t svc, lsvc, distance, count, depending_by, depending_on;
} kmz_tail_detail;
/* cohesion: service svc has `consumes` distinct endpoints that consumer
 * service `consumer` calls at distance 1 (EndpointDependencies.ts:569-596) */
typedef struct kmz_tail_pair {
  uint32_t svc, consumer, consumes;
} kmz_tail_pair;
/* upload the maps (host memory; kept until replaced) */
int kmz_tail_map_set(kmz_ctx *ctx, const kmz_tail_map *map);
/* run the tail over the context's current edge set (after KMZ_RUN_DEPS and
 * any kmz_merge_triples); synchronous, returns the result sizes */
int kmz_tail_run(kmz_ctx *ctx, uint64_t *n_details, uint64_t *n_pairs);
/* kmz_tail_run in two halves: _begin enqueues the tail on the context's
 * stream (no wait), _end waits for it (repeating it with larger tables when
 * one overflowed) and returns the result sizes.  Between them the host is
 * free (a step's fetch and host finish run while the GPU computes the tail).
 * The next kmz_run_begin may come before _end: its kernels follow the tail's
 * on the stream and _end waits for the tail alone (if the tail then has to be
 * repeated with larger tables, _end fails with KMZ_E_STATE: the run has
 * replaced its inputs).  kmz_tail_map_set and the tail's getters are refused
 * while a tail is open. */
int kmz_tail_begin(kmz_ctx *ctx);
int kmz_tail_end(kmz_ctx *ctx, uint64_t *n_details, uint64_t *n_pairs);
/* per-service counters of the last tail run, 8 u32 per service id:
 *   [0] linked services with dependingBy > 0, [1] with dependingOn > 0
 *       (toServiceInstability, EndpointDependencies.ts:618-628)
 *   [2] distance-1 details with dependingBy > 0 (AIS without the gateway +1),
 *   [3] distance-1 details with dependingOn > 0 (ADS)   (RiskAnalyzer.ts:150-166)
 *   [4] distance-1 consumer services, [5] sum of their consumes
 *       (toServiceEndpointCohesion, EndpointDependencies.ts:569-596)
 *   [6] endpoints with a row (totalEndpoints, EndpointDependencies.ts:566-573, 606)
 *   [7] 1 if some row has an empty dependingBy (a gateway, RiskAnalyzer.ts:155-158)
 * and by_dist[svc * n_dist + d] = sum of dependingBy at distance d
 * (RelyingFactor, RiskAnalyzer.ts:124-137).  *n_dist = 0 when some distance
 * exceeded the dense table (the caller then sums the details).  Copied back
 * by kmz_tail_run itself: no device synchronisation here. */
int kmz_tail_service_stats(kmz_ctx *ctx, uint32_t *stats, uint64_t scap, uint32_t *by_dist, uint64_t dcap,
                           uint32_t *n_dist);
/* per service id: the global index of its first row (UINT64_MAX: no row) --
 * toServiceDependencies' service order (EndpointDependencies.ts:372-384) */
int kmz_tail_service_first(kmz_ctx *ctx, uint64_t *first, uint64_t cap);

/* ---- RiskAnalyzer.RealtimeRisk's per-service sums (RiskAnalyzer.ts:18, 228-248) */
/* Over the finalised groups of the last stats run (after any multi-GPU merge):
 * the groups of stats endpoint e belong to service sid_of_ep[e]; is_5xx[s]
 * marks status id s as a 5xx.  Per service, over its groups with combined > 0:
 *   wsum  = sum(cv * combined), in ascending group index (bit-equal to the
 *           host's per-row sum in that order)
 *   count = sum(combined), err = sum(combined of 5xx groups)
 *   first = smallest first index (UINT64_MAX: no group) -- the service order */
typedef struct kmz_service_sum {
  double wsum, count, err;
  uint64_t first;
} kmz_service_sum;
int kmz_service_map_set(kmz_ctx *ctx, const uint32_t *sid_of_ep, uint32_t n_ep, uint32_t n_sid, const uint8_t *is_5xx,
                        uint32_t n_status);
int kmz_service_sums(kmz_ctx *ctx, kmz_service_sum *out, uint64_t cap);
/* kmz_service_sums in two halves (enqueue; wait and copy out), as the tail;
 * _end waits for the sums alone (a run may be enqueued in between) */
int kmz_service_sums_begin(kmz_ctx *ctx);
int kmz_service_sums_end(kmz_ctx *ctx, kmz_service_sum *out, uint64_t cap);
/* copy the results: details and pairs in no particular order; has_in[e] = 1
 * when endpoint e's merged row has a non-empty dependingBy */
int kmz_tail_get(kmz_ctx *ctx, kmz_tail_detail *details, uint64_t dcap, kmz_tail_pair *pairs, uint64_t pcap,
                 uint8_t *has_in, uint64_t hcap);

/* ---- pinned host memory for result buffers (fast D2H) ---------------------- */
void *kmz_host_alloc(uint64_t bytes);
void kmz_host_free(void *p);

/* ---- per-kernel timing (HIP events around each launch) ------------------- */
/* One id per kernel of the hot path (small helper launches are folded into the
 * kernel they serve), so bench.py can price each launch against the roofline. */
#define KMZ_K_MEMSET 0   /* memsets of the per-run workspace                     */
#define KMZ_K_BUILD 1    /* K1 span-id table build (repeated ids only)           */
#define KMZ_K_FIXUP 2    /* K1 duplicate-id fixup (repeated ids only)            */
#define KMZ_K_RESOLVE 3  /* K2 table resolve / window-join MISS + PEND fix-ups    */
#define KMZ_K_STATS 4    /* K3 k3_produce (or the one-pass LDS k_stats)           */
#define KMZ_K_WALK 5     /* K4 k4_chain alone (or the global k_walk for repeated ids) */
#define KMZ_K_FINAL 6    /* finalise, collapse, edge-set compaction               */
#define KMZ_K_JOIN 7     /* K2 k_join_window: parent join + CLIENT contraction    */
#define KMZ_K_CERT 8     /* uniqueness certificate pass 2 (k_cert_split)          */
#define KMZ_K_REDUCE 9   /* K3 k3_reduce + k3_combine                             */
#define KMZ_K_PEND 10    /* K4 chains whose ancestry leaves the LDS window        */
#define KMZ_K_CHECK 11   /* uniqueness certificate pass 3 (k_cert_check)          */
#define KMZ_K_SETTLE 12  /* K4 k_chain_settle: staged keys + deferred chain checks */
#define KMZ_K_TAIL 13    /* service tail: k_tail_links + k_tail_compact           */
#define KMZ_K_ORDER 14   /* entry order of the reduced graph (KMZ_RUN_DEP_ORDER)  */
#define KMZ_K_JSON 15    /* K1 on the device: kmz_json_parse's kernels            */
#define KMZ_K_JOINWALK 16 /* K2 + K4 fused: k_join_chain (join, contraction, chain walk) */
#define KMZ_K_COUNT 17
int kmz_set_profiling(kmz_ctx *ctx, int on);
/* time only the kernel ids whose bit is set in mask (1 << KMZ_K_*; 0 = off).
 * Each timed id costs an event pair on the stream, and each event record a
 * short pipeline gap before the next launch: a benchmark that prices one
 * kernel times only that one (bench.py).  While more than one id is timed,
 * runs keep every kernel on one stream (no side-stream overlap), so that each
 * kernel's time is its own. */
int kmz_set_profiling_mask(kmz_ctx *ctx, uint32_t mask);
/* ms[KMZ_K_COUNT] accumulated since the last reset, calls[KMZ_K_COUNT] */
int kmz_kernel_times(kmz_ctx *ctx, double *ms, uint64_t *calls, int reset);

/* ---- synthetic workload (BASELINE.json configs 2-5), generated in HBM ---- */
#define KMZ_SYNTH_BOOKINFO 2
#define KMZ_SYNTH_MESH 3
#define KMZ_SYNTH_POWER 5 /* power-law fan-out mesh, 50k endpoints, depth-16 chains, hot endpoints */
typedef struct kmz_synth_desc {
  uint32_t n_shapes, n_status;
  uint32_t n_endpoints;
} kmz_synth_desc;
int kmz_synth_describe(int config, kmz_synth_desc *out);
/* Generate traces [trace_begin, trace_end) of `config` into the context as its
 * loaded batch (device resident); index_base = number of spans in the traces
 * before trace_begin (computed by the call). Returns the span count. */
int kmz_synth_load(kmz_ctx *ctx, int config, uint64_t seed, uint64_t trace_begin, uint64_t trace_end,
                   uint64_t *n_spans_out);
/* The traces of [trace_begin, trace_end) whose synthetic traceId (the 128-bit
 * t * 0x9E3779B97F4A7C15) has kmz_trace_shard == rank, with their global
 * flatten indices (the index map is set by the call). */
int kmz_synth_load_shard(kmz_ctx *ctx, int config, uint64_t seed, uint64_t trace_begin, uint64_t trace_end,
                         uint32_t world, uint32_t rank, uint64_t *n_spans_out);
/* Host-side generation of the same traces into caller arrays (cap spans);
 * trace_off receives trace_end-trace_begin+1 offsets. */
int kmz_synth_host(int config, uint64_t seed, uint64_t trace_begin, uint64_t trace_end, uint64_t cap,
                   uint64_t *span_id, uint64_t *parent_id, uint8_t *kind, uint32_t *shape, uint16_t *status,
                   uint32_t *duration, int64_t *timestamp, uint64_t *trace_off, uint64_t *n_spans_out);
/* identity tables of a synthetic config (shape == endpoint for synthetic) */
int kmz_synth_shape_ids(int config, uint32_t *rt_ep, uint32_t *tag_ep, uint32_t *dep_ep, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* KMZ_H */
