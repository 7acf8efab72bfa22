// kmz_api.hip -- context, buffers, launch sequencing and the C ABI (kmz.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string>
#include <unordered_map>
#include <vector>

#include "kmz_kernels.h"
#include "kmz_walkw.h"

using namespace kmz;

namespace {

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
};

struct EventPair {
  hipEvent_t a = nullptr, b = nullptr;
  int kernel = 0;
};

}  // namespace

constexpr uint64_t SIG_SEED0 = 0x4B4D5A5349470001ull;  // the K4 ancestry-hash seed of a fresh context

struct kmz_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;

  // loaded batch
  bool loaded = false;
  uint64_t n = 0, index_base = 0;
  const uint64_t *sid = nullptr, *pid = nullptr;
  const uint8_t *kind = nullptr;
  const uint32_t *shape = nullptr;
  const uint16_t *status = nullptr;
  const uint32_t *dur = nullptr;
  const int64_t *ts = nullptr;
  DevBuf in_sid, in_pid, in_kind, in_shape, in_status, in_dur, in_ts;

  // shapes
  uint32_t n_shapes = 0, n_rt = 0, n_tag = 0, n_dep = 0, n_status = 0;
  DevBuf d_rt, d_tag, d_dep;

  // workspace
  DevBuf table, dups, dkey, dval, cparent, rowpos, grp, grp_final, epp, trip, trip_out, counters, stats64, scratch;
  DevBuf synth_cnt, synth_off, dur_table;
  DevBuf k3pool, k3dir, k3part, tile_tmp, sgrp;
  DevBuf dp, cpool1, cpool2, ccur, cdir, mkey, mval;  // window join + certificate
  DevBuf ctab, plist, kstage, kstage_n, kdefer, kdefer_n, cetab;  // K4 chain interning
  DevBuf kbucket, kbucket_n;  // staged keys partitioned by edge-set slice (k_key_part)
  DevBuf mkeys_in, mtab;                                 // kmz_merge_triples staging / fallback set
  DevBuf gd_out, gd_in, gd_set, gd_cnt;  // sharding guard (kmz_guard.hip)
  DevBuf rt_hist, rt_tot, rt_out, rt_ctr;  // cross-shard repeated-id guard: routing scratch, certificate counters
  DevBuf rt_pool1, rt_dir, rt_pool2, rt_cur;  // ... and its own certificate buffers (the run's stay as the run left them)
  DevBuf rt_tsz;                               // ... segment tile sizes (kmz_id_repeats_seg_begin)
  DevBuf rt_jcur;                              // ... the join-folded routing's per-owner cursors (128 B each)
  DevBuf gu_ids, gu_grp, gu_bcnt;              // the used groups compacted (kmz_fetch_used)
  bool gu_ok = false;    // grp_final's used groups are compacted in gu_* (G <= 2^22)
  bool gu_host = false;  // ... and their count is in the run's read-back (not after kmz_finalize)
  // kmz_id_repeats_seg_begin/_end: the open check's stream, segment size, plan
  // and pinned read-back (counters, then the largest count)
  bool rs_open = false;
  hipStream_t rs_stream = nullptr;
  uint64_t rs_seg = 0;
  void *rs_pin = nullptr;
  // device JSON ingest (kmz_json.hip)
  DevBuf j_buf, j_elem, j_state, j_jsc, j_mask, j_cnt, j_off, j_csc, j_small, j_starts, j_slices, j_tslot, j_stab,
      j_ttab, j_reps, j_smap, j_tmap;
  uint64_t j_n = 0, j_scap = 0, j_tcap = 0;
  bool j_ready = false;
  std::vector<uint64_t> j_sfields, j_tfields;  // raw shapes / statuses, first-occurrence order
  std::vector<uint32_t> j_sslots, j_tslots;    // their table slots
  // identities across batches: raw JSON text of a shape's seven fields (or of
  // a status) -> the id the caller gave it in kmz_json_load
  std::unordered_map<std::string, uint32_t> j_known_s, j_known_t;
  std::vector<std::string> j_skeys, j_tkeys;  // the current batch's raw keys
  DevBuf o_key, o_val, o_out, o_rts, o_rsh;  // reduced-graph entry order (kmz_order.hip; o_key = the slot table)
  uint64_t o_n = 0;
  DevBuf imap_l, imap_g;  // local -> global flatten-index runs of a non-contiguous shard (kmz_shard.hip)
  uint64_t imap_n = 0;     // 0: contiguous batch (index_base + i)
  DevBuf ctile;           // K4 per-workgroup stats (apart from K3's tile_tmp: the two run concurrently)
  DevBuf kwpos, kwpos_n;  // chain-table slots written by a run (cleared after it: no per-run memset)
  // service tail (kmz_tail.hip): maps, pair set / table, outputs, link-key buckets
  DevBuf tl_svc, tl_cls, tl_lsvc, tl_pset, tl_pkey, tl_pval, tl_hasin, tl_det, tl_pairs, tl_rb,
      tl_lbkt, tl_lbn;
  uint32_t tl_n_ep = 0, tl_n_cls = 0, tl_n_svc = 0, tl_n_dist = 64, tl_deep = 0;
  uint32_t tl_rel_dist = 0;  // distances in the last run's relying table (0: not complete, use the details)
  bool tl_map = false, tl_ran = false;
  bool tl_open = false;       // kmz_tail_begin enqueued, kmz_tail_end not yet
  uint64_t tl_nt = 0;         // ... its edge-key count
  uint32_t tl_nd_run = 0;     // ... its relying-table width
  bool tl_run_after = false;  // ... a run was begun behind it (a repeat is then impossible)
  uint64_t tl_acap = 0, tl_pacap = 0, tl_pcap = 0, tl_nd = 0, tl_np = 0, tl_bcap = 0;
  uint32_t tl_bbits = 0;  // link-key buckets: 2^tl_bbits
  // tl_rb: the tail's read-back in one device buffer, laid out as its pinned
  // host copy: counters [64 B], stats [n_svc x 8 u32], first rows [n_svc u64]
  // (k_tail_service_rows), relying table [n_svc x n_dist u32] -- one copy
  void *tl_host = nullptr;       // pinned: the tail's counters, per-service stats, relying table, first rows
  size_t tl_host_bytes = 0;
  // RiskAnalyzer.RealtimeRisk's per-service sums (k_service_sums): CSR of the
  // services' stats endpoints, 5xx status mask, output
  DevBuf sv_off, sv_eps, sv_5xx, sv_out;
  void *sv_host = nullptr;    // kmz_service_sums_begin's read-back (pinned)
  size_t sv_host_bytes = 0;
  bool sv_open = false;
  uint32_t sv_n_ep = 0, sv_n_sid = 0, sv_n_status = 0;
  bool sv_map = false;
  bool ctab_dirty = true;  // the chain table holds entries no list records (new, or a list overflowed)
  int path = 0;             // kmz_info.path of the last dependency run
  bool sstats = false;      // shape-level K3 partials computed in this run
  bool chain_ran = false;   // this run's dependency graph came from k4_chain's chain interning
  bool walk_once = false;   // a K4 wait ran out (F_SPIN): this run is redone on the exact per-row walk
  bool k4_now = false;      // this kmz_run's K4 mode (direct enumeration), decided once per call
  bool dep_valid = false;   // every shape's dependency endpoint is < n_dep (chain elements by shape)
  uint64_t shape_gen = 0;   // counts shape tables whose dependency endpoints differ from the last (load_shapes)
  std::vector<uint32_t> dep_host;  // the last table's dependency endpoints
  uint64_t alloc_gen = 0;   // counts device allocations (ensure)
  uint64_t etab_key = 0;    // (shape table, seed, buffer) the walk's gather table cetab holds; 0: none
  // hipGraphs of a whole run for small batches (launch-bound): a run whose
  // launch sequence (kmz_run key) repeats is captured once and replayed
  struct RunGraph {
    uint64_t key = 0;
    hipGraphExec_t exec = nullptr;
    uint64_t used = 0;
    // host-side state the captured enqueue left (restored on a replay)
    int path = 0;
    bool sstats = false, chain_ran = false, k4_direct_ran = false, ctab_dirty = false;
    uint32_t G = 0, ep_mode = 0, k4_lb1 = 0, k4_nsl = 0, k4_ng = 0;
  };
  RunGraph graphs[4];
  uint64_t graph_seen = 0, graph_clock = 0, graph_launches = 0;
  // K4 mode: chain interning, or direct enumeration (every row stages all its
  // keys) when most rows start a new chain -- chosen from the last interning
  // run's chains/rows for this shape table, measured again every 64 runs
  uint64_t k4_key = ~0ull;
  bool k4_auto_direct = false, k4_direct_ran = false;
  uint32_t k4_since = 0;
  uint32_t k4_lb1 = 0, k4_nsl = 0, k4_ng = 0;  // the last K4 run's staging layout (kmz__debug_k4)
  uint64_t cap = 0, tcap = 1ull << 16, ccap = 1ull << 20;
  uint64_t sig_seed = SIG_SEED0;  // K4 ancestry-hash seed (changed after a collision)
  uint32_t dcap = 1024;
  uint32_t scap = 1u << 15;  // K4 staged keys per persistent workgroup (grown when it overflows)
  uint32_t mcap = 1u << 16;   // window-join miss table slots (grown on F_MISS_OVERFLOW)
  bool no_cert = false;       // KMZ_RUN_NO_CERT: the caller's guard checks the ids (no certificate in the run)
  bool table_hint = false;    // the loaded batch failed the uniqueness certificate: go to the table path
  void *hpin = nullptr;       // pinned host copy of counters + stats64 (one read-back per run)
  bool hpin_valid = false;    // hpin holds the last completed run's values
  void *hep = nullptr;        // pinned staging for the endpoint partials
  size_t hep_bytes = 0;

  // last run
  uint32_t ran = 0;
  uint32_t G = 0;        // group slots of the last stats run
  uint32_t ep_mode = 0;  // which ep table the groups use
  bool links = false;
  uint32_t ablate = 0;  // diagnostic knobs (KMZ_ABLATE env), never set in production
  uint32_t ablate2 = 0;  // more knobs (KMZ_ABLATE2): bit 0 = 8-byte key staging (no compact keys), bit 1 = 2^20-slot edge set, bits 2/3 = chain table load <= 1/2 / 1/4, bit 4 = join + walk never fused, bit 5 = fused at any size, bit 6 = 2^8 certificate bins at any size, bit 7 = never, bit 8 = chain interning on the persistent k4_chain (not k4_tile), bit 9 = kmz_fetch_begin's copies to the host by the runtime's blit (not the DMA engines), bit 10 = chain interning on the 16-byte-record k4_tile (not k4_tile8), bit 11 = k4_tile8's chain elements by endpoint even where the table would allow shapes, bit 12 = kmz_route_ids_fixed by histogram / scan / scatter (not one pass), bit 13 = the certificate from the start of the run beside the join (pass 1 by k_cert_bin), bit 14 = the certificate behind K3 on the side stream (not on a stream of its own), bit 15 = with a chain table past the MALL, the certificate beside the settle (not on the main stream between the join and the walk), bit 16 = k_key_part without its LDS cache of written keys, bit 17 = K3 on the main stream between the join and the walk, bit 18 = K3 beside the join on the side stream on the chain-tile path too (not after the walk on the main stream), bit 20 = the run's counters zeroed by hipMemsetAsync (not k_fill), bit 21 = on the direct walk, K3 beside the join on the side stream (not from the end of the walk, beside the settle), bit 22 = chain interning on k4_tile8 (not k4_tile9), bit 23 = no run graphs (as KMZ_HIPGRAPH=0)

  // side stream: K3 and the uniqueness certificate run beside the join and the
  // chain walk (they share no buffers; fork/join by events)
  hipStream_t main = nullptr, side = nullptr;
  // the certificate's side stream: `side` when K3 is not on it this run (the
  // chain-tile path, K3 after the walk); else a second one, created on first
  // use (a run's streams stay within HIP's default 4 hardware queues: a
  // fifth shares one, measured 0.206 against 0.192 ms on Bookinfo), its
  // completion event, and whether this run used it
  bool k3_on_side = false;
  hipStream_t side2 = nullptr;
  hipEvent_t ev_cert = nullptr;
  bool cert2 = false;
  // a chain table past the MALL (config 5): the certificate waits for the
  // end of the walk and runs beside the settle (launch_cert_deferred)
  bool cert_defer = false;
  CertPlan cert_pl{};
  bool k3_settle = false;  // K3 on the side stream from the end of the direct walk (run_enqueue)
  bool k3_ran = false;     // ... and it has been enqueued
  uint32_t k3_mode = 0;    // this run's K3 mode (run_stats)
  bool k3_late = false;  // the shape-level K3 on the main stream after the chain walk (run_chain_tiles)
  bool epp_filled = false;  // this run's endpoint partials were filled with its counters (run_enqueue)
  hipEvent_t ev_fork = nullptr, ev_k3 = nullptr, ev_join = nullptr, ev_done = nullptr;
  bool overlap = false;  // this run uses the side stream
  // kmz_route_ids_join: the next run routes its span ids into these fixed
  // segments (in the join where it can, else by kmz_route_ids_fixed's pass),
  // then records ev_route; kmz_route_wait makes a stream wait for it
  JoinRoute rt_arm;
  bool rt_armed = false, rt_routed = false, rt_in_join = false;
  hipEvent_t ev_route = nullptr;
  // the service tail's and the service sums' read-backs: their _end calls
  // wait for these, not for the stream, so that the next run may be enqueued
  // behind an open tail (the bench's step pipelining)
  hipEvent_t ev_tail = nullptr, ev_sums = nullptr;
  // KMZ_RUNBEGIN_PROFILE=1 (diagnostic): host time of kmz_run_begin's stages
  // (what the enqueue costs before the GPU has the run's big kernels)
  bool rb_prof = false;
  std::vector<std::pair<const char *, double>> rb_marks;

  // profiling
  // kmz_fetch_begin / _end: transfer stream, snapshot of the results, the open fetch
  hipStream_t xfer = nullptr;
  hipEvent_t ev_snap = nullptr;
  DevBuf f_grp, f_trip, f_ep;
  void *fhep = nullptr;
  size_t fhep_bytes = 0;
  bool fetch_open = false;
  // kmz_run_begin / _end: a run enqueued and not yet waited for
  bool run_open = false;
  uint32_t run_flags = 0;
  kmz_endpoint *f_eps = nullptr;
  uint32_t f_ndep = 0;

  bool prof = false;
  // run graphs for batches below 2^23 spans (run_enqueue_graphed): on unless
  // KMZ_HIPGRAPH=0 or KMZ_ABLATE2 bit 23
  bool graphs_on = true;
  uint32_t prof_mask = 0;  // kernel ids timed while prof (kmz_set_profiling_mask)
  std::vector<EventPair> pending;
  std::vector<hipEvent_t> pool;
  double ms[KMZ_K_COUNT] = {0};
  uint64_t calls[KMZ_K_COUNT] = {0};
};

namespace {

int fail(kmz_ctx *c, int code, const std::string &msg) {
  if (c) {
    c->err = msg;
    c->etab_key = 0;  // (after any failure the walk's gather table is rebuilt)
  }
  return code;
}

int run_busy(kmz_ctx *c) { return fail(c, KMZ_E_STATE, "a run is open: kmz_run_end first"); }

#define HIPCHK(c, x)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return fail((c), KMZ_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

int ensure(kmz_ctx *c, DevBuf &b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return 0;
  if (b.p) {  // (both streams may still use it)
    hipStreamSynchronize(c->stream);
    if (c->side) hipStreamSynchronize(c->side);
    if (c->side2) hipStreamSynchronize(c->side2);
    if (c->main && c->main != c->stream) hipStreamSynchronize(c->main);
    hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) return fail(c, KMZ_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  b.bytes = bytes;
  ++c->alloc_gen;
  return 0;
}

template <class T>
T *P(DevBuf &b) {
  return reinterpret_cast<T *>(b.p);
}

hipEvent_t ev_get(kmz_ctx *c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // device-scope timing events: no system-scope fence (and no pipeline bubble
  // for one) between the kernels they bracket
  hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}

struct Timed {
  kmz_ctx *c;
  EventPair ep;
  bool on;
  Timed(kmz_ctx *ctx, int k) : c(ctx), on(ctx->prof && ((ctx->prof_mask >> k) & 1u)) {
    if (!on) return;
    ep.kernel = k;
    ep.a = ev_get(c);
    ep.b = ev_get(c);
    hipEventRecord(ep.a, c->stream);
  }
  ~Timed() {
    if (!on) return;
    hipEventRecord(ep.b, c->stream);
    c->pending.push_back(ep);
  }
};

static void rb_mark(kmz_ctx *c, const char *what) {
  if (c->rb_prof)
    c->rb_marks.emplace_back(what, std::chrono::duration<double, std::micro>(
                                       std::chrono::steady_clock::now().time_since_epoch()).count());
}

void harvest(kmz_ctx *c) {
  for (auto &ep : c->pending) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, ep.a, ep.b) == hipSuccess) {
      c->ms[ep.kernel] += t;
      c->calls[ep.kernel] += 1;
    }
    c->pool.push_back(ep.a);
    c->pool.push_back(ep.b);
  }
  c->pending.clear();
}

// ---- lognormal(ln 2000us, 0.75) quantile table (host computed, shared) ----
double inv_norm(double p) {  // Acklam's rational approximation, |rel err| < 1.2e-9
  static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                             1.383577518672690e+02,  -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                             6.680131188771972e+01,  -1.328068155288572e+01};
  static const double cc[] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                              -2.549732539343734e+00, 4.374664141464968e+00,  2.938163982698783e+00};
  static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                             3.754408661907416e+00};
  const double pl = 0.02425, ph = 1 - pl;
  if (p < pl) {
    double q = std::sqrt(-2 * std::log(p));
    return (((((cc[0] * q + cc[1]) * q + cc[2]) * q + cc[3]) * q + cc[4]) * q + cc[5]) /
           ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  }
  if (p <= ph) {
    double q = p - 0.5, r = q * q;
    return (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
           (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
  }
  double q = std::sqrt(-2 * std::log(1 - p));
  return -(((((cc[0] * q + cc[1]) * q + cc[2]) * q + cc[3]) * q + cc[4]) * q + cc[5]) /
         ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
}

const std::vector<uint32_t> &dur_table_host() {
  static std::vector<uint32_t> t;
  if (t.empty()) {
    const uint32_t n = 1u << SYN_DUR_BITS;
    t.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
      double z = inv_norm((i + 0.5) / n);
      double v = std::exp(std::log(2000.0) + 0.75 * z);
      double r = std::floor(v + 0.5);
      if (r < 50) r = 50;
      if (r > 1e7) r = 1e7;
      t[i] = (uint32_t)r;
    }
  }
  return t;
}

int check_flags(kmz_ctx *c, uint32_t flags) {
  if (flags & F_CYCLE) return fail(c, KMZ_E_CYCLE, "cyclic parentId chain (depth > 16384)");
  if (flags & F_ZERO_ID) return fail(c, KMZ_E_ZERO_ID, "span_id 0 is reserved");
  if (flags & F_RANGE) return fail(c, KMZ_E_RANGE, "shape/status/endpoint id out of range");
  if (flags & F_TABLE_FULL) return fail(c, KMZ_E_OVERFLOW, "span table full");
  return KMZ_OK;
}

}  // namespace

extern "C" {

int kmz_abi_version(void) { return KMZ_ABI_VERSION; }

kmz_ctx *kmz_create(int device, void *stream) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  kmz_ctx *c = new kmz_ctx();
  c->device = device;
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      return nullptr;
    }
    c->own_stream = true;
  }
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_cert, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_k3, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_route, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_tail, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_sums, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return nullptr;
  }
  if (const char *a = getenv("KMZ_ABLATE")) c->ablate = (uint32_t)strtoul(a, nullptr, 0);
  if (const char *a = getenv("KMZ_RUNBEGIN_PROFILE")) c->rb_prof = atoi(a) != 0;
  if (const char *a = getenv("KMZ_ABLATE2")) c->ablate2 = (uint32_t)strtoul(a, nullptr, 0);
  // run graphs: on by default (round 6); KMZ_HIPGRAPH=0 or KMZ_ABLATE2 bit 23
  // turn them off, KMZ_ABLATE bit 13 (or KMZ_HIPGRAPH=1) keeps them on
  if (const char *a = getenv("KMZ_HIPGRAPH")) c->graphs_on = atoi(a) != 0;
  if (c->ablate2 & (1u << 23)) c->graphs_on = false;
  if (c->ablate & (1u << 13)) c->graphs_on = true;
  if (c->ablate2 & 2u) c->tcap = 1ull << 20;  // test knob: an edge set large enough for compact staging from the start
  if (c->ablate & (1u << 30)) c->scap = 256;  // test knob: tiny key staging (overflow + growth paths)
  // counters (u32) and statistics (u64) in one allocation: one fill and one
  // read-back per run (stats64 is a view, not freed on its own)
  if (ensure(c, c->counters, C_COUNT * 4 + S_COUNT * 8)) {
    delete c;
    return nullptr;
  }
  c->stats64.p = static_cast<char *>(c->counters.p) + C_COUNT * 4;
  c->stats64.bytes = S_COUNT * 8;
  return c;
}

void kmz_destroy(kmz_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->side) hipStreamSynchronize(c->side);
  if (c->side2) hipStreamSynchronize(c->side2);
  hipStreamSynchronize(c->stream);
  if (c->xfer) hipStreamSynchronize(c->xfer);
  harvest(c);
  for (auto e : c->pool) hipEventDestroy(e);
  DevBuf *bufs[] = {&c->in_sid, &c->in_pid,    &c->in_kind,  &c->in_shape,  &c->in_status, &c->in_dur,
                    &c->in_ts,  &c->d_rt,      &c->d_tag,    &c->d_dep,     &c->table,     &c->dups,
                    &c->dkey,   &c->dval,      &c->cparent,  &c->rowpos,    &c->grp,       &c->grp_final,
                    &c->epp,    &c->trip,      &c->trip_out, &c->counters,  &c->scratch,
                    &c->synth_cnt, &c->synth_off, &c->dur_table, &c->k3pool, &c->k3dir, &c->k3part,
                    &c->tile_tmp, &c->sgrp, &c->dp, &c->cpool1, &c->cpool2, &c->ccur, &c->cdir, &c->mkey,
                    &c->mval, &c->ctab, &c->cetab, &c->plist, &c->kstage, &c->kstage_n, &c->kdefer, &c->kdefer_n,
                    &c->kbucket, &c->kbucket_n, &c->mkeys_in, &c->mtab, &c->kwpos, &c->kwpos_n, &c->ctile, &c->gd_out, &c->gd_in, &c->gd_set, &c->gd_cnt, &c->rt_hist, &c->rt_tot, &c->rt_out, &c->rt_ctr, &c->rt_pool1, &c->rt_dir, &c->rt_pool2, &c->rt_cur, &c->rt_tsz, &c->rt_jcur, &c->gu_ids, &c->gu_grp, &c->gu_bcnt, &c->imap_l, &c->imap_g, &c->tl_svc, &c->tl_cls, &c->tl_lsvc,
                    &c->tl_pset, &c->tl_pkey, &c->tl_pval,
                    &c->tl_hasin, &c->tl_det, &c->tl_pairs, &c->tl_rb,
                    &c->tl_lbkt, &c->tl_lbn, &c->sv_off, &c->sv_eps, &c->sv_5xx, &c->sv_out,
                    &c->o_key, &c->o_val, &c->o_out,
                    &c->o_rts, &c->o_rsh, &c->j_buf, &c->j_elem, &c->j_state, &c->j_jsc, &c->j_mask,
                    &c->j_cnt, &c->j_off, &c->j_csc, &c->j_small, &c->j_starts, &c->j_slices, &c->j_tslot,
                    &c->j_stab, &c->j_ttab, &c->j_reps, &c->j_smap, &c->j_tmap, &c->f_grp, &c->f_trip, &c->f_ep};
  if (c->rs_open && c->rs_stream) hipStreamSynchronize(c->rs_stream);  // (an open guard check reads its buffers)
  for (DevBuf *b : bufs)
    if (b->p) hipFree(b->p);
  for (auto &g : c->graphs)
    if (g.exec) hipGraphExecDestroy(g.exec);
  if (c->hpin) hipHostFree(c->hpin);
  if (c->rs_pin) hipHostFree(c->rs_pin);
  if (c->hep) hipHostFree(c->hep);
  if (c->sv_host) hipHostFree(c->sv_host);
  if (c->fhep) hipHostFree(c->fhep);
  if (c->xfer) hipStreamDestroy(c->xfer);
  if (c->ev_snap) hipEventDestroy(c->ev_snap);
  if (c->tl_host) hipHostFree(c->tl_host);
  if (c->side) {
    hipStreamSynchronize(c->side);
    hipStreamDestroy(c->side);
  }
  if (c->side2) {
    hipStreamSynchronize(c->side2);
    hipStreamDestroy(c->side2);
  }
  for (hipEvent_t e : {c->ev_fork, c->ev_k3, c->ev_join, c->ev_done, c->ev_cert, c->ev_route, c->ev_tail, c->ev_sums})
    if (e) hipEventDestroy(e);
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
}

const char *kmz_last_error(kmz_ctx *c) { return c ? c->err.c_str() : "null context"; }

int kmz_sync(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  harvest(c);
  return KMZ_OK;
}

static int load_shapes(kmz_ctx *c, const kmz_shapes *sh) {
  if (!sh || !sh->rt_ep || !sh->tag_ep || !sh->dep_ep) return fail(c, KMZ_E_ARG, "shape table missing");
  if (sh->n_dep_ep >= (1u << 24) || sh->n_status == 0 || sh->n_status > 65535)
    return fail(c, KMZ_E_ARG, "endpoint/status count out of range");
  c->n_shapes = sh->n_shapes;
  c->n_rt = sh->n_rt_ep;
  c->n_tag = sh->n_tag_ep;
  c->n_dep = sh->n_dep_ep;
  c->n_status = sh->n_status;
  // (the walk's chain elements may be shapes -- each maps to one endpoint in
  // range, and a shape id fits an edge key's 24 bits below NONE's)
  // (a reload of the same dependency endpoints -- every kmz_load of a realtime
  // tick -- keeps the walk's gather table, etab_cached)
  if (c->dep_host.size() != sh->n_shapes ||
      (sh->n_shapes && memcmp(c->dep_host.data(), sh->dep_ep, (size_t)sh->n_shapes * 4) != 0)) {
    c->dep_host.assign(sh->dep_ep, sh->dep_ep + sh->n_shapes);
    ++c->shape_gen;
  }
  c->dep_valid = sh->n_shapes < 0xFFFFFFu;
  for (uint32_t s = 0; s < sh->n_shapes && c->dep_valid; ++s) c->dep_valid = sh->dep_ep[s] < sh->n_dep_ep;
  size_t b = (size_t)sh->n_shapes * 4;
  if (ensure(c, c->d_rt, b) || ensure(c, c->d_tag, b) || ensure(c, c->d_dep, b)) return KMZ_E_HIP;
  if (b) {
    HIPCHK(c, hipMemcpyAsync(c->d_rt.p, sh->rt_ep, b, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_tag.p, sh->tag_ep, b, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_dep.p, sh->dep_ep, b, hipMemcpyHostToDevice, c->stream));
  }
  return KMZ_OK;
}

int kmz_load(kmz_ctx *c, const kmz_spans *s, const kmz_shapes *sh, int where) {
  if (!c || !s) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  hipSetDevice(c->device);
  if (s->n >= 0xFFFFFFFFull) return fail(c, KMZ_E_ARG, "batch too large (n must be < 2^32-1)");
  if (s->n && (!s->span_id || !s->parent_id || !s->kind || !s->shape || !s->status || !s->duration || !s->timestamp))
    return fail(c, KMZ_E_ARG, "null column");
  int r = load_shapes(c, sh);
  if (r) return r;
  c->n = s->n;
  c->index_base = s->index_base;
  c->imap_n = 0;
  c->ran = 0;
  c->table_hint = false;
  c->hpin_valid = false;
  if (where == KMZ_MEM_DEVICE) {
    c->sid = s->span_id;
    c->pid = s->parent_id;
    c->kind = s->kind;
    c->shape = s->shape;
    c->status = s->status;
    c->dur = s->duration;
    c->ts = s->timestamp;
  } else {
    size_t n = s->n;
    if (ensure(c, c->in_sid, n * 8) || ensure(c, c->in_pid, n * 8) || ensure(c, c->in_kind, n) ||
        ensure(c, c->in_shape, n * 4) || ensure(c, c->in_status, n * 2) || ensure(c, c->in_dur, n * 4) ||
        ensure(c, c->in_ts, n * 8))
      return KMZ_E_HIP;
    if (n) {
      HIPCHK(c, hipMemcpyAsync(c->in_sid.p, s->span_id, n * 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->in_pid.p, s->parent_id, n * 8, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->in_kind.p, s->kind, n, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->in_shape.p, s->shape, n * 4, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->in_status.p, s->status, n * 2, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->in_dur.p, s->duration, n * 4, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->in_ts.p, s->timestamp, n * 8, hipMemcpyHostToDevice, c->stream));
    }
    c->sid = P<uint64_t>(c->in_sid);
    c->pid = P<uint64_t>(c->in_pid);
    c->kind = P<uint8_t>(c->in_kind);
    c->shape = P<uint32_t>(c->in_shape);
    c->status = P<uint16_t>(c->in_status);
    c->dur = P<uint32_t>(c->in_dur);
    c->ts = P<int64_t>(c->in_ts);
  }
  c->loaded = true;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

// ---- K1 on the device: Zipkin JSON -> columns (kmz_json.hip) -----------------
namespace {
// the distinct entries of one interning table, sorted by first occurrence:
// fields (offset, length) pairs and table slots
int json_collect(kmz_ctx *c, DevBuf &tab, uint64_t cap, uint32_t first, uint32_t nf, uint64_t nspan,
                 std::vector<uint64_t> &fields, std::vector<uint32_t> &slots) {
  unsigned long long *cnt = P<unsigned long long>(c->j_small) + 4;
  uint64_t ocap = std::min<uint64_t>(cap, 1ull << 16);
  for (;;) {
    if (ensure(c, c->j_reps, ocap * (2 + nf) * 8)) return KMZ_E_HIP;
    HIPCHK(c, hipMemsetAsync(cnt, 0, 8, c->stream));
    launch_json_reps(c->stream, P<unsigned long long>(tab), cap, P<unsigned long long>(c->j_slices), first, nf,
                     P<unsigned long long>(c->j_reps), ocap, nspan, cnt);
    HIPCHK(c, hipGetLastError());
    unsigned long long m = 0;
    HIPCHK(c, hipMemcpyAsync(&m, cnt, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (m > ocap) {
      ocap = m;
      continue;
    }
    std::vector<uint64_t> h((size_t)m * (2 + nf));
    if (m) HIPCHK(c, hipMemcpy(h.data(), c->j_reps.p, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> order((size_t)m);
    for (uint32_t k = 0; k < m; ++k) order[k] = k;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return h[(size_t)a * (2 + nf)] < h[(size_t)b * (2 + nf)]; });
    fields.assign((size_t)m * nf * 2, 0);
    slots.assign((size_t)m, 0);
    for (uint32_t r = 0; r < m; ++r) {
      const uint64_t *e = &h[(size_t)order[r] * (2 + nf)];
      slots[r] = (uint32_t)e[1];
      for (uint32_t f = 0; f < nf; ++f) {
        const uint64_t sl = e[2 + f], ln = sl & 0xFFFFFFull;
        fields[((size_t)r * nf + f) * 2] = ln == 0xFFFFFFull ? 0 : (sl >> 24);
        fields[((size_t)r * nf + f) * 2 + 1] = ln == 0xFFFFFFull ? KMZ_JSON_ABSENT : ln;
      }
    }
    return KMZ_OK;
  }
}
// the raw keys (per field: u32 length or ~0 + bytes) of the distinct entries,
// from the caller's buffer (host) or gathered on the device
int json_keys(kmz_ctx *c, const char *json, int mem, uint32_t nf, const std::vector<uint64_t> &fields,
              std::vector<std::string> &keys) {
  const size_t m = fields.size() / (2 * nf);
  keys.assign(m, std::string());
  std::vector<char> dev;
  const char *src = json;
  if (mem != KMZ_MEM_HOST) {  // copy the spans' byte range once (fields are offsets into it)
    uint64_t lo = ~0ull, hi = 0;
    for (size_t k = 0; k < fields.size(); k += 2)
      if (fields[k + 1] != KMZ_JSON_ABSENT) {
        lo = std::min(lo, fields[k]);
        hi = std::max(hi, fields[k] + fields[k + 1]);
      }
    if (hi > lo) {
      dev.resize(hi - lo);
      HIPCHK(c, hipMemcpy(dev.data(), json + lo, hi - lo, hipMemcpyDeviceToHost));
      src = dev.data() - lo;
    }
  }
  for (size_t e = 0; e < m; ++e) {
    std::string &k = keys[e];
    for (uint32_t f = 0; f < nf; ++f) {
      const uint64_t off = fields[(e * nf + f) * 2], len = fields[(e * nf + f) * 2 + 1];
      const uint32_t l32 = len == KMZ_JSON_ABSENT ? 0xFFFFFFFFu : (uint32_t)len;
      k.append(reinterpret_cast<const char *>(&l32), 4);
      if (len != KMZ_JSON_ABSENT) k.append(src + off, (size_t)len);
    }
  }
  return KMZ_OK;
}
}  // namespace

int kmz_json_known(kmz_ctx *c, uint32_t *shape_of_raw, uint32_t *status_of_raw) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->j_ready) return fail(c, KMZ_E_STATE, "kmz_json_known before a successful kmz_json_parse");
  for (size_t k = 0; shape_of_raw && k < c->j_skeys.size(); ++k) {
    auto it = c->j_known_s.find(c->j_skeys[k]);
    shape_of_raw[k] = it == c->j_known_s.end() ? KMZ_NONE : it->second;
  }
  for (size_t k = 0; status_of_raw && k < c->j_tkeys.size(); ++k) {
    auto it = c->j_known_t.find(c->j_tkeys[k]);
    status_of_raw[k] = it == c->j_known_t.end() ? KMZ_NONE : it->second;
  }
  return KMZ_OK;
}

int kmz_json_forget(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  c->j_known_s.clear();
  c->j_known_t.clear();
  return KMZ_OK;
}

int kmz_json_parse(kmz_ctx *c, const char *json, uint64_t len, int mem, uint64_t *n_spans, uint32_t *n_shapes,
                   uint32_t *n_statuses) {
  if (!c || (!json && len) || !n_spans || !n_shapes || !n_statuses) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  hipSetDevice(c->device);
  c->j_ready = false;
  c->loaded = false;  // the context's columns are rewritten
  c->ran = 0;
  c->hpin_valid = false;
  if (len == 0) return KMZ_E_UNSUPPORTED;
  const uint64_t nch = (len + JCHUNK - 1) / JCHUNK;
  const uint8_t *b = reinterpret_cast<const uint8_t *>(json);
  if (mem == KMZ_MEM_HOST) {
    if (ensure(c, c->j_buf, len + JCHUNK)) return KMZ_E_HIP;
    HIPCHK(c, hipMemcpyAsync(c->j_buf.p, json, len, hipMemcpyHostToDevice, c->stream));
    b = P<uint8_t>(c->j_buf);
  }
  const uint64_t sc = json_scan_scratch(nch);
  if (ensure(c, c->j_elem, nch * sizeof(JElem)) || ensure(c, c->j_state, nch * sizeof(JElem)) ||
      ensure(c, c->j_jsc, sc * sizeof(JElem)) || ensure(c, c->j_mask, nch * 8) || ensure(c, c->j_cnt, nch * 4) ||
      ensure(c, c->j_off, nch * 4) || ensure(c, c->j_csc, sc * 4) || ensure(c, c->j_small, 64))
    return KMZ_E_HIP;
  // j_small: [0..12) JElem total, [16) u32 count total, [20) u32 flags, [32) u64 rep count
  uint8_t *sm = P<uint8_t>(c->j_small);
  unsigned int *flags = reinterpret_cast<unsigned int *>(sm + 20);
  HIPCHK(c, hipMemsetAsync(sm, 0, 64, c->stream));
  {
    Timed t(c, KMZ_K_JSON);
    launch_json_structure(c->stream, b, len, nch, P<JElem>(c->j_elem), P<JElem>(c->j_state),
                          reinterpret_cast<JElem *>(sm), P<JElem>(c->j_jsc), P<unsigned long long>(c->j_mask),
                          P<uint32_t>(c->j_cnt), P<uint32_t>(c->j_off), reinterpret_cast<uint32_t *>(sm + 16),
                          P<uint32_t>(c->j_csc), flags);
  }
  HIPCHK(c, hipGetLastError());
  uint8_t hs[32];
  HIPCHK(c, hipMemcpyAsync(hs, sm, 32, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  JElem tot;
  uint32_t n32, fl;
  memcpy(&tot, hs, sizeof(tot));
  memcpy(&n32, hs + 16, 4);
  memcpy(&fl, hs + 20, 4);
  if ((fl & JF_BAD) || !(fl & JF_TOP) || tot.p != 0 || tot.d0 != 0) return KMZ_E_UNSUPPORTED;
  const uint64_t n = n32;
  // interning tables at load <= 1/2 for the shapes a realtime window has
  // (tens of thousands); a fuller table flags JF_FULL and the spans are parsed
  // again with a larger one
  uint64_t scap = 1024, tcap = 4096;
  while (scap < 2 * n + 1024 && scap < (1ull << 20)) scap *= 2;
  if (ensure(c, c->j_starts, (n + 1) * 8) || ensure(c, c->in_sid, (n + 1) * 8) || ensure(c, c->in_pid, (n + 1) * 8) ||
      ensure(c, c->in_kind, n + 1) || ensure(c, c->in_shape, (n + 1) * 4) || ensure(c, c->in_status, (n + 1) * 2) ||
      ensure(c, c->in_dur, (n + 1) * 4) || ensure(c, c->in_ts, (n + 1) * 8) || ensure(c, c->j_slices, (n + 1) * 64) ||
      ensure(c, c->j_tslot, (n + 1) * 4))
    return KMZ_E_HIP;
  {
    Timed t(c, KMZ_K_JSON);
    launch_json_starts(c->stream, P<unsigned long long>(c->j_mask), P<uint32_t>(c->j_off), nch,
                       P<unsigned long long>(c->j_starts));
  }
  {  // starts[n] = len: the end of the last span (the span kernels' staging bound)
    const uint64_t end = len;
    HIPCHK(c, hipMemcpyAsync(P<uint64_t>(c->j_starts) + n, &end, 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  for (int attempt = 0;; ++attempt) {
    if (ensure(c, c->j_stab, scap * 16) || ensure(c, c->j_ttab, tcap * 16)) return KMZ_E_HIP;
    HIPCHK(c, hipMemsetAsync(c->j_stab.p, 0, scap * 16, c->stream));
    HIPCHK(c, hipMemsetAsync(c->j_ttab.p, 0, tcap * 16, c->stream));
    HIPCHK(c, hipMemsetAsync(flags, 0, 4, c->stream));
    {
      Timed t(c, KMZ_K_JSON);
      launch_json_spans(c->stream, b, len, P<unsigned long long>(c->j_starts), n, P<uint64_t>(c->in_sid),
                        P<uint64_t>(c->in_pid), P<uint8_t>(c->in_kind), P<uint32_t>(c->in_dur), P<int64_t>(c->in_ts),
                        P<unsigned long long>(c->j_slices), P<uint32_t>(c->in_shape), P<uint32_t>(c->j_tslot),
                        P<unsigned long long>(c->j_stab), scap, P<unsigned long long>(c->j_ttab), tcap, flags);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(&fl, flags, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (fl & JF_BAD) return KMZ_E_UNSUPPORTED;
    if (!(fl & JF_FULL)) {
      if (fl & JF_COLLIDE) return KMZ_E_UNSUPPORTED;
      break;
    }
    if (attempt >= 6) return KMZ_E_UNSUPPORTED;
    scap *= 4;
    tcap *= 4;
  }
  int r = json_collect(c, c->j_stab, scap, 0, 7, n, c->j_sfields, c->j_sslots);
  if (!r) r = json_collect(c, c->j_ttab, tcap, 7, 1, n, c->j_tfields, c->j_tslots);
  if (r) return r;
  if ((r = json_keys(c, json, mem, 7, c->j_sfields, c->j_skeys)) || (r = json_keys(c, json, mem, 1, c->j_tfields, c->j_tkeys)))
    return r;
  c->j_n = n;
  c->j_scap = scap;
  c->j_tcap = tcap;
  c->j_ready = true;
  *n_spans = n;
  *n_shapes = (uint32_t)c->j_sslots.size();
  *n_statuses = (uint32_t)c->j_tslots.size();
  return KMZ_OK;
}

int kmz_json_fields(kmz_ctx *c, uint64_t *shape_fields, uint64_t *status_fields) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->j_ready) return fail(c, KMZ_E_STATE, "kmz_json_fields before a successful kmz_json_parse");
  if (shape_fields && !c->j_sfields.empty()) memcpy(shape_fields, c->j_sfields.data(), c->j_sfields.size() * 8);
  if (status_fields && !c->j_tfields.empty()) memcpy(status_fields, c->j_tfields.data(), c->j_tfields.size() * 8);
  return KMZ_OK;
}

int kmz_json_load(kmz_ctx *c, const uint32_t *shape_of_raw, const uint32_t *status_of_raw, const kmz_shapes *shapes,
                  uint64_t index_base) {
  if (!c || !shapes) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->j_ready) return fail(c, KMZ_E_STATE, "kmz_json_load before a successful kmz_json_parse");
  const size_t ns = c->j_sslots.size(), nt = c->j_tslots.size();
  if ((ns && !shape_of_raw) || (nt && !status_of_raw)) return KMZ_E_ARG;
  std::vector<uint32_t> sm(c->j_scap, 0), tm(c->j_tcap, 0);
  for (size_t k = 0; k < ns; ++k) sm[c->j_sslots[k]] = shape_of_raw[k];
  for (size_t k = 0; k < nt; ++k) {
    if (status_of_raw[k] > 0xFFFFu) return fail(c, KMZ_E_RANGE, "status id >= 65536");
    tm[c->j_tslots[k]] = status_of_raw[k];
  }
  // remembered for kmz_json_known on later batches
  for (size_t k = 0; k < ns; ++k) c->j_known_s[c->j_skeys[k]] = shape_of_raw[k];
  for (size_t k = 0; k < nt; ++k) c->j_known_t[c->j_tkeys[k]] = status_of_raw[k];
  int r = load_shapes(c, shapes);
  if (r) return r;
  if (ensure(c, c->j_smap, sm.size() * 4) || ensure(c, c->j_tmap, tm.size() * 4)) return KMZ_E_HIP;
  HIPCHK(c, hipMemcpyAsync(c->j_smap.p, sm.data(), sm.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->j_tmap.p, tm.data(), tm.size() * 4, hipMemcpyHostToDevice, c->stream));
  launch_json_remap(c->stream, c->j_n, P<uint32_t>(c->in_shape), P<uint32_t>(c->j_tslot), P<uint16_t>(c->in_status),
                    P<uint32_t>(c->j_smap), P<uint32_t>(c->j_tmap));
  HIPCHK(c, hipGetLastError());
  c->n = c->j_n;
  c->index_base = index_base;
  c->imap_n = 0;
  c->ran = 0;
  c->table_hint = false;
  c->hpin_valid = false;
  c->sid = P<uint64_t>(c->in_sid);
  c->pid = P<uint64_t>(c->in_pid);
  c->kind = P<uint8_t>(c->in_kind);
  c->shape = P<uint32_t>(c->in_shape);
  c->status = P<uint16_t>(c->in_status);
  c->dur = P<uint32_t>(c->in_dur);
  c->ts = P<int64_t>(c->in_ts);
  c->loaded = true;
  c->j_ready = false;  // the columns now hold the caller's ids
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

// the stream the certificate runs on beside the walk (see kmz_ctx::side2);
// nullptr if the second stream cannot be created
static hipStream_t cert_stream(kmz_ctx *c) {
  if (!c->k3_on_side) return c->side;
  if (!c->side2 && hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking) != hipSuccess) c->side2 = nullptr;
  return c->side2;
}

// whether cetab already holds this shape table's gather table under this seed
// (k_chain_etab is then skipped: one launch less per run); marks it as held.
// Never under run graphs (a replay must not depend on what an earlier run left).
static bool etab_cached(kmz_ctx *c) {
  const uint64_t key = (mix64(c->shape_gen * 0x9E3779B97F4A7C15ull ^ c->sig_seed ^ (c->alloc_gen << 40)) ^
                        (uint64_t)(uintptr_t)c->cetab.p ^ c->n_shapes) | 1;
  const bool ok = key == c->etab_key && !c->graphs_on;
  c->etab_key = c->graphs_on ? 0 : key;
  return ok;
}

// The certificate split + check deferred by run_join (a chain table past the
// MALL, config 5): on side2 from here, i.e. beside the settle's probe-bound
// k_key_part / k_key_slice instead of between the join and the walk (the
// walk's HBM-resident chain table and the certificate slow each other down).
static int launch_cert_deferred(kmz_ctx *c) {
  if (!c->cert_defer) return KMZ_OK;
  c->cert_defer = false;
  const uint32_t n = (uint32_t)c->n;
  const CertPlan &pl = c->cert_pl;
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned int *cur2 = P<unsigned int>(c->ccur);
  hipStream_t cs = cert_stream(c);
  if (!cs) return fail(c, KMZ_E_HIP, "hipStreamCreateWithFlags (certificate stream)");
  HIPCHK(c, hipEventRecord(c->ev_join, c->stream));
  HIPCHK(c, hipStreamWaitEvent(cs, c->ev_join, 0));
  hipStream_t keep = c->stream;
  c->stream = cs;
  c->cert2 = cs == c->side2;
  {
    Timed t(c, KMZ_K_CERT);
    launch_cert_split(c->stream, n, P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir), pl,
                      P<unsigned long long>(c->cpool2), cur2, cnt);
  }
  {
    Timed t(c, KMZ_K_CHECK);
    launch_cert_check(c->stream, n, pl, P<unsigned long long>(c->cpool2), cur2, cnt);
  }
  c->stream = keep;
  return KMZ_OK;
}

// K1': window join + uniqueness certificate.  *ok = false when the batch
// needs the global table (a repeated span id, or a batch too large for the
// certificate's two partition levels).
static int run_join(kmz_ctx *c, bool *ok) {
  const uint32_t n = (uint32_t)c->n;
  *ok = false;
  rb_mark(c, "join:entry");
  // The certificate beside the join and the walk only while the chain table
  // fits the 256 MB MALL: then the walk's probes leave HBM to the certificate
  // (measured: mesh 5.21 -> 5.12 ms, Bookinfo 0.385 -> 0.323 ms); a chain
  // table in HBM (config 5, 4 GB) and the certificate slow each other down
  // (19.3 -> 25.7 ms)
  const bool cert_side = c->overlap && !(c->ablate & (1u << 26)) && c->ccap * CHAIN_ENTRY_BYTES <= (256ull << 20);
  // (KMZ_ABLATE2 bit 13, for comparison: the certificate from the start of
  // the run -- pass 1 by its own kernel, k_cert_bin over the span ids, on the
  // side stream, none in the join -- so that it runs beside the join too.
  // Measured slower on config 3: 3.81 against 3.59 ms; the certificate's
  // workgroups take CUs from the VALU-bound join, while beside the walk,
  // whose probes wait on the MALL, they fill idle issue slots;
  // profiles/r05/ab/early/.)
  const bool early = cert_side && !c->no_cert && (c->ablate2 & 8192u);
  CertPlan pl;
  // (KMZ_ABLATE2 bit 6, test knob: the certificate's 2^8 pass-1 bins at any
  // size; bit 7: never, for comparison.  k_cert_bin bins by 2^6.)
  if (n == 0 || !cert_plan(n, &pl, !early && !(c->ablate2 & 128u), !early && (c->ablate2 & 64u) != 0) ||
      c->table_hint || (c->ablate & 32))
    return KMZ_OK;
  if (ensure(c, c->dp, (size_t)(n + 1) * 4) || ensure(c, c->cpool1, cert_pool1_words(n) * 8) ||
      ensure(c, c->cpool2, cert_pool2_bytes(pl)) || ensure(c, c->ccur, cert_cur_words(pl) * 4) ||
      ensure(c, c->cdir, cert_dir_entries(n, pl) * 2))
    return KMZ_E_HIP;
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned int *cur2 = P<unsigned int>(c->ccur);
  if (ensure(c, c->mkey, (size_t)c->mcap * 8) || ensure(c, c->mval, (size_t)c->mcap * 4)) return KMZ_E_HIP;
  // an armed routing (kmz_route_ids_join) rides in the join's pass 1 when the
  // run has no certificate of its own and the owners fit the pass-1 bins
  rb_mark(c, "join:ensure");
  JoinRoute rt;
  if (c->rt_armed && c->no_cert && !early && c->rt_arm.world <= (1u << pl.B1)) {
    if (ensure(c, c->rt_jcur, (size_t)c->rt_arm.world * ROUTE_CUR_STRIDE * 8)) return KMZ_E_HIP;
    rt = c->rt_arm;
    rt.cur = P<unsigned long long>(c->rt_jcur);
  }
  if (early) {  // (behind the side stream's K3: the main stream waits for that one near the end)
    c->stream = c->side;
    {
      Timed t(c, KMZ_K_MEMSET);
      FillArgs f;
      f.add(cur2, cert_cur_words(pl) * 4, 0);
      launch_fill(c->stream, f);
    }
    {
      Timed t(c, KMZ_K_CERT);
      launch_cert_bin(c->stream, reinterpret_cast<const unsigned long long *>(c->sid), n,
                      P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir));
      launch_cert_split(c->stream, n, P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir), pl,
                        P<unsigned long long>(c->cpool2), cur2, cnt);
    }
    {
      Timed t(c, KMZ_K_CHECK);
      launch_cert_check(c->stream, n, pl, P<unsigned long long>(c->cpool2), cur2, cnt);
    }
    c->stream = c->main;
  }
  {
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    if (!early) f.add(cur2, cert_cur_words(pl) * 4, 0);
    if (rt.out) f.add(rt.cur, (size_t)rt.world * ROUTE_CUR_STRIDE * 8, 0);
    f.add(c->mkey.p, (size_t)c->mcap * 8, 0);
    f.add(c->mval.p, (size_t)c->mcap * 4, 0xFF);  // ids not in the batch: NONE
    launch_fill(c->stream, f);
  }
  {
    Timed t(c, KMZ_K_JOIN);
    // (no pass 1 in the join -- bit 6 of its knobs -- when the certificate
    // bins on its own or KMZ_RUN_NO_CERT leaves it to the caller)
    launch_join(c->stream, c->sid, c->pid, c->kind, n, P<uint32_t>(c->cparent), P<uint32_t>(c->dp),
                P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir), cnt, pl,
                c->ablate | ((c->no_cert && !rt.out) || early ? 64u : 0u), rt);
  }
  rb_mark(c, "join:fill+launch");
  if (rt.out) {  // the segments' counts, then the event the exchange waits for
    launch_route_counts(c->stream, rt.world, rt.segw, rt.cur, ROUTE_CUR_STRIDE, rt.out);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev_route, c->stream));
    c->rt_armed = false;
    c->rt_routed = c->rt_in_join = true;
  }
  // (KMZ_ABLATE2 bit 15, for comparison: with a chain table past the MALL
  // the certificate beside the settle instead of on the main stream between
  // the join and the walk.  Config 5: 8.31 against 8.00 ms, the settle's
  // probes and the certificate slow each other down; profiles/r05/ab/defer/)
  if (!early && !c->no_cert && !cert_side && c->overlap && (c->ablate2 & 32768u)) {
    c->cert_defer = true;
    c->cert_pl = pl;
  } else if (!early && !c->no_cert) {
    if (cert_side) {  // the certificate checks the join's ids beside the chain walk (read after the run)
      // on a stream of its own, from the end of the join, not behind K3 on
      // the side stream (KMZ_ABLATE2 bit 14: behind it, for comparison)
      hipStream_t cs = (c->ablate2 & 16384u) ? c->side : cert_stream(c);
      if (!cs) return fail(c, KMZ_E_HIP, "hipStreamCreateWithFlags (certificate stream)");
      HIPCHK(c, hipEventRecord(c->ev_join, c->stream));
      HIPCHK(c, hipStreamWaitEvent(cs, c->ev_join, 0));
      c->stream = cs;
      c->cert2 = cs == c->side2;
    }
    {
      Timed t(c, KMZ_K_CERT);
      launch_cert_split(c->stream, n, P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir), pl,
                        P<unsigned long long>(c->cpool2), cur2, cnt);
    }
    {
      Timed t(c, KMZ_K_CHECK);
      launch_cert_check(c->stream, n, pl, P<unsigned long long>(c->cpool2), cur2, cnt);
    }
    c->stream = c->main;
  }
  {
    // parents outside the window / chains leaving it: these kernels read the
    // join's counters and return at once when there is nothing to do, so the
    // host never waits here.  The certificate is read after the run: if an id
    // repeats, kmz_run discards the run and takes the table path.
    Timed t(c, KMZ_K_RESOLVE);
    launch_miss(c->stream, c->sid, c->pid, P<uint32_t>(c->dp), n, P<unsigned long long>(c->mkey),
                P<uint32_t>(c->mval), c->mcap, cnt);
    launch_pend(c->stream, c->kind, P<uint32_t>(c->dp), n, P<uint32_t>(c->cparent), cnt);
  }
  *ok = true;
  return KMZ_OK;
}

// K1 (global span-id table) + K2: any batch, including repeated span ids
static int run_table(kmz_ctx *c) {
  const uint32_t n = (uint32_t)c->n;
  c->cap = c->n * 5 / 3 + 64;  // load factor 0.6
  if (ensure(c, c->table, c->cap * 8) || ensure(c, c->dups, (size_t)(n + 1) * sizeof(DupEntry)) ||
      ensure(c, c->dkey, (size_t)c->dcap * 4) || ensure(c, c->dval, (size_t)c->dcap * 4))
    return KMZ_E_HIP;
  unsigned int *cnt = P<unsigned int>(c->counters);
  {
    Timed t(c, KMZ_K_MEMSET);
    HIPCHK(c, hipMemsetAsync(c->table.p, 0, c->cap * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(c->dkey.p, 0, (size_t)c->dcap * 4, c->stream));
    HIPCHK(c, hipMemsetAsync(c->dval.p, 0xFF, (size_t)c->dcap * 4, c->stream));
  }
  {
    Timed t(c, KMZ_K_BUILD);
    launch_build(c->stream, c->sid, n, P<unsigned long long>(c->table), c->cap, P<DupEntry>(c->dups), n + 1, cnt);
  }
  {
    Timed t(c, KMZ_K_FIXUP);
    launch_fixup(c->stream, P<DupEntry>(c->dups), cnt, n + 1, P<unsigned long long>(c->table), P<unsigned int>(c->dkey),
                 P<unsigned int>(c->dval), c->dcap);
  }
  {
    Timed t(c, KMZ_K_RESOLVE);
    launch_resolve(c->stream, c->sid, c->pid, c->kind, n, P<unsigned long long>(c->table), c->cap,
                   P<uint32_t>(c->cparent), cnt);
  }
  return KMZ_OK;
}

// K3 once per batch over (shape x status); every grouping the path needs is a
// union of these groups (k_collapse_groups / k_collapse_endpoints).
static int run_stats(kmz_ctx *c, uint32_t mode);

static int run_shape_stats(kmz_ctx *c) {
  const uint32_t n = (uint32_t)c->n;
  const uint64_t Gs = (uint64_t)c->n_shapes * c->n_status;
  if (Gs >= 0xFFFFFFFFull) return fail(c, KMZ_E_ARG, "too many (shape x status) groups");
  // (the shape-level group partials, then the partitioned K3's escape block E)
  if (ensure(c, c->sgrp, (Gs + 1) * 48 * 2)) return KMZ_E_HIP;
  unsigned long long *sg = P<unsigned long long>(c->sgrp);
  unsigned long long *E = sg + 6 * Gs;
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned long long *nsrv = P<unsigned long long>(c->stats64) + S_SERVER;
  const bool part = Gs > 1024 && k3_partitions((uint32_t)Gs) <= k3_pmax() && !(c->ablate & 8);
  {
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    f.add(sg, Gs * 40, 0);
    f.add(sg + 5 * Gs, Gs * 8, 0xFF);
    if (part) {
      f.add(E, Gs * 40, 0);
      f.add(E + 5 * Gs, Gs * 8, 0xFF);
    }
    launch_fill(c->stream, f);
  }
  if (part) {
    const uint32_t Pp = k3_partitions((uint32_t)Gs), nt = k3_tiles(n);
    // slices per partition: enough workgroups to fill the GPU at scale; one
    // for small batches, whose reduce then writes the group partials directly
    // (no k3_combine over S x G: at a 2 500-trace tick of the mesh, 34 slices
    // x 6 x 60k groups made the combine cost more than the records)
#ifndef KMZ_K3_SMALL_S
#define KMZ_K3_SMALL_S 1
#endif
    const uint32_t S = (KMZ_K3_SMALL_S && nt <= 64) ? 1u
                                                     : std::max<uint32_t>(1, std::min<uint32_t>({64u, 2048 / Pp,
                                                                                                  std::max(nt / 32, 1u)}));
    // larger batches: work items sized by each partition's records (the
    // partitions are far from equal: hot endpoints); KMZ_ABLATE bit 14: S
    // fixed slices per partition, for comparison
    const bool bal = S > 1 && !(c->ablate & (1u << 14));
    const uint32_t Sd = bal ? 1u : S;  // the directory's slices ([partition][tile] for the balanced reduce)
    if (ensure(c, c->k3pool, k3_pool_bytes(n)) || ensure(c, c->k3dir, (k3_dir_words(n, Pp, Sd) + k3_plan_words(Pp) + 1) * 4) ||
        ensure(c, c->k3part, bal ? k3_bal_part_bytes((uint32_t)Gs) : k3_slice_part_bytes((uint32_t)Gs, S)) ||
        ensure(c, c->tile_tmp, (size_t)nt * 16))
      return KMZ_E_HIP;
    {
      Timed t(c, KMZ_K_STATS);
      launch_k3_produce(c->stream, c->kind, c->shape, c->status, c->dur, c->ts, n, nullptr, c->n_shapes, c->n_shapes,
                        c->n_status, Sd, cnt, nsrv, c->k3pool.p, P<uint32_t>(c->k3dir), P<uint32_t>(c->tile_tmp));
    }
    {
      Timed t(c, KMZ_K_REDUCE);
      if (bal)
        launch_k3_reduce_bal(c->stream, n, (uint32_t)Gs, c->k3pool.p, P<uint32_t>(c->k3dir),
                             P<uint32_t>(c->k3dir) + k3_dir_words(n, Pp, 1), P<unsigned long long>(c->k3part), sg,
                             (c->ablate & (1u << 15)) != 0);  // (bit 15, test knob: unpacked accumulators)
      else
        launch_k3_reduce(c->stream, n, (uint32_t)Gs, c->k3pool.p, P<uint32_t>(c->k3dir),
                         P<unsigned long long>(c->k3part), S, sg);
      launch_k3_first(c->stream, c->kind, c->shape, c->status, n, nullptr, c->n_shapes, c->n_status, c->index_base,
                      (uint32_t)Gs, sg, cnt);
      launch_k3_escapes(c->stream, c->kind, c->shape, c->status, c->dur, c->ts, n, nullptr, c->n_shapes, c->n_status,
                        c->index_base, c->k3pool.p, cnt, E, (uint32_t)Gs, sg);
    }
  } else if (Gs <= 1024 && !(c->ablate & 8)) {
    const uint32_t nb = k3_small_blocks(n);
    if (ensure(c, c->k3part, (size_t)nb * 6 * Gs * 8) || ensure(c, c->tile_tmp, (size_t)nb * 16)) return KMZ_E_HIP;
    Timed t(c, KMZ_K_STATS);
    launch_k3_small(c->stream, c->kind, c->shape, c->status, c->dur, c->ts, n, nullptr, c->n_shapes, c->n_shapes,
                    c->n_status, c->index_base, cnt, nsrv, P<unsigned long long>(c->k3part), P<uint32_t>(c->tile_tmp), sg);
  } else {
    Timed t(c, KMZ_K_STATS);
    launch_stats(c->stream, c->kind, c->shape, c->status, c->dur, c->ts, n, nullptr, c->n_shapes, c->n_shapes,
                 c->n_status, c->index_base, sg, cnt, nsrv);
  }
  c->sstats = true;
  return KMZ_OK;
}

// bytes of K4 key staging (and as many again of slice buckets): 4 GB, or
// 40 B per span for larger batches (HBM is 288 GB)
static uint64_t stage_limit(uint64_t n) { return std::max<uint64_t>(4ull << 30, 40ull * n); }

static bool k4_direct(kmz_ctx *c) {
  if (c->ablate & (1u << 28)) return true;  // test knobs: force direct enumeration / chain interning
  if (c->ablate & (1u << 29)) return false;
  const uint64_t key = ((uint64_t)c->n_shapes << 32) | c->n_dep;
  if (key != c->k4_key) {
    c->k4_key = key;
    c->k4_auto_direct = false;
    c->k4_since = 0;
  }
  // (small batches: either mode is quick, keep interning)
  return c->k4_auto_direct && c->n >= (1u << 20) && (++c->k4_since % 64) != 0;
}

// The join and the chain walk of chain interning as one kernel per LDS window
// (kmz_fuse.hip), then the certificate, the MISS / PEND fix-ups, the settle of
// the staged keys and deferred checks, and the pending ancestries -- the same
// outputs as run_join + the chain path of run_deps.  Taken by window-join runs
// that intern chains on batches of [KMZ_FUSE_MIN, KMZ_FUSE_MAX) spans: there
// one kernel instead of two pays (mesh 10^6: 0.57 -> 0.49 ms/step, 4*10^6:
// 0.70 -> 0.67; Bookinfo 10^6: 0.37 -> 0.24).  At 10^8 spans the fused kernel
// (64 KB of LDS and ~112 VGPRs per 512-thread workgroup: 2 workgroups per CU,
// each a chain of dependent round trips: loads, probes, claims) took 2.72 ms
// against 1.09 + 1.11 ms for k_join_window + the persistent, prefetching
// k4_chain; at a 2 500-trace tick (68k mesh / 142k config-5 spans: 33 / 70
// workgroups) 320 / 569 us against 304 / 487 us per run.  KMZ_ABLATE2 bit 4:
// never fused; bit 5: fused at any size (tests/bench_tick.py).
#ifndef KMZ_FUSE_MIN
#define KMZ_FUSE_MIN (1u << 19)
#endif
#ifndef KMZ_FUSE_MAX
#define KMZ_FUSE_MAX (1u << 23)
#endif
static bool fused_eligible(kmz_ctx *c) {
  CertPlan pl;
  const bool size_ok = (c->n >= KMZ_FUSE_MIN && c->n < KMZ_FUSE_MAX) || (c->ablate2 & 32u);
  return c->n > 0 && size_ok && !c->k4_now && !(c->ablate2 & 16u) && !c->table_hint && !(c->ablate & (32u | 16u)) &&
         !c->walk_once && cert_plan((uint32_t)c->n, &pl, true, (c->ablate2 & 64u) != 0) &&
         pl.B1 == 6;  // (the fused kernel bins by 2^6)
}

static int run_fused(kmz_ctx *c, bool links) {
  const uint32_t n = (uint32_t)c->n;
  CertPlan pl;  // (the plan fused_eligible accepted: same arguments)
  if (!cert_plan(n, &pl, true, (c->ablate2 & 64u) != 0) || pl.B1 != 6)
    return fail(c, KMZ_E_STATE, "fused join + walk: certificate plan is not the kernel's 2^6 pass-1 binning");
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned int *cur2 = P<unsigned int>(c->ccur);
  unsigned long long *st = P<unsigned long long>(c->stats64);
  unsigned long long *epp = P<unsigned long long>(c->epp);
  if (!c->sstats) {
    int r = run_shape_stats(c);
    if (r) return r;
  }
  // the global lists: staged keys (as many as the per-workgroup runs of the
  // two-kernel path hold), deferred checks (KMZ_ABLATE bit 10, test knob: 4,
  // so that leaders fall through to the in-place chain_put waits), claimed slots
  while (!(c->ablate & (1u << 30)) && (uint64_t)c->scap * chain_grid(n) < 8ull * n &&
         (uint64_t)chain_grid(n) * c->scap * 2 * 8 <= stage_limit(n))
    c->scap *= 2;
  const uint32_t ng = chain_grid(n), wcap = 1u << 16;
  // (staged keys: only new chains stage; <= 2^28 keys, 2 GB, whatever the batch)
  const uint64_t stot = std::min<uint64_t>((uint64_t)ng * c->scap, 1ull << 28), dtot = (c->ablate & (1u << 10)) ? 4u : (uint64_t)ng << 12,
                 gtot = ((uint64_t)ng + 1) * wcap;
  if (stot >= (1ull << 32) || dtot >= (1ull << 32) || gtot >= (1ull << 32))
    return fail(c, KMZ_E_ARG, "fused join + walk: list sizes past 2^32");
  void *old_ctab = c->ctab.p;
  if (ensure(c, c->dp, (size_t)(n + 1) * 4) || ensure(c, c->cpool1, cert_pool1_words(n) * 8) ||
      ensure(c, c->cpool2, cert_pool2_bytes(pl)) || ensure(c, c->ccur, cert_cur_words(pl) * 4) ||
      ensure(c, c->cdir, cert_dir_entries(n, pl) * 2) || ensure(c, c->mkey, (size_t)c->mcap * 8) ||
      ensure(c, c->mval, (size_t)c->mcap * 4) || ensure(c, c->ctab, c->ccap * CHAIN_ENTRY_BYTES) ||
      ensure(c, c->ctile, (size_t)chain_tiles(n) * 16) || ensure(c, c->plist, (size_t)(n + 1) * 4) ||
      ensure(c, c->kstage, stot * 8) || ensure(c, c->kdefer, dtot * 16) || ensure(c, c->kwpos, gtot * 4) ||
      ensure(c, c->cetab, ((size_t)c->n_shapes + 1) * 16))
    return KMZ_E_HIP;
  cur2 = P<unsigned int>(c->ccur);
  if (c->ctab.p != old_ctab) c->ctab_dirty = true;
  uint32_t *gpos = P<uint32_t>(c->kwpos);
  {
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    f.add(cur2, cert_cur_words(pl) * 4, 0);
    f.add(c->mkey.p, (size_t)c->mcap * 8, 0);
    f.add(c->mval.p, (size_t)c->mcap * 4, 0xFF);  // ids not in the batch: NONE
    if (c->ctab_dirty) f.add(c->ctab.p, c->ccap * CHAIN_ENTRY_BYTES, 0);
    f.add(c->trip.p, c->tcap * 8, 0);
    launch_fill(c->stream, f);
  }
  c->ctab_dirty = true;  // until this run's slots are cleared below
  {
    Timed t(c, KMZ_K_JOINWALK);
    launch_join_chain(c->stream, c->sid, c->pid, c->kind, c->shape, c->ts, n, P<uint32_t>(c->d_dep), c->n_shapes,
                      c->n_dep, c->index_base, c->sig_seed, P<uint32_t>(c->cparent), P<uint32_t>(c->dp),
                      P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir), cnt, c->ctab.p, c->ccap,
                      P<unsigned long long>(c->trip), c->tcap, epp, links ? P<unsigned long long>(c->rowpos) : nullptr,
                      P<uint32_t>(c->plist), n + 1, P<uint32_t>(c->ctile), P<unsigned long long>(c->kstage),
                      (uint32_t)stot, P<unsigned long long>(c->kdefer), (uint32_t)dtot, gpos, (uint32_t)gtot,
                      P<uint4>(c->cetab),
                      // (test knob 24 forces sig collisions on the first seed only)
                      c->sig_seed == SIG_SEED0 ? c->ablate : (c->ablate & ~(1u << 24)), n > 0 && etab_cached(c));
  }
  // the certificate beside the settle (small batches), as run_join
  const bool cert_side = c->overlap && !(c->ablate & (1u << 26)) && c->ccap * CHAIN_ENTRY_BYTES <= (256ull << 20);
  if (cert_side && !c->no_cert) {
    HIPCHK(c, hipEventRecord(c->ev_join, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_join, 0));
    c->stream = c->side;
  }
  if (!c->no_cert) {  // (KMZ_RUN_NO_CERT: the fused kernel's pass 1 still runs, unread)
    {
      Timed t(c, KMZ_K_CERT);
      launch_cert_split(c->stream, n, P<unsigned long long>(c->cpool1), P<uint16_t>(c->cdir), pl,
                        P<unsigned long long>(c->cpool2), cur2, cnt);
    }
    {
      Timed t(c, KMZ_K_CHECK);
      launch_cert_check(c->stream, n, pl, P<unsigned long long>(c->cpool2), cur2, cnt);
    }
  }
  c->stream = c->main;
  {
    Timed t(c, KMZ_K_RESOLVE);
    launch_miss(c->stream, c->sid, c->pid, P<uint32_t>(c->dp), n, P<unsigned long long>(c->mkey),
                P<uint32_t>(c->mval), c->mcap, cnt);
    launch_pend(c->stream, c->kind, P<uint32_t>(c->dp), n, P<uint32_t>(c->cparent), cnt);
  }
  {
    Timed t(c, KMZ_K_SETTLE);
    launch_chain_settle_list(c->stream, join_tiles(n), c->ctab.p, c->ccap, P<unsigned long long>(c->trip), c->tcap, cnt,
                             P<uint32_t>(c->ctile), st, P<unsigned long long>(c->kstage), (uint32_t)stot,
                             P<unsigned long long>(c->kdefer), (uint32_t)dtot, gpos, (uint32_t)gtot, c->ablate);
  }
  {
    Timed t(c, KMZ_K_PEND);
    launch_chain_pend(c->stream, P<uint32_t>(c->plist), n + 1, c->kind, c->shape, c->ts, P<uint32_t>(c->cparent), n,
                      P<uint32_t>(c->d_dep), c->n_shapes, c->n_dep, c->sig_seed, c->ctab.p, c->ccap,
                      P<unsigned long long>(c->trip), c->tcap, epp, cnt, st, gpos, (uint32_t)gtot, false, c->ablate);
  }
  if (c->overlap) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_k3, 0));  // the shape-level K3 partials
  {
    Timed t(c, KMZ_K_FINAL);
    launch_compact(c->stream, P<unsigned long long>(c->trip), c->tcap, P<unsigned long long>(c->trip_out),
                   st + S_TRIP_OUT);
    launch_collapse_endpoints(c->stream, P<unsigned long long>(c->sgrp), c->n_shapes, c->n_status,
                              P<uint32_t>(c->d_dep), c->n_dep, P<uint32_t>(c->cparent), c->index_base, epp,
                              epp + c->n_dep, cnt);
    launch_chain_clear_list(c->stream, c->ctab.p, gpos, (uint32_t)gtot, cnt);
  }
  c->ctab_dirty = false;  // (set again after the run if the list overflowed: F_CTAB_DIRTY)
  c->path = 1 | 2 | 16;
  c->chain_ran = true;
  c->k4_direct_ran = false;
  c->k4_lb1 = 0;
  c->k4_ng = ng;
  return KMZ_OK;
}

// K4 by chain interning with one workgroup per tile (k4_tile, kmz_walk.hip):
// the same global lists, settle, pending pass and slot clearing as the fused
// kernel's tail (run_fused), after the window join (run_join / run_table).
static int run_chain_tiles(kmz_ctx *c, bool links, bool joined) {
  rb_mark(c, "chain:entry");
  const uint32_t n = (uint32_t)c->n;
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned long long *st = P<unsigned long long>(c->stats64);
  unsigned long long *epp = P<unsigned long long>(c->epp);
  // the global lists (as run_fused): staged keys of new chains, deferred checks
  // (KMZ_ABLATE bit 10, test knob: 4), claimed slots
  while (!(c->ablate & (1u << 30)) && (uint64_t)c->scap * chain_grid(n) < 8ull * n &&
         (uint64_t)chain_grid(n) * c->scap * 2 * 8 <= stage_limit(n))
    c->scap *= 2;
  const uint32_t nt = walk_tiles(n), ng = chain_grid(n), wcap = 1u << 16;
  const uint64_t stot = std::min<uint64_t>((uint64_t)ng * c->scap, 1ull << 28),
                 dtot = (c->ablate & (1u << 10)) ? 4u : (uint64_t)ng << 12, gtot = ((uint64_t)ng + 1) * wcap;
  if (stot >= (1ull << 32) || dtot >= (1ull << 32) || gtot >= (1ull << 32))
    return fail(c, KMZ_E_ARG, "chain walk: list sizes past 2^32");
  void *old_ctab = c->ctab.p;
  if (ensure(c, c->ctab, c->ccap * CHAIN_ENTRY_BYTES) || ensure(c, c->ctile, (size_t)nt * 16) ||
      ensure(c, c->plist, (size_t)(n + 1) * 4) || ensure(c, c->kstage, stot * 8) || ensure(c, c->kdefer, dtot * 16) ||
      ensure(c, c->kwpos, gtot * 4) || ensure(c, c->cetab, ((size_t)c->n_shapes + 1) * 16))
    return KMZ_E_HIP;
  const bool w8 = !(c->ablate2 & 1024u), by_shape = w8 && c->dep_valid && !(c->ablate2 & 2048u);
  // k4_tile9 where the ids fit its 19-bit record field (KMZ_ABLATE2 bit 22:
  // k4_tile8, for comparison)
  const bool w9 = w8 && !(c->ablate2 & (1u << 22)) && chain_tile9_fits(by_shape ? c->n_shapes : c->n_dep);
  if (c->ctab.p != old_ctab) c->ctab_dirty = true;
  uint32_t *gpos = P<uint32_t>(c->kwpos);
  {
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    if (c->ctab_dirty) f.add(c->ctab.p, c->ccap * CHAIN_ENTRY_BYTES, 0);
    f.add(c->trip.p, c->tcap * 8, 0);
    launch_fill(c->stream, f);
  }
  c->ctab_dirty = true;  // until this run's slots are cleared below
  {
    ChainRun a;
    a.ts = c->ts;
    a.ctab = P<unsigned long long>(c->ctab);
    a.ccap = c->ccap;
    a.trip = P<unsigned long long>(c->trip);
    a.tcap = c->tcap;
    a.ep_ts = epp;
    a.rowpos_out = links ? P<unsigned long long>(c->rowpos) : nullptr;
    a.plist = P<uint32_t>(c->plist);
    a.pcap = n + 1;
    a.counters = cnt;
    a.stage = P<unsigned long long>(c->kstage);
    a.scap = (uint32_t)stot;
    a.defer = P<unsigned long long>(c->kdefer);
    a.dcap = (uint32_t)dtot;
    a.gpos = gpos;
    a.gcap = (uint32_t)gtot;
    a.n_ep = c->n_dep;
    a.index_base = c->index_base;
    a.seed = c->sig_seed;
    // (test knob 24 forces sig collisions on the first seed only)
    a.ablate = c->sig_seed == SIG_SEED0 ? c->ablate : (c->ablate & ~(1u << 24));
    // k4_tile8 (8-byte window records; KMZ_ABLATE2 bit 10: the 16-byte
    // k4_tile, for comparison).  Its chain elements are shapes when the
    // dependency table maps every shape into range (bit 11: endpoints
    // anyway): no gather before the window is built; the leaders map their
    // keys' shapes to endpoints
    a.id_ep = by_shape ? P<uint32_t>(c->d_dep) : nullptr;
    a.n_ids = c->n_shapes;
    {
      Timed t(c, KMZ_K_WALK);
      if (w9)
        launch_chain_tile9(c->stream, c->kind, c->shape, P<uint32_t>(c->cparent), n, P<uint32_t>(c->d_dep),
                           c->n_shapes, P<uint32_t>(c->ctile), a);
      else if (w8)
        launch_chain_tile8(c->stream, c->kind, c->shape, P<uint32_t>(c->cparent), n, P<uint32_t>(c->d_dep),
                           c->n_shapes, P<uint32_t>(c->ctile), a);
      else
        launch_chain_tile(c->stream, c->kind, c->shape, P<uint32_t>(c->cparent), n, P<uint32_t>(c->d_dep),
                          c->n_shapes, P<uint4>(c->cetab), P<uint32_t>(c->ctile), a);
    }
  }
  rb_mark(c, "walk:launch");
  if (int r2 = launch_cert_deferred(c)) return r2;
  if (c->k3_late && !c->sstats)
    if (int r2 = run_shape_stats(c)) return r2;
  {
    Timed t(c, KMZ_K_SETTLE);
    launch_chain_settle_list(c->stream, nt, c->ctab.p, c->ccap, P<unsigned long long>(c->trip), c->tcap, cnt,
                             P<uint32_t>(c->ctile), st, P<unsigned long long>(c->kstage), (uint32_t)stot,
                             P<unsigned long long>(c->kdefer), (uint32_t)dtot, gpos, (uint32_t)gtot, c->ablate,
                             by_shape ? P<uint32_t>(c->d_dep) : nullptr, c->n_shapes);
  }
  {
    Timed t(c, KMZ_K_PEND);
    launch_chain_pend(c->stream, P<uint32_t>(c->plist), n + 1, c->kind, c->shape, c->ts, P<uint32_t>(c->cparent), n,
                      P<uint32_t>(c->d_dep), c->n_shapes, c->n_dep, c->sig_seed, c->ctab.p, c->ccap,
                      P<unsigned long long>(c->trip), c->tcap, epp, cnt, st, gpos, (uint32_t)gtot, false, c->ablate, by_shape);
  }
  if (c->overlap) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_k3, 0));  // the shape-level K3 partials
  {
    Timed t(c, KMZ_K_FINAL);
    launch_compact(c->stream, P<unsigned long long>(c->trip), c->tcap, P<unsigned long long>(c->trip_out),
                   st + S_TRIP_OUT);
    launch_collapse_endpoints(c->stream, P<unsigned long long>(c->sgrp), c->n_shapes, c->n_status,
                              P<uint32_t>(c->d_dep), c->n_dep, P<uint32_t>(c->cparent), c->index_base, epp,
                              epp + c->n_dep, cnt);
    launch_chain_clear_list(c->stream, c->ctab.p, gpos, (uint32_t)gtot, cnt);
  }
  c->ctab_dirty = false;  // (set again after the run if the list overflowed: F_CTAB_DIRTY)
  c->path = (joined ? 1 : 0) | 2 | 32 | (w9 ? 64 : 0);
  c->chain_ran = true;
  c->k4_direct_ran = false;
  c->k4_lb1 = 0;
  c->k4_ng = ng;
  return KMZ_OK;
}

static int run_deps(kmz_ctx *c, bool links) {
  const uint32_t n = (uint32_t)c->n;
  // unique edge keys are far fewer than spans; start at ~n/32 (grown on overflow)
  while (c->tcap < (1ull << 26) && c->tcap * 32 < c->n) c->tcap *= 2;
  if (ensure(c, c->cparent, (size_t)(n + 1) * 4) || ensure(c, c->epp, (size_t)(c->n_dep + 1) * 16) ||
      (links && ensure(c, c->rowpos, (size_t)(n + 1) * 8)))
    return KMZ_E_HIP;
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned long long *st = P<unsigned long long>(c->stats64);
  unsigned long long *epp = P<unsigned long long>(c->epp);
  if (!c->epp_filled) {  // (run_enqueue fills it with the counters)
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    f.add(epp, (size_t)c->n_dep * 8, 0);
    f.add(epp + c->n_dep, (size_t)c->n_dep * 8, 0xFF);
    launch_fill(c->stream, f);
  }
  if (fused_eligible(c)) {
    if (ensure(c, c->trip, c->tcap * 8) || ensure(c, c->trip_out, c->tcap * 8)) return KMZ_E_HIP;
    return run_fused(c, links);
  }
  bool joined = false;
  int r = run_join(c, &joined);
  if (r) return r;
  uint32_t dups = 0;
  if (!joined) {
    c->cap = 0;
    if ((r = run_table(c))) return r;
    unsigned int hc[C_COUNT];
    HIPCHK(c, hipMemcpyAsync(hc, c->counters.p, sizeof(hc), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dups = hc[C_DUPS];
  }
  if (ensure(c, c->trip, c->tcap * 8) || ensure(c, c->trip_out, c->tcap * 8)) return KMZ_E_HIP;
  if (dups == 0 && !(c->ablate & 16) && !c->walk_once && !c->k4_now && !(c->ablate2 & 256u)) {
    // unique span ids, chain interning: one workgroup per tile (kmz_walk.hip)
    if (!c->sstats && !c->k3_late && (r = run_shape_stats(c))) return r;
    return run_chain_tiles(c, links, joined);
  }
  if (dups == 0 && !(c->ablate & 16) && !c->walk_once) {
    // unique span ids: rows are the SERVER spans; chain interning (kmz_chain.hip)
    if (!c->sstats && !c->k3_settle && (r = run_shape_stats(c))) return r;
    const uint32_t nt = chain_tiles(n);
    const bool direct = c->k4_now;
    // per persistent workgroup: staged keys (of candidate new chains, or of
    // every row when direct) in one run per coarse bin of the edge set's
    // slices, and deferred chain checks (overflow is handled in place, just
    // slower) and the slots each workgroup claims in the chain table (wcap
    // each; the run's global list of wcap more follows them); the staged keys
    // partitioned per slice (as many again)
    // (a batch starts with staging for ~8 keys per span -- direct enumeration
    // of config 5 stages ~4.5 -- within the staging limit)
    while (!(c->ablate & (1u << 30)) && (uint64_t)c->scap * chain_grid(n) < 8ull * n &&
           (uint64_t)chain_grid(n) * c->scap * 2 * 8 <= stage_limit(n))
      c->scap *= 2;
    // deferred chain checks per workgroup (KMZ_ABLATE bit 10, test knob: 4, so
    // that leaders fall through to the in-place chain_put waits)
    const uint32_t scap = c->scap, dcap = (c->ablate & (1u << 10)) ? 4u : 1u << 12, wcap = 1u << 16,
                   ng = chain_grid(n);
    uint32_t lb1, lb2;
    if (!key_bins(c->tcap, &lb1, &lb2)) return fail(c, KMZ_E_ARG, "edge-set capacity is not ESLICE * 2^k");
    // slice buckets (direct enumeration): KMZ_BUCKET_X times the mean fill --
    // hot endpoints concentrate keys in a few slices (config 5: the fullest
    // slice holds ~3x the mean), and what overflows is inserted in place
#ifndef KMZ_BUCKET_X
#define KMZ_BUCKET_X 3  // (x1 -> x3: config 5's k_key_part + k_key_slice 2.97 -> 2.69 ms)
#endif
    const uint64_t nsl = c->tcap / ESLICE, bmean = ((uint64_t)ng * scap + nsl - 1) / nsl;
    const uint64_t bcap = direct ? std::min<uint64_t>(bmean * KMZ_BUCKET_X, std::max<uint64_t>(bmean, (12ull << 30) / 8 / nsl))
                                 : bmean;
    // direct enumeration stages 4-byte keys where every edge key of the batch
    // can be compact (dependency endpoints < 2^16; a key with a distance >= 32
    // is inserted in place) -- half the bytes of the walk's staging writes,
    // k_key_part and k_key_slice (KMZ_ABLATE2 bit 0: 8-byte keys, for comparison)
    const bool cmode = direct && compact_staging(c->tcap, c->n_dep) && !(c->ablate2 & 1u);
    void *old_ctab = c->ctab.p;
    c->k4_lb1 = direct ? lb1 : 0;
    c->k4_nsl = (uint32_t)nsl;
    c->k4_ng = ng;
    if (ensure(c, c->ctab, c->ccap * CHAIN_ENTRY_BYTES) || ensure(c, c->ctile, (size_t)nt * 16) ||
        ensure(c, c->plist, (size_t)(n + 1) * 4) || ensure(c, c->kstage, (size_t)ng * scap * 8) ||
        ensure(c, c->kstage_n, ((size_t)ng << lb1) * 4) || ensure(c, c->kdefer, (size_t)ng * dcap * 16) ||
        ensure(c, c->kdefer_n, (size_t)ng * 4) || ensure(c, c->kwpos, ((size_t)ng + 1) * wcap * 4) ||
        ensure(c, c->kwpos_n, (size_t)ng * 4) || ensure(c, c->cetab, ((size_t)c->n_shapes + 1) * 16) ||
        ensure(c, c->kbucket, nsl * bcap * 8) || ensure(c, c->kbucket_n, nsl * 4))
      return KMZ_E_HIP;
    if (c->ctab.p != old_ctab) c->ctab_dirty = true;
    uint32_t *wpos = P<uint32_t>(c->kwpos), *gpos = wpos + (size_t)ng * wcap;
    {
      Timed t(c, KMZ_K_MEMSET);
      // the chain table is cleared entry by entry after each run; a full
      // memset only when it is new or a list overflowed
      FillArgs f;
      if (c->ctab_dirty && !direct) f.add(c->ctab.p, c->ccap * CHAIN_ENTRY_BYTES, 0);
      f.add(c->trip.p, c->tcap * 8, 0);
      f.add(c->kbucket_n.p, nsl * 4, 0);
      launch_fill(c->stream, f);
    }
    const bool was_dirty = c->ctab_dirty;
    if (!direct) c->ctab_dirty = true;  // until this run's slots are cleared below
    {
      Timed t(c, KMZ_K_WALK);
      launch_chain(c->stream, c->kind, c->shape, c->ts, P<uint32_t>(c->cparent), n, P<uint32_t>(c->d_dep),
                   c->n_shapes, c->n_dep, c->index_base, c->sig_seed, c->ctab.p, c->ccap,
                   P<unsigned long long>(c->trip), c->tcap, epp, links ? P<unsigned long long>(c->rowpos) : nullptr,
                   P<uint32_t>(c->plist), n + 1, cnt, P<uint32_t>(c->ctile), st, P<unsigned long long>(c->kstage),
                   scap, P<uint32_t>(c->kstage_n), P<unsigned long long>(c->kdefer), dcap, P<uint32_t>(c->kdefer_n),
                   wpos, wcap, P<uint32_t>(c->kwpos_n), P<uint4>(c->cetab), direct,
                   // (test knob 24 forces sig collisions on the first seed only)
                   c->sig_seed == SIG_SEED0 ? c->ablate : (c->ablate & ~(1u << 24)), cmode,
                   n > 0 && etab_cached(c));
    }
    if (int r2 = launch_cert_deferred(c)) return r2;
    if (c->k3_settle) {  // K3 beside the settle (run_enqueue)
      HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
      HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
      c->stream = c->side;
      const int r2 = run_stats(c, c->k3_mode);
      c->stream = c->main;
      if (r2) return r2;
      HIPCHK(c, hipEventRecord(c->ev_k3, c->side));
      c->k3_ran = true;
    }
    {
      Timed t(c, KMZ_K_SETTLE);
      launch_chain_settle(c->stream, n, direct, c->ctab.p, c->ccap, P<unsigned long long>(c->trip), c->tcap, cnt,
                          P<uint32_t>(c->ctile), st, P<unsigned long long>(c->kstage), scap,
                          P<uint32_t>(c->kstage_n), P<unsigned long long>(c->kbucket), bcap,
                          P<uint32_t>(c->kbucket_n), P<unsigned long long>(c->kdefer), dcap, P<uint32_t>(c->kdefer_n),
                          gpos, wcap, c->ablate, cmode, c->ablate2);
    }
    {  // ancestries that left their window: one pass, sized on the device (no host round trip)
      Timed t(c, KMZ_K_PEND);
      launch_chain_pend(c->stream, P<uint32_t>(c->plist), n + 1, c->kind, c->shape, c->ts, P<uint32_t>(c->cparent),
                        n, P<uint32_t>(c->d_dep), c->n_shapes, c->n_dep, c->sig_seed, c->ctab.p, c->ccap,
                        P<unsigned long long>(c->trip), c->tcap, epp, cnt, st, gpos, wcap, direct, c->ablate);
    }
    if (c->overlap) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_k3, 0));  // the shape-level K3 partials
    {
      Timed t(c, KMZ_K_FINAL);
      launch_compact(c->stream, P<unsigned long long>(c->trip), c->tcap, P<unsigned long long>(c->trip_out),
                     st + S_TRIP_OUT);
      launch_collapse_endpoints(c->stream, P<unsigned long long>(c->sgrp), c->n_shapes, c->n_status,
                                P<uint32_t>(c->d_dep), c->n_dep, P<uint32_t>(c->cparent), c->index_base, epp,
                                epp + c->n_dep, cnt);
      if (!direct) launch_chain_clear(c->stream, n, c->ctab.p, wpos, wcap, P<uint32_t>(c->kwpos_n), gpos, wcap, cnt);
    }
    // (set again after the run if a list overflowed: F_CTAB_DIRTY)
    c->ctab_dirty = direct ? was_dirty : false;
    c->path = (joined ? 1 : 0) | 2 | (direct ? 4 : 0);
    c->chain_ran = !direct;
    c->k4_direct_ran = direct;
    return KMZ_OK;
  }
  // repeated span ids: the row of an id is its last occurrence at its first
  // position; one global walk per row over the table path's links.  Also the
  // exact redo of a run whose chain-table wait ran out (F_SPIN): with unique
  // ids the walk reads no table.
  c->path = (joined ? 1 : 0) | (c->walk_once ? 8 : 0);
  HIPCHK(c, hipMemsetAsync(c->trip.p, 0, c->tcap * 8, c->stream));
  {
    // the table is read only for repeated ids (dups > 0), which implies run_table
    Timed t(c, KMZ_K_WALK);
    launch_walk(c->stream, c->sid, c->kind, c->shape, c->ts, P<uint32_t>(c->cparent), n, P<uint32_t>(c->d_dep),
                c->n_shapes, c->n_dep, c->index_base, P<unsigned long long>(c->table), c->cap,
                P<unsigned int>(c->dkey), P<unsigned int>(c->dval), c->dcap, P<unsigned long long>(c->trip), c->tcap,
                epp, epp + c->n_dep, links ? P<unsigned long long>(c->rowpos) : nullptr, cnt, st, c->ablate);
  }
  {
    Timed t(c, KMZ_K_FINAL);
    launch_compact(c->stream, P<unsigned long long>(c->trip), c->tcap, P<unsigned long long>(c->trip_out),
                   st + S_TRIP_OUT);
  }
  return KMZ_OK;
}

// finalisation of the endpoint groups, with the used groups compacted beside
// it where G allows (kmz_fetch_used)
static int finalize_groups(kmz_ctx *c) {
  const uint32_t G = c->G;
  c->gu_ok = G && used_chunks(G) <= USED_MAX_CHUNKS;
  if (c->gu_ok && (ensure(c, c->gu_ids, (size_t)G * 4) || ensure(c, c->gu_grp, (size_t)G * sizeof(kmz_group)) ||
                   ensure(c, c->gu_bcnt, (size_t)used_chunks(G) * 4)))
    return KMZ_E_HIP;
  GroupsUsed u{P<uint32_t>(c->gu_ids), P<uint32_t>(c->gu_bcnt), P<kmz_group>(c->gu_grp),
               P<unsigned long long>(c->stats64) + S_GUSED};
  launch_finalize(c->stream, P<unsigned long long>(c->grp), G, P<kmz_group>(c->grp_final), c->gu_ok ? &u : nullptr);
  return KMZ_OK;
}

static int run_stats(kmz_ctx *c, uint32_t mode) {
  uint32_t n_ep = mode == KMZ_RUN_STATS_RT ? c->n_rt : c->n_tag;
  const uint32_t *tab = mode == KMZ_RUN_STATS_RT ? P<uint32_t>(c->d_rt) : P<uint32_t>(c->d_tag);
  uint64_t G = (uint64_t)n_ep * c->n_status;
  if (G >= 0xFFFFFFFFull) return fail(c, KMZ_E_ARG, "too many groups");
  c->G = (uint32_t)G;
  c->ep_mode = mode;
  int r;
  if (!c->sstats && (r = run_shape_stats(c))) return r;
  if (ensure(c, c->grp, (G + 1) * 48) || ensure(c, c->grp_final, (G + 1) * sizeof(kmz_group))) return KMZ_E_HIP;
  unsigned long long *grp = P<unsigned long long>(c->grp);
  {
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    f.add(grp, G * 40, 0);
    f.add(grp + 5 * G, G * 8, 0xFF);
    launch_fill(c->stream, f);
  }
  {
    Timed t(c, KMZ_K_FINAL);
    launch_collapse_groups(c->stream, P<unsigned long long>(c->sgrp), c->n_shapes, c->n_status, tab, n_ep, grp,
                           P<unsigned int>(c->counters));
    if (int r2 = finalize_groups(c)) return r2;
  }
  return KMZ_OK;
}

// Entry order of the reduced graph (kmz_order.hip): after a successful
// dependency run with span links; synchronous (the record count sizes the
// index remap of a non-contiguous shard).
static int run_dep_order(kmz_ctx *c, uint64_t n_keys, bool dups) {
  const uint32_t n = (uint32_t)c->n;
  // by-entries and on-entries are each at most one per edge key: load <= 1/2
  uint64_t ecap = 1024;
  while (ecap < 4 * n_keys + 64) ecap *= 2;
  const uint64_t ocap = 2 * n_keys + 1;
  if (ensure(c, c->o_key, ecap * dep_order_slot_bytes()) || ensure(c, c->o_out, ocap * sizeof(kmz_dep_entry)) ||
      ensure(c, c->o_rts, ((size_t)c->n_dep + 1) * 8) || ensure(c, c->o_rsh, ((size_t)c->n_dep + 1) * 4) ||
      (dups && ensure(c, c->o_val, ((size_t)n + 1) * 4)))
    return KMZ_E_HIP;
  unsigned long long *cnt = P<unsigned long long>(c->stats64) + S_DEPENT;
  {
    Timed t(c, KMZ_K_ORDER);
    HIPCHK(c, hipMemsetAsync(c->o_key.p, 0xFF, ecap * dep_order_slot_bytes(), c->stream));
    HIPCHK(c, hipMemsetAsync(cnt, 0, 8, c->stream));
    launch_dep_order(c->stream, c->kind, c->shape, c->ts, P<uint32_t>(c->cparent), P<unsigned long long>(c->rowpos),
                     n, P<uint32_t>(c->d_dep), c->n_shapes, c->n_dep, c->index_base, c->o_key.p, ecap,
                     dups ? P<uint32_t>(c->o_val) : nullptr, P<unsigned long long>(c->epp) + c->n_dep,
                     P<kmz_dep_entry>(c->o_out), cnt, P<int64_t>(c->o_rts), P<uint32_t>(c->o_rsh),
                     P<unsigned int>(c->counters));
  }
  HIPCHK(c, hipGetLastError());
  unsigned long long m = 0;
  unsigned int fl = 0;
  HIPCHK(c, hipMemcpyAsync(&m, cnt, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&fl, P<unsigned int>(c->counters) + C_FLAGS, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((fl & F_TABLE_FULL) || m > ocap) return fail(c, KMZ_E_OVERFLOW, "entry-order table overflow");
  c->o_n = m;
  if (c->imap_n && m) {
    const uint64_t *ls = P<uint64_t>(c->imap_l), *gs = P<uint64_t>(c->imap_g);
    unsigned long long *o = P<unsigned long long>(c->o_out);
    for (int col = 1; col <= 3; ++col)  // row, span, pos
      launch_remap_index(c->stream, o + col, m, sizeof(kmz_dep_entry) / 8, 0, ls, gs, c->imap_n);
    HIPCHK(c, hipGetLastError());
  }
  return KMZ_OK;
}

int kmz_get_dep_entries(kmz_ctx *c, kmz_dep_entry *out, uint64_t cap, uint64_t *n_out, int64_t *row_ts,
                        uint32_t *row_shape, uint64_t row_cap) {
  if (!c || !n_out) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & KMZ_RUN_DEP_ORDER)) return fail(c, KMZ_E_STATE, "run with KMZ_RUN_DEPS|KMZ_RUN_DEP_ORDER first");
  *n_out = c->o_n;
  if (out && cap < c->o_n) return fail(c, KMZ_E_ARG, "output too small");
  if ((row_ts || row_shape) && row_cap < c->n_dep) return fail(c, KMZ_E_ARG, "output too small");
  if (out && c->o_n)
    HIPCHK(c, hipMemcpyAsync(out, c->o_out.p, c->o_n * sizeof(kmz_dep_entry), hipMemcpyDeviceToHost, c->stream));
  if (row_ts && c->n_dep) HIPCHK(c, hipMemcpyAsync(row_ts, c->o_rts.p, (size_t)c->n_dep * 8, hipMemcpyDeviceToHost, c->stream));
  if (row_shape && c->n_dep)
    HIPCHK(c, hipMemcpyAsync(row_shape, c->o_rsh.p, (size_t)c->n_dep * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

// A non-contiguous shard (kmz_set_index_map): the run used local flatten
// indices; map the order keys it reports to global ones (kmz_shard.hip).
static int remap_results(kmz_ctx *c, uint32_t flags, bool links) {
  const uint64_t *ls = P<uint64_t>(c->imap_l), *gs = P<uint64_t>(c->imap_g);
  if (flags & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG)) {
    launch_remap_index(c->stream, P<unsigned long long>(c->grp) + 5ull * c->G, c->G, 1, 0, ls, gs, c->imap_n);
    launch_remap_index(c->stream, P<unsigned long long>(c->grp_final) + 1, c->G, sizeof(kmz_group) / 8, 0, ls, gs,
                       c->imap_n);
    if (c->gu_ok)  // (entries past the used count are remapped too: harmless)
      launch_remap_index(c->stream, P<unsigned long long>(c->gu_grp) + 1, c->G, sizeof(kmz_group) / 8, 0, ls, gs,
                         c->imap_n);
  }
  if (flags & KMZ_RUN_DEPS) {
    launch_remap_index(c->stream, P<unsigned long long>(c->epp) + c->n_dep, c->n_dep, 1, 1, ls, gs, c->imap_n);
    if (links) launch_remap_index(c->stream, P<unsigned long long>(c->rowpos), c->n, 1, 0, ls, gs, c->imap_n);
  }
  HIPCHK(c, hipGetLastError());
  return KMZ_OK;
}

int kmz_set_index_map(kmz_ctx *c, const uint64_t *local_start, const uint64_t *global_start, uint64_t n_runs) {
  if (!c || (n_runs && (!local_start || !global_start))) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_set_index_map before kmz_load");
  if (n_runs == 0) {
    c->imap_n = 0;
    return KMZ_OK;
  }
  if (local_start[0] != 0) return fail(c, KMZ_E_ARG, "the first run must start at local index 0");
  for (uint64_t k = 1; k < n_runs; ++k)
    if (local_start[k] < local_start[k - 1] || (local_start[k] > local_start[k - 1] &&
                                                global_start[k] < global_start[k - 1] + (local_start[k] - local_start[k - 1])))
      return fail(c, KMZ_E_ARG, "index map runs must be ordered and non-overlapping");
  if (ensure(c, c->imap_l, n_runs * 8) || ensure(c, c->imap_g, n_runs * 8)) return KMZ_E_HIP;
  HIPCHK(c, hipMemcpyAsync(c->imap_l.p, local_start, n_runs * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->imap_g.p, global_start, n_runs * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->imap_n = n_runs;
  c->index_base = 0;  // the run works on local indices; results are mapped
  c->ran = 0;
  c->hpin_valid = false;
  return KMZ_OK;
}

uint32_t kmz_trace_shard(const char *trace_id, uint64_t len, uint32_t world) {
  if (world <= 1) return 0;
  uint64_t hi = 0, lo = 0;
  bool hex = trace_id && (len == 16 || len == 32);
  for (uint64_t i = 0; hex && i < len; ++i) {
    const char ch = trace_id[i];
    const uint64_t v = ch >= '0' && ch <= '9' ? (uint64_t)(ch - '0') : (ch >= 'a' && ch <= 'f' ? (uint64_t)(ch - 'a' + 10) : 16);
    if (v == 16) {
      hex = false;
      break;
    }
    hi = (hi << 4) | (lo >> 60);
    lo = (lo << 4) | v;
  }
  if (!hex) {  // any other traceId string: FNV-1a of its bytes
    hi = ~0ull;
    lo = 0xcbf29ce484222325ull;
    for (uint64_t i = 0; trace_id && i < len; ++i) lo = (lo ^ (uint8_t)trace_id[i]) * 0x100000001b3ull;
  }
  return shard_of(hi, lo, world);
}

// Everything one kmz_run attempt puts on the stream, up to the read-back of
// the counters into pinned memory: no host synchronisation inside on the
// window-join path (run_table, the repeated-id path, synchronises).
static int run_enqueue(kmz_ctx *c, uint32_t flags, bool links, unsigned int *h, unsigned long long *s64) {
  const uint32_t smode = flags & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG);
  c->sstats = false;
  c->chain_ran = false;
  c->cert2 = false;
  c->cert_defer = false;
  // (by our fill kernel, not hipMemsetAsync: the runtime's fill is a blit
  // kernel that waited behind the previous fetch's device-to-host blit on the
  // transfer stream, ~0.13 ms at the head of every pipelined step;
  // KMZ_ABLATE2 bit 20: the runtime's fill, for comparison)
  // (with DEPS, the endpoint partials' fill rides in the same launch)
  c->epp_filled = false;
  if (c->ablate2 & (1u << 20)) {
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, C_COUNT * 4 + S_COUNT * 8, c->stream));
  } else {
    FillArgs f;
    f.add(c->counters.p, C_COUNT * 4 + S_COUNT * 8, 0);
    if (flags & KMZ_RUN_DEPS) {
      if (ensure(c, c->epp, (size_t)(c->n_dep + 1) * 16)) return KMZ_E_HIP;
      unsigned long long *epp = P<unsigned long long>(c->epp);
      f.add(epp, (size_t)c->n_dep * 8, 0);
      f.add(epp + c->n_dep, (size_t)c->n_dep * 8, 0xFF);
      c->epp_filled = true;
    }
    launch_fill(c->stream, f);
  }
  rb_mark(c, "fill");
  int r;
  c->main = c->stream;
  // (KMZ_ABLATE2 bit 17, for comparison: K3 on the main stream between the
  // join and the walk -- run_deps runs the shape-level K3 before its walk --
  // instead of beside the join on the side stream)
  // On the chain-tile path K3 runs on the main stream after the walk
  // (run_chain_tiles), so that the join has the CUs to itself and the
  // certificate's split, which cannot share a CU with the walk, shares them
  // with K3 instead: mesh 3.39 -> 3.36 ms (profiles/r05/ab/k3late, wide).
  // KMZ_ABLATE2 bit 18: beside the join on the side stream, for comparison
  // (and elsewhere: config 5's direct walk measured 7.58 against 7.44 ms
  // with K3 on the main stream, profiles/r05/ab/k3mid5)
  c->k3_late = smode && (flags & KMZ_RUN_DEPS) && !(c->ablate2 & 262144u) && !c->k4_now && !fused_eligible(c) &&
               !(c->ablate & 16) && !(c->ablate2 & 256u);
  // On the direct walk (config 5) K3 runs on the side stream from the end of
  // the walk, beside the settle, so that the join has the CUs to itself:
  // 7.28-7.31 -> 7.15-7.19 ms (profiles/r05/ab/k3s, k3s2; KMZ_ABLATE2 bit 21:
  // beside the join, for comparison)
  c->k3_settle = c->overlap && smode && (flags & KMZ_RUN_DEPS) && !(c->ablate2 & (1u << 21)) && !c->k3_late &&
                 c->k4_now && !fused_eligible(c) && !(c->ablate & 16);
  c->k3_ran = false;
  c->k3_mode = smode;
  const bool k3_mid = smode && (flags & KMZ_RUN_DEPS) && ((c->ablate2 & 131072u) || c->k3_late || c->k3_settle);
  c->k3_on_side = c->overlap && smode && !k3_mid;
  if (c->overlap && !k3_mid) {
    HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
    c->stream = c->side;
  }
  r = smode && !k3_mid ? run_stats(c, smode) : 0;
  if (c->overlap && !k3_mid) {
    c->stream = c->main;
    HIPCHK(c, hipEventRecord(c->ev_k3, c->side));
  }
  if (c->overlap && k3_mid) {  // (nothing on the side stream before the certificate: the waits pass at once)
    HIPCHK(c, hipEventRecord(c->ev_k3, c->main));
    HIPCHK(c, hipEventRecord(c->ev_fork, c->main));
    HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
  }
  if (r) return r;
  rb_mark(c, "k3/fork");
  if ((flags & KMZ_RUN_DEPS) && (r = run_deps(c, links))) {
    c->stream = c->main;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipStreamIsCapturing(c->main, &cs);
    if (c->overlap && cs == hipStreamCaptureStatusNone) {
      hipStreamSynchronize(c->side);
      if (c->side2) hipStreamSynchronize(c->side2);
    }
    return r;
  }
  if ((r = launch_cert_deferred(c))) return r;  // (a path with no walk after the join)
  if (c->rt_armed) {  // an armed routing the join did not take (fused or table path, a certificate, world past
    // the bins): kmz_route_ids_fixed's pass on the main stream
    if (ensure(c, c->rt_tot, (size_t)c->rt_arm.world * 8)) return KMZ_E_HIP;
    if (!launch_route_fixed(c->stream, c->sid, (uint32_t)c->n, c->rt_arm.world, c->rt_arm.segw,
                            P<unsigned long long>(c->rt_tot), c->rt_arm.out))
      return fail(c, KMZ_E_HIP, "routing launch");
    HIPCHK(c, hipEventRecord(c->ev_route, c->stream));
    c->rt_armed = false;
    c->rt_routed = true;
  }
  if (k3_mid && !c->k3_ran && (r = run_stats(c, smode))) return r;  // (its shape level ran inside run_deps)
  if (c->overlap) {  // everything queued on the side stream, before the read-back
    HIPCHK(c, hipEventRecord(c->ev_done, c->side));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_done, 0));
  }
  if (c->cert2) {  // ... and on the certificate's
    HIPCHK(c, hipEventRecord(c->ev_cert, c->side2));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_cert, 0));
  }
  rb_mark(c, "deps");
  static_assert(C_COUNT * 4 % 8 == 0, "the statistics follow the counters in one buffer and in hpin");
  (void)s64;
  HIPCHK(c, hipMemcpyAsync(h, c->counters.p, C_COUNT * 4 + S_COUNT * 8, hipMemcpyDeviceToHost, c->stream));
  return KMZ_OK;
}

// The launch sequence of a run is a function of this state (buffer addresses
// and sizes, table capacities, seeds, modes, the batch's shape counts): runs
// with equal keys enqueue identical work.
static uint64_t run_key(kmz_ctx *c, uint32_t flags) {
  uint64_t k = 0xcbf29ce484222325ull;
  auto mix = [&](uint64_t v) { k = mix64(k ^ v) + 0x9E3779B97F4A7C15ull; };
  for (uint64_t v : {(uint64_t)flags, c->n, c->index_base, (uint64_t)c->n_shapes, (uint64_t)c->n_status,
                     (uint64_t)c->n_rt, (uint64_t)c->n_tag, (uint64_t)c->n_dep, c->tcap, c->ccap, (uint64_t)c->scap,
                     (uint64_t)c->mcap, (uint64_t)c->dcap, c->sig_seed, (uint64_t)c->ablate, (uint64_t)c->ablate2, (uint64_t)c->overlap,
                     (uint64_t)c->k4_now, (uint64_t)c->ctab_dirty, (uint64_t)c->walk_once,
                     (uint64_t)(uintptr_t)c->stream, (uint64_t)(uintptr_t)c->side, (uint64_t)(uintptr_t)c->hpin,
                     (uint64_t)(uintptr_t)c->sid, (uint64_t)(uintptr_t)c->pid, (uint64_t)(uintptr_t)c->kind,
                     (uint64_t)(uintptr_t)c->shape, (uint64_t)(uintptr_t)c->status, (uint64_t)(uintptr_t)c->dur,
                     (uint64_t)(uintptr_t)c->ts, (uint64_t)(uintptr_t)c->d_rt.p, (uint64_t)(uintptr_t)c->d_tag.p,
                     (uint64_t)(uintptr_t)c->d_dep.p, (uint64_t)chain_grid((uint32_t)c->n)})
    mix(v);
  for (DevBuf *b : {&c->table, &c->dups, &c->dkey, &c->dval, &c->cparent, &c->rowpos, &c->grp, &c->grp_final, &c->epp,
                    &c->trip, &c->trip_out, &c->counters, &c->stats64, &c->k3pool, &c->k3dir, &c->k3part,
                    &c->tile_tmp, &c->sgrp, &c->dp, &c->cpool1, &c->cpool2, &c->ccur, &c->cdir, &c->mkey, &c->mval,
                    &c->ctab, &c->plist, &c->kstage, &c->kstage_n, &c->kdefer, &c->kdefer_n, &c->cetab, &c->kbucket,
                    &c->kbucket_n, &c->ctile, &c->kwpos, &c->kwpos_n}) {
    mix((uint64_t)(uintptr_t)b->p);
    mix(b->bytes);
  }
  return k;
}

// Small batches (< 2^23 spans) are launch-bound: ~25 kernels and memsets per
// run.  A run whose key was seen on the previous run is captured into a
// hipGraph (stream capture, both streams) and replayed while the key holds;
// the first run of a key (and any run that grows a buffer) is enqueued
// directly, so a capture never allocates.  On by default since round 6: at
// the 2 500-trace tick the replays measured faster than direct launches on
// all three configs (round 5: 135 / 289 / 559 against 162 / 305 / 572 us per
// run + fetch, Bookinfo / mesh / config 5); KMZ_HIPGRAPH=0 turns them off.
// (Not while kernels are timed: the bench's live events keep them off.)
static int run_enqueue_graphed(kmz_ctx *c, uint32_t flags, bool links, unsigned int *h, unsigned long long *s64) {
  const bool eligible = c->n > 0 && c->n < (1ull << 23) && !c->prof && c->graphs_on && !c->rt_armed &&
                        !c->table_hint && !c->walk_once && !(c->ablate & (32u | 16u));
  if (!eligible) return run_enqueue(c, flags, links, h, s64);
  const uint64_t key = run_key(c, flags);
  ++c->graph_clock;
  for (auto &g : c->graphs) {
    if (!g.exec || g.key != key) continue;
    HIPCHK(c, hipGraphLaunch(g.exec, c->stream));
    g.used = c->graph_clock;
    ++c->graph_launches;
    c->path = g.path;
    c->sstats = g.sstats;
    c->chain_ran = g.chain_ran;
    c->k4_direct_ran = g.k4_direct_ran;
    c->ctab_dirty = g.ctab_dirty;
    c->G = g.G;
    c->ep_mode = g.ep_mode;
    c->k4_lb1 = g.k4_lb1;
    c->k4_nsl = g.k4_nsl;
    c->k4_ng = g.k4_ng;
    c->main = c->stream;
    return KMZ_OK;
  }
  if (c->graph_seen != key) {  // first run of this key: direct (buffers settle)
    c->graph_seen = key;
    return run_enqueue(c, flags, links, h, s64);
  }
  // second run of this key: capture it (the host state the enqueue changes is
  // restored if the capture fails, then the run is enqueued directly)
  const bool dirty0 = c->ctab_dirty;
  hipStream_t s0 = c->stream;
  hipGraph_t graph = nullptr;
  bool ok = hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal) == hipSuccess;
  int r = ok ? run_enqueue(c, flags, links, h, s64) : KMZ_OK;
  c->stream = s0;
  if (ok) ok = hipStreamEndCapture(s0, &graph) == hipSuccess && graph && r == KMZ_OK && run_key(c, flags) == key;
  hipGraphExec_t exec = nullptr;
  if (ok) ok = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
  if (graph) hipGraphDestroy(graph);
  if (!ok) {
    if (exec) hipGraphExecDestroy(exec);
    (void)hipGetLastError();
    c->ctab_dirty = dirty0;
    c->graph_seen = 0;
    c->err.clear();
    return run_enqueue(c, flags, links, h, s64);
  }
  auto *slot = &c->graphs[0];
  for (auto &g : c->graphs)
    if (!g.exec || g.used < slot->used) slot = &g;
  if (slot->exec) hipGraphExecDestroy(slot->exec);
  slot->key = key;
  slot->exec = exec;
  slot->used = c->graph_clock;
  slot->path = c->path;
  slot->sstats = c->sstats;
  slot->chain_ran = c->chain_ran;
  slot->k4_direct_ran = c->k4_direct_ran;
  slot->ctab_dirty = c->ctab_dirty;
  slot->G = c->G;
  slot->ep_mode = c->ep_mode;
  slot->k4_lb1 = c->k4_lb1;
  slot->k4_nsl = c->k4_nsl;
  slot->k4_ng = c->k4_ng;
  HIPCHK(c, hipGraphLaunch(exec, s0));
  ++c->graph_launches;
  return KMZ_OK;
}

// one attempt of a run: the stream layout, then every launch and the read-back
static int run_attempt(kmz_ctx *c, uint32_t flags, bool links, unsigned int *h, unsigned long long *s64) {
  const uint32_t smode = flags & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG);
  // K3 (+ the certificate, see run_join) on the side stream while the main
  // stream joins and walks (KMZ_ABLATE bit 25: serial, for comparison).
  // Small batches are launch- and latency-bound (Bookinfo 1M: 0.369 -> 0.323
  // ms/step).  At 10^8 spans the kernels of round 1 each filled the GPU and
  // overlap bought <= 3 % or lost (profiles/r01_overlap_ab/); since round 4
  // the VALU-bound join shares the CUs with the memory-bound K3, and the
  // latency-bound walk with the certificate: mesh 3.96 -> 3.76, config 5
  // 8.56 -> 8.43 ms/step (profiles/r04/ab/overlap/).  Below 2^18 spans (a
  // 2 500-trace tick) the second stream's fork / join costs more than the
  // overlap gives: Bookinfo 164 -> 149 us, mesh 320 -> 300 us per run serial
  // (tools/bench_tick.py); config 5's tick (1.4*10^5 spans) 833 -> 805 us per
  // tick serial (profiles/r05/m3/tick.json).  While more than one kernel id is timed
  // (kmz_set_profiling_mask) runs stay on one stream, so that each kernel's
  // time is its own.  KMZ_ABLATE bit 27 forces the overlap.
  const bool timing_many = c->prof && (c->prof_mask & (c->prof_mask - 1));
  c->overlap = smode && (flags & KMZ_RUN_DEPS) && !(c->ablate & (1u << 25)) &&
               ((c->n >= (1ull << 18) && !timing_many) || (c->ablate & (1u << 27)));
  return run_enqueue_graphed(c, flags, links, h, s64);
}

int kmz_run(kmz_ctx *c, uint32_t flags) {
  const int r = kmz_run_begin(c, flags);
  return r ? r : kmz_run_end(c);
}

int kmz_run_begin(kmz_ctx *c, uint32_t flags) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return fail(c, KMZ_E_STATE, "kmz_run_begin while a run is open (kmz_run_end first)");
  // (a run may begin behind an open service tail: its kernels follow the
  // tail's on the stream, and kmz_tail_end waits for the tail's event only)
  if (c->tl_open) c->tl_run_after = true;
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_run before kmz_load");
  uint32_t smode = flags & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG);
  if (smode == (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG)) return fail(c, KMZ_E_ARG, "choose one stats identity per run");
  if ((flags & KMZ_RUN_DEP_ORDER) && !(flags & KMZ_RUN_DEPS)) return fail(c, KMZ_E_ARG, "KMZ_RUN_DEP_ORDER needs KMZ_RUN_DEPS");
  const bool links = (flags & (KMZ_RUN_SPAN_LINKS | KMZ_RUN_DEP_ORDER)) != 0;
  hipSetDevice(c->device);
  c->hpin_valid = false;
  c->walk_once = false;
  // one read-back per run: counters + statistics into pinned host memory
  if (!c->hpin && hipHostMalloc(&c->hpin, C_COUNT * 4 + S_COUNT * 8, hipHostMallocDefault) != hipSuccess) {
    c->hpin = nullptr;
    return fail(c, KMZ_E_HIP, "hipHostMalloc (run read-back)");
  }
  unsigned int *h = reinterpret_cast<unsigned int *>(c->hpin);
  unsigned long long *s64 = reinterpret_cast<unsigned long long *>(h + C_COUNT);
  if (c->rb_prof) {
    c->rb_marks.clear();
    rb_mark(c, "begin");
  }
  c->k4_now = (flags & KMZ_RUN_DEPS) ? k4_direct(c) : false;
  c->no_cert = (flags & KMZ_RUN_NO_CERT) != 0;
  c->rt_routed = c->rt_in_join = false;  // (kmz_route_wait: this run's routing only)
  c->gu_host = true;
  if (int r = run_attempt(c, flags, links, h, s64)) {
    c->rt_armed = false;
    return r;
  }
  c->run_open = true;
  c->run_flags = flags;
  if (c->rb_prof) {
    rb_mark(c, "end");
    for (size_t k = 1; k < c->rb_marks.size(); ++k)
      fprintf(stderr, "%s%s %.1f", k == 1 ? "run_begin us:" : ",", c->rb_marks[k].first,
              c->rb_marks[k].second - c->rb_marks[k - 1].second);
    fprintf(stderr, "\n");
  }
  return KMZ_OK;
}

// waits for the run's read-back; a run that must grow a table or change a
// seed is repeated here (each repeat enqueued and waited for in turn)
int kmz_run_end(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (!c->run_open) return fail(c, KMZ_E_STATE, "kmz_run_end without kmz_run_begin");
  c->run_open = false;
  const uint32_t flags = c->run_flags;
  const bool links = (flags & (KMZ_RUN_SPAN_LINKS | KMZ_RUN_DEP_ORDER)) != 0;
  unsigned int *h = reinterpret_cast<unsigned int *>(c->hpin);
  unsigned long long *s64 = reinterpret_cast<unsigned long long *>(h + C_COUNT);
  for (int attempt = 0; attempt < 8; ++attempt) {
    if (attempt > 0) {
      int r = run_attempt(c, flags, links, h, s64);
      if (r) return r;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    harvest(c);
    if (h[C_FLAGS] & F_CTAB_DIRTY) c->ctab_dirty = true;
    // staged keys overflowed (low chain reuse, config 5): the overflow was
    // inserted in place, correct but serial per leader; stage more next time
    // (<= 8 GB of staging)
    if (h[C_FLAGS] & F_STAGE_FULL) {  // x4, or as far as the staging limit allows
      const uint64_t ng = chain_grid((uint32_t)c->n);
      uint64_t want = (uint64_t)c->scap * 4;
      while (want > c->scap && ng * want * 8 > stage_limit(c->n)) want /= 2;
      c->scap = (uint32_t)want;
    }
    if ((flags & KMZ_RUN_DEPS) && (c->path & 1) && h[C_CERT]) {  // a repeated span id: the table path, same run
      c->table_hint = true;
      continue;
    }
    // hash-table load factors: grow for the next run (correctness never
    // depends on it: an overfull probe raises the overflow flags below)
    // chain table at load factor <= 1/8 while it fits the 256 MB MALL, else
    // <= 1/4: a found chain is then almost always at its home slot (each
    // extra slot is another dependent probe round trip)
    // most rows start a new chain (config 5): enumerate directly next time
    if (c->chain_ran) c->k4_auto_direct = s64[S_CHAINS] * 2 > s64[S_ROWS];
    // (KMZ_ABLATE2 bits 2 / 3, for comparison: load <= 1/2 / <= 1/4 whatever the size)
    const uint64_t lf_small = (c->ablate2 & 4u) ? 2 : (c->ablate2 & 8u) ? 4 : 8;
    const uint64_t lf_big = (c->ablate2 & 4u) ? 2 : 4;
    while (c->chain_ran && c->ccap < (1ull << 31) &&
           (s64[S_CHAINS] * lf_big > c->ccap ||
            (s64[S_CHAINS] * lf_small > c->ccap && c->ccap * CHAIN_ENTRY_BYTES < (256ull << 20))))
      c->ccap *= 2;
    if ((flags & KMZ_RUN_DEPS) && ((c->ablate & (1u << 31)) ? s64[S_TRIP_OUT] * 8 > c->tcap * 7
                                                           : s64[S_TRIP_OUT] * 2 > c->tcap))
      c->tcap *= 2;  // (knob 31: diagnostic, a MALL-sized edge set at load <= 7/8)
    bool retry = false;
    if (h[C_FLAGS] & F_MISS_OVERFLOW) {
      c->mcap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(2ull * c->mcap, 2ull * h[C_MISS] + 64), 0xFFFFFFF0ull);
      retry = true;
    }
    if (h[C_FLAGS] & F_TRIPLE_OVERFLOW) {
      c->tcap *= 4;
      retry = true;
    }
    if ((flags & KMZ_RUN_DEPS) && (h[C_FLAGS] & F_SPIN) && !c->walk_once) {
      // a chain-table wait ran out: some check, row or key may be missing.
      // Redo this run on the exact per-row walk (kmz_info.path bit 3 says so)
      c->walk_once = true;
      c->ctab_dirty = true;  // (entries may be half written: a full clear next time)
      retry = true;
    }
    if (h[C_FLAGS] & F_SIG) {  // an ancestry-hash collision: same run, another seed
      c->sig_seed = mix64(c->sig_seed + 0x9E3779B97F4A7C15ull);
      retry = true;
    }
    if (h[C_FLAGS] & F_CHAIN_OVERFLOW) {
      if (c->ccap >= (1ull << 31)) return fail(c, KMZ_E_OVERFLOW, "chain table full");
      c->ccap *= 4;
      retry = true;
    }
    if ((flags & KMZ_RUN_DEPS) && (uint64_t)h[C_DUPS] * 2 > c->dcap) {
      c->dcap = (uint32_t)std::min<uint64_t>(4ull * h[C_DUPS] + 1024, 0xFFFFFFF0ull);
      retry = true;
    }
    if (!retry) {
      int e = check_flags(c, h[C_FLAGS]);
      if (e) return e;
      if ((flags & KMZ_RUN_DEP_ORDER) && (e = run_dep_order(c, s64[S_TRIP_OUT], h[C_DUPS] != 0))) return e;
      if (c->imap_n && (e = remap_results(c, flags, links))) return e;
      c->ran = flags;
      c->links = links;
      c->hpin_valid = true;
      return KMZ_OK;
    }
  }
  return fail(c, KMZ_E_OVERFLOW, "table growth did not converge");
}

int kmz_get_graph_stats(kmz_ctx *c, uint64_t *launches, uint32_t *cached) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (launches) *launches = c->graph_launches;
  if (cached) {
    uint32_t k = 0;
    for (auto &g : c->graphs) k += g.exec != nullptr;
    *cached = k;
  }
  return KMZ_OK;
}

int kmz_get_info(kmz_ctx *c, kmz_info *out) {
  if (!c || !out) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  unsigned int hb[C_COUNT];
  unsigned long long sb[S_COUNT];
  const unsigned int *h = hb;
  const unsigned long long *s = sb;
  if (c->hpin_valid) {  // the last run's read-back (nothing has run since)
    h = reinterpret_cast<const unsigned int *>(c->hpin);
    s = reinterpret_cast<const unsigned long long *>(h + C_COUNT);
  } else {
    HIPCHK(c, hipMemcpyAsync(hb, c->counters.p, sizeof(hb), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(sb, c->stats64.p, sizeof(sb), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  memset(out, 0, sizeof(*out));
  out->n_spans = c->n;
  out->n_server = s[S_SERVER];
  out->n_rows = s[S_ROWS];
  out->n_relations = s[S_REL];
  out->n_triples = s[S_TRIP_OUT];
  out->n_dups = h[C_DUPS];
  out->max_depth = s[S_MAXD];
  out->n_groups = c->G;
  out->flags = h[C_FLAGS];
  out->path = (uint32_t)c->path;
  out->n_chains = c->chain_ran ? s[S_CHAINS] : 0;
  return KMZ_OK;
}

int kmz_get_groups(kmz_ctx *c, kmz_group *out, uint64_t cap) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
  if (cap < c->G) return fail(c, KMZ_E_ARG, "output too small");
  if (c->G) HIPCHK(c, hipMemcpyAsync(out, c->grp_final.p, (size_t)c->G * sizeof(kmz_group), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_get_endpoints(kmz_ctx *c, kmz_endpoint *out, uint64_t cap) {
  return kmz_fetch(c, nullptr, 0, nullptr, 0, nullptr, out, cap);
}

int kmz_get_triples(kmz_ctx *c, uint64_t *out, uint64_t cap, uint64_t *n_out) {
  if (!c || !n_out) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  return kmz_fetch(c, nullptr, 0, out, cap, n_out, nullptr, 0);
}

namespace {

// kmz_fetch's argument checks; the edge-key count from the run's read-back
int fetch_check(kmz_ctx *c, kmz_group *groups, uint64_t gcap, uint64_t *trip, uint64_t tcap, uint64_t *n_trip,
                kmz_endpoint *eps, uint64_t ecap, uint64_t *nt) {
  if (!c) return KMZ_E_ARG;
  const bool want_deps = trip || n_trip || eps;
  if (groups && !(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
  if (want_deps && !(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
  if (groups && gcap < c->G) return fail(c, KMZ_E_ARG, "output too small");
  if (eps && ecap < c->n_dep) return fail(c, KMZ_E_ARG, "output too small");
  *nt = 0;
  if (want_deps) {
    if (c->hpin_valid) {
      *nt = reinterpret_cast<const unsigned long long *>(reinterpret_cast<const unsigned int *>(c->hpin) + C_COUNT)[S_TRIP_OUT];
    } else {
      unsigned long long s[S_COUNT];
      HIPCHK(c, hipMemcpyAsync(s, c->stats64.p, sizeof(s), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      *nt = s[S_TRIP_OUT];
    }
    if (n_trip) *n_trip = *nt;
    if (trip && tcap < *nt) return fail(c, KMZ_E_ARG, "output too small");
  }
  return KMZ_OK;
}

// per endpoint {last timestamp ^ bias, first row << 1 | internal} -> kmz_endpoint
void endpoints_from(const uint64_t *h, uint32_t n_dep, kmz_endpoint *eps) {
  for (uint32_t e = 0; e < n_dep; ++e) {
    const uint64_t tsx = h[e], f = h[n_dep + e];
    eps[e].last_ts = tsx == 0 ? INT64_MIN : (int64_t)(tsx ^ TS_BIAS);
    eps[e].has_row = f != ~0ull;
    eps[e].first_row = f == ~0ull ? ~0ull : (f >> 1);
    eps[e].external = f == ~0ull ? 0u : (uint32_t)((f & 1) == 0);
  }
}

// the device address of page-locked host memory (hipHostMalloc / registered), else null
void *host_pinned_dev(void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // (pageable memory: not an error of the fetch)
    return nullptr;
  }
  return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

int pinned_staging(kmz_ctx *c, void *&p, size_t &have, size_t bytes) {
  if (have >= bytes) return KMZ_OK;
  if (p) hipHostFree(p);
  p = nullptr;
  have = 0;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    p = nullptr;
    return fail(c, KMZ_E_HIP, "hipHostMalloc (endpoint staging)");
  }
  have = bytes;
  return KMZ_OK;
}

}  // namespace

int kmz_fetch(kmz_ctx *c, kmz_group *groups, uint64_t gcap, uint64_t *trip, uint64_t tcap, uint64_t *n_trip,
              kmz_endpoint *eps, uint64_t ecap) {
  if (c && c->run_open) return run_busy(c);
  if (c && c->fetch_open) {
    const int r = kmz_fetch_end(c);
    if (r) return r;
  }
  uint64_t nt = 0;
  if (int r = fetch_check(c, groups, gcap, trip, tcap, n_trip, eps, ecap, &nt)) return r;
  bool any = false;
  if (groups && c->G) {
    HIPCHK(c, hipMemcpyAsync(groups, c->grp_final.p, (size_t)c->G * sizeof(kmz_group), hipMemcpyDeviceToHost, c->stream));
    any = true;
  }
  if (trip && nt) {
    HIPCHK(c, hipMemcpyAsync(trip, c->trip_out.p, nt * 8, hipMemcpyDeviceToHost, c->stream));
    any = true;
  }
  const size_t eb = (size_t)c->n_dep * 16;
  if (eps && c->n_dep) {
    if (int r = pinned_staging(c, c->hep, c->hep_bytes, eb)) return r;
    HIPCHK(c, hipMemcpyAsync(c->hep, c->epp.p, eb, hipMemcpyDeviceToHost, c->stream));
    any = true;
  }
  if (any) HIPCHK(c, hipStreamSynchronize(c->stream));
  if (eps) endpoints_from(reinterpret_cast<const uint64_t *>(c->hep), c->n_dep, eps);
  return KMZ_OK;
}

int kmz_fetch_used(kmz_ctx *c, uint32_t *ids, kmz_group *groups, uint64_t gcap, uint64_t *n_used, uint64_t *trip,
                   uint64_t tcap, uint64_t *n_trip, kmz_endpoint *eps, uint64_t ecap) {
  if (!c || !n_used || (gcap && (!ids || !groups))) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (c->fetch_open) {
    const int r = kmz_fetch_end(c);
    if (r) return r;
  }
  uint64_t nt = 0;
  if (int r = fetch_check(c, nullptr, 0, trip, tcap, n_trip, eps, ecap, &nt)) return r;
  if (!(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
  if (!c->gu_ok) return fail(c, KMZ_E_UNSUPPORTED, "more than 2^22 groups: kmz_fetch the dense groups");
  uint64_t nu;
  if (c->hpin_valid && c->gu_host) {
    nu = reinterpret_cast<const unsigned long long *>(reinterpret_cast<const unsigned int *>(c->hpin) + C_COUNT)[S_GUSED];
  } else {
    unsigned long long v = 0;
    HIPCHK(c, hipMemcpyAsync(&v, P<unsigned long long>(c->stats64) + S_GUSED, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    nu = v;
  }
  *n_used = nu;
  if (!gcap && !trip && !eps) return KMZ_OK;  // (the count only)
  if (gcap < nu) return fail(c, KMZ_E_ARG, "output too small");
  if (nu) {
    HIPCHK(c, hipMemcpyAsync(ids, c->gu_ids.p, nu * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(groups, c->gu_grp.p, nu * sizeof(kmz_group), hipMemcpyDeviceToHost, c->stream));
  }
  if (trip && nt) HIPCHK(c, hipMemcpyAsync(trip, c->trip_out.p, nt * 8, hipMemcpyDeviceToHost, c->stream));
  const size_t eb = (size_t)c->n_dep * 16;
  if (eps && c->n_dep) {
    if (int r = pinned_staging(c, c->hep, c->hep_bytes, eb)) return r;
    HIPCHK(c, hipMemcpyAsync(c->hep, c->epp.p, eb, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (eps) endpoints_from(reinterpret_cast<const uint64_t *>(c->hep), c->n_dep, eps);
  return KMZ_OK;
}

int kmz_fetch_begin(kmz_ctx *c, kmz_group *groups, uint64_t gcap, uint64_t *trip, uint64_t tcap, uint64_t *n_trip,
                    kmz_endpoint *eps, uint64_t ecap) {
  if (c && c->run_open) return run_busy(c);
  if (c && c->fetch_open) {
    const int r = kmz_fetch_end(c);
    if (r) return r;
  }
  uint64_t nt = 0;
  if (int r = fetch_check(c, groups, gcap, trip, tcap, n_trip, eps, ecap, &nt)) return r;
  if (!c->xfer) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->xfer, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_snap, hipEventDisableTiming));
  }
  const size_t gb = groups ? (size_t)c->G * sizeof(kmz_group) : 0, tb = trip ? (size_t)nt * 8 : 0,
               eb = eps ? (size_t)c->n_dep * 16 : 0;
  // the device copy: the next run is free to overwrite the results at once
  if (ensure(c, c->f_grp, gb) || ensure(c, c->f_trip, tb) || ensure(c, c->f_ep, eb))
    return fail(c, KMZ_E_HIP, "hipMalloc (fetch snapshot)");
  if (eb) {
    if (int r = pinned_staging(c, c->fhep, c->fhep_bytes, eb)) return r;
  }
  {  // (one copy kernel; the runtime's copies where a range is not 8-byte aligned)
    CopyArgs cp;
    cp.add(c->grp_final.p, c->f_grp.p, gb);
    cp.add(c->trip_out.p, c->f_trip.p, tb);
    cp.add(c->epp.p, c->f_ep.p, eb);
    if (!launch_copy8(c->stream, cp)) {
      if (gb) HIPCHK(c, hipMemcpyAsync(c->f_grp.p, c->grp_final.p, gb, hipMemcpyDeviceToDevice, c->stream));
      if (tb) HIPCHK(c, hipMemcpyAsync(c->f_trip.p, c->trip_out.p, tb, hipMemcpyDeviceToDevice, c->stream));
      if (eb) HIPCHK(c, hipMemcpyAsync(c->f_ep.p, c->epp.p, eb, hipMemcpyDeviceToDevice, c->stream));
    }
  }
  HIPCHK(c, hipEventRecord(c->ev_snap, c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->xfer, c->ev_snap, 0));
  // to page-locked host memory by the DMA engines (hipMemcpyDeviceToDeviceNoCU
  // on the buffer's device address): the runtime's device-to-host copy is a
  // blit kernel over the whole GPU whose waves wait on PCIe, and the next
  // run's first kernels waited ~0.13 ms for it.  Pageable memory, or KMZ_ABLATE2
  // bit 9 (for comparison): the runtime's copy.
  const void *from[3] = {c->f_grp.p, c->f_trip.p, c->f_ep.p};
  void *to[3] = {groups, trip, c->fhep};
  const size_t nb[3] = {gb, tb, eb};
  for (int k = 0; k < 3; ++k) {
    if (!nb[k]) continue;
    void *dev = (c->ablate2 & (1u << 9)) ? nullptr : host_pinned_dev(to[k]);
    if (dev)
      HIPCHK(c, hipMemcpyAsync(dev, from[k], nb[k], hipMemcpyDeviceToDeviceNoCU, c->xfer));
    else
      HIPCHK(c, hipMemcpyAsync(to[k], from[k], nb[k], hipMemcpyDeviceToHost, c->xfer));
  }
  c->fetch_open = true;
  c->f_eps = eps;
  c->f_ndep = eb ? c->n_dep : 0;
  return KMZ_OK;
}

int kmz_fetch_end(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->fetch_open) return KMZ_OK;
  c->fetch_open = false;
  HIPCHK(c, hipStreamSynchronize(c->xfer));
  if (c->f_eps && c->f_ndep) endpoints_from(reinterpret_cast<const uint64_t *>(c->fhep), c->f_ndep, c->f_eps);
  c->f_eps = nullptr;
  return KMZ_OK;
}

int kmz_get_spans(kmz_ctx *c, uint64_t *span_id, uint64_t *parent_id, uint8_t *kind, uint32_t *shape,
                  uint16_t *status, uint32_t *duration, int64_t *timestamp, uint64_t cap) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "no batch loaded");
  if (cap < c->n) return fail(c, KMZ_E_ARG, "output too small");
  const uint64_t n = c->n;
  if (n) {
    if (span_id) HIPCHK(c, hipMemcpyAsync(span_id, c->sid, n * 8, hipMemcpyDeviceToHost, c->stream));
    if (parent_id) HIPCHK(c, hipMemcpyAsync(parent_id, c->pid, n * 8, hipMemcpyDeviceToHost, c->stream));
    if (kind) HIPCHK(c, hipMemcpyAsync(kind, c->kind, n, hipMemcpyDeviceToHost, c->stream));
    if (shape) HIPCHK(c, hipMemcpyAsync(shape, c->shape, n * 4, hipMemcpyDeviceToHost, c->stream));
    if (status) HIPCHK(c, hipMemcpyAsync(status, c->status, n * 2, hipMemcpyDeviceToHost, c->stream));
    if (duration) HIPCHK(c, hipMemcpyAsync(duration, c->dur, n * 4, hipMemcpyDeviceToHost, c->stream));
    if (timestamp) HIPCHK(c, hipMemcpyAsync(timestamp, c->ts, n * 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_get_span_links(kmz_ctx *c, uint32_t *cparent, uint64_t *rowpos, uint64_t cap) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & KMZ_RUN_DEPS) || !c->links) return fail(c, KMZ_E_STATE, "run with KMZ_RUN_DEPS|KMZ_RUN_SPAN_LINKS first");
  if (cap < c->n) return fail(c, KMZ_E_ARG, "output too small");
  if (c->n) {
    if (cparent) HIPCHK(c, hipMemcpyAsync(cparent, c->cparent.p, c->n * 4, hipMemcpyDeviceToHost, c->stream));
    if (rowpos) HIPCHK(c, hipMemcpyAsync(rowpos, c->rowpos.p, c->n * 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_group_partials(kmz_ctx *c, void **dev_ptr, uint64_t *n_groups) {
  if (!c || !dev_ptr || !n_groups) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
  *dev_ptr = c->grp.p;
  *n_groups = c->G;
  return KMZ_OK;
}

int kmz_endpoint_partials(kmz_ctx *c, void **dev_ptr, uint64_t *n_ep) {
  if (!c || !dev_ptr || !n_ep) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
  *dev_ptr = c->epp.p;
  *n_ep = c->n_dep;
  return KMZ_OK;
}

int kmz_partials_size(kmz_ctx *c, int which, uint64_t *words) {
  if (!c || !words) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (which == KMZ_PART_GROUPS) {
    if (!(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
    *words = 6ull * c->G;
  } else if (which == KMZ_PART_ENDPOINTS) {
    if (!(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
    *words = 2ull * c->n_dep;
  } else if (which == KMZ_PART_TRIPLES) {
    if (!(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
    if (c->hpin_valid) {
      *words = reinterpret_cast<const unsigned long long *>(reinterpret_cast<const unsigned int *>(c->hpin) + C_COUNT)[S_TRIP_OUT];
    } else {
      unsigned long long s[S_COUNT];
      HIPCHK(c, hipMemcpyAsync(s, c->stats64.p, sizeof(s), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      *words = s[S_TRIP_OUT];
    }
  } else {
    return fail(c, KMZ_E_ARG, "unknown partial");
  }
  return KMZ_OK;
}

int kmz_partials_copy(kmz_ctx *c, int which, void *buf, uint64_t words, int mem, int direction) {
  if (c && c->run_open) return run_busy(c);
  uint64_t need = 0;
  int r = kmz_partials_size(c, which, &need);
  if (r) return r;
  if (words < need) return fail(c, KMZ_E_ARG, "buffer too small");
  if (which == KMZ_PART_TRIPLES && direction) return fail(c, KMZ_E_ARG, "triples are export-only");
  void *mine = which == KMZ_PART_GROUPS ? c->grp.p : (which == KMZ_PART_ENDPOINTS ? c->epp.p : c->trip_out.p);
  hipMemcpyKind k = direction ? (mem == KMZ_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                              : (mem == KMZ_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost);
  if (need) {
    if (direction)
      HIPCHK(c, hipMemcpyAsync(mine, buf, need * 8, k, c->stream));
    else
      HIPCHK(c, hipMemcpyAsync(buf, mine, need * 8, k, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

// replace: the keys become the edge set (kmz_set_triples), else they join it
static int merge_or_set_triples(kmz_ctx *c, const uint64_t *keys, uint64_t n, int mem, bool replace) {
  if (!c || (n && !keys)) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
  uint64_t nl = 0;
  int r = kmz_partials_size(c, KMZ_PART_TRIPLES, &nl);
  if (r) return r;
  if (replace) {
    HIPCHK(c, hipMemsetAsync(c->trip.p, 0, c->tcap * 8, c->stream));
    nl = 0;
  }
  const unsigned long long *src = reinterpret_cast<const unsigned long long *>(keys);
  if (n && mem == KMZ_MEM_HOST) {
    if (ensure(c, c->mkeys_in, n * 8)) return KMZ_E_HIP;
    HIPCHK(c, hipMemcpyAsync(c->mkeys_in.p, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    src = P<unsigned long long>(c->mkeys_in);
  }
  unsigned int *cnt = P<unsigned int>(c->counters);
  unsigned long long *st = P<unsigned long long>(c->stats64);
  // the run's edge set is intact: insert the incoming keys into it (they are
  // mostly already there), then compact again
  HIPCHK(c, hipMemsetAsync(cnt + C_FLAGS, 0, 4, c->stream));
  {
    Timed t(c, KMZ_K_FINAL);
    launch_key_insert(c->stream, src, n, P<unsigned long long>(c->trip), c->tcap, cnt);
  }
  unsigned int fl = 0;
  HIPCHK(c, hipMemcpyAsync(&fl, cnt + C_FLAGS, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  unsigned long long *tab = P<unsigned long long>(c->trip);
  uint64_t cap = c->tcap;
  if (fl & F_TRIPLE_OVERFLOW) {  // the union outgrew the set: a fresh one, large enough for every key
    cap = 1ull << 16;
    while (cap < 2 * (nl + n) + 64) cap *= 2;
    if (ensure(c, c->mtab, cap * 8)) return KMZ_E_HIP;
    tab = P<unsigned long long>(c->mtab);
    HIPCHK(c, hipMemsetAsync(tab, 0, cap * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(cnt + C_FLAGS, 0, 4, c->stream));
    launch_key_insert(c->stream, P<unsigned long long>(c->trip_out), nl, tab, cap, cnt);  // this rank's keys
    launch_key_insert(c->stream, src, n, tab, cap, cnt);
    HIPCHK(c, hipMemcpyAsync(&fl, cnt + C_FLAGS, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (fl & F_TRIPLE_OVERFLOW) return fail(c, KMZ_E_OVERFLOW, "edge-key union overflow");
    if (ensure(c, c->trip_out, cap * 8)) return KMZ_E_HIP;
  }
  HIPCHK(c, hipMemsetAsync(st + S_TRIP_OUT, 0, 8, c->stream));
  {
    Timed t(c, KMZ_K_FINAL);
    launch_compact(c->stream, tab, cap, P<unsigned long long>(c->trip_out), st + S_TRIP_OUT);
  }
  unsigned long long nt = 0;
  HIPCHK(c, hipMemcpyAsync(&nt, st + S_TRIP_OUT, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->hpin_valid)
    reinterpret_cast<unsigned long long *>(reinterpret_cast<unsigned int *>(c->hpin) + C_COUNT)[S_TRIP_OUT] = nt;
  return KMZ_OK;
}

int kmz_get_global_index(kmz_ctx *c, uint64_t *out, uint64_t cap, int mem) {
  if (!c || (c->n && !out)) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_get_global_index before kmz_load");
  if (cap < c->n) return fail(c, KMZ_E_ARG, "output too small");
  unsigned long long *dst = reinterpret_cast<unsigned long long *>(out);
  if (mem != KMZ_MEM_DEVICE) {
    if (ensure(c, c->rt_out, (size_t)c->n * 8 + 8)) return KMZ_E_HIP;
    dst = P<unsigned long long>(c->rt_out);
  }
  launch_iota(c->stream, dst, c->n, c->imap_n ? 0 : c->index_base);
  if (c->imap_n)
    launch_remap_index(c->stream, dst, c->n, 1, 0, P<uint64_t>(c->imap_l), P<uint64_t>(c->imap_g), c->imap_n);
  HIPCHK(c, hipGetLastError());
  if (mem != KMZ_MEM_DEVICE && c->n) HIPCHK(c, hipMemcpyAsync(out, dst, (size_t)c->n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_merge_triples(kmz_ctx *c, const uint64_t *keys, uint64_t n, int mem) {
  return merge_or_set_triples(c, keys, n, mem, false);
}

int kmz_set_triples(kmz_ctx *c, const uint64_t *keys, uint64_t n, int mem) {
  return merge_or_set_triples(c, keys, n, mem, true);
}

static uint64_t pow2_at_least(uint64_t x) {
  uint64_t c = 1024;
  while (c < x) c *= 2;
  return c;
}

int kmz_tail_map_set(kmz_ctx *c, const kmz_tail_map *m) {
  if (c && c->tl_open) return fail(c, KMZ_E_STATE, "kmz_tail_map_set while a service tail is open");
  if (!c || !m || !m->svc || !m->cls || (m->n_cls && !m->lsvc)) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  const uint32_t lim = 1u << 24;
  if (m->n_svc >= lim || m->n_cls >= lim || m->n_lsvc >= lim || m->n_ep >= lim) return fail(c, KMZ_E_ARG, "tail ids must be < 2^24");
  for (uint32_t e = 0; e < m->n_ep; ++e)
    if (m->svc[e] >= m->n_svc || m->cls[e] >= m->n_cls) return fail(c, KMZ_E_RANGE, "tail map id out of range");
  for (uint32_t k = 0; k < m->n_cls; ++k)
    if (m->lsvc[k] >= m->n_lsvc) return fail(c, KMZ_E_RANGE, "tail link-class id out of range");
  if (ensure(c, c->tl_svc, (size_t)m->n_ep * 4) || ensure(c, c->tl_cls, (size_t)m->n_ep * 4) ||
      ensure(c, c->tl_lsvc, (size_t)m->n_cls * 4) || ensure(c, c->tl_hasin, m->n_ep))
    return KMZ_E_HIP;
  if (m->n_ep) {
    HIPCHK(c, hipMemcpyAsync(c->tl_svc.p, m->svc, (size_t)m->n_ep * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->tl_cls.p, m->cls, (size_t)m->n_ep * 4, hipMemcpyHostToDevice, c->stream));
  }
  if (m->n_cls) HIPCHK(c, hipMemcpyAsync(c->tl_lsvc.p, m->lsvc, (size_t)m->n_cls * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->tl_n_ep = m->n_ep;
  c->tl_n_cls = m->n_cls;
  c->tl_n_svc = m->n_svc;
  c->tl_map = true;
  c->tl_ran = false;
  return KMZ_OK;
}

// one attempt of the service tail, enqueued on the context's stream up to
// the read-back of its counters and per-service outputs (kmz_tail_begin, and
// kmz_tail_end's repeats)
static int tail_enqueue(kmz_ctx *c) {
  const uint64_t nt = c->tl_nt;
  unsigned long long *st = P<unsigned long long>(c->stats64);
  const uint64_t acap = c->tl_acap, pacap = c->tl_pacap, pcap = c->tl_pcap;
  // link-key buckets: two link keys per edge key at most, spread by a hash
  // of their (service, linked service) pair, each pass-A workgroup writing
  // its own slab of every bucket (2 x its mean share + 64: hot pairs weigh
  // some buckets); grown on overflow
  const uint32_t bits = c->tl_bbits, nbk = 1u << bits, nwg = tail_part_grid(nt);
  c->tl_bcap = std::max<uint64_t>(c->tl_bcap, (2 * nt) / ((uint64_t)nbk * nwg) * 2 + 64);
  const uint64_t slab = c->tl_bcap;
  if (slab >= 0xFFFFFFFFull) return fail(c, KMZ_E_OVERFLOW, "service tail buckets");
  if (ensure(c, c->tl_lbkt, slab * nbk * nwg * 8) || ensure(c, c->tl_lbn, (size_t)nbk * nwg * 4) ||
      ensure(c, c->tl_pset, pcap * 8) || ensure(c, c->tl_pkey, pacap * 8) || ensure(c, c->tl_pval, pacap * 4) ||
      ensure(c, c->tl_det, acap * sizeof(kmz_tail_detail)) || ensure(c, c->tl_pairs, pacap * sizeof(kmz_tail_pair)) ||
      ensure(c, c->tl_rb, 64 + (size_t)c->tl_n_svc * 40 + (size_t)c->tl_n_svc * c->tl_n_dist * 4 + 8))
    return KMZ_E_HIP;
  // the read-back (pinned): counters [64 B], stats [n_svc x 8 u32], first rows [n_svc u64], relying table
  const uint32_t nd_run = c->tl_n_dist;
  c->tl_nd_run = nd_run;
  const size_t hb = 64 + (size_t)c->tl_n_svc * 40 + (size_t)c->tl_n_svc * nd_run * 4;
  if (c->tl_host_bytes < hb) {
    if (c->tl_host) hipHostFree(c->tl_host);
    c->tl_host_bytes = 0;
    if (hipHostMalloc(&c->tl_host, hb, hipHostMallocDefault) != hipSuccess) {
      c->tl_host = nullptr;
      return fail(c, KMZ_E_HIP, "hipHostMalloc (tail read-back)");
    }
    c->tl_host_bytes = hb;
  }
  char *rb = static_cast<char *>(c->tl_rb.p);
  unsigned int *rb_cnt = reinterpret_cast<unsigned int *>(rb);
  uint32_t *rb_sstat = reinterpret_cast<uint32_t *>(rb + 64);
  unsigned long long *rb_sfirst = reinterpret_cast<unsigned long long *>(rb + 64 + (size_t)c->tl_n_svc * 32);
  uint32_t *rb_rel = reinterpret_cast<uint32_t *>(rb + 64 + (size_t)c->tl_n_svc * 40);
  {
    Timed t(c, KMZ_K_MEMSET);
    FillArgs f;
    f.add(c->tl_pset.p, pcap * 8, 0);
    f.add(c->tl_pkey.p, pacap * 8, 0);
    f.add(c->tl_pval.p, pacap * 4, 0);
    f.add(c->tl_hasin.p, c->tl_n_ep ? c->tl_n_ep : 1, 0);
    f.add(rb_cnt, 64, 0);
    if (c->tl_n_svc) {
      f.add(rb_sstat, (size_t)c->tl_n_svc * 32, 0);
      f.add(rb_rel, (size_t)c->tl_n_svc * nd_run * 4, 0);
      f.add(rb_sfirst, (size_t)c->tl_n_svc * 8, 0xFF);
    }
    launch_fill(c->stream, f);
  }
  unsigned long long *cnt64 = reinterpret_cast<unsigned long long *>(rb_cnt);  // [0] flags (u32), [1] details, [2] pairs
  {
    Timed t(c, KMZ_K_TAIL);
    launch_tail(c->stream, P<unsigned long long>(c->trip_out), st + S_TRIP_OUT, nt, P<uint32_t>(c->tl_svc),
                P<uint32_t>(c->tl_cls), P<uint32_t>(c->tl_lsvc), P<uint32_t>(c->tl_svc), c->tl_n_ep, c->tl_n_cls,
                bits, P<unsigned long long>(c->tl_lbkt), (uint32_t)slab, P<uint32_t>(c->tl_lbn),
                P<unsigned long long>(c->tl_pset), pcap, P<unsigned long long>(c->tl_pkey), P<uint32_t>(c->tl_pval),
                pacap, P<uint8_t>(c->tl_hasin), rb_sstat, rb_rel, nd_run,
                rb_cnt, P<kmz_tail_detail>(c->tl_det), acap, P<uint32_t>(c->tl_pairs), cnt64 + 1,
                // diagnostic knobs (timing only, wrong results): KMZ_ABLATE bit 7 skips the
                // link keys, bit 12 the cohesion pairs
                ((c->ablate >> 7) & 1u) | (((c->ablate >> 12) & 1u) << 1));
    launch_tail_service_rows(c->stream, P<unsigned long long>(c->epp) + c->n_dep, P<uint32_t>(c->tl_svc),
                             P<uint8_t>(c->tl_hasin), c->tl_n_ep, rb_sstat, rb_sfirst);
  }
  // one read-back and one synchronisation for the counters and every per-service output
  char *hh = static_cast<char *>(c->tl_host);
  HIPCHK(c, hipMemcpyAsync(hh, rb, hb, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_tail, c->stream));
  return KMZ_OK;
}

// kmz_tail_end's wait for one attempt: 1 = done, 0 = repeat (tables grown), else an error
static int tail_finish(kmz_ctx *c, int attempt, uint64_t *n_details, uint64_t *n_pairs) {
  const uint64_t nt = c->tl_nt;
  char *hh = static_cast<char *>(c->tl_host);
  HIPCHK(c, hipEventSynchronize(c->ev_tail));
  if (!c->tl_run_after) harvest(c);  // (else the run behind it is timed too: its kmz_run_end harvests both)
  unsigned long long h[6];
  memcpy(h, hh, sizeof(h));
  const uint32_t fl = (uint32_t)h[0];
  if (fl & F_RANGE) return fail(c, KMZ_E_RANGE, "edge key endpoint outside the tail map");
  const bool bucket_full = (uint32_t)h[5] != 0;  // (u32 word 10) a bucket outgrew its LDS tables
  if ((fl & F_TRIPLE_OVERFLOW) || bucket_full) {
    if (attempt >= 3) return fail(c, KMZ_E_OVERFLOW, "service tail table overflow");
    if (c->tl_run_after)  // (a run enqueued behind the open tail has overwritten the edge keys it read)
      return fail(c, KMZ_E_STATE, "service tail tables overflowed after the next run began: kmz_tail_run again");
    if (bucket_full) {
      if (c->tl_bbits >= tail_bucket_bits_max()) return fail(c, KMZ_E_OVERFLOW, "service tail: too many link keys");
      ++c->tl_bbits;
    }
    if (fl & F_TRIPLE_OVERFLOW) {
      c->tl_acap = std::max(c->tl_acap * 4, pow2_at_least(nt / 2 + 4096));
      c->tl_pacap = std::max(c->tl_pacap * 4, pow2_at_least(nt / 4 + 4096));
      c->tl_pcap = std::max(c->tl_pcap * 4, pow2_at_least(2 * nt + 64));
      c->tl_bcap *= 2;
    }
    return 0;
  }
  const uint64_t won_p = (uint32_t)(h[4] >> 32);
  c->tl_pcap = pow2_at_least(2 * won_p + 4096);  // the next run's pair set (this run's pairs at load <= 1/2)
  // the detail output / pair tables at 2x this run's counts for the next
  // run (they start at nt / 2 and nt / 4); a larger next batch overflows and
  // repeats the tail 4x larger
  c->tl_acap = pow2_at_least(2 * h[1] + 4096);
  c->tl_pacap = pow2_at_least(2 * h[2] + 4096);
  c->tl_nd = h[1];
  c->tl_np = h[2];
  // relying-factor distances beyond the dense table: reported, and the
  // table grows for the next run (the host takes them from the details)
  c->tl_deep = (uint32_t)h[3];
  if (c->tl_deep >= c->tl_n_dist && (uint64_t)c->tl_n_svc * (c->tl_deep + 1) <= (1ull << 26))
    c->tl_n_dist = c->tl_deep + 1;
  c->tl_rel_dist = c->tl_deep ? 0 : c->tl_nd_run;
  c->tl_ran = true;
  if (n_details) *n_details = h[1];
  if (n_pairs) *n_pairs = h[2];
  return 1;
}

int kmz_tail_begin(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (c->tl_open) return fail(c, KMZ_E_STATE, "kmz_tail_begin while a tail is open (kmz_tail_end first)");
  if (!(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
  if (!c->tl_map) return fail(c, KMZ_E_STATE, "kmz_tail_map_set first");
  if (c->tl_n_ep != c->n_dep) return fail(c, KMZ_E_ARG, "tail map size differs from the dependency endpoints");
  unsigned long long *st = P<unsigned long long>(c->stats64);
  uint64_t nt = 0;
  if (c->hpin_valid) {
    nt = reinterpret_cast<const unsigned long long *>(reinterpret_cast<const unsigned int *>(c->hpin) + C_COUNT)[S_TRIP_OUT];
  } else {
    unsigned long long s[S_COUNT];
    HIPCHK(c, hipMemcpyAsync(s, c->stats64.p, sizeof(s), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    nt = s[S_TRIP_OUT];
  }
  // link keys <= 2 per edge key (load <= 1/2); pairs <= 1 per edge key; the
  // detail / pair tables start smaller and grow on overflow
  // pair set: sized by the previous run's first occurrences (load <= 1/2), or
  // by the worst case (one pair per edge key) on the first run; grown on overflow
  if (!c->tl_bbits) c->tl_bbits = 11;
  if (!c->tl_pcap) c->tl_pcap = pow2_at_least(2 * nt + 64);
  if (!c->tl_acap) c->tl_acap = pow2_at_least(nt / 2 + 4096);
  if (!c->tl_pacap) c->tl_pacap = pow2_at_least(nt / 4 + 4096);
  c->tl_nt = nt;
  if (int r = tail_enqueue(c)) return r;
  c->tl_open = true;
  c->tl_run_after = false;
  return KMZ_OK;
}

int kmz_tail_end(kmz_ctx *c, uint64_t *n_details, uint64_t *n_pairs) {
  if (!c) return KMZ_E_ARG;
  if (!c->tl_open) return fail(c, KMZ_E_STATE, "kmz_tail_end without kmz_tail_begin");
  c->tl_open = false;
  for (int attempt = 0;; ++attempt) {
    const int r = tail_finish(c, attempt, n_details, n_pairs);
    if (r == 1) return KMZ_OK;
    if (r != 0) return r;
    if (int e = tail_enqueue(c)) return e;
  }
}

int kmz_tail_run(kmz_ctx *c, uint64_t *n_details, uint64_t *n_pairs) {
  const int r = kmz_tail_begin(c);
  return r ? r : kmz_tail_end(c, n_details, n_pairs);
}

int kmz_tail_service_stats(kmz_ctx *c, uint32_t *stats, uint64_t scap, uint32_t *by_dist, uint64_t dcap,
                           uint32_t *n_dist) {
  if (!c || !n_dist) return KMZ_E_ARG;
  // (a host copy: readable while a run behind the tail is open)
  if (c->tl_open) return fail(c, KMZ_E_STATE, "service tail open (kmz_tail_end first)");
  if (!c->tl_ran) return fail(c, KMZ_E_STATE, "no tail run");
  *n_dist = c->tl_rel_dist;
  const uint64_t ns = (uint64_t)c->tl_n_svc * 8, nd = (uint64_t)c->tl_n_svc * c->tl_rel_dist;
  if ((stats && scap < ns) || (by_dist && dcap < nd)) return fail(c, KMZ_E_ARG, "output too small");
  const char *hh = static_cast<const char *>(c->tl_host);  // (copied back by kmz_tail_run)
  if (stats && ns) memcpy(stats, hh + 64, ns * 4);
  if (by_dist && nd) memcpy(by_dist, hh + 64 + (size_t)c->tl_n_svc * 40, nd * 4);
  return KMZ_OK;
}

int kmz_tail_service_first(kmz_ctx *c, uint64_t *first, uint64_t cap) {
  if (!c || (!first && cap)) return KMZ_E_ARG;
  // (a host copy: readable while a run behind the tail is open)
  if (c->tl_open) return fail(c, KMZ_E_STATE, "service tail open (kmz_tail_end first)");
  if (!c->tl_ran) return fail(c, KMZ_E_STATE, "no tail run");
  if (cap < c->tl_n_svc) return fail(c, KMZ_E_ARG, "output too small");
  if (c->tl_n_svc) memcpy(first, static_cast<const char *>(c->tl_host) + 64 + (size_t)c->tl_n_svc * 32, (size_t)c->tl_n_svc * 8);
  return KMZ_OK;
}

int kmz_service_map_set(kmz_ctx *c, const uint32_t *sid_of_ep, uint32_t n_ep, uint32_t n_sid, const uint8_t *is_5xx,
                        uint32_t n_status) {
  if (!c || (n_ep && !sid_of_ep) || (n_status && !is_5xx) || !n_status) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  std::vector<uint32_t> off((size_t)n_sid + 1, 0), eps(n_ep);
  for (uint32_t e = 0; e < n_ep; ++e) {
    if (sid_of_ep[e] >= n_sid) return fail(c, KMZ_E_RANGE, "service id out of range");
    ++off[sid_of_ep[e] + 1];
  }
  for (uint32_t v = 0; v < n_sid; ++v) off[v + 1] += off[v];
  std::vector<uint32_t> at(off.begin(), off.end() - 1);
  for (uint32_t e = 0; e < n_ep; ++e) eps[at[sid_of_ep[e]]++] = e;  // ascending within each service
  if (ensure(c, c->sv_off, off.size() * 4) || ensure(c, c->sv_eps, (size_t)n_ep * 4 + 4) ||
      ensure(c, c->sv_5xx, n_status) || ensure(c, c->sv_out, (size_t)n_sid * sizeof(kmz_service_sum) + 8))
    return KMZ_E_HIP;
  HIPCHK(c, hipMemcpyAsync(c->sv_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice, c->stream));
  if (n_ep) HIPCHK(c, hipMemcpyAsync(c->sv_eps.p, eps.data(), (size_t)n_ep * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->sv_5xx.p, is_5xx, n_status, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->sv_n_ep = n_ep;
  c->sv_n_sid = n_sid;
  c->sv_n_status = n_status;
  c->sv_map = true;
  return KMZ_OK;
}

int kmz_service_sums_begin(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->sv_map) return fail(c, KMZ_E_STATE, "kmz_service_map_set first");
  if (!(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
  if ((uint64_t)c->sv_n_ep * c->sv_n_status != c->G) return fail(c, KMZ_E_ARG, "service map size differs from the groups");
  if (c->sv_open) return fail(c, KMZ_E_STATE, "kmz_service_sums_begin while sums are open (kmz_service_sums_end first)");
  c->sv_open = true;
  if (!c->sv_n_sid) return KMZ_OK;
  const size_t bytes = (size_t)c->sv_n_sid * sizeof(kmz_service_sum);
  if (int r = pinned_staging(c, c->sv_host, c->sv_host_bytes, bytes)) {
    c->sv_open = false;
    return r;
  }
  launch_service_sums(c->stream, P<kmz_group>(c->grp_final), c->sv_n_status, P<uint32_t>(c->sv_off),
                      P<uint32_t>(c->sv_eps), P<uint8_t>(c->sv_5xx), c->sv_n_sid, P<kmz_service_sum>(c->sv_out));
  HIPCHK(c, hipMemcpyAsync(c->sv_host, c->sv_out.p, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_sums, c->stream));
  return KMZ_OK;
}

int kmz_service_sums_end(kmz_ctx *c, kmz_service_sum *out, uint64_t cap) {
  if (!c || (!out && cap)) return KMZ_E_ARG;
  if (!c->sv_open) return fail(c, KMZ_E_STATE, "kmz_service_sums_end without kmz_service_sums_begin");
  if (cap < c->sv_n_sid) return fail(c, KMZ_E_ARG, "output too small");
  c->sv_open = false;
  if (!c->sv_n_sid) return KMZ_OK;
  HIPCHK(c, hipEventSynchronize(c->ev_sums));
  memcpy(out, c->sv_host, (size_t)c->sv_n_sid * sizeof(kmz_service_sum));
  return KMZ_OK;
}

int kmz_service_sums(kmz_ctx *c, kmz_service_sum *out, uint64_t cap) {
  if (!c || (!out && cap)) return KMZ_E_ARG;
  if (c->sv_map && cap < c->sv_n_sid) return fail(c, KMZ_E_ARG, "output too small");
  const int r = kmz_service_sums_begin(c);
  return r ? r : kmz_service_sums_end(c, out, cap);
}

int kmz_tail_get(kmz_ctx *c, kmz_tail_detail *det, uint64_t dcap, kmz_tail_pair *pairs, uint64_t pcap,
                 uint8_t *has_in, uint64_t hcap) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (c->tl_open) return fail(c, KMZ_E_STATE, "service tail open (kmz_tail_end first)");
  if (!c->tl_ran) return fail(c, KMZ_E_STATE, "no tail run");
  if ((det && dcap < c->tl_nd) || (pairs && pcap < c->tl_np) || (has_in && hcap < c->tl_n_ep))
    return fail(c, KMZ_E_ARG, "output too small");
  if (det && c->tl_nd)
    HIPCHK(c, hipMemcpyAsync(det, c->tl_det.p, c->tl_nd * sizeof(kmz_tail_detail), hipMemcpyDeviceToHost, c->stream));
  if (pairs && c->tl_np)
    HIPCHK(c, hipMemcpyAsync(pairs, c->tl_pairs.p, c->tl_np * sizeof(kmz_tail_pair), hipMemcpyDeviceToHost, c->stream));
  if (has_in && c->tl_n_ep) HIPCHK(c, hipMemcpyAsync(has_in, c->tl_hasin.p, c->tl_n_ep, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_unresolved_parents(kmz_ctx *c, uint64_t *ids, uint64_t cap, uint64_t *n_out, int mem) {
  if (!c || !n_out) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & KMZ_RUN_DEPS)) return fail(c, KMZ_E_STATE, "no dependency run");
  if (!(c->path & 1)) return fail(c, KMZ_E_UNSUPPORTED, "span-table path: no per-span parent resolution to export");
  if (c->hpin_valid && reinterpret_cast<const unsigned int *>(c->hpin)[C_MISS] == 0) {
    *n_out = 0;  // every parent was found in its own window: nothing is unresolved (no scan)
    return KMZ_OK;
  }
  if (ensure(c, c->gd_cnt, 16)) return KMZ_E_HIP;
  unsigned long long *cnt = P<unsigned long long>(c->gd_cnt);
  HIPCHK(c, hipMemsetAsync(cnt, 0, 8, c->stream));
  unsigned long long *out = nullptr;
  if (ids && cap) {
    if (mem == KMZ_MEM_DEVICE) {
      out = reinterpret_cast<unsigned long long *>(ids);
    } else {
      if (ensure(c, c->gd_out, cap * 8)) return KMZ_E_HIP;
      out = P<unsigned long long>(c->gd_out);
    }
  }
  launch_unresolved(c->stream, c->pid, P<uint32_t>(c->dp), (uint32_t)c->n, out, out ? cap : 0, cnt);
  unsigned long long n = 0;
  HIPCHK(c, hipMemcpyAsync(&n, cnt, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *n_out = n;
  if (out && n > cap) return fail(c, KMZ_E_ARG, "output too small");
  if (out && mem != KMZ_MEM_DEVICE && n) {
    HIPCHK(c, hipMemcpyAsync(ids, out, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return KMZ_OK;
}

int kmz_count_ids(kmz_ctx *c, const uint64_t *ids, uint64_t n, int mem, uint64_t *found) {
  if (!c || !found || (n && !ids)) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_count_ids before kmz_load");
  uint64_t cap = 1024;
  while (cap < 2 * n + 64) cap *= 2;
  if (ensure(c, c->gd_set, cap * 8) || ensure(c, c->gd_cnt, 16)) return KMZ_E_HIP;
  const unsigned long long *src = reinterpret_cast<const unsigned long long *>(ids);
  if (n && mem == KMZ_MEM_HOST) {
    if (ensure(c, c->gd_in, n * 8)) return KMZ_E_HIP;
    HIPCHK(c, hipMemcpyAsync(c->gd_in.p, ids, n * 8, hipMemcpyHostToDevice, c->stream));
    src = P<unsigned long long>(c->gd_in);
  }
  unsigned long long *cnt = P<unsigned long long>(c->gd_cnt);
  HIPCHK(c, hipMemsetAsync(c->gd_set.p, 0, cap * 8, c->stream));
  HIPCHK(c, hipMemsetAsync(cnt + 1, 0, 8, c->stream));
  launch_ids_count(c->stream, src, n, P<unsigned long long>(c->gd_set), cap, c->sid, (uint32_t)c->n, cnt + 1);
  unsigned long long f = 0;
  HIPCHK(c, hipMemcpyAsync(&f, cnt + 1, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *found = f;
  return KMZ_OK;
}

int kmz_route_ids(kmz_ctx *c, uint32_t world, uint64_t *out, uint64_t cap, int mem, uint64_t *counts) {
  if (!c || !counts || world == 0 || (c->n && !out)) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_route_ids before kmz_load");
  if (cap < c->n) return fail(c, KMZ_E_ARG, "output too small");
  const uint32_t n = (uint32_t)c->n;
  if (ensure(c, c->rt_hist, (size_t)route_chunks(n) * world * 4) || ensure(c, c->rt_tot, (size_t)world * 8))
    return KMZ_E_HIP;
  unsigned long long *dst = reinterpret_cast<unsigned long long *>(out);
  if (mem != KMZ_MEM_DEVICE) {
    if (ensure(c, c->rt_out, (size_t)n * 8)) return KMZ_E_HIP;
    dst = P<unsigned long long>(c->rt_out);
  }
  if (!launch_route(c->stream, c->sid, n, world, P<uint32_t>(c->rt_hist), P<unsigned long long>(c->rt_tot), dst))
    return fail(c, KMZ_E_ARG, "world must be 1..1024");
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(counts, c->rt_tot.p, (size_t)world * 8, hipMemcpyDeviceToHost, c->stream));
  if (mem != KMZ_MEM_DEVICE && n) HIPCHK(c, hipMemcpyAsync(out, dst, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_route_ids_fixed(kmz_ctx *c, uint32_t world, uint64_t seg, uint64_t *out, int mem) {
  if (!c || world == 0 || seg < 2 || !out) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_route_ids_fixed before kmz_load");
  const uint32_t n = (uint32_t)c->n;
  if (ensure(c, c->rt_hist, (size_t)route_chunks(n) * world * 4) || ensure(c, c->rt_tot, (size_t)world * 8))
    return KMZ_E_HIP;
  unsigned long long *dst = reinterpret_cast<unsigned long long *>(out);
  const size_t words = (size_t)world * seg;
  if (mem != KMZ_MEM_DEVICE) {
    if (ensure(c, c->rt_out, words * 8)) return KMZ_E_HIP;
    dst = P<unsigned long long>(c->rt_out);
  }
  // (KMZ_ABLATE2 bit 12, for comparison: the histogram / scan / scatter form)
  const bool ok = (c->ablate2 & 4096u)
                      ? launch_route(c->stream, c->sid, n, world, P<uint32_t>(c->rt_hist),
                                     P<unsigned long long>(c->rt_tot), dst, seg)
                      : launch_route_fixed(c->stream, c->sid, n, world, seg, P<unsigned long long>(c->rt_tot), dst);
  if (!ok) return world > 1024 ? fail(c, KMZ_E_ARG, "world must be 1..1024") : fail(c, KMZ_E_HIP, "kmz_route_ids_fixed launch");
  HIPCHK(c, hipGetLastError());
  if (mem != KMZ_MEM_DEVICE) {  // (host memory: copied back; device memory: enqueued only)
    HIPCHK(c, hipMemcpyAsync(out, dst, words * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return KMZ_OK;
}

int kmz_route_ids_join(kmz_ctx *c, uint32_t world, uint64_t seg, uint64_t *out) {
  if (!c || world == 0 || world > 1024 || seg < 2 || !out) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!c->loaded) return fail(c, KMZ_E_STATE, "kmz_route_ids_join before kmz_load");
  c->rt_arm.world = world;
  c->rt_arm.segw = seg;
  c->rt_arm.out = reinterpret_cast<unsigned long long *>(out);
  c->rt_armed = true;
  c->rt_routed = false;
  return KMZ_OK;
}

int kmz_route_wait(kmz_ctx *c, void *stream, int *in_join) {
  if (!c) return KMZ_E_ARG;
  if (!c->rt_routed) return fail(c, KMZ_E_STATE, "kmz_route_wait: no routed run (kmz_route_ids_join, then kmz_run_begin)");
  HIPCHK(c, hipStreamWaitEvent(stream ? (hipStream_t)stream : c->stream, c->ev_route, 0));
  if (in_join) *in_join = c->rt_in_join ? 1 : 0;
  return KMZ_OK;
}

int kmz_id_repeats(kmz_ctx *c, const uint64_t *vals, uint64_t n, int mem, uint32_t *repeated) {
  if (!c || !repeated || (n && !vals)) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (c->rs_open) return fail(c, KMZ_E_STATE, "kmz_id_repeats while kmz_id_repeats_seg_begin is open");
  *repeated = 0;
  if (n < 2) return KMZ_OK;
  CertPlan pl;
  if (n >= 0xFFFFFFFFull || !cert_plan((uint32_t)n, &pl, false))  // (k_cert_bin bins by 2^6)
    return fail(c, KMZ_E_UNSUPPORTED, "too many values for the certificate: check on the host");
  const uint32_t m = (uint32_t)n;
  // (the guard's own certificate buffers: reusing the run's would resize them
  // between runs, changing the run's addresses -- and its hipGraph key -- every
  // multi-GPU step)
  if (ensure(c, c->rt_pool1, cert_pool1_words(m) * 8) || ensure(c, c->rt_dir, cert_dir_entries(m, pl) * 2) ||
      ensure(c, c->rt_pool2, cert_pool2_bytes(pl)) || ensure(c, c->rt_cur, cert_cur_words(pl) * 4) ||
      ensure(c, c->rt_ctr, C_COUNT * 4))
    return KMZ_E_HIP;
  const unsigned long long *src = reinterpret_cast<const unsigned long long *>(vals);
  if (mem != KMZ_MEM_DEVICE) {
    if (ensure(c, c->rt_out, (size_t)m * 8)) return KMZ_E_HIP;
    HIPCHK(c, hipMemcpyAsync(c->rt_out.p, vals, (size_t)m * 8, hipMemcpyHostToDevice, c->stream));
    src = P<unsigned long long>(c->rt_out);
  }
  unsigned int *cnt = P<unsigned int>(c->rt_ctr);
  unsigned int *cur2 = P<unsigned int>(c->rt_cur);
  HIPCHK(c, hipMemsetAsync(cnt, 0, C_COUNT * 4, c->stream));
  HIPCHK(c, hipMemsetAsync(cur2, 0, cert_cur_words(pl) * 4, c->stream));
  launch_cert_bin(c->stream, src, m, P<unsigned long long>(c->rt_pool1), P<uint16_t>(c->rt_dir));
  launch_cert_split(c->stream, m, P<unsigned long long>(c->rt_pool1), P<uint16_t>(c->rt_dir), pl,
                    P<unsigned long long>(c->rt_pool2), cur2, cnt);
  launch_cert_check(c->stream, m, pl, P<unsigned long long>(c->rt_pool2), cur2, cnt);
  HIPCHK(c, hipGetLastError());
  unsigned int h[C_COUNT];
  HIPCHK(c, hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (h[C_CERT] & CERT_DUP) {
    *repeated = 1;
    return KMZ_OK;
  }
  if (h[C_CERT] & CERT_OVF) return fail(c, KMZ_E_UNSUPPORTED, "certificate overflow: check on the host");
  return KMZ_OK;
}

// The guard's certificate straight over the fixed segments an all-to-all
// delivered (IdGuard): no compaction of the segments first, and enqueued only,
// on the caller's stream (the one that waits for the exchange), so that it
// runs beside the rank's own run; kmz_id_repeats_seg_end waits for it.
int kmz_id_repeats_seg_begin(kmz_ctx *c, const uint64_t *segs, uint32_t world, uint64_t seg, void *stream) {
  if (!c || !segs || world == 0 || seg < 2) return KMZ_E_ARG;
  if (c->rs_open) return fail(c, KMZ_E_STATE, "kmz_id_repeats_seg_begin while one is open");
  hipSetDevice(c->device);
  const uint64_t jt = cert_pool1_words(1);  // (values per pass-1 tile)
  const uint64_t tps = (seg - 1 + jt - 1) / jt, tiles = tps * world;
  CertPlan pl;
  if (tiles * jt >= 0xFFFFFFFFull || !cert_plan((uint32_t)(tiles * jt), &pl, false))
    return fail(c, KMZ_E_UNSUPPORTED, "too many values for the certificate: check on the host");
  const uint32_t m = (uint32_t)(tiles * jt);  // (an upper bound: the plan's pools are sized for it)
  if (ensure(c, c->rt_pool1, cert_pool1_words(m) * 8) || ensure(c, c->rt_dir, cert_dir_entries(m, pl) * 2) ||
      ensure(c, c->rt_pool2, cert_pool2_bytes(pl)) || ensure(c, c->rt_cur, cert_cur_words(pl) * 4) ||
      ensure(c, c->rt_ctr, C_COUNT * 4 + 8) || ensure(c, c->rt_tsz, tiles * 2))
    return KMZ_E_HIP;
  if (!c->rs_pin && hipHostMalloc(&c->rs_pin, C_COUNT * 4 + 8, hipHostMallocDefault) != hipSuccess) {
    c->rs_pin = nullptr;
    return fail(c, KMZ_E_HIP, "hipHostMalloc (guard read-back)");
  }
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
  unsigned int *cnt = P<unsigned int>(c->rt_ctr);
  unsigned long long *maxc = reinterpret_cast<unsigned long long *>(cnt + C_COUNT);
  static_assert(C_COUNT * 4 % 8 == 0, "the largest count follows the counters");
  unsigned int *cur2 = P<unsigned int>(c->rt_cur);
  HIPCHK(c, hipMemsetAsync(cnt, 0, C_COUNT * 4 + 8, s));
  HIPCHK(c, hipMemsetAsync(cur2, 0, cert_cur_words(pl) * 4, s));
  const unsigned long long *src = reinterpret_cast<const unsigned long long *>(segs);
  launch_cert_bin_seg(s, src, world, seg, (uint32_t)tps, P<unsigned long long>(c->rt_pool1), P<uint16_t>(c->rt_dir),
                      P<uint16_t>(c->rt_tsz), maxc);
  launch_cert_split(s, m, P<unsigned long long>(c->rt_pool1), P<uint16_t>(c->rt_dir), pl,
                    P<unsigned long long>(c->rt_pool2), cur2, cnt, P<uint16_t>(c->rt_tsz));
  launch_cert_check(s, m, pl, P<unsigned long long>(c->rt_pool2), cur2, cnt);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->rs_pin, cnt, C_COUNT * 4 + 8, hipMemcpyDeviceToHost, s));
  c->rs_stream = s;
  c->rs_seg = seg;
  c->rs_open = true;
  return KMZ_OK;
}

int kmz_id_repeats_seg_end(kmz_ctx *c, uint32_t *repeated, uint64_t *max_count) {
  if (!c || !repeated || !max_count) return KMZ_E_ARG;
  if (!c->rs_open) return fail(c, KMZ_E_STATE, "kmz_id_repeats_seg_end without kmz_id_repeats_seg_begin");
  c->rs_open = false;
  HIPCHK(c, hipStreamSynchronize(c->rs_stream));
  const unsigned int *h = reinterpret_cast<const unsigned int *>(c->rs_pin);
  const uint64_t mc = *reinterpret_cast<const unsigned long long *>(h + C_COUNT);
  *max_count = mc;
  *repeated = 0;
  if (mc >= c->rs_seg) return KMZ_OK;  // a segment overflowed: the caller redoes the exchange exactly
  if (h[C_CERT] & CERT_DUP) {
    *repeated = 1;
    return KMZ_OK;
  }
  if (h[C_CERT] & CERT_OVF) return fail(c, KMZ_E_UNSUPPORTED, "certificate overflow: check on the host");
  return KMZ_OK;
}

int kmz_finalize(kmz_ctx *c) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  if (!(c->ran & (KMZ_RUN_STATS_RT | KMZ_RUN_STATS_TAG))) return fail(c, KMZ_E_STATE, "no stats run");
  {
    Timed t(c, KMZ_K_FINAL);
    if (int r = finalize_groups(c)) return r;
  }
  c->gu_host = false;  // (the used count is on the device only)
  return kmz_sync(c);
}

void kmz_finalize_host(const uint64_t *p, uint64_t G, kmz_group *out) {
  for (uint64_t g = 0; g < G; ++g) {
    kmz_group r;
    r.combined = p[g];
    r.first = p[5 * G + g];
    r.latest_timestamp = (int64_t)(p[4 * G + g] ^ TS_BIAS);
    finalize_moments(p[g], p[G + g], p[2 * G + g], p[3 * G + g], &r.mean, &r.cv);
    out[g] = r;
  }
}

void kmz_host_exp(const double *in, double *out, uint64_t n) {
#pragma clang loop vectorize(disable)  // (the scalar libm exp: no vector math library)
  for (uint64_t i = 0; i < n; ++i) out[i] = exp(in[i]);
}

void *kmz_host_alloc(uint64_t bytes) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 8, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void kmz_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

int kmz_set_profiling(kmz_ctx *c, int on) { return kmz_set_profiling_mask(c, on ? (1u << KMZ_K_COUNT) - 1 : 0u); }

int kmz_set_profiling_mask(kmz_ctx *c, uint32_t mask) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  c->prof_mask = mask & ((1u << KMZ_K_COUNT) - 1);
  c->prof = c->prof_mask != 0;
  // create the timing events now, and record each once (the first record of
  // an event allocates its completion signal: ~0.5 ms, not inside a timed run)
  std::vector<hipEvent_t> tmp;
  while (c->prof && c->pool.size() + tmp.size() < 4 * KMZ_K_COUNT) tmp.push_back(ev_get(c));
  for (auto e : tmp) c->pool.push_back(e);
  if (c->prof) {
    for (auto e : c->pool) HIPCHK(c, hipEventRecord(e, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float t = 0.f;  // and the elapsed-time path once per pair
    for (size_t k = 0; k + 1 < c->pool.size(); k += 2) hipEventElapsedTime(&t, c->pool[k], c->pool[k + 1]);
  }
  return KMZ_OK;
}

int kmz_kernel_times(kmz_ctx *c, double *ms, uint64_t *calls, int reset) {
  if (!c) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  int r = kmz_sync(c);
  if (r) return r;
  for (int k = 0; k < KMZ_K_COUNT; ++k) {
    if (ms) ms[k] = c->ms[k];
    if (calls) calls[k] = c->calls[k];
    if (reset) {
      c->ms[k] = 0;
      c->calls[k] = 0;
    }
  }
  return KMZ_OK;
}

// ---- synthetic ---------------------------------------------------------------
int kmz_synth_describe(int config, kmz_synth_desc *out) {
  if (!out) return KMZ_E_ARG;
  if (config == KMZ_SYNTH_BOOKINFO) {
    out->n_shapes = out->n_endpoints = BOOK_EPS;
  } else if (config == KMZ_SYNTH_MESH) {
    out->n_shapes = out->n_endpoints = MESH_EPS;
  } else if (config == KMZ_SYNTH_POWER) {
    out->n_shapes = out->n_endpoints = PL_EPS;
  } else {
    return KMZ_E_ARG;
  }
  out->n_status = 3;
  return KMZ_OK;
}

int kmz_synth_shape_ids(int config, uint32_t *rt, uint32_t *tag, uint32_t *dep, uint32_t cap) {
  kmz_synth_desc d;
  if (kmz_synth_describe(config, &d)) return KMZ_E_ARG;
  if (cap < d.n_shapes) return KMZ_E_ARG;
  for (uint32_t i = 0; i < d.n_shapes; ++i) {
    if (rt) rt[i] = i;
    if (tag) tag[i] = i;
    if (dep) dep[i] = i;
  }
  return KMZ_OK;
}

// spans of the synthetic traces [0, t0): the global flatten index of trace t0's first span
static int synth_base(kmz_ctx *c, int config, uint64_t seed, uint64_t t0, uint64_t *base) {
  *base = 0;
  if (!t0) return KMZ_OK;
  size_t tmp_bytes = 0;
  if (t0 >= (1ull << 31)) return fail(c, KMZ_E_ARG, "trace range too large");
  if (ensure(c, c->synth_cnt, t0 * 8) || ensure(c, c->synth_off, 16)) return KMZ_E_HIP;
  launch_synth_count(c->stream, config, seed, 0, t0, P<uint64_t>(c->synth_cnt));
  HIPCHK(c, hipcub::DeviceReduce::Sum(nullptr, tmp_bytes, P<uint64_t>(c->synth_cnt), P<uint64_t>(c->synth_off),
                                       (int)t0, c->stream));
  if (ensure(c, c->scratch, tmp_bytes)) return KMZ_E_HIP;
  HIPCHK(c, hipcub::DeviceReduce::Sum(c->scratch.p, tmp_bytes, P<uint64_t>(c->synth_cnt), P<uint64_t>(c->synth_off),
                                       (int)t0, c->stream));
  HIPCHK(c, hipMemcpyAsync(base, c->synth_off.p, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KMZ_OK;
}

int kmz_synth_load(kmz_ctx *c, int config, uint64_t seed, uint64_t t0, uint64_t t1, uint64_t *n_out) {
  if (!c || t1 < t0) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  kmz_synth_desc d;
  if (kmz_synth_describe(config, &d)) return fail(c, KMZ_E_ARG, "unknown synthetic config");
  hipSetDevice(c->device);
  const auto &dt = dur_table_host();
  if (ensure(c, c->dur_table, dt.size() * 4)) return KMZ_E_HIP;
  HIPCHK(c, hipMemcpyAsync(c->dur_table.p, dt.data(), dt.size() * 4, hipMemcpyHostToDevice, c->stream));
  uint64_t nt = t1 - t0;
  uint64_t base = 0;
  int rb = synth_base(c, config, seed, t0, &base);
  if (rb) return rb;
  size_t tmp_bytes = 0;
  if (ensure(c, c->synth_cnt, (nt + 1) * 8) || ensure(c, c->synth_off, (nt + 1) * 8)) return KMZ_E_HIP;
  launch_synth_count(c->stream, config, seed, t0, nt, P<uint64_t>(c->synth_cnt));
  tmp_bytes = 0;
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, P<uint64_t>(c->synth_cnt), P<uint64_t>(c->synth_off),
                                              (int)nt, c->stream));
  if (ensure(c, c->scratch, tmp_bytes)) return KMZ_E_HIP;
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->scratch.p, tmp_bytes, P<uint64_t>(c->synth_cnt),
                                              P<uint64_t>(c->synth_off), (int)nt, c->stream));
  uint64_t last_off = 0, last_cnt = 0;
  if (nt) {
    HIPCHK(c, hipMemcpyAsync(&last_off, P<uint64_t>(c->synth_off) + nt - 1, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&last_cnt, P<uint64_t>(c->synth_cnt) + nt - 1, 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint64_t n = last_off + last_cnt;
  if (n >= 0xFFFFFFFFull) return fail(c, KMZ_E_ARG, "synthetic batch too large for one context");
  if (ensure(c, c->in_sid, n * 8) || ensure(c, c->in_pid, n * 8) || ensure(c, c->in_kind, n) ||
      ensure(c, c->in_shape, n * 4) || ensure(c, c->in_status, n * 2) || ensure(c, c->in_dur, n * 4) ||
      ensure(c, c->in_ts, n * 8))
    return KMZ_E_HIP;
  SynthOut o{P<uint64_t>(c->in_sid), P<uint64_t>(c->in_pid), P<uint8_t>(c->in_kind), P<uint32_t>(c->in_shape),
             P<uint16_t>(c->in_status), P<uint32_t>(c->in_dur), P<int64_t>(c->in_ts)};
  launch_synth_fill(c->stream, config, seed, t0, nt, P<uint64_t>(c->synth_off), base, P<uint32_t>(c->dur_table), o);
  HIPCHK(c, hipGetLastError());
  std::vector<uint32_t> ids(d.n_shapes);
  kmz_synth_shape_ids(config, ids.data(), nullptr, nullptr, d.n_shapes);
  kmz_shapes sh{d.n_shapes, ids.data(), ids.data(), ids.data(), d.n_endpoints, d.n_endpoints, d.n_endpoints,
                d.n_status};
  int r = load_shapes(c, &sh);
  if (r) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->n = n;
  c->index_base = base;
  c->imap_n = 0;
  c->sid = o.span_id;
  c->pid = o.parent_id;
  c->kind = o.kind;
  c->shape = o.shape;
  c->status = o.status;
  c->dur = o.duration;
  c->ts = o.timestamp;
  c->loaded = true;
  c->ran = 0;
  c->table_hint = false;
  c->hpin_valid = false;
  if (n_out) *n_out = n;
  return KMZ_OK;
}

int kmz_synth_load_shard(kmz_ctx *c, int config, uint64_t seed, uint64_t t0, uint64_t t1, uint32_t world,
                         uint32_t rank, uint64_t *n_out) {
  if (!c || t1 < t0 || world == 0 || rank >= world) return KMZ_E_ARG;
  if (c->run_open) return run_busy(c);
  kmz_synth_desc d;
  if (kmz_synth_describe(config, &d)) return fail(c, KMZ_E_ARG, "unknown synthetic config");
  hipSetDevice(c->device);
  const uint64_t nt = t1 - t0;
  if (nt >= (1ull << 31)) return fail(c, KMZ_E_ARG, "trace range too large");
  const auto &dt = dur_table_host();
  if (ensure(c, c->dur_table, dt.size() * 4)) return KMZ_E_HIP;
  HIPCHK(c, hipMemcpyAsync(c->dur_table.p, dt.data(), dt.size() * 4, hipMemcpyHostToDevice, c->stream));
  uint64_t base = 0;
  int rb = synth_base(c, config, seed, t0, &base);
  if (rb) return rb;
  // per trace: spans (cnt), spans if it is this rank's (sel); their exclusive
  // sums are the global (imap_g) and local (imap_l) starts of every trace
  if (ensure(c, c->synth_cnt, (nt + 1) * 8) || ensure(c, c->synth_off, (nt + 1) * 8) ||
      ensure(c, c->imap_l, (nt + 1) * 8) || ensure(c, c->imap_g, (nt + 1) * 8))
    return KMZ_E_HIP;
  uint64_t *cnt = P<uint64_t>(c->synth_cnt), *sel = P<uint64_t>(c->synth_off);
  uint64_t *loff = P<uint64_t>(c->imap_l), *goff = P<uint64_t>(c->imap_g);
  launch_synth_count(c->stream, config, seed, t0, nt, cnt);
  launch_shard_select(c->stream, t0, nt, world, rank, cnt, sel);
  size_t tmp_bytes = 0;
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, goff, (int)nt, c->stream));
  if (ensure(c, c->scratch, tmp_bytes)) return KMZ_E_HIP;
  if (nt) {
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->scratch.p, tmp_bytes, cnt, goff, (int)nt, c->stream));
    HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->scratch.p, tmp_bytes, sel, loff, (int)nt, c->stream));
  }
  uint64_t last_off = 0, last_cnt = 0;
  if (nt) {
    HIPCHK(c, hipMemcpyAsync(&last_off, loff + nt - 1, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&last_cnt, sel + nt - 1, 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t n = last_off + last_cnt;
  if (n >= 0xFFFFFFFFull) return fail(c, KMZ_E_ARG, "synthetic shard too large for one context");
  if (ensure(c, c->in_sid, n * 8) || ensure(c, c->in_pid, n * 8) || ensure(c, c->in_kind, n) ||
      ensure(c, c->in_shape, n * 4) || ensure(c, c->in_status, n * 2) || ensure(c, c->in_dur, n * 4) ||
      ensure(c, c->in_ts, n * 8))
    return KMZ_E_HIP;
  SynthOut o{P<uint64_t>(c->in_sid), P<uint64_t>(c->in_pid), P<uint8_t>(c->in_kind), P<uint32_t>(c->in_shape),
             P<uint16_t>(c->in_status), P<uint32_t>(c->in_dur), P<int64_t>(c->in_ts)};
  launch_synth_fill_shard(c->stream, config, seed, t0, nt, world, rank, goff, loff, base, P<uint32_t>(c->dur_table), o);
  launch_add_base(c->stream, goff, nt, base);
  HIPCHK(c, hipGetLastError());
  std::vector<uint32_t> ids(d.n_shapes);
  kmz_synth_shape_ids(config, ids.data(), nullptr, nullptr, d.n_shapes);
  kmz_shapes sh{d.n_shapes, ids.data(), ids.data(), ids.data(), d.n_endpoints, d.n_endpoints, d.n_endpoints,
                d.n_status};
  int r = load_shapes(c, &sh);
  if (r) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->n = n;
  c->index_base = 0;
  c->imap_n = nt;  // one run per trace (foreign traces repeat a local start: skipped by the map)
  c->sid = o.span_id;
  c->pid = o.parent_id;
  c->kind = o.kind;
  c->shape = o.shape;
  c->status = o.status;
  c->dur = o.duration;
  c->ts = o.timestamp;
  c->loaded = true;
  c->ran = 0;
  c->table_hint = false;
  c->hpin_valid = false;
  if (n_out) *n_out = n;
  return KMZ_OK;
}

int kmz_synth_host(int config, uint64_t seed, uint64_t t0, uint64_t t1, uint64_t cap, uint64_t *span_id,
                   uint64_t *parent_id, uint8_t *kind, uint32_t *shape, uint16_t *status, uint32_t *duration,
                   int64_t *timestamp, uint64_t *trace_off, uint64_t *n_out) {
  if (t1 < t0 || (config != KMZ_SYNTH_BOOKINFO && config != KMZ_SYNTH_MESH && config != KMZ_SYNTH_POWER))
    return KMZ_E_ARG;
  const auto &dt = dur_table_host();
  auto gen = [&](uint64_t t, uint64_t gbase, uint64_t lbase, const uint32_t *tab, const SynthOut *o) -> uint32_t {
    if (config == KMZ_SYNTH_BOOKINFO) return synth_trace<2>(seed, t, gbase, lbase, tab, o);
    if (config == KMZ_SYNTH_POWER) return synth_trace<5>(seed, t, gbase, lbase, tab, o);
    return synth_trace<3>(seed, t, gbase, lbase, tab, o);
  };
  uint64_t base = 0;
  for (uint64_t t = 0; t < t0; ++t) base += gen(t, 0, 0, nullptr, nullptr);
  SynthOut o{span_id, parent_id, kind, shape, status, duration, timestamp};
  uint64_t off = 0;
  for (uint64_t t = t0; t < t1; ++t) {
    const uint32_t cnt = gen(t, 0, 0, nullptr, nullptr);
    if (trace_off) trace_off[t - t0] = off;
    if (span_id && off + cnt > cap) return KMZ_E_ARG;
    if (span_id) gen(t, base + off, off, dt.data(), &o);
    off += cnt;
  }
  if (trace_off) trace_off[t1 - t0] = off;
  if (n_out) *n_out = off;
  return KMZ_OK;
}

}  // extern "C"

// diagnostic (tools/diag_power.py): K4 staging occupancy of the last run --
// scap, staged keys (sum, max per run), bucket fill (sum, max), bucket
// capacity, slices, coarse bins
extern "C" int kmz__debug_k4(kmz_ctx *c, unsigned long long *out) {
  if (!c || !out) return KMZ_E_ARG;
  const uint32_t ng = c->k4_ng, lb1 = c->k4_lb1;
  const uint64_t nsl = c->k4_nsl;
  if (!ng) return KMZ_E_STATE;
  std::vector<uint32_t> sn((size_t)ng << lb1), bn(nsl);
  if (hipMemcpy(sn.data(), c->kstage_n.p, sn.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(bn.data(), c->kbucket_n.p, bn.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return KMZ_E_HIP;
  unsigned long long s1 = 0, m1 = 0, s2 = 0, m2 = 0;
  for (uint32_t v : sn) s1 += v, m1 = std::max<unsigned long long>(m1, v);
  for (uint32_t v : bn) s2 += v, m2 = std::max<unsigned long long>(m2, v);
  out[0] = c->scap;
  out[1] = s1;
  out[2] = m1;
  out[3] = s2;
  out[4] = m2;
  out[5] = ((uint64_t)ng * c->scap + nsl - 1) / nsl;
  out[6] = nsl;
  out[7] = 1ull << lb1;
  return KMZ_OK;
}

// diagnostic (tools/diag_lists.py): the chain walk's global lists in the last
// run -- staged keys, deferred checks, claimed slots (outside the tile kernel's
// per-workgroup reservations: all of them for k4_tile8/9), pending spans
extern "C" int kmz__debug_chain_lists(kmz_ctx *c, unsigned long long *out) {
  if (!c || !out) return KMZ_E_ARG;
  unsigned int cnt[16];
  if (hipMemcpy(cnt, c->counters.p, sizeof(cnt), hipMemcpyDeviceToHost) != hipSuccess) return KMZ_E_HIP;
  out[0] = cnt[kmz::C_FSTAGE];
  out[1] = cnt[kmz::C_FDEFER];
  out[2] = cnt[kmz::C_WPOS];
  out[3] = cnt[kmz::C_PLIST];
  return KMZ_OK;
}
