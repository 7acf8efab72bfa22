// kmz_kernels.h -- kernel launchers shared between kmz_kernels.hip and kmz_api.hip
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kmz.h"
#include "kmz_common.h"
#include "kmz_synth.h"

namespace kmz {

constexpr uint8_t KIND_SERVER = KMZ_KIND_SERVER;
constexpr uint8_t KIND_CLIENT = KMZ_KIND_CLIENT;

// A window slot's packed (kind, element id) word (k4_tile8's 8-byte records):
// kind in bits 30-31, the id in bits 0-29 -- the span's shape, or its
// dependency endpoint -- and EPK_NONE for none (a CLIENT span, an unknown
// shape).  Edge keys hold endpoints in 24 bits, so every endpoint id fits.
constexpr uint32_t EPK_NONE = 0x3FFFFFFFu;
__host__ __device__ __forceinline__ uint32_t epk_pack(uint32_t kind, uint32_t ep) {
  return ((kind & 3u) << 30) | (ep < EPK_NONE ? ep : EPK_NONE);
}
__host__ __device__ __forceinline__ uint32_t epk_kind(uint32_t e) { return e >> 30; }
__host__ __device__ __forceinline__ uint32_t epk_ep(uint32_t e) {
  return (e & EPK_NONE) == EPK_NONE ? NONE : (e & EPK_NONE);
}

// u32 device counters
enum {
  C_FLAGS = 0,
  C_DUPS = 1,
  C_TRIPLES = 2,
  C_MISS = 3,
  C_PEND = 4,
  C_CERT = 5,
  C_PLIST = 6,  // K4 spans whose ancestry leaves their LDS window (pending list length)
  C_WPOS = 7,   // K4 chain-table slots written outside the tile kernel (cleared after the run)
  C_FSTAGE = 8,  // fused join + walk: keys staged in the global list
  C_FDEFER = 9,  // fused join + walk: deferred chain checks in the global list
  C_K3ESC = 10,  // partitioned K3: spans without a record (escapes)
  C_COUNT = 12   // (even: the u64 statistics follow the counters)
};
// C_CERT bits: the window join's answers cannot be used (global table path)
constexpr uint32_t CERT_DUP = 1u, CERT_OVF = 2u;
constexpr uint32_t MISSV = 0xFFFFFFFDu;  // dp: parent id not in the span's window
constexpr uint32_t PEND = 0xFFFFFFFCu;   // cparent: CLIENT chain leaves the window
// u64 device statistics
enum { S_ROWS = 0, S_REL = 1, S_MAXD = 2, S_CHAINS = 3, S_SERVER = 4, S_TRIP_OUT = 5, S_DEPENT = 6, S_GUSED = 7, S_COUNT = 8 };

struct DupEntry {
  uint32_t pos, idx, winner, pad;
};

// up to FILL_MAX buffer fills (byte value each) in one launch (k_fill)
constexpr uint32_t FILL_MAX = 12;
struct FillArgs {
  void *p[FILL_MAX];
  uint64_t bytes[FILL_MAX];
  uint32_t val[FILL_MAX];
  uint32_t n = 0;
  void add(void *ptr, uint64_t nbytes, uint32_t byte) {
    if (!nbytes) return;
    if (n >= FILL_MAX) __builtin_trap();  // (a programming error: never corrupt the launch arguments)
    p[n] = ptr;
    bytes[n] = nbytes;
    val[n] = byte;
    ++n;
  }
};
void launch_fill(hipStream_t s, const FillArgs &a);
// up to 4 device copies (8-byte multiples, 8-byte aligned) in one launch;
// false (nothing launched) if a range is not
struct CopyArgs {
  const void *src[4];
  void *dst[4];
  uint64_t bytes[4];
  uint32_t n = 0;
  void add(const void *from, void *to, uint64_t nbytes) {
    if (!nbytes) return;
    if (n >= 4) __builtin_trap();
    src[n] = from;
    dst[n] = to;
    bytes[n] = nbytes;
    ++n;
  }
};
bool launch_copy8(hipStream_t s, const CopyArgs &a);

void launch_build(hipStream_t s, const uint64_t *sid, uint32_t n, unsigned long long *table, uint64_t cap,
                  DupEntry *dups, uint32_t dup_cap, unsigned int *counters);
void launch_fixup(hipStream_t s, const DupEntry *dups, const unsigned int *counters, uint32_t dup_cap,
                  unsigned long long *table, unsigned int *dkey, unsigned int *dval, uint32_t dcap);
void launch_resolve(hipStream_t s, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind, uint32_t n,
                    const unsigned long long *table, uint64_t cap, uint32_t *cparent, unsigned int *counters);
void launch_stats(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status, const uint32_t *dur,
                  const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape, uint32_t n_shapes, uint32_t n_ep,
                  uint32_t n_status, uint64_t index_base, unsigned long long *grp, unsigned int *counters,
                  unsigned long long *n_server);
void launch_walk(hipStream_t s, const uint64_t *sid, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                 const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                 uint64_t index_base, const unsigned long long *table, uint64_t cap, const unsigned int *dkey,
                 const unsigned int *dval, uint32_t dcap, unsigned long long *trip, uint64_t tcap,
                 unsigned long long *ep_ts, unsigned long long *ep_first, unsigned long long *rowpos,
                 unsigned int *counters, unsigned long long *stats64, uint32_t ablate = 0);
// the used groups (combined > 0) compacted in ascending id beside the dense
// finalisation (kmz_fetch_used): ids, groups, per-chunk counts, the total
struct GroupsUsed {
  uint32_t *ids, *bcnt;
  kmz_group *groups;
  unsigned long long *total;
};
constexpr uint32_t USED_MAX_CHUNKS = 4096;  // (1024 groups a chunk: G <= 2^22)
uint32_t used_chunks(uint32_t G);
void launch_finalize(hipStream_t s, unsigned long long *grp, uint32_t G, kmz_group *out,
                     const GroupsUsed *u = nullptr);
void launch_compact(hipStream_t s, const unsigned long long *trip, uint64_t tcap, unsigned long long *out,
                    unsigned long long *count);
void launch_synth_count(hipStream_t s, int config, uint64_t seed, uint64_t t0, uint64_t nt, uint64_t *cnt);
void launch_synth_fill(hipStream_t s, int config, uint64_t seed, uint64_t t0, uint64_t nt, const uint64_t *off,
                       uint64_t gbase, const uint32_t *dur_table, SynthOut out);

// partitioned K3 / K4 (kmz_part.hip)
void launch_k3_produce(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                       const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                       uint32_t n_shapes, uint32_t n_ep, uint32_t n_status, uint32_t S, unsigned int *counters,
                       unsigned long long *n_server, void *pool, uint32_t *dir, uint32_t *tile_tmp);
// balanced K3 reduce (directory [partition][tile], i.e. produced with S = 1):
// plan = k3_plan_words(P) u32 scratch, part = k3_bal_part_bytes(G)
void launch_k3_reduce_bal(hipStream_t s, uint32_t n, uint32_t G, const void *pool,
                          const uint32_t *dir, uint32_t *plan, unsigned long long *part, unsigned long long *grp,
                          bool unpacked = false);
uint32_t k3_bal_items(uint32_t G);
uint32_t k3_plan_words(uint32_t P);
uint64_t k3_bal_part_bytes(uint32_t G);
uint64_t k3_slice_part_bytes(uint32_t G, uint32_t S);
// the reduce leaves each group's first 16-span block; launch_k3_first turns it
// into the first span index (before launch_k3_escapes)
void launch_k3_first(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status, uint32_t n,
                     const uint32_t *ep_of_shape, uint32_t n_shapes, uint32_t n_status, uint64_t index_base,
                     uint32_t G, unsigned long long *grp, unsigned int *counters);
void launch_k3_reduce(hipStream_t s, uint32_t n, uint32_t G, const void *pool,
                      const uint32_t *dir, unsigned long long *part, uint32_t S, unsigned long long *grp);
// small key spaces (G <= 1024): per-chunk LDS partials, part = [k3_small_blocks(n)][6][G] u64
uint32_t k3_small_blocks(uint32_t n);
void launch_k3_small(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                     const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                     uint32_t n_shapes, uint32_t n_ep, uint32_t n_status, uint64_t index_base,
                     unsigned int *counters, unsigned long long *n_server, unsigned long long *part,
                     uint32_t *tile_tmp, unsigned long long *grp);
uint32_t k3_partitions(uint32_t G);
uint32_t k3_pmax();
uint64_t k3_pool_bytes(uint32_t n);
uint64_t *k3_tbase(void *pool, uint32_t n);
uint32_t *k3_esc(void *pool, uint32_t n);
// the partitioned K3's escapes (spans whose duration or timestamp do not fit an
// 8-byte record, counted in C_K3ESC): into E ([6][G] u64, zero / max 0 / min
// ~0 filled before the run), then folded into the group partials grp
void launch_k3_escapes(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint16_t *status,
                       const uint32_t *dur, const int64_t *ts, uint32_t n, const uint32_t *ep_of_shape,
                       uint32_t n_shapes, uint32_t n_status, uint64_t index_base, void *pool,
                       const unsigned int *counters, unsigned long long *E, uint32_t G, unsigned long long *grp);
uint32_t k3_tiles(uint32_t n);
uint64_t k3_dir_words(uint32_t n, uint32_t P, uint32_t S);
void launch_tile_sum(hipStream_t s, const uint32_t *v, uint32_t ntiles, uint32_t stride, uint32_t fields,
                     unsigned long long *out, uint32_t max_field);

// K4 by ancestor-chain interning (kmz_chain.hip)
uint32_t chain_tiles(uint32_t n);
void launch_chain(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                  const uint32_t *cparent, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes, uint32_t n_ep,
                  uint64_t index_base, uint64_t seed, void *ctab, uint64_t ccap, unsigned long long *trip,
                  uint64_t tcap, unsigned long long *ep_ts, unsigned long long *rowpos, uint32_t *plist,
                  uint32_t pcap, unsigned int *counters, uint32_t *tile_stats, unsigned long long *stats64,
                  unsigned long long *stage, uint32_t scap, uint32_t *stage_n, unsigned long long *defer,
                  uint32_t dcap, uint32_t *defer_n, uint32_t *wpos, uint32_t wcap, uint32_t *wpos_n,
                  uint4 *etab, bool direct, uint32_t ablate = 0, bool cmode = false, bool etab_ok = false);
uint32_t chain_grid(uint32_t n);
// coarse bins per tile workgroup (2^lb1) and slices per coarse bin (2^lb2) of
// an edge set of tcap slots; false if tcap is not ESLICE * a power of two
bool key_bins(uint64_t tcap, uint32_t *lb1, uint32_t *lb2);
// direct enumeration may stage 4-byte keys (kmz_common.h, compact edge keys)
bool compact_staging(uint64_t tcap, uint32_t n_ep);
constexpr uint64_t CHAIN_ENTRY_BYTES = 16;  // {sig, parent sig}
void launch_key_insert(hipStream_t s, const unsigned long long *keys, uint64_t n, unsigned long long *trip,
                       uint64_t tcap, unsigned int *counters);
// staged keys -> edge set (k_key_part, k_key_slice), deferred chain checks
// (chain mode), run totals
void launch_chain_settle(hipStream_t s, uint32_t n, bool direct, void *ctab, uint64_t ccap, unsigned long long *trip,
                         uint64_t tcap, unsigned int *counters, const uint32_t *wg_stats, unsigned long long *stats64,
                         const unsigned long long *stage, uint32_t scap, const uint32_t *stage_n,
                         unsigned long long *bucket, uint64_t bcap, uint32_t *bucket_n,
                         const unsigned long long *defer, uint32_t dcap, const uint32_t *defer_n, uint32_t *gpos,
                         uint32_t gcap, uint32_t ablate = 0, bool cmode = false, uint32_t ablate2 = 0);
// per shape: dependency endpoint + SERVER element hash under `seed` (the walk's gather table)
void launch_chain_etab(hipStream_t s, const uint32_t *dep_ep, uint32_t n_shapes, uint64_t seed, uint4 *etab);
// K2 + K4 fused over one LDS window, chain interning (kmz_fuse.hip); its
// staged keys, deferred checks and claimed slots are global lists
// (counters C_FSTAGE, C_FDEFER, C_WPOS), settled by launch_chain_settle_list
void launch_join_chain(hipStream_t s, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind,
                       const uint32_t *shape, const int64_t *ts, uint32_t n, const uint32_t *dep_ep, uint32_t n_shapes,
                       uint32_t n_ep, uint64_t index_base, uint64_t seed, uint32_t *cparent, uint32_t *dp,
                       unsigned long long *pool1, uint16_t *jdir, unsigned int *counters, void *ctab, uint64_t ccap,
                       unsigned long long *trip, uint64_t tcap, unsigned long long *ep_ts, unsigned long long *rowpos,
                       uint32_t *plist, uint32_t pcap, uint32_t *tile_stats, unsigned long long *stage, uint32_t scap,
                       unsigned long long *defer, uint32_t dcap, uint32_t *gpos, uint32_t gcap, uint4 *etab,
                       uint32_t ablate = 0, bool etab_ok = false);
// (nt: the tile kernel's tiles, whose tile_stats rows are summed)
void launch_chain_settle_list(hipStream_t s, uint32_t nt, void *ctab, uint64_t ccap, unsigned long long *trip,
                              uint64_t tcap, unsigned int *counters, const uint32_t *tile_stats,
                              unsigned long long *stats64, const unsigned long long *stage, uint32_t scap,
                              const unsigned long long *defer, uint32_t dcap, uint32_t *gpos, uint32_t gcap,
                              uint32_t ablate = 0, const uint32_t *id_ep = nullptr, uint32_t n_ids = 0);
// K4 chain interning, one workgroup per tile (kmz_walk.hip); same global
// lists as the fused kernel (settled by launch_chain_settle_list over walk_tiles)
struct ChainRun;
uint32_t walk_tiles(uint32_t n);
void launch_chain_tile(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint32_t *cparent, uint32_t n,
                       const uint32_t *dep_ep, uint32_t n_shapes, uint4 *etab, uint32_t *tile_stats, const ChainRun &a);
// k4_tile8: 8-byte window records; chain elements by shape (a.id_ep set: the
// dependency table maps every shape into range) or by endpoint (gathered)
void launch_chain_tile8(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint32_t *cparent, uint32_t n,
                        const uint32_t *dep_ep, uint32_t n_shapes, uint32_t *tile_stats, const ChainRun &a);
// k4_tile9 (round 6): k4_tile8's chains with the element hashes kept in LDS
// and sentinel-terminated walks; ids (shapes, or gathered endpoints) below
// 2^19 - 1 (chain_tile9_fits)
bool chain_tile9_fits(uint32_t n_ids);
void launch_chain_tile9(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const uint32_t *cparent, uint32_t n,
                        const uint32_t *dep_ep, uint32_t n_shapes, uint32_t *tile_stats, const ChainRun &a);
// zero the chain-table entries this run wrote (instead of a memset of the table)
void launch_chain_clear(hipStream_t s, uint32_t n, void *ctab, const uint32_t *wpos, uint32_t wcap,
                        const uint32_t *wpos_n, const uint32_t *gpos, uint32_t gcap, const unsigned int *counters);
// (the global list only: the fused kernel's claimed slots)
void launch_chain_clear_list(hipStream_t s, void *ctab, const uint32_t *gpos, uint32_t gcap, const unsigned int *counters);
void launch_chain_pend(hipStream_t s, const uint32_t *plist, uint32_t pcap, const uint8_t *kind,
                       const uint32_t *shape, const int64_t *ts, const uint32_t *cparent, uint32_t n,
                       const uint32_t *dep_ep,
                       uint32_t n_shapes, uint32_t n_ep, uint64_t seed, void *ctab, uint64_t ccap,
                       unsigned long long *trip, uint64_t tcap, unsigned long long *ep_ts, unsigned int *counters,
                       unsigned long long *stats64, uint32_t *gpos, uint32_t gcap, bool direct, uint32_t ablate = 0,
                       bool by_shape = false);
// shape-level K3 partials -> endpoint groups / dependency-endpoint records
void launch_collapse_groups(hipStream_t s, const unsigned long long *sg, uint32_t n_shapes, uint32_t S,
                            const uint32_t *map, uint32_t n_ep, unsigned long long *grp, unsigned int *counters);
void launch_collapse_endpoints(hipStream_t s, const unsigned long long *sg, uint32_t n_shapes, uint32_t S,
                               const uint32_t *dep_map, uint32_t n_dep, const uint32_t *cparent, uint64_t index_base,
                               unsigned long long *ep_ts, unsigned long long *ep_first, unsigned int *counters);

// service-level tail over the compacted edge keys (kmz_tail.hip)
// link keys are bucketed by their (service, linked service) pair first, each
// pass-A workgroup into its own slab of every bucket: lbkt = 2^bits x
// tail_part_grid(n_max) x slab u64, lbn = as many u32 fills (written by the
// kernel); bits = tail_bucket_bits_max() or one less; details are written
// to links_out (dcap records, count in out_counts[0]); counters word 10 set:
// a bucket outgrew its LDS tables (redo with more buckets)
uint32_t tail_bucket_bits_max();
uint32_t tail_part_grid(uint64_t n_max);
void launch_tail(hipStream_t s, const unsigned long long *keys, const unsigned long long *n_keys, uint64_t n_max,
                 const uint32_t *svc, const uint32_t *cls, const uint32_t *lsvc_of_cls, const uint32_t *usn,
                 uint32_t n_ep, uint32_t n_cls, uint32_t bits, unsigned long long *lbkt, uint32_t slab, uint32_t *lbn,
                 unsigned long long *pset, uint64_t pcap, unsigned long long *pkey, uint32_t *pval, uint64_t pacap,
                 uint8_t *hasin, uint32_t *sstat, uint32_t *rel, uint32_t n_dist, unsigned int *counters,
                 kmz_tail_detail *links_out, uint64_t dcap, uint32_t *pairs_out, unsigned long long *out_counts,
                 uint32_t knobs = 0);
// per service: rows / gateway into sstat slots 6 / 7, first row into sfirst (after launch_tail)
void launch_tail_service_rows(hipStream_t s, const unsigned long long *epf, const uint32_t *svc, const uint8_t *hasin,
                              uint32_t n_ep, uint32_t *sstat, unsigned long long *sfirst);
// RiskAnalyzer.RealtimeRisk's per-service sums over the finalised groups
void launch_service_sums(hipStream_t s, const kmz_group *grp, uint32_t n_status, const uint32_t *off, const uint32_t *eps,
                         const uint8_t *is5, uint32_t n_sid, kmz_service_sum *out);

// multi-GPU sharding guard (kmz_guard.hip)
void launch_unresolved(hipStream_t s, const uint64_t *pid, const uint32_t *dp, uint32_t n, unsigned long long *out,
                       uint64_t cap, unsigned long long *count);
// cross-shard repeated ids: hashes of the span ids grouped by owner rank;
// hist [route_chunks(n) * world] u32 scratch, tot [world] counts
uint32_t route_chunks(uint32_t n);
bool launch_route(hipStream_t s, const uint64_t *sid, uint32_t n, uint32_t world, uint32_t *hist,
                  unsigned long long *tot, unsigned long long *out, uint64_t segw = 0);
// ... into fixed segments of segw words in one pass over the ids (no
// histogram pass): cur [world] u64 scratch (zeroed here)
bool launch_route_fixed(hipStream_t s, const uint64_t *sid, uint32_t n, uint32_t world, uint64_t segw,
                        unsigned long long *cur, unsigned long long *out);
void launch_ids_count(hipStream_t s, const unsigned long long *ids, uint64_t m, unsigned long long *set, uint64_t cap,
                      const uint64_t *sid, uint32_t n, unsigned long long *found);

// traceId sharding + local -> global index map (kmz_shard.hip)
void launch_shard_select(hipStream_t s, uint64_t t0, uint64_t nt, uint32_t world, uint32_t rank, const uint64_t *cnt,
                         uint64_t *sel);
void launch_synth_fill_shard(hipStream_t s, int config, uint64_t seed, uint64_t t0, uint64_t nt, uint32_t world,
                             uint32_t rank, const uint64_t *goff, const uint64_t *loff, uint64_t gbase,
                             const uint32_t *dur_table, SynthOut out);
void launch_add_base(hipStream_t s, uint64_t *v, uint64_t n, uint64_t base);
void launch_iota(hipStream_t s, unsigned long long *v, uint64_t n, uint64_t base);
void launch_remap_index(hipStream_t s, unsigned long long *v, uint64_t n, uint32_t stride, uint32_t shift,
                        const uint64_t *lstart, const uint64_t *gstart, uint64_t nruns);

// window parent join + uniqueness certificate (kmz_join.hip)
struct CertPlan {
  uint32_t B1, B2, cap2, chunks;  // 2^B1 pass-1 bins, 2^B2 sub-bins per bin
  // past 2^29 ids a single pass 2 would write runs of ~2 records: pass 2 then
  // splits into 2^B2 and a second split pass into 2^B3 more (0: no third level)
  uint32_t B3 = 0, cap3 = 0, chunks3 = 0;
};
// the certificate's pass-2 pool (bytes: level 2, then level 3) and sub-bin
// counters (u32 words) for a plan
uint64_t cert_pool2_bytes(const CertPlan &pl);
uint64_t cert_cur_words(const CertPlan &pl);
// wide: pass 1 may use 2^8 bins (the window join; the guard's k_cert_bin
// always bins by 2^6); force_wide: 2^8 bins at any size (test knob)
bool cert_plan(uint32_t n, CertPlan *pl, bool wide = true, bool force_wide = false);
uint64_t cert_pool1_words(uint32_t n);
uint64_t cert_dir_entries(uint32_t n, const CertPlan &pl);
__host__ __device__ uint32_t join_tiles(uint32_t n);
// The guard's routing folded into the join (kmz_route_ids_join): with `out`
// set, the join's certificate pass 1 bins the tile's hashed ids by owner rank
// (id_owner, world <= the pass-1 bins) and writes them into the owners' fixed
// segments of segw words (word 0 the count, kmz_route_ids_fixed's layout),
// each (tile, owner) run reserved by one device atomic on cur[owner * 16]
// (one 128-byte line per owner); no pool1 / directory.
struct JoinRoute {
  uint32_t world = 0;
  uint64_t segw = 0;
  unsigned long long *cur = nullptr, *out = nullptr;
};
constexpr uint32_t ROUTE_CUR_STRIDE = 16;
void launch_join(hipStream_t s, const uint64_t *sid, const uint64_t *pid, const uint8_t *kind, uint32_t n,
                 uint32_t *cparent, uint32_t *dp, unsigned long long *pool1, uint16_t *jdir, unsigned int *counters,
                 const CertPlan &pl, uint32_t ablate = 0, const JoinRoute &rt = JoinRoute());
// the segments' count words from cur[owner * stride] (after the routing)
void launch_route_counts(hipStream_t s, uint32_t world, uint64_t segw, const unsigned long long *cur, uint32_t stride,
                         unsigned long long *out);
// tsz: per-tile sizes (the guard's segment tiles, launch_cert_bin_seg); null: dense tiles of n values
void launch_cert_split(hipStream_t s, uint32_t n, const unsigned long long *pool1, const uint16_t *jdir,
                       const CertPlan &pl, unsigned long long *pool2, unsigned int *cur2, unsigned int *counters,
                       const uint16_t *tsz = nullptr);
void launch_cert_check(hipStream_t s, uint32_t n, const CertPlan &pl, const unsigned long long *pool2,
                       const unsigned int *cur2, unsigned int *counters);
// pass 1 of the certificate over a plain value array (cross-shard id guard)
void launch_cert_bin(hipStream_t s, const unsigned long long *v, uint32_t n, unsigned long long *pool1,
                     uint16_t *jdir);
// ... over fixed segments as received (count word, values): tps tiles per
// segment, their sizes into tsz, the largest count into *maxc (atomicMax)
void launch_cert_bin_seg(hipStream_t s, const unsigned long long *segs, uint32_t world, uint64_t segw, uint32_t tps,
                         unsigned long long *pool1, uint16_t *jdir, uint16_t *tsz, unsigned long long *maxc);
void launch_miss(hipStream_t s, const uint64_t *sid, const uint64_t *pid, uint32_t *dp, uint32_t n,
                 unsigned long long *mkey, uint32_t *mval, uint32_t mcap, const unsigned int *counters);
void launch_pend(hipStream_t s, const uint8_t *kind, const uint32_t *dp, uint32_t n, uint32_t *cparent,
                 const unsigned int *counters);

// entry order of the reduced dependency graph (kmz_order.hip)
void launch_dep_order(hipStream_t s, const uint8_t *kind, const uint32_t *shape, const int64_t *ts,
                      const uint32_t *cparent, const unsigned long long *rowpos, uint32_t n, const uint32_t *dep_ep,
                      uint32_t n_shapes, uint32_t n_ep, uint64_t index_base, void *tab, uint64_t ecap, uint32_t *val,
                      const unsigned long long *ep_first, kmz_dep_entry *out, unsigned long long *count,
                      int64_t *row_ts, uint32_t *row_shape, unsigned int *counters);
uint64_t dep_order_slot_bytes();

// Zipkin JSON -> columns on the device (kmz_json.hip)
struct JElem {
  int p, d0, d1;  // quote parity; depth change if the chunk starts outside / inside a string
};
constexpr uint32_t JCHUNK = 64;
constexpr uint32_t JF_BAD = 1, JF_COLLIDE = 2, JF_TOP = 4, JF_FULL = 8;
uint64_t json_scan_scratch(uint64_t n);
void launch_json_structure(hipStream_t s, const uint8_t *b, uint64_t len, uint64_t nch, JElem *elem, JElem *state,
                           JElem *jtotal, JElem *jscratch, unsigned long long *mask, uint32_t *cnt, uint32_t *off,
                           uint32_t *ctotal, uint32_t *cscratch, unsigned int *flags);
void launch_json_starts(hipStream_t s, const unsigned long long *mask, const uint32_t *off, uint64_t nch,
                        unsigned long long *starts);
void launch_json_spans(hipStream_t s, const uint8_t *b, uint64_t len, const unsigned long long *starts, uint64_t n,
                       uint64_t *sid, uint64_t *pid, uint8_t *kind, uint32_t *dur, int64_t *ts,
                       unsigned long long *slices, uint32_t *shape_slot, uint32_t *status_slot, unsigned long long *stab,
                       uint64_t scap, unsigned long long *ttab, uint64_t tcap, unsigned int *flags);
void launch_json_reps(hipStream_t s, const unsigned long long *tab, uint64_t cap, const unsigned long long *slices,
                      uint32_t first, uint32_t nf, unsigned long long *out, uint64_t ocap, uint64_t nspan,
                      unsigned long long *count);
void launch_json_remap(hipStream_t s, uint64_t n, uint32_t *shape, const uint32_t *status_slot, uint16_t *status,
                       const uint32_t *smap, const uint32_t *tmap);

}  // namespace kmz
