"""Benchmark: spans/sec through the endpoint dependency graph + combined stats.

One step = one pass of the hot path over one device-resident synthetic batch:
K1 build + K2 resolve + K4 walk (dependency graph) and K3 (combined stats),
finalisation, the multi-GPU merge (N > 1, RCCL via torch.distributed) and the
download of the results (groups, endpoint records, edge keys) to the host.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config mesh|bookinfo|power]

Workloads: one GPU runs config 3 (the 500-service mesh, 1e8 spans); N > 1
GPUs run config 4: 1e9 spans of the same mesh, sharded by h(traceId) mod N
(kmz_synth_load_shard), so the total work is fixed as N grows
(strong scaling, over N = 2/4/8).  --spans / --scaling override.  Rank 0
prints one JSON line.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic bytes per launch of each hot-path kernel (DESIGN.md section 3;
# SURVEY.md 8d budgets K2 57 B/span, K3 19 B/span, K4 12 B/relation).
#   join   k_join_window  K2 parent join + CLIENT contraction   57 B/span
#   stats  k3_produce     K3 (read ep/status/kind/dur/ts)       19 B/span
#   reduce k3_reduce      K3 second pass: the partitioned records it must
#                         read (dur 4 + ts 8 + key/index 4)      16 B/SERVER span
#   walk   k4_tile9       K4 traversal (k4_tile8, k4_tile, k4_chain: knobs / direct)  12 B/relation
#   cert   k_cert_split   uniqueness certificate: one radix split of the
#                         8-B hashed span id (read + write)      16 B/span
#   check  k_cert_check   certificate check: one read of it       8 B/span
#   tail   k_tail_links   service tail: one read of each edge key  8 B/key
#          (+ k_tail_compact; config 5 only)
#   joinwalk k_join_chain the join and the chain walk fused (batches of
#                         2^19..2^23 spans): K2's + K4's bytes  57 B/span + 12 B/relation
def alg_bytes(kernel, n, n_server, relations, n_keys=0):
    return {"join": 57 * n, "stats": 19 * n, "reduce": 16 * n_server, "walk": 12 * relations,
            "cert": 16 * n, "check": 8 * n, "tail": 8 * n_keys, "joinwalk": 57 * n + 12 * relations}.get(kernel, 0)


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")


def build_id() -> str:
    """Digest of the engine's sources (kernels, ABI, headers): which build a
    committed PMC traffic figure was measured on."""
    import glob
    import hashlib

    h = hashlib.sha1()
    root = os.path.dirname(os.path.abspath(__file__))
    files = sorted(glob.glob(os.path.join(root, "kmamiz_amd", "csrc", "*")) + [os.path.join(root, "include", "kmz.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:12]


def traffic_of(kernel, config, n_local):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC pass
    (tools/traffic.sh -> profiles/traffic_*.json: 2 x FETCH_SIZE + WRITE_SIZE)
    of THIS build on this workload; else None (never a stale build's figure)."""
    import glob

    bid = build_id()
    for f in sorted(glob.glob(os.path.join(PROFILES, "traffic_*.json")), reverse=True):
        try:
            t = json.load(open(f))
        except Exception:
            continue
        if t.get("build") != bid or t.get("config") != config or abs(t.get("n_spans", 0) - n_local) > 0.02 * n_local:
            continue
        # (template instances, e.g. k4_chain<false>, count as their kernel)
        ks = [v for name, v in t.get("kernels", {}).items() if name.split("<")[0] == kernel]
        if not ks:
            return None
        lower = sum(v.get("traffic_lower_bytes", 0) for v in ks) if all("traffic_lower_bytes" in v for v in ks) else None
        hits = [v["l2_hit_rate"] for v in ks if "l2_hit_rate" in v]
        return (sum(v["traffic_bytes"] for v in ks), os.path.basename(f), lower, hits[0] if len(hits) == 1 else None)
    return None


def progress(msg):
    """Progress on stderr (stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["mesh", "bookinfo", "power"], default="mesh")
    ap.add_argument("--spans", type=float, default=None,
                    help="spans of the whole job (default: mesh 1e8 on one GPU = config 3, 1e9 on N > 1 GPUs = "
                         "config 4; bookinfo 1e6; power 1e8)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: --spans is the job's total, sharded by h(traceId) mod N; weak: --spans per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-fetch", action="store_true", help="leave results on the device")
    ap.add_argument("--no-h2d", action="store_true", help="skip the host-to-device copy timing of the batch")
    ap.add_argument("--fetch", choices=["pipelined", "sync"], default="pipelined",
                    help="pipelined: each step's results are copied on the device and cross PCIe on a transfer "
                         "stream while the next step's kernels run (kmz_fetch_begin/_end; the last step's copies "
                         "land inside the timed region); sync: kmz_fetch after each run")
    ap.add_argument("--kernel-times", choices=["split", "live"], default="split",
                    help="split: every kernel timed in a profiled pass of --steps steps before the timed region, "
                         "only the dominant kernel's events live inside it; live: every kernel's events inside the "
                         "timed region (each event pair adds launch gaps to the step)")
    ap.add_argument("--tail", choices=["auto", "on", "off"], default="auto",
                    help="service-level tail (instability/coupling/cohesion/risk) in every step; auto = config 5")
    return ap.parse_args()


def cpu_baseline(config, target_seconds, tail=None):
    """The all-core OpenMP restatement (oracle/kmz_cpu_omp.c: per-thread group
    moments, a concurrent span-id table, one walk per row into per-thread edge
    sets) on a bounded prefix of the same synthetic workload, timed on this
    host's cores (OMP_NUM_THREADS; 16 on the GPU box).  ``tail(stats, keys,
    endpoints)``, when given, is the step's service tail on the CPU, timed
    with it (oracle/tail_np.py + the same host finish)."""
    from kmamiz_amd import synth
    from oracle import c_oracle

    table = synth.shape_table(config)

    def run(ntr):
        batch, _ = synth.host_batch(config, 0, ntr)
        t = time.perf_counter()
        st = c_oracle.omp_stats(batch, table.tag_ep, table.n_tag_ep, table.n_status)
        keys, ep, _ = c_oracle.omp_deps(batch, table.dep_ep, table.n_dep_ep)
        if tail is not None:
            tail(st, keys, ep)
        return len(batch), time.perf_counter() - t

    run(2000)  # warm (thread pool, page faults)
    n0, t0 = run(20000)
    rate0 = n0 / max(t0, 1e-6)
    ntr = max(20000, int(20000 * target_seconds * rate0 / n0))
    n, t = run(ntr)
    threads = c_oracle.omp_threads()
    return {
        "value": n / t,
        "unit": "spans/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {ntr} traces ({n} spans) of the same synthetic workload, seed 0x4B4D414D495A, "
        f"oracle/kmz_cpu_omp.c stats+deps on {threads} OpenMP threads"
        + (" + service tail (oracle/tail_np.py, metrics, realtime risk; numpy)" if tail is not None else "")
        + f", {t:.1f} s",
    }


def main():
    args = parse()
    if os.environ.get("KMZ_BENCH_TRACE"):  # diagnostic: Python stacks every 30 s
        import faulthandler

        faulthandler.dump_traceback_later(30, repeat=True)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist

    # (KMZ_DIST_BACKEND=gloo and more ranks than GPUs: a rehearsal of the
    # multi-rank path on a one-GPU box; the driver's runs use RCCL, one GPU per rank)
    backend = os.environ.get("KMZ_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    config = {"mesh": synth.MESH, "bookinfo": synth.BOOKINFO, "power": synth.POWER}[args.config]
    if args.spans:
        target = int(args.spans) * (world if args.scaling == "weak" else 1)
    else:  # config 3 on one GPU, config 4 (1e9 spans over the node) on several
        target = int(1e6 if args.config == "bookinfo" else (1e9 if world > 1 and args.config == "mesh" else 1e8))
    sample_tr = 20000
    per_trace = synth.count_spans(config, 0, sample_tr) / sample_tr
    n_traces = max(1, int(round(target / per_trace)))

    # one stream for torch, the collectives and the engine: a stream of its
    # own (torch's default stream has handle 0, which kmz_create would take
    # for "create your own" -- a non-blocking stream unordered with torch's)
    stream = torch.cuda.Stream(device=local)
    torch.cuda.set_stream(stream)
    eng = Engine(local, stream=stream.cuda_stream)
    if world > 1:  # this rank's traces: shard(traceId) == rank, global flatten indices
        n_local = eng.load_synthetic_shard(config, synth.SEED, 0, n_traces, world, rank)
    else:
        n_local = eng.load_synthetic(config, synth.SEED, 0, n_traces)
    progress(f"loaded {n_local} spans")
    digest = synth.table_digest(config)  # every rank indexes partials by the same synthetic id tables
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    if world > 1:
        # every step's id guard (IdGuard, below) routes and checks every span
        # id of every shard, this rank's own included: the run skips its own
        # uniqueness certificate (a repeat anywhere sends the merge to the
        # exact unsharded pass)
        flags |= L.RUN_NO_CERT
    dev = torch.device("cuda", local)
    state = {}
    tail_on = args.tail == "on" or (args.tail == "auto" and config == synth.POWER)
    if tail_on:  # interned service names of the synthetic shapes (static per config, built once)
        import numpy as np

        from kmamiz_amd.ingest import SHAPE_TAGS, UNDEFINED, tag_identity
        from kmamiz_amd.tail import maps_for_synth, realtime_risk_columns, realtime_risk_from_sums, tail_begin, tail_end

        args.no_fetch = False
        tmaps = maps_for_synth(config)
        n_shapes, n_status, _ = synth.describe(config)
        sid_of, sid_names = {}, []
        tag_sid = np.zeros(n_shapes, dtype=np.int64)
        for sh in range(n_shapes):
            name, tags = synth.shape_tags(config, sh)
            usn = tag_identity((name,) + tuple(tags.get(t, UNDEFINED) for t in SHAPE_TAGS))["uniqueServiceName"]
            if usn not in sid_of:
                sid_of[usn] = len(sid_names)
                sid_names.append(usn)
            tag_sid[sh] = sid_of[usn]
        is_5xx = np.array([str(x).startswith("5") for x in synth.STATUSES[:n_status]], dtype=bool)
        eng.set_service_map(tag_sid, len(sid_names), is_5xx)  # the groups' services, for kmz_service_sums

    phases = {}  # (KMZ_BENCH_TRACE: host wall time per step phase)

    def mark(name, t):
        now = time.perf_counter()
        phases[name] = phases.get(name, 0.0) + (now - t)
        return now

    tail_sync = os.environ.get("KMZ_BENCH_TAIL_SYNC", "0") == "1"

    def service_tail_begin():
        # the device half: what reads this run's buffers (the edge keys where
        # the run left them in HBM; the combined groups), enqueued right after
        # the run so that the GPU goes on while the host fetches
        tp = time.perf_counter()
        tail_begin(eng, tmaps)
        # RiskAnalyzer.RealtimeRisk: the per-service sums over the combined
        # groups on the device (kmz_service_sums, bit-equal to the host's row
        # sums), the rest over the ~10^3 services on the host
        eng.service_sums_begin()
        mark("tail_begin", tp)

    def service_tail_end():
        state["tail_open"] = False
        tp = time.perf_counter()
        t = tail_end(eng, tmaps)
        sums = eng.service_sums_end()
        mark("tail_end", tp)
        state["tail_host"] = (t, sums)

    def tail_host():
        # the host half (metrics, risk): pure host work on what the device half
        # read back, done while the next step's run is on the GPU
        if "tail_host" not in state:
            return
        t, sums = state.pop("tail_host")
        tp = time.perf_counter()
        state["metrics"] = t.metrics()
        tp = mark("tail_metrics", tp)
        state["risk"] = realtime_risk_from_sums(t, sid_names, *sums)
        mark("risk", tp)

    def fetch_done():
        if tail_on:
            tail_host()
        out = eng.fetch_end()
        if out is not None:
            state["groups"], state["keys"], state["endpoints"] = out

    def step():
        # N > 1: the repeated-span-id guard routes this batch's ids and posts
        # its all-to-all before the run, so the exchange overlaps the kernels
        tg = time.perf_counter()
        # (fold: the routing rides in the run's join, kmz_route_ids_join, and
        # post() exchanges once the join is done, beside the rest of the run)
        guard = kdist.IdGuard(eng, dev).start(fold=True) if world > 1 else None
        state["guard_start_s"] = state.get("guard_start_s", 0.0) + (time.perf_counter() - tg)
        tp = time.perf_counter()
        eng.run_begin(flags)
        if state.get("tail_open"):  # the previous step's tail, done while this run was being enqueued
            service_tail_end()
        if guard is not None:
            tg = time.perf_counter()
            guard.post()
            state["guard_start_s"] += time.perf_counter() - tg
        if tail_on:
            tail_host()  # the previous step's host finish, beside this step's kernels
            tp = mark("run_begin+tail_host", tp)
        eng.run_end()
        tp = mark("run", tp)
        if world > 1:
            gw = eng.partials_words(L.PART_GROUPS)
            ew = eng.partials_words(L.PART_ENDPOINTS)
            tw = eng.partials_words(L.PART_TRIPLES)
            g = torch.empty(gw, dtype=torch.int64, device=dev)
            e = torch.empty(ew, dtype=torch.int64, device=dev)
            t = torch.empty(max(1, tw), dtype=torch.int64, device=dev)
            eng.export_partials(L.PART_GROUPS, g.data_ptr(), gw, True)
            eng.export_partials(L.PART_ENDPOINTS, e.data_ptr(), ew, True)
            eng.export_partials(L.PART_TRIPLES, t.data_ptr(), tw, True)
            # three collectives: SUM moments, MAX of max / negated min fields
            # + key count, all-gather of the keys (union in the engine's set)
            kdist.merge_all(g, gw // 6, e, ew // 2, t[:tw], engine=eng, digest=digest, check_ids=guard)
            eng.import_partials(L.PART_GROUPS, g.data_ptr(), gw, True)
            eng.import_partials(L.PART_ENDPOINTS, e.data_ptr(), ew, True)
            eng.finalize()
        # (KMZ_BENCH_TAIL_SYNC=1, for comparison: the tail after the fetch,
        # each half right after the other, as before round 6)
        if tail_on and not tail_sync:
            service_tail_begin()
            state["tail_open"] = True  # (ended by the next step, behind its run_begin)
        if not args.no_fetch:  # the three result sets (with the tail on, the edge keys stay
            # in HBM for kmz_tail_run: the service tail is the output)
            if args.fetch == "pipelined":
                fetch_done()  # the previous step's copies, landed while this step's kernels ran
                eng.fetch_begin(keys=not tail_on)
            else:
                state["groups"], state["keys"], state["endpoints"] = eng.fetch(keys=not tail_on)
            mark("fetch", tp)
        if tail_on and tail_sync:
            service_tail_begin()
            service_tail_end()

    for w in range(args.warmup):
        step()
        progress(f"warmup step {w + 1}/{args.warmup}")
    fetch_done()
    # no collector pause inside the timed region (one measured 7 ms); collected
    # here, before the steps that follow keep the GPU busy and its clock up
    gc.collect()
    gc.disable()
    info = eng.info()
    A = info["n_relations"]

    def kernel_table(ktimes):
        per_kernel = {}
        for k, (ms, calls) in ktimes.items():
            if not calls:
                continue
            avg = ms / calls
            alg = alg_bytes(k, n_local, info["n_server"], A, info["n_triples"]) if calls == args.steps else 0
            per_kernel[k] = {"ms_per_step": round(ms / args.steps, 4), "calls_per_step": round(calls / args.steps, 2),
                             "avg_ms": round(avg, 4), "alg_bytes": alg,
                             "gbs": round(alg / (avg * 1e-3) / 1e9, 1) if alg else None}
        return per_kernel

    eng.kernel_times(reset=True)
    if args.kernel_times == "split":
        # every kernel's events in a profiled pass of the same steps, outside
        # the timed region; inside it only the dominant kernel's (an event
        # record is a ~8 us gap before the next launch: ~20 per mesh step)
        eng.set_profiling(True)
        for _ in range(args.steps):
            step()
        fetch_done()
        per_kernel = kernel_table(eng.kernel_times(reset=True))
        dom = max((k for k in per_kernel if per_kernel[k]["alg_bytes"]), key=lambda k: per_kernel[k]["avg_ms"])
        eng.set_profiling([dom])
    else:
        eng.set_profiling(True)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    state["guard_start_s"] = 0.0
    phases.clear()
    t0 = time.perf_counter()
    marks = []
    for _ in range(args.steps):
        step()
        marks.append(time.perf_counter())
    fetch_done()  # (the last step's results on the host)
    barrier()
    t1 = time.perf_counter()
    if state.get("tail_open"):  # (the last step's tail: its GPU half ran inside the timed region)
        service_tail_end()
        tail_host()
    gc.enable()
    if os.environ.get("KMZ_BENCH_TRACE"):  # diagnostic: per-step wall times
        print("step ms:", [round((b - a) * 1e3, 3) for a, b in zip([t0] + marks, marks + [t1])], file=sys.stderr)
        print("phase ms/step:", {k: round(v / args.steps * 1e3, 4) for k, v in phases.items()}, file=sys.stderr)
    eng.set_profiling(False)
    ktimes = eng.kernel_times(reset=True)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev if world > 1 else "cpu")
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        tot = torch.tensor([n_local], dtype=torch.int64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        n_total = int(tot.item())
    else:
        n_total = n_local
    secs = float(elapsed.item())
    spans_per_s = n_total * args.steps / secs

    # roofline of the dominant kernel: HIP events around its launches on the
    # engine's stream, live in the timed region
    live = kernel_table(ktimes)
    if args.kernel_times == "live":
        per_kernel = live
        dom = max((k for k in per_kernel if per_kernel[k]["alg_bytes"]), key=lambda k: per_kernel[k]["avg_ms"])
    d = live[dom]
    kern_ms = sum(v["ms_per_step"] for v in per_kernel.values())
    # the step's SURVEY.md 8d bytes: K2 57 + K3 19 per span, K4 12 per relation
    # (K1 is not in the step: the batch is generated on the device); the
    # certificate's and the reduce's extra passes are overhead, not 8d work
    pipe_bytes = (57 + 19) * n_local + 12 * A
    overhead = {k: per_kernel[k]["alg_bytes"] for k in ("cert", "check", "reduce", "tail") if k in per_kernel}
    # (the walk: k4_tile9 for chain interning, kmz_info.path bits 5 + 6 --
    # k4_tile8 with KMZ_ABLATE2 bit 22, k4_tile with bit 10; the persistent
    # k4_chain otherwise)
    tile = ("k4_tile" if int(os.environ.get("KMZ_ABLATE2", "0"), 0) & 1024
            else ("k4_tile9" if info.get("path", 0) & 64 else "k4_tile8"))
    kname = {"join": "k_join_window", "stats": "k3_produce" if "reduce" in per_kernel else "k_stats",
             "reduce": "k3_reduce_bal", "walk": tile if info.get("path", 0) & 32 else "k4_chain",
             "cert": "k_cert_split", "check": "k_cert_check", "tail": "k_tail_part", "joinwalk": "k_join_chain"}[dom]
    tr = traffic_of(kname, config, n_local)
    # SURVEY.md 8d's kernels as whole units (every launch that does that
    # unit's work), next to the pieces: K2 = join + certificate + its fix-ups,
    # K3 = produce + reduce (or the one-pass k_stats / k3_small), K4 = the walk
    # + settle + pending ancestries
    units = {}
    unit_defs = [("K2", ("join", "cert", "check", "resolve"), 57 * n_local), ("K3", ("stats", "reduce"), 19 * n_local),
                 ("K4", ("walk", "settle", "pend"), 12 * A)]
    if "joinwalk" in per_kernel:  # (the fused kernel does K2's join and K4's walk: one unit)
        unit_defs = [("K2+K4", ("joinwalk", "cert", "check", "resolve", "settle", "pend"), 57 * n_local + 12 * A),
                     unit_defs[1]]
    for u, parts, alg in unit_defs:
        ms = sum(per_kernel[k]["ms_per_step"] for k in parts if k in per_kernel)
        if ms:
            gbs = alg / (ms * 1e-3) / 1e9
            units[u] = {"ms_per_step": round(ms, 4), "alg_bytes": alg, "gbs": round(gbs, 1),
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "pieces": [k for k in parts if k in per_kernel]}
    h2d = None
    if rank == 0 and not args.no_h2d:
        # the kmz_spans columns (35 B/span) from pinned host memory, as kmz_load
        # copies a host-parsed batch: reported beside the device-resident rate
        nbytes = 35 * n_local
        host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        devb = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        devb.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        devb.copy_(host, non_blocking=True)
        ev1.record()
        torch.cuda.synchronize()
        h2d_ms = ev0.elapsed_time(ev1)
        step_ms = secs / args.steps * 1e3
        h2d = {"bytes": nbytes, "ms": round(h2d_ms, 3), "GB_per_s": round(nbytes / (h2d_ms * 1e-3) / 1e9, 1),
               "pcie_inclusive_spans_per_s": round(n_local / ((h2d_ms + step_ms) * 1e-3), 1),
               "note": "35 B/span kmz_spans columns, pinned host -> HBM, one GPU; not part of `value`"}
        del host, devb
    if rank == 0:
        cpu = None
        if args.cpu_seconds > 0 and world == 1:  # (the CPU baseline is an N = 1 figure)
            cpu_tail = None
            if tail_on:
                def cpu_tail(st, keys, ep):
                    from oracle.tail_np import tail_np

                    first = np.where(ep["has_row"], ep["first"], np.iinfo(np.uint64).max).astype(np.uint64)
                    t = tail_np(keys, tmaps, ep["has_row"], first)
                    t.metrics()
                    used = np.nonzero(st["combined"] > 0)[0]
                    realtime_risk_columns(t, tag_sid[used // n_status], sid_names, st["combined"][used],
                                          st["cv"][used], is_5xx[used % n_status], first=st["first"][used])
            cpu = cpu_baseline(config, args.cpu_seconds, cpu_tail)
        line = {
            "metric": "spans/sec -> endpoint dependency graph + combined stats (node); % HBM roofline",
            "value": round(spans_per_s, 1),
            "unit": "spans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(secs / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int64+f64",
            "data": "synthetic (device-generated, seed 0x4B4D414D495A)",
            "config": {
                "workload": {synth.MESH: "config3: 500-service/20k-endpoint mesh, depth-8 chains, ",
                             synth.BOOKINFO: "config2: Bookinfo-shaped mesh, ",
                             synth.POWER: "config5: power-law fan-out mesh, 50k endpoints, depth-16 chains, "
                                          "hot endpoints, "}[config]
                + f"{n_total} spans ({n_traces} traces)"
                + (f", sharded by h(traceId) mod {world} ({n_local} spans on rank 0)" if world > 1 else "")
                + (" = config 4" if config == synth.MESH and world > 1 and n_total >= 9e8 else "")
                + (", + service tail (instability/coupling/cohesion/risk) per step" if tail_on else ""),
                "spans_per_gpu": n_local,
                "spans_total": n_total,
                "relations_per_gpu": A,
                "edge_keys": info["n_triples"],
                "parallelism": f"traceId-shard x{world}" if world > 1 else "single GPU",
                "sharding_guards": ("in every timed step: id-table/size agreement, unresolved parents, "
                                    "cross-shard repeated span ids (all-to-all of hashed ids, overlapping the run, "
                                    "+ certificate)" if world > 1 else None),
                # (IdGuard.start: kmz_route_ids + the blocking counts all-to-all,
                # host time per step before the run is queued)
                "guard_start_ms_per_step": (round(state["guard_start_s"] / args.steps * 1e3, 4)
                                            if world > 1 else None),
                "service_tail": tail_on,
                "fetched": ("nothing (--no-fetch)" if args.no_fetch else
                            ("groups + endpoints to the host; the edge keys stay in HBM, where "
                             "kmz_tail_run reads them" if tail_on else "groups + edge keys + endpoints")
                            + (" (pipelined: copied to the host while the next step's kernels run)"
                               if args.fetch == "pipelined" else "")),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": d["gbs"],
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(d["gbs"] / HBM_PEAK_GBS, 4),
                # HBM-side bytes per launch from the PMC passes: 2 x FETCH_SIZE +
                # WRITE_SIZE (every read request 128 B: the upper figure), and
                # FETCH_SIZE + WRITE_SIZE (every request 64 B, as a random 16-B
                # probe registers: the lower one); the L2 hit rate of its requests
                "traffic": (tr[0] if tr else None),
                "traffic_lower": (tr[2] if tr else None),
                "l2_hit_rate": (tr[3] if tr else None),
                "traffic_source": (f"profiles/{tr[1]} (build {build_id()})" if tr else
                                   f"no PMC pass of build {build_id()} on this workload committed"),
                "pipeline_bytes": pipe_bytes,
                "pipeline_gbs": round(pipe_bytes / (kern_ms * 1e-3) / 1e9, 1),
                "kernel_ms_per_step": round(kern_ms, 4),
                # the whole step (bench clock) against 8d's bytes: (57 + 19) N + 12 A
                "step_gbs": round(pipe_bytes / (secs / args.steps) / 1e9, 1),
                "step_frac": round(pipe_bytes / (secs / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "overhead_bytes": overhead,
                "kernels": per_kernel,
                "kernels_source": ("a profiled pass of the same --steps steps before the timed region, every kernel "
                                   "timed and on one stream; in the timed region (side-stream overlap on) only "
                                   f"{dom}'s events ({kname}, `achieved`)" if args.kernel_times == "split"
                                   else "every kernel's events inside the timed region (one stream)"),
                "units": units,
            },
            "cpu_baseline": cpu,
            "h2d": h2d,
        }
        print(json.dumps(line))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
