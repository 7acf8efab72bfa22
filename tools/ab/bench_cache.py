"""Timing of the cache-layer step at scale: one 5 s tick
of a realtime worker whose window is config 3's mesh.

  device   kmz_run(STATS_TAG | DEPS | DEP_ORDER) on the resident window; the
           entry-order pass alone (kernel "order", HIP events)
  fetch    kmz_fetch + kmz_get_dep_entries (D2H of the reduced graph's records)
  columns  ReducedDependencies.from_window + CombinedColumns.from_groups
  merge    cached.combineWith(window) for both caches (the cache already holds
           the previous, half-overlapping window)
  json     toJSON() of the merged dependency cache (what Mongo would get)

usage: python tools/bench_cache.py [traces_per_window] -> one JSON line
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402
from kmamiz_amd.cache import CombinedColumns, ReducedDependencies  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 366000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = synth.MESH
    d = synth.dictionary(cfg)
    dep_f = d.shape_ident["dep"]
    tag_f = d.shape_ident["tag"]
    n_status = len(d.statuses)
    eng = Engine(0)
    eng.set_profiling(True)
    flags = L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_DEP_ORDER

    def window(t0, reg=None, like=None):
        n = eng.load_synthetic(cfg, synth.SEED, t0, t0 + T)
        t = time.perf_counter()
        eng.run(flags)
        eng.sync()
        t_run = time.perf_counter() - t
        t = time.perf_counter()
        g, _, ep = eng.fetch(groups=True, deps=True)
        ents, rts, rsh = eng.dep_entries()
        t_fetch = time.perf_counter() - t
        t = time.perf_counter()
        rd = ReducedDependencies.from_window(ents, rts, rsh, ep, d.ep_names["dep"], lambda s: dep_f[s].fields, reg)
        cc = CombinedColumns.from_groups(g, n_status, lambda e: tag_f[e].fields, d.statuses, like)
        t_cols = time.perf_counter() - t
        return n, rd, cc, len(ents), t_run, t_fetch, t_cols

    n0, cache_d, cache_c, _, _, _, _ = window(0)
    eng.kernel_times(reset=True)
    res = []
    for _ in range(reps):
        n, rd, cc, ne, t_run, t_fetch, t_cols = window(T // 2, cache_d.reg, cache_c)
        t = time.perf_counter()
        md = cache_d.combineWith(rd)
        mc = cache_c.combineWith(cc.filter_service())
        t_merge = time.perf_counter() - t
        res.append((t_run, t_fetch, t_cols, t_merge))
    kt = eng.kernel_times()
    t = time.perf_counter()
    js = md.toJSON()
    t_json = time.perf_counter() - t
    med = [statistics.median(x[i] for x in res) for i in range(4)]
    order_ms = kt["order"][0] / max(1, kt["order"][1])
    out = {
        "tool": "tools/bench_cache.py", "workload": f"config3 mesh, {n} spans per window ({T} traces), "
        "cache = previous half-overlapping window",
        "spans": n, "entries": ne, "cache_rows": len(md), "cache_entries": md.n_entries(),
        "combined_groups": len(mc),
        "device_run_ms": round(med[0] * 1e3, 3), "order_kernel_ms": round(order_ms, 3),
        "fetch_ms": round(med[1] * 1e3, 3), "columns_ms": round(med[2] * 1e3, 3),
        "merge_ms": round(med[3] * 1e3, 3), "json_ms": round(t_json * 1e3, 1), "json_rows": len(js),
        "kernels_ms_per_run": {k: round(v[0] / max(1, v[1]), 4) for k, v in kt.items() if v[1]},
    }
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
