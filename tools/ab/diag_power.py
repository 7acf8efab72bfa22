"""Where config 5's step time goes (bench.py --config power): device run,
result fetch, device tail, host tail finish (metrics, realtime risk).
usage: python tools/diag_power.py [traces] -> one JSON line of median ms"""
import ctypes as C
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
from kmamiz_amd.tail import (maps_for_synth, realtime_risk_arrays, realtime_risk_columns, realtime_risk_from_sums,
                             run_tail, service_sums_grid)  # noqa: E402


def main():
    cfg = synth.POWER
    ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    eng = Engine(0)
    if not ntr:  # 1e8 spans, as bench.py sizes it
        lo, hi = 1, 1 << 24
        while lo < hi:
            mid = (lo + hi) // 2
            if synth.count_spans(cfg, 0, mid) < 100_000_000:
                lo = mid + 1
            else:
                hi = mid
        ntr = lo
    n = eng.load_synthetic(cfg, synth.SEED, 0, ntr)
    print("loaded", n, file=sys.stderr, flush=True)
    from kmamiz_amd.ingest import SHAPE_TAGS, UNDEFINED, tag_identity

    tmaps = maps_for_synth(cfg)
    n_shapes, n_status, _ = synth.describe(cfg)
    sid_of, sid_names = {}, []
    tag_sid = np.zeros(n_shapes, dtype=np.int64)
    for sh in range(n_shapes):
        name, tags = synth.shape_tags(cfg, sh)
        usn = tag_identity((name,) + tuple(tags.get(t, UNDEFINED) for t in SHAPE_TAGS))["uniqueServiceName"]
        if usn not in sid_of:
            sid_of[usn] = len(sid_names)
            sid_names.append(usn)
        tag_sid[sh] = sid_of[usn]
    is_5xx_st = np.array([str(x).startswith("5") for x in synth.STATUSES[:n_status]], dtype=bool)
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    marks = {k: [] for k in ("run", "fetch_all", "fetch_no_keys", "tail_device", "metrics", "risk", "risk_dicts", "risk_grid")}
    dbg_fn = L.lib().kmz__debug_k4
    dbg_fn.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    k4 = []  # scap, staged sum, max per run, bucket sum, max, bcap, slices, coarse bins, flags, path
    for rep in range(6):
        t = time.perf_counter()
        eng.run(flags)
        eng.sync()
        marks["run"].append(time.perf_counter() - t)
        dbg = (C.c_ulonglong * 8)()
        L.check(eng.ctx, dbg_fn(eng.ctx, dbg))
        k4.append([int(x) for x in dbg] + [eng.info()["flags"], eng.info()["path"]])
        print("rep", rep, k4[-1], round(marks["run"][-1] * 1e3, 3), file=sys.stderr, flush=True)
        t = time.perf_counter()
        g, k, e = eng.fetch()
        nk = len(k)
        marks["fetch_all"].append(time.perf_counter() - t)
        t = time.perf_counter()
        g, _, e = eng.fetch(keys=False)
        marks["fetch_no_keys"].append(time.perf_counter() - t)
        t = time.perf_counter()
        tl = run_tail(eng, tmaps, e)
        marks["tail_device"].append(time.perf_counter() - t)
        t = time.perf_counter()
        tl.metrics()
        marks["metrics"].append(time.perf_counter() - t)
        t = time.perf_counter()
        used = np.nonzero(g["combined"] > 0)[0]
        realtime_risk_columns(tl, tag_sid[used // n_status], sid_names, g["combined"][used], g["cv"][used],
                              is_5xx_st[used % n_status], first=g["first"][used])
        marks["risk"].append(time.perf_counter() - t)
        t = time.perf_counter()
        realtime_risk_arrays(tl, tag_sid[used // n_status], sid_names, g["combined"][used], g["cv"][used],
                             is_5xx_st[used % n_status], first=g["first"][used])
        marks["risk_dicts"].append(time.perf_counter() - t)
        t = time.perf_counter()
        realtime_risk_from_sums(tl, sid_names, *service_sums_grid(g["combined"], g["cv"], g["first"], is_5xx_st,
                                                                   tag_sid[: len(g) // n_status], len(sid_names)))
        marks["risk_grid"].append(time.perf_counter() - t)
    out = {k: round(statistics.median(v[1:]) * 1e3, 3) for k, v in marks.items()}
    out["spans"] = n
    out["edge_keys"] = int(nk)
    out["k4"] = k4
    out["tail_details"], out["tail_pairs"] = int(tl.n_details), int(tl.n_pairs)
    out["info"] = {k: v for k, v in eng.info().items() if isinstance(v, int)}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
