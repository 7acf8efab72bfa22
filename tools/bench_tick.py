"""Production-tick latency: the reference's realtime worker
takes up to 2 500 traces per 5-s tick (RealtimeWorkerImpl.ts:31-35).  Per tick
on one GPU: kmz_load of the host columns (H2D) + kmz_run (stats + dependency
graph) + kmz_fetch of the results, timed over many ticks, with the run's
join + chain walk fused (default) or as two kernels, hipGraph replay on (the
default since round 6) or off (KMZ_ABLATE2 bit 23).  Prints one JSON object;
kernel traces of a tick come from rocprofv3 over tools/tick_trace.py.

    python tools/bench_tick.py [--traces 2500] [--ticks 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--traces", type=int, default=2500)
    ap.add_argument("--ticks", type=int, default=200)
    args = ap.parse_args()
    import numpy as np

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    out = {"metric": "per-tick latency, 2 500 traces per call (RealtimeWorkerImpl.ts:31-35)", "unit": "us",
           "ticks": args.ticks, "configs": {}}
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    for name, cfg in (("bookinfo", synth.BOOKINFO), ("mesh", synth.MESH), ("power", synth.POWER)):
        batch, _ = synth.host_batch(cfg, 0, args.traces)
        table = synth.shape_table(cfg)
        res = {"spans": len(batch)}
        # default: hipGraph replay (since round 6), the join + chain walk fused
        # (kmz_fuse.hip) where the batch allows; separate: k_join_window + the
        # tile walk (KMZ_ABLATE2 bit 4); direct: launches one at a time
        # (KMZ_ABLATE2 bit 23, = KMZ_HIPGRAPH=0); serial: no side stream (bit 25)
        # used: default, fetching only the used groups (kmz_fetch_used, round 6)
        for mode, knob, knob2 in (("default", 0, 0), ("used", 0, 0), ("separate", 0, 16), ("direct", 0, 1 << 23),
                                  ("serial", 1 << 25, 0)):
            os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"] = str(knob), str(knob2)
            e = Engine(0)
            del os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"]
            fetch = e.fetch_used if mode == "used" else e.fetch
            for _ in range(10):  # warm: buffers, the graph capture
                e.load(batch, table)
                e.run(flags)
                fetch()
            t_run, t_tick, t_fetch = [], [], []
            for _ in range(args.ticks):
                t0 = time.perf_counter()
                e.load(batch, table)
                t1 = time.perf_counter()
                e.run(flags)
                tf = time.perf_counter()
                fetch()
                t2 = time.perf_counter()
                t_run.append(t2 - t1)
                t_tick.append(t2 - t0)
                t_fetch.append(t2 - tf)
            res[mode] = {"run_fetch_us_median": round(float(np.median(t_run)) * 1e6, 1),
                         "fetch_us_median": round(float(np.median(t_fetch)) * 1e6, 1),
                         "groups": int(e.info()["n_groups"]), "groups_used": int(len(e.fetch_used()[0])),
                         "tick_us_median": round(float(np.median(t_tick)) * 1e6, 1),
                         "tick_us_p99": round(float(np.percentile(t_tick, 99)) * 1e6, 1),
                         "graph_replays": e.graph_stats()[0]}
            e.close()
        out["configs"][name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
