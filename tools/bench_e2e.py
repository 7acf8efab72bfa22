"""End-to-end timing from Zipkin JSON bytes to the reference's result objects
(SURVEY.md 8d timing scope: "the MockData config is also timed end-to-end from
JSON"; "the H2D of host-parsed spans is reported separately").

Stages, each timed on its own and as one chain (median of `reps`):
  parse     kmz_parse_zipkin + the once-per-shape identity rules (ingest_json)
  load      kmz_load: columns host -> HBM (PCIe)
  run       kmz_run(STATS_TAG | DEPS) on the device
  results   kmz_fetch + the objects: combined rows (toCombinedRealtimeData),
            and the reduced dependency graph (MockData: the exact per-row
            toEndpointDependencies() JSON and combineWith([]).trim())

and the same chain with K1 on the GPU (kmz_json_parse, kmz_json.hip): the JSON
bytes go to HBM (from pageable memory, and from a pinned buffer as an HTTP
client would receive into), are parsed there, the distinct shapes come back
for the identity rules, and the batch is loaded without a column H2D.

usage: python tools/bench_e2e.py [config2_traces]  -> one JSON line
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kmamiz_amd import EndpointDependencies, Engine, Traces, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402
from kmamiz_amd.ingest import ingest_json  # noqa: E402


def med(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), out


def mockdata(eng, reps=20):
    fx = os.path.join(ROOT, "tests", "fixtures")
    book = json.load(open(os.path.join(fx, "MockTrace.json")))
    pdas = [json.load(open(os.path.join(fx, "MockTracePDAS.json")))]
    out = {}
    for name, traces in (("MockTrace(Bookinfo)", book), ("MockTracePDAS", pdas)):
        data = json.dumps(traces).encode()
        n = sum(len(t) for t in traces)

        def chain():
            t = Traces.from_json(data, engine=eng)
            comb = t.combineLogsToRealtimeData([]).toCombinedRealtimeData().toJSON()
            deps = t.toEndpointDependencies()
            rows = deps.toJSON()
            red = EndpointDependencies([]).combineWith(deps).trim().toJSON()
            return len(comb), len(rows), len(red)

        chain()  # warm (identity cache, pinned buffers)
        t, res = med(chain, reps)
        out[name] = {"spans": n, "json_bytes": len(data), "ms": round(t * 1e3, 3), "spans_per_s": round(n / t, 1),
                     "groups/rows/reduced_rows": res}
    return out


def config2(eng, ntr, reps=5):
    b, off = synth.host_batch(synth.BOOKINFO, 0, ntr)
    data = json.dumps(synth.to_traces(synth.BOOKINFO, b, off)).encode()
    n = len(b)
    tp, (batch, d) = med(lambda: ingest_json(data), reps)
    table = d.shape_table()
    tl, _ = med(lambda: eng.load(batch, table), reps)

    def run():
        eng.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        eng.sync()

    tr, _ = med(run, reps)

    def results():
        from kmamiz_amd.classes import _combine_native

        g, k, e = eng.fetch()
        comb = _combine_native(g, 0, batch, d, "tag", None)
        return len(comb), len(k)

    tf, res = med(results, reps)

    def chain():
        bt, dd = ingest_json(data)
        eng.load(bt, dd.shape_table())
        eng.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        from kmamiz_amd.classes import _combine_native

        g, k, e = eng.fetch()
        return len(_combine_native(g, 0, bt, dd, "tag", None)), len(k)

    tc, _ = med(chain, reps)
    return {"config2(Bookinfo-shaped)": {
        "spans": n, "json_bytes": len(data), "json_bytes_per_span": round(len(data) / n, 1),
        "parse_ms": round(tp * 1e3, 2), "h2d_load_ms": round(tl * 1e3, 2), "run_ms": round(tr * 1e3, 3),
        "results_ms": round(tf * 1e3, 3), "chain_ms": round(tc * 1e3, 2),
        "parse_spans_per_s": round(n / tp), "h2d_GB_per_s": round(35 * n / tl / 1e9, 1),
        "end_to_end_spans_per_s": round(n / tc), "device_resident_run_spans_per_s": round(n / tr),
        "groups/edge_keys": res}}


def device_json(eng, config, ntr, reps=5):
    """K1 on the GPU through DeviceIngest (a worker's persistent dictionary):
    the first window runs the identity rules for every shape ("cold"), later
    windows only look the raw shapes up (kmz_json_known, "warm")."""
    import ctypes as C

    from kmamiz_amd.ingest import DeviceIngest

    b, off = synth.host_batch(config, 0, ntr)
    data = json.dumps(synth.to_traces(config, b, off)).encode()
    n = len(b)
    pin = L.lib().kmz_host_alloc(len(data))
    C.memmove(pin, data, len(data))
    di = DeviceIngest(eng)
    t0 = time.perf_counter()
    assert di.ingest(data, ptr=pin) == n
    cold = time.perf_counter() - t0
    eng.set_profiling(True)

    def parse(pinned):
        r = eng.json_parse(ptr=pin, length=len(data)) if pinned else eng.json_parse(data)
        assert r is not None and r[0] == n
        return r

    tp, _ = med(lambda: parse(False), reps)
    eng.kernel_times(reset=True)
    tq, r = med(lambda: parse(True), reps)
    kt = eng.kernel_times(reset=True)
    json_ms = kt["json"][0] / reps

    def run():
        eng.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        eng.sync()

    di.ingest(data, ptr=pin)  # (a bare json_parse leaves nothing loaded)
    tr, _ = med(run, reps)

    def chain():
        di.ingest(data, ptr=pin)
        run()
        g, k, e = eng.fetch()
        return len(k)

    tc, _ = med(chain, reps)
    eng.set_profiling(False)
    L.lib().kmz_host_free(C.c_void_p(pin))
    return {f"config{config} device JSON": {
        "spans": n, "json_bytes": len(data), "distinct_shapes": r[1], "parse_pageable_ms": round(tp * 1e3, 2),
        "parse_pinned_ms": round(tq * 1e3, 2), "json_kernels_ms": round(json_ms, 3),
        "kernel_GB_per_s": round(len(data) / (json_ms * 1e-3) / 1e9, 1) if json_ms else None,
        "first_window_ingest_ms": round(cold * 1e3, 2), "run_ms": round(tr * 1e3, 3),
        "chain_ms": round(tc * 1e3, 2), "end_to_end_spans_per_s": round(n / tc),
        "parse_pinned_spans_per_s": round(n / tq)}}


def main():
    ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 136000
    eng = Engine(0)
    out = {"tool": "tools/bench_e2e.py", **mockdata(eng), **config2(eng, ntr), **device_json(eng, 2, ntr),
           **device_json(eng, 3, ntr // 4)}
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
