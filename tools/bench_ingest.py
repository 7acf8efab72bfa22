"""Host ingest throughput: Zipkin Trace[][] JSON bytes ->
kmz_spans columns, native parser (kmz_parse_zipkin) vs the general path
(json.loads + ingest_traces), on the synthetic mesh rendered as JSON.

usage: python tools/bench_ingest.py [traces] [config]   -> one JSON line"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmamiz_amd import synth  # noqa: E402
from kmamiz_amd.ingest import ingest_json, ingest_traces  # noqa: E402

ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
config = int(sys.argv[2]) if len(sys.argv) > 2 else synth.MESH
batch, off = synth.host_batch(config, 0, ntr)
data = json.dumps(synth.to_traces(config, batch, off)).encode()
n = len(batch)


def best(fn, reps=3):
    t = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t = min(t, time.perf_counter() - t0)
    return t


cores = min(16, os.cpu_count())


def parse_only(threads):
    import ctypes as C

    from kmamiz_amd import _lib as L

    out = C.POINTER(L.ZipkinBatch)()
    assert L.lib().kmz_parse_zipkin(data, len(data), threads, C.byref(out)) == 0
    L.lib().kmz_zipkin_free(out)


tp1 = best(lambda: parse_only(1))
tpn = best(lambda: parse_only(0))
t1 = best(lambda: ingest_json(data, threads=1))
tn = best(lambda: ingest_json(data, threads=0))
tg = best(lambda: ingest_traces(json.loads(data)), reps=1)
node = {}
if shutil.which("node") and os.path.exists(os.path.join(ROOT, "js", "kmz.node")):
    with tempfile.NamedTemporaryFile(suffix=".json") as f:
        f.write(data)
        f.flush()
        r = subprocess.run(["node", os.path.join(ROOT, "tools", "bench_ingest_node.js"), f.name],
                           capture_output=True, text=True, timeout=600)
        node = json.loads(r.stdout) if r.returncode == 0 else {"node_error": r.stderr[-300:]}
print(json.dumps({
    "workload": f"config{config} synthetic, {ntr} traces, {n} spans, {len(data) / n:.0f} B/span of JSON",
    "native_1thread_spans_per_s": round(n / t1), "native_all_threads_spans_per_s": round(n / tn),
    "threads": cores, "general_path_spans_per_s": round(n / tg),
    "native_GB_per_s_1thread": round(len(data) / t1 / 1e9, 3),
    "parse_only_GB_per_s_1thread": round(len(data) / tp1 / 1e9, 3),
    "parse_only_GB_per_s_all_threads": round(len(data) / tpn / 1e9, 3), "speedup_1thread": round(tg / t1, 1),
    **node,
}))
