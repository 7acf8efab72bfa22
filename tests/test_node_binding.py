"""The Node side of the boundary (js/): N-API addon + JS ingest.

CPU: the addon loads (context-aware N-API), its JS ExplodeUrl / ToEndpointInfo
/ ingest agree with the oracle.  GPU: the whole path through Node equals the
oracle (order-exact dependencies, 1e-9 latency stats)."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import FIX, ROOT, fixture
from oracle import kmz_oracle as O

NODE = shutil.which("node")
ADDON = os.path.join(ROOT, "js", "kmz.node")
pytestmark = pytest.mark.skipif(not NODE or not os.path.exists(ADDON), reason="node or js/kmz.node not available")


def node(script, *args):
    r = subprocess.run([NODE, "-e", script, *args], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_addon_exports():
    out = node("const k=require('./js/kmz.node');process.stdout.write(JSON.stringify(Object.keys(k)))")
    assert {"create", "load", "run", "groups", "endpoints", "triples", "spanLinks", "info"} <= set(out)


def test_js_explode_url_and_endpoint_info():
    urls = ["http://example.com:8080/test/test", "https://192.168.1.1/test#123",
            "service.test.svc.cluster.local:80/test/endpoint", "e.svc.cluster.local/q", "dsvc.ns3.svc:81/z"]
    got = node(
        "const {explodeUrl}=require('./js/kmamiz_native');"
        "const u=JSON.parse(process.argv[1]);"
        "process.stdout.write(JSON.stringify(u.map(x=>[explodeUrl(x),explodeUrl(x,true)])))",
        json.dumps(urls),
    )
    for u, (a, b) in zip(urls, got):
        assert a == [None if v is O.UNDEF else v for v in O.explode_url(u)]
        assert b == [None if v is O.UNDEF else v for v in O.explode_url(u, True)]
    traces = fixture("MockTrace")
    info = node(
        "const {NativeTraces}=require('./js/kmamiz_native');const fs=require('fs');"
        "const t=JSON.parse(fs.readFileSync(process.argv[1]));"
        "process.stdout.write(JSON.stringify([].concat(...t).map(s=>NativeTraces.ToEndpointInfo(s))))",
        os.path.join(FIX, "MockTrace.json"),
    )
    assert info == [O.strip_undef(O.Traces.ToEndpointInfo(s)) for tr in traces for s in tr]


_SAME_BATCH_JS = """
const {ingest, ingestJSON} = require('./js/kmamiz_native'); const fs = require('fs');
const raw = fs.readFileSync(process.argv[1]);
const a = ingestJSON(raw, Number(process.argv[2])), b = ingest(JSON.parse(raw.toString('utf8')));
const out = {};
for (const k of ['span_id', 'parent_id', 'kind', 'shape', 'status', 'duration', 'timestamp'])
  out[k] = a.spans[k].length === b.spans[k].length && a.spans[k].every((x, i) => x === b.spans[k][i]);
out.table = JSON.stringify(Object.keys(b.shapesTable).map(k => Array.from(a.shapesTable[k].length !== undefined
  ? a.shapesTable[k] : [a.shapesTable[k]]))) === JSON.stringify(Object.keys(b.shapesTable).map(k =>
  Array.from(b.shapesTable[k].length !== undefined ? b.shapesTable[k] : [b.shapesTable[k]])));
out.statuses = JSON.stringify(a.statuses) === JSON.stringify(b.statuses);
out.ident = JSON.stringify(a.ident) === JSON.stringify(b.ident);
out.n = a.spans.span_id.length;
process.stdout.write(JSON.stringify(out));
"""


@pytest.mark.parametrize("src", ["MockTracePDAS", "MockTrace", "MockData2_traces", "mesh"])
def test_js_ingest_json_equals_object_ingest(src, tmp_path):
    """NativeTraces.fromJSON's batch (native parser through parseZipkin) is
    the batch the object ingest builds: columns, identity tables, statuses."""
    if src == "mesh":
        from kmamiz_amd import synth

        batch, off = synth.host_batch(3, 0, 3000)
        traces = synth.to_traces(3, batch, off)
    else:
        traces = fixture(src)
        if src != "MockTrace":
            traces = [traces]
    p = tmp_path / "t.json"
    p.write_text(json.dumps(traces))
    out = node(_SAME_BATCH_JS, str(p), "4")
    assert out.pop("n") == sum(len(t) for t in traces)
    assert all(out.values()), out


@pytest.mark.gpu
@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
@pytest.mark.parametrize("mode", ["objects", "json"])
def test_node_path_vs_oracle(fx, mode, tmp_path):
    traces = fixture(fx)
    if fx != "MockTrace":
        traces = [traces]
    p = tmp_path / "t.json"
    p.write_text(json.dumps(traces))
    r = subprocess.run([NODE, "js/run_fixture.js", str(p), mode], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    ref = O.Traces(traces)
    assert out["deps"] == O.strip_undef(ref.toEndpointDependencies().toJSON())
    assert out["rl"] == O.strip_undef(ref.toRealTimeData().toJSON())
    reps = [{"uniqueServiceName": "details\tbook\tv1", "replicas": 3}]
    for key, exp in (("crl_rt", ref.toRealTimeData(reps)), ("crl_tag", ref.combineLogsToRealtimeData([], reps))):
        e = O.strip_undef(exp.toCombinedRealtimeData().toJSON())
        g = out[key]
        assert [(x["uniqueEndpointName"], x["status"], x["combined"], x["latestTimestamp"], x.get("avgReplica"))
                for x in g] == [(x["uniqueEndpointName"], x["status"], x["combined"], x["latestTimestamp"],
                                 x.get("avgReplica")) for x in e]
        for a, b in zip(g, e):
            assert a["latency"]["mean"] == pytest.approx(b["latency"]["mean"], rel=1e-9)
            assert a["latency"]["cv"] == pytest.approx(b["latency"]["cv"], rel=1e-9, abs=1e-13)


_TAIL_JS = """
const {NativeTraces} = require('./js/kmamiz_native'); const fs = require('fs');
const t = new NativeTraces(JSON.parse(fs.readFileSync(process.argv[1])));
const lm = process.argv[2] ? JSON.parse(fs.readFileSync(process.argv[2])) : undefined;
process.stdout.write(JSON.stringify(t.serviceTail(lm)));
"""


@pytest.mark.gpu
@pytest.mark.parametrize("src", ["MockTrace", "MockTracePDAS", "mesh", "power", "mesh-labels"])
def test_node_service_tail_vs_oracle(src, tmp_path):
    """NativeTraces.serviceTail (addon serviceTail -> kmz_tail_run) against
    the oracle's tail of the reduced graph (EndpointDependencies.ts:565-657,
    RiskAnalyzer.ts:124-169)."""
    lm = None
    if src in ("mesh", "power", "mesh-labels"):
        from kmamiz_amd import synth

        cfg = 5 if src == "power" else 3
        batch, off = synth.host_batch(cfg, 0, 200)
        traces = synth.to_traces(cfg, batch, off)
    else:
        traces = fixture(src)
        if src != "MockTrace":
            traces = [traces]
    ref = O.Traces(traces)
    red = O.strip_undef(O.EndpointDependencies([]).combineWith(ref.toEndpointDependencies()).trim().toJSON())
    od = O.EndpointDependencies(red)
    if src == "mesh-labels":
        lm = {r["endpoint"]["uniqueEndpointName"]: "/L%d" % (i % 3) for i, r in enumerate(red)}
        od = O.EndpointDependencies(od.label(lm))
    p = tmp_path / "t.json"
    p.write_text(json.dumps(traces))
    q = tmp_path / "labels.json"
    q.write_text(json.dumps(lm))
    got = node(_TAIL_JS, str(p), str(q) if lm else "")
    inst, coup, coh = od.toServiceInstability(), od.toServiceCoupling(), od.toServiceEndpointCohesion()
    rf = {x["uniqueServiceName"]: x["factor"] for x in O.RiskAnalyzer.RelyingFactor(od.toServiceDependencies())}
    assert [g["uniqueServiceName"] for g in got] == [x["uniqueServiceName"] for x in inst]
    for g, i, c, h in zip(got, inst, coup, coh):
        assert (g["name"], g["dependingBy"], g["dependingOn"]) == (i["name"], i["dependingBy"], i["dependingOn"])
        assert g["instability"] == pytest.approx(i["instability"], rel=1e-12)
        assert (g["ais"], g["ads"], g["acs"]) == (c["ais"], c["ads"], c["acs"])
        assert (g["totalEndpoints"], g["consumers"]) == (h["totalEndpoints"], len(h["consumers"]))
        assert g["endpointUsageCohesion"] == pytest.approx(h["endpointUsageCohesion"], rel=1e-9)
        assert g["relyingFactor"] == pytest.approx(rf[g["uniqueServiceName"]], rel=1e-9)


def test_addon_loads_in_worker_threads():
    """The realtime step runs in a worker_threads Worker in the reference
    (RealtimeWorkerImpl.ts:29-84, ServiceOperator.ts:57-64): the addon must be
    context-aware.  Four Workers load kmz.node (through js/realtime_worker.js)
    at once."""
    r = subprocess.run([NODE, "js/worker_seam_run.js", os.path.join(FIX, "MockTrace.json"), "4", "load"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout) == {"loaded": 4}


@pytest.mark.gpu
@pytest.mark.parametrize("src", ["MockTrace", "mesh"])
def test_worker_threads_run_the_path_concurrently(src, tmp_path):
    """Two (and four) Workers, each with its own engine context on the GPU,
    run the worker step on the same batch at the same time (half from
    objects, half from the raw JSON bytes); every answer equals the oracle."""
    if src == "mesh":
        from kmamiz_amd import synth

        batch, off = synth.host_batch(3, 0, 300)
        traces = synth.to_traces(3, batch, off)
    else:
        traces = fixture(src)
    p = tmp_path / "t.json"
    p.write_text(json.dumps(traces))
    ref = O.Traces(traces)
    exp_deps = O.strip_undef(ref.toEndpointDependencies().toJSON())
    exp_rl = O.strip_undef(ref.combineLogsToRealtimeData([]).toCombinedRealtimeData().toJSON())
    for nw in (2, 4):
        r = subprocess.run([NODE, "js/worker_seam_run.js", str(p), str(nw), "gpu"], cwd=ROOT, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        res = json.loads(r.stdout)["results"]
        assert len(res) == nw
        for x in res:
            assert "error" not in x, x.get("error")
            assert x["dependencies"] == exp_deps
            got = x["rlDataList"]
            assert [(g["uniqueEndpointName"], g["status"], g["combined"], g["latestTimestamp"]) for g in got] == \
                [(e["uniqueEndpointName"], e["status"], e["combined"], e["latestTimestamp"]) for e in exp_rl]
            for a, b in zip(got, exp_rl):
                assert a["latency"]["mean"] == pytest.approx(b["latency"]["mean"], rel=1e-9)
                assert a["latency"]["cv"] == pytest.approx(b["latency"]["cv"], rel=1e-9, abs=1e-13)
