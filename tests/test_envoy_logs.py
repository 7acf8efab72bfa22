"""Traces.combineLogsToRealtimeData with Envoy logs
(Traces.ts:55-106).  The per-span log join (traceId/id, parent fallback for
missing or fallback logs) adds request/response bodies and content types to
the realtime rows; toCombinedRealtimeData keeps the first row's content types
(RealtimeDataList.ts:53-89).  Rows and combined data must equal the oracle's.
application/json bodies (MergeStringBody, JSON.parse, schemas) are covered by
test_envoy_structuring.py."""
import random

import pytest

from conftest import fixture
from oracle import kmz_oracle as O

CTS = ["text/plain", "text/html", None, "application/xml"]  # (None: no contentType property)


def make_logs(traces, rng, ct_choices=CTS):
    logs = []
    for tr in traces:
        entries = []
        for s in tr:
            if rng.random() < 0.6:
                e = {"traceId": s["traceId"], "spanId": s["id"], "isFallback": rng.random() < 0.2,
                     "request": {"body": f"req{rng.randint(0, 9)}"}, "response": {"body": f"res{rng.randint(0, 9)}"}}
                for side in ("request", "response"):
                    ct = rng.choice(ct_choices)
                    if ct is not None:
                        e[side]["contentType"] = ct
                entries.append(e)
        if rng.random() < 0.1:
            entries = []
        logs.append({"traces": entries})
    return logs


def _check(traces, logs, engine):
    from kmamiz_amd import Traces

    ours = Traces(traces, engine=engine).combineLogsToRealtimeData(logs)
    ref = O.Traces(traces).combineLogsToRealtimeData(logs)
    assert ours.toJSON() == O.strip_undef(ref.toJSON())
    return ours, ref


@pytest.mark.parametrize("fx", ["MockTrace", "MockTracePDAS"])
@pytest.mark.parametrize("seed", range(3))
def test_rows_with_logs_equal_oracle_cpu(fx, seed):
    """The realtime rows (host side only: no GPU needed)."""
    traces = fixture(fx)
    if fx != "MockTrace":
        traces = [traces]
    _check(traces, make_logs(traces, random.Random(seed)), None)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_combined_with_logs_equal_oracle(engine, seed):
    from kmamiz_amd import synth
    from test_gpu_parity import _stats_equal

    rng = random.Random(seed)
    batch, off = synth.host_batch(2 if seed % 2 else 3, 0, 150)
    traces = synth.to_traces(2 if seed % 2 else 3, batch, off)
    ours, ref = _check(traces, make_logs(traces, rng), engine)
    got = ours.toCombinedRealtimeData().toJSON()
    exp = O.strip_undef(ref.toCombinedRealtimeData().toJSON())
    _stats_equal(got, exp)
    for a, b in zip(got, exp):
        for k in ("requestContentType", "responseContentType"):
            assert a.get(k) == b.get(k), k


def test_log_without_response_raises_like_the_reference():
    """`log?.response.body` (Traces.ts:94-97) throws when the picked log has
    no response: the oracle and the mirror both raise TypeError."""
    from kmamiz_amd import Traces

    traces = [fixture("MockTracePDAS")]
    s = next(x for x in traces[0] if x["kind"] == "SERVER")
    logs = [{"traces": [{"traceId": s["traceId"], "spanId": s["id"], "isFallback": False,
                         "request": {"body": "x"}}]}]
    with pytest.raises(TypeError):
        O.Traces(traces).combineLogsToRealtimeData(logs)
    with pytest.raises(TypeError):
        Traces(traces).combineLogsToRealtimeData(logs).toJSON()


_NODE_JS = """
const {NativeTraces} = require('./js/kmamiz_native'); const fs = require('fs');
const traces = JSON.parse(fs.readFileSync(process.argv[1])), logs = JSON.parse(fs.readFileSync(process.argv[2]));
const l = new NativeTraces(traces).combineLogsToRealtimeData(logs);
const out = {rows: l.toJSON()};
if (process.argv[3] === 'gpu') out.combined = l.toCombinedRealtimeData();
process.stdout.write(JSON.stringify(out));
"""


def _node(tmp_path, traces, logs, gpu):
    import json
    import os
    import shutil
    import subprocess

    from conftest import ROOT

    node = shutil.which("node")
    if not node or not os.path.exists(os.path.join(ROOT, "js", "kmz.node")):
        pytest.skip("node or js/kmz.node not available")
    p, q = tmp_path / "t.json", tmp_path / "l.json"
    p.write_text(json.dumps(traces))
    q.write_text(json.dumps(logs))
    r = subprocess.run([node, "-e", _NODE_JS, str(p), str(q), "gpu" if gpu else "cpu"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("seed", range(2))
def test_node_rows_with_logs_equal_oracle_cpu(seed, tmp_path):
    traces = fixture("MockTrace")
    logs = make_logs(traces, random.Random(seed))
    out = _node(tmp_path, traces, logs, False)
    assert out["rows"] == O.strip_undef(O.Traces(traces).combineLogsToRealtimeData(logs).toJSON())


@pytest.mark.gpu
def test_node_combined_with_logs_equal_oracle(tmp_path):
    from kmamiz_amd import synth

    batch, off = synth.host_batch(3, 0, 100)
    traces = synth.to_traces(3, batch, off)
    logs = make_logs(traces, random.Random(5))
    out = _node(tmp_path, traces, logs, True)
    ref = O.Traces(traces).combineLogsToRealtimeData(logs)
    assert out["rows"] == O.strip_undef(ref.toJSON())
    exp = O.strip_undef(ref.toCombinedRealtimeData().toJSON())
    def key(rows):
        return [(x["uniqueEndpointName"], x["status"], x["combined"], x.get("requestContentType"),
                 x.get("responseContentType")) for x in rows]

    assert key(out["combined"]) == key(exp)


@pytest.mark.gpu
def test_node_combined_with_json_bodies_equal_oracle(tmp_path):
    """The Node mirror folds application/json bodies (MergeStringBody, JSON.parse,
    ObjectToInterfaceString) like the oracle; bodies whose schema needs
    json-to-ts's nested naming or quoted members are left out (not restated)."""
    from kmamiz_amd import synth
    from test_envoy_structuring import JSON_BODIES, json_logs

    batch, off = synth.host_batch(2, 0, 120)
    traces = synth.to_traces(2, batch, off)
    # (a string body spread into an object gives "0", "1", ... members, whose
    # interface json-to-ts quotes: not restated either)
    logs = json_logs(traces, random.Random(9), [b for b in JSON_BODIES if "deep" not in b and b != '"str"'])
    out = _node(tmp_path, traces, logs, True)
    ref = O.Traces(traces).combineLogsToRealtimeData(logs)
    assert out["rows"] == O.strip_undef(ref.toJSON())
    exp = O.strip_undef(ref.toCombinedRealtimeData().toJSON())
    assert len(out["combined"]) == len(exp)
    for a, b in zip(out["combined"], exp):
        for k in ("uniqueEndpointName", "status", "combined", "requestContentType", "responseContentType",
                  "requestBody", "requestSchema", "responseBody", "responseSchema"):
            assert a.get(k) == b.get(k), k
