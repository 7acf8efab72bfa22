"""The cache layer's merges in Node (js/kmz_cache.js)
against the Python oracle's object merges.

CPU: the columnar EndpointDependencies merge (fromJSON + combineWith) and the
combined-data merge (CombinedColumns, pooled CV with the decimal shift) over
ticks, from the oracle's window objects.  GPU: the same ticks with each window
taken straight from the engine through the addon (depEntries: the reduced
graph in entry order; groups), and the worker seam (realtime_worker.step with
existingDep), i.e. RealtimeWorkerImpl.ts:67-70, CEndpointDependencies.ts:46-48
and CCombinedRealtimeData.ts:47-53 without a per-row object."""
import copy
import json
import os
import shutil
import subprocess

import pytest

from conftest import ROOT
from oracle import kmz_oracle as O
from shard_util import mixed_traces
from test_cache import _messy, _ticks

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(not NODE, reason="node not available")
REL = 1e-9


def _node(script, inp, tmp_path):
    f = tmp_path / "in.json"
    f.write_text(json.dumps(inp))
    r = subprocess.run([NODE, "--max-old-space-size=8192", "-e", script, str(f)], cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def _oracle_ticks(windows):
    """Per tick: the dependency cache (trimmed) and the combined cache, as the
    reference's worker + caches leave them."""
    odeps = ocomb = None
    out = []
    for w in windows:
        newdep = O.Traces(copy.deepcopy(w)).toEndpointDependencies()
        odeps = (O.EndpointDependencies(copy.deepcopy(odeps)).combineWith(newdep) if odeps is not None
                 else newdep).trim().toJSON()
        odeps = O.strip_undef(odeps)
        upd = O.strip_undef(O.Traces(copy.deepcopy(w)).combineLogsToRealtimeData([], None)
                            .toCombinedRealtimeData().toJSON())
        f = [r for r in upd if O.truthy(O.get(r, "service"))]
        ocomb = O.strip_undef((O.CombinedRealtimeDataList(copy.deepcopy(ocomb)).combineWith(
            O.CombinedRealtimeDataList(f)) if ocomb is not None else O.CombinedRealtimeDataList(f)).toJSON())
        out.append((odeps, ocomb, upd, O.strip_undef(newdep.toJSON())))
    return out


def _same_combined(got, exp, exact):
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        if exact:
            assert a == b
            continue
        for k in set(a) | set(b):
            if k != "latency":
                assert a.get(k) == b.get(k), k
        for k in ("mean", "cv"):  # window stats: engine vs sequential Welford (north_star 1e-9)
            assert a["latency"][k] == pytest.approx(b["latency"][k], rel=REL, abs=1e-13)


_CPU_JS = """
const fs = require('fs');
const C = require('./js/kmz_cache');
const N = require('./js/kmamiz_native');
const inp = JSON.parse(fs.readFileSync(process.argv[1]));
let state = null;
const comb = N.newCombinedCache();
const out = [];
for (const t of inp.ticks) {
  state = state === null ? C.trimRows(t.newdep)
                         : C.ReducedDependencies.fromJSON(state, false)
                             .combineWith(C.ReducedDependencies.fromJSON(t.newdep, true)).trim().toJSON();
  comb.setData(C.CombinedColumns.fromJSON(t.update, comb.getData()));
  out.push([state, comb.getData().toJSON()]);
}
process.stdout.write(JSON.stringify(out));
"""


def test_js_cache_ticks_equal_oracle(tmp_path):
    traces = mixed_traces(240) + _messy(7, 80)
    for t in traces[10:14] + traces[130:133]:  # rows with a falsy service: dropped by the combined cache
        for s in t:
            s.get("tags", {}).pop("istio.canonical_service", None)
    windows = _ticks(traces, [0, 40, 95, 150, len(traces)])
    exp = _oracle_ticks(windows)
    got = _node(_CPU_JS, {"ticks": [{"newdep": e[3], "update": e[2]} for e in exp]}, tmp_path)
    for k, ((gd, gc), (ed, ec, _, _)) in enumerate(zip(got, exp)):
        assert gd == ed, k
        _same_combined(gc, ec, exact=True)


_GPU_JS = """
const fs = require('fs');
const N = require('./js/kmamiz_native');
const C = N.cache;
const { step } = require('./js/realtime_worker');
const inp = JSON.parse(fs.readFileSync(process.argv[1]));
let state = null;
const comb = N.newCombinedCache();
const out = [];
inp.windows.forEach((w, k) => {
  const t = new N.NativeTraces(w, 0);
  // the worker tick: the first returns newDep (per row), later ones existingDep.combineWith(newDep)
  const dep = state === null ? t.toEndpointDependencies()
                             : C.ReducedDependencies.fromJSON(state, false).combineWith(t.toReducedDependencies()).toJSON();
  state = C.trimRows(dep);  // CEndpointDependencies.setData -> trim()
  comb.setData(t.combineLogsToRealtimeData([]).toCombinedColumns(comb.getData()));
  // the worker seam itself, fed the same existingDep
  const viaWorker = k ? step({ uniqueId: k, traces: w, existingDep: inp.prev[k] }).dependencies : null;
  out.push([state, comb.getData().toJSON(), viaWorker]);
});
process.stdout.write(JSON.stringify(out));
"""


@pytest.mark.gpu
def test_js_cache_ticks_from_the_engine(tmp_path):
    if not os.path.exists(os.path.join(ROOT, "js", "kmz.node")):
        pytest.skip("js/kmz.node not built")
    traces = mixed_traces(240) + _messy(7, 80)
    windows = _ticks(traces, [0, 40, 95, 150, len(traces)])
    exp = _oracle_ticks(windows)
    prev = [None] + [e[0] for e in exp[:-1]]
    got = _node(_GPU_JS, {"windows": windows, "prev": prev}, tmp_path)
    for k, ((gd, gc, gw), (ed, ec, _, _)) in enumerate(zip(got, exp)):
        assert gd == ed, k
        _same_combined(gc, ec, exact=False)
        if k:
            assert O.strip_undef(O.EndpointDependencies(gw).trim().toJSON()) == ed, k
