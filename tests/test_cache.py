"""Cache-layer merges in columnar form (kmamiz_amd/cache.py)
against the Python oracle's object merges, on CPU.

The window side is fed from the C oracle's entry records (oracle_dep_entries,
the restatement kmz_order.hip is checked against in test_gpu_cache.py), so
these tests pin the host columns + merges, and the records' semantics, without
a GPU:
  * one window: ReducedDependencies == EndpointDependencies([]).combineWith(
    toEndpointDependencies()).trim()  (EndpointDependencies.ts:91-112, 499-542);
  * a cache over several windows: existing.combineWith(window).trim() per tick
    (RealtimeWorkerImpl.ts:67-70, CEndpointDependencies.ts:46-48);
  * CCombinedRealtimeData.setData: service filter + combineWith
    (CCombinedRealtimeData.ts:47-53, CombinedRealtimeDataList.ts:183-332).
"""
import copy
import json

import numpy as np
import pytest

from conftest import fixture
from oracle import c_oracle
from oracle import kmz_oracle as O
from shard_util import mixed_traces


def _window(traces, reg=None):
    from kmamiz_amd.cache import ReducedDependencies
    from kmamiz_amd.ingest import ingest_traces

    batch, d, _ = ingest_traces(traces)
    t = d.shape_table()
    entries, rts, rsh = c_oracle.dep_entries(batch, t.dep_ep, t.n_dep_ep)
    _, ep, _ = c_oracle.deps(batch, t.dep_ep, t.n_dep_ep)
    idents = d.shape_ident["dep"]
    return ReducedDependencies.from_columns(entries, rts, rsh, ep["first"], ep["has_row"], ep["external"], ep["last"],
                                            np.zeros(t.n_dep_ep, bool), d.ep_names["dep"],
                                            lambda s: idents[s].fields, reg)


def _oracle_reduced(traces):
    return O.EndpointDependencies([]).combineWith(O.Traces(traces).toEndpointDependencies()).trim()


def _messy(seed, n_traces=60):
    """Traces with repeated span ids, CLIENT chains, non-SERVER ancestors and
    parents in other traces (the span map is global, Traces.ts:117-123)."""
    rng = np.random.default_rng(seed)
    names = ["a.ns1.svc.cluster.local:80/x", "b.ns1.svc.cluster.local:9080/*", "c.ns2.svc.c2:80/y",
             "d.ns2.svc.cluster.local:80/z", "e.ns3.svc.cluster.local:80/w"]
    out, nid = [], 1
    pool = []
    for t in range(n_traces):
        spans = []
        for k in range(int(rng.integers(1, 9))):
            if pool and rng.random() < 0.08:
                sid = pool[int(rng.integers(len(pool)))]  # repeated id
            else:
                sid = f"{nid:016x}"
                nid += 1
            pool.append(sid)
            kind = ["SERVER", "CLIENT", "PRODUCER"][int(rng.choice(3, p=[0.6, 0.3, 0.1]))]
            par = None
            if spans and rng.random() < 0.85:
                par = spans[int(rng.integers(len(spans)))]["id"]
            elif pool and rng.random() < 0.1:
                par = pool[int(rng.integers(len(pool)))]
            nm = names[int(rng.integers(len(names)))]
            sp = {"traceId": f"{t:032x}", "id": sid, "kind": kind, "name": nm,
                  "timestamp": 1_650_000_000_000_000 + int(rng.integers(0, 10**9)), "duration": int(rng.integers(1, 9999)),
                  "tags": {"http.method": "GET", "http.url": "http://" + nm.split(":")[0] + "/p",
                           "istio.canonical_revision": "v1", "istio.canonical_service": nm.split(".")[0],
                           "istio.namespace": nm.split(".")[1], "istio.mesh_id": "cluster.local",
                           "http.status_code": "200"}}
            if par is not None and par != sid:
                sp["parentId"] = par
            spans.append(sp)
        out.append(spans)
    return out


@pytest.mark.parametrize("fx", ["MockTrace", "MockTracePDAS"])
def test_window_reduced_graph_equals_oracle(fx):
    traces = fixture(fx) if fx == "MockTrace" else [fixture(fx)]
    got = _window(traces).toJSON()
    assert got == O.strip_undef(_oracle_reduced(traces).toJSON())


def test_window_reduced_graph_mixed_and_messy():
    for traces in (mixed_traces(120), _messy(1), _messy(2), _messy(3, 200)):
        got = _window(copy.deepcopy(traces)).toJSON()
        exp = O.strip_undef(_oracle_reduced(copy.deepcopy(traces)).toJSON())
        assert got == exp


def _ticks(traces, cuts):
    return [traces[a:b] for a, b in zip(cuts[:-1], cuts[1:])]


def test_cache_over_windows_equals_oracle_ticks():
    """Initializer (EndpointDependencies([]).combineWith(today)) then worker
    ticks existing.combineWith(newDep), setData -> trim, each round-tripping
    through the cache's JSON form as the worker message does."""
    from kmamiz_amd.cache import CEndpointDependencies, ReducedDependencies, worker_dependencies

    traces = mixed_traces(240) + _messy(7, 80)
    windows = _ticks(traces, [0, 40, 95, 150, len(traces)])
    cache = CEndpointDependencies()
    ocache = None
    for k, w in enumerate(windows):
        win = _window(copy.deepcopy(w))
        existing = cache.getData()
        if k == 0:
            dep = ReducedDependencies().combineWith(win)
        else:
            # the worker gets existingDep as JSON (ServiceOperator.ts:290-298)
            existing = ReducedDependencies.from_json(existing.toJSON())
            dep = worker_dependencies(existing, win)
        cache.setData(dep)
        newdep = O.Traces(copy.deepcopy(w)).toEndpointDependencies()
        base = O.EndpointDependencies(copy.deepcopy(ocache) if ocache is not None else [])
        ocache = base.combineWith(newdep).trim().toJSON()
        assert cache.getData().toJSON() == O.strip_undef(ocache), k
    # getData(namespace) (CEndpointDependencies.ts:51-59)
    exp = [d for d in O.strip_undef(ocache) if d["endpoint"].get("namespace") == "book"]
    assert cache.getData("book").toJSON() == exp


def test_reduced_json_round_trip_and_dup_rows():
    from kmamiz_amd.cache import ReducedDependencies

    traces = mixed_traces(80)
    r = _window(traces)
    js = r.toJSON()
    assert ReducedDependencies.from_json(js).toJSON() == js
    # `this` with a repeated endpoint row: Map.set keeps the LAST row at the
    # first one's position (EndpointDependencies.ts:508-513)
    rows = O.strip_undef(O.Traces(copy.deepcopy(traces)).toEndpointDependencies().toJSON())
    other = _window(mixed_traces(40))
    exp = O.EndpointDependencies(copy.deepcopy(rows)).combineWith(
        O.EndpointDependencies(other.toJSON())).trim().toJSON()
    got = ReducedDependencies.from_json(rows).combineWith(other).toJSON()
    assert got == O.strip_undef(exp)
    # the argument with repeated rows: they merge (514-535)
    exp2 = O.EndpointDependencies(copy.deepcopy(js)).combineWith(O.EndpointDependencies(copy.deepcopy(rows))).trim()
    got2 = ReducedDependencies.from_json(js).combineWith(ReducedDependencies.from_json(rows, merge_rows=True))
    assert got2.toJSON() == O.strip_undef(exp2.toJSON())


# ---------------------------------------------------------------------------
# combined realtime data cache
# ---------------------------------------------------------------------------
def _combined(traces):
    return O.Traces(traces).combineLogsToRealtimeData([], None).toCombinedRealtimeData()


def test_combined_columns_merge_equals_oracle():
    from kmamiz_amd.cache import CombinedColumns

    traces = mixed_traces(200)
    a = O.strip_undef(_combined(copy.deepcopy(traces[:90])).toJSON())
    b = O.strip_undef(_combined(copy.deepcopy(traces[60:])).toJSON())
    exp = O.CombinedRealtimeDataList(copy.deepcopy(a)).combineWith(O.CombinedRealtimeDataList(copy.deepcopy(b)))
    got = CombinedColumns.from_json(a).combineWith(CombinedColumns.from_json(b))
    assert got.toJSON() == O.strip_undef(exp.toJSON())
    # the host object mirror agrees too
    from kmamiz_amd import CombinedRealtimeDataList

    mir = CombinedRealtimeDataList(copy.deepcopy(a)).combineWith(CombinedRealtimeDataList(copy.deepcopy(b)))
    assert got.toJSON() == mir.toJSON()


def test_combined_cache_ticks_with_service_filter():
    """CCombinedRealtimeData.setData over ticks: rows with a falsy service are
    dropped before the merge (CCombinedRealtimeData.ts:47-53)."""
    from kmamiz_amd.cache import CCombinedRealtimeData

    traces = mixed_traces(240)
    # spans without istio tags: service undefined in the tag identity
    for t in traces[10:14] + traces[130:133]:
        for s in t:
            s.get("tags", {}).pop("istio.canonical_service", None)
    from kmamiz_amd.cache import CombinedColumns

    cache = CCombinedRealtimeData()
    ocache = None
    dropped = 0
    for k, w in enumerate(_ticks(traces, [0, 50, 120, 170, len(traces)])):
        upd = O.strip_undef(_combined(copy.deepcopy(w)).toJSON())
        dropped += sum(1 for r in upd if not r.get("service"))

        cache.setData(CombinedColumns.from_json(upd))
        f = [r for r in copy.deepcopy(upd) if O.truthy(O.get(r, "service"))]
        ocache = (O.CombinedRealtimeDataList(copy.deepcopy(ocache)).combineWith(O.CombinedRealtimeDataList(f))
                  if ocache is not None else O.CombinedRealtimeDataList(f)).toJSON()
        ocache = O.strip_undef(ocache)
        assert cache.getData().toJSON() == ocache, k
    assert dropped > 0
    assert cache.getData("book").toJSON() == [r for r in ocache if r.get("namespace") == "book"]


def test_pooled_matches_scalar_fold():
    """The vectorised combineLatencyCVAndMean equals the scalar restatement on
    awkward magnitudes (decimal shifts across powers of ten, zeros)."""
    from kmamiz_amd.cache import pooled

    rng = np.random.default_rng(5)
    m1 = np.concatenate([10.0 ** rng.uniform(-4, 6, 500), [0.0, 1.0, 10.0, 999.9999999999999, 1e-3]])
    m2 = np.concatenate([10.0 ** rng.uniform(-4, 6, 500), [5.0, 0.0, 0.1, 1000.0, 0.0]])
    c1, c2 = rng.uniform(0, 3, len(m1)), rng.uniform(0, 3, len(m1))
    n1, n2 = rng.integers(0, 10**6, len(m1)), rng.integers(1, 10**6, len(m1))
    gm, gc = pooled(n1, m1, c1, n2, m2, c2)
    for k in range(len(m1)):
        em, ec = O.combine_latency_cv_and_mean(int(n1[k]), float(m1[k]), float(c1[k]), int(n2[k]), float(m2[k]),
                                               float(c2[k]))
        assert gm[k] == em and gc[k] == ec, k


def test_combined_columns_from_engine_groups():
    """CombinedColumns.from_groups (the engine's dense groups -> columns) equals
    the drop-in rows built from the same groups (classes._combine_native), on
    the C oracle's groups of a mixed batch; and merges like them."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd.cache import CombinedColumns
    from kmamiz_amd.classes import CombinedRealtimeDataList, _combine_native, _UsedGroups
    from kmamiz_amd.ingest import ingest_traces

    def groups_of(traces):
        batch, d, _ = ingest_traces(traces)
        t = d.shape_table()
        o = c_oracle.stats(batch, t.tag_ep, t.n_tag_ep, t.n_status)
        g = np.zeros(len(o["combined"]), L.GROUP_DTYPE)
        for f in L.GROUP_DTYPE.names:
            g[f] = o[f]
        return g, batch, d, t

    traces = mixed_traces(160)
    parts = []
    for w in (traces[:70], traces[50:]):
        g, batch, d, t = groups_of(copy.deepcopy(w))
        rows = _combine_native(g, 0, batch, d, "tag", None)
        idents = d.shape_ident["tag"]
        first_shape = {}
        for sh, e in enumerate(d.shape_ep["tag"]):
            first_shape.setdefault(e, sh)
        cols = CombinedColumns.from_groups(g, t.n_status, lambda e: idents[first_shape[e]].fields, d.statuses)
        assert cols.toJSON() == rows
        # the used groups alone (kmz_fetch_used's form): the same columns and rows
        used = np.nonzero(g["combined"] > 0)[0]
        cu = CombinedColumns.from_groups(g[used].copy(), t.n_status, lambda e: idents[first_shape[e]].fields,
                                         d.statuses, used=used.astype(np.uint32))
        assert cu.toJSON() == rows
        assert _combine_native(_UsedGroups(used, g[used].copy()), 0, batch, d, "tag", None) == rows
        parts.append((cols, rows))
    got = parts[0][0].combineWith(parts[1][0]).toJSON()
    exp = CombinedRealtimeDataList(copy.deepcopy(parts[0][1])).combineWith(
        CombinedRealtimeDataList(copy.deepcopy(parts[1][1]))).toJSON()
    assert got == exp
