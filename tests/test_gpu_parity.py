"""GPU parity: the HIP path (through the C ABI) against the oracles.

* reference fixtures (MockData) through the drop-in classes vs the reference's
  own expected outputs / the Python oracle (order-exact JSON);
* randomized "messy" batches (duplicate ids, cross-trace and missing parents,
  CLIENT chains, non-SERVER ancestors, unparsable names) vs the Python oracle;
* synthetic configs 2/3 vs the C oracle (bit-exact integers, 1e-9 latency);
* size-independent properties at BASELINE.json's full sizes.
"""
import math
import os
import random

import numpy as np
import pytest

from conftest import fixture
from oracle import c_oracle
from oracle import kmz_oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-9  # north_star tolerance for latency statistics


def _stats_equal(got, exp):
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        for k in ("uniqueEndpointName", "uniqueServiceName", "service", "namespace", "version", "method", "status",
                  "combined", "latestTimestamp", "avgReplica"):
            assert a.get(k) == b.get(k), (k, a.get(k), b.get(k))
        for k in ("mean", "cv"):
            assert a["latency"][k] == pytest.approx(b["latency"][k], rel=REL, abs=1e-13), k


def _run_both(traces, replicas=None):
    from kmamiz_amd import Traces

    ours = Traces(traces)
    ref = O.Traces(traces)
    return ours, ref


# ---------------------------------------------------------------------------
# reference fixtures
# ---------------------------------------------------------------------------
def test_pdas_endpoint_dependencies_exact(engine):
    from kmamiz_amd import Traces

    deps = Traces([fixture("MockTracePDAS")], engine=engine).toEndpointDependencies()
    assert deps.toJSON() == fixture("MockEndpointDependenciesPDAS")  # Traces.test.ts:16-20


def test_pdas_realtime_rows_exact(engine):
    from kmamiz_amd import Traces

    rl = Traces([fixture("MockTracePDAS")], engine=engine).toRealTimeData()
    assert rl.toJSON() == fixture("MockRlDataPDAS")  # Traces.test.ts:11-14


def test_endpoint_info_exact():
    from kmamiz_amd import Traces

    assert Traces.ToEndpointInfo(fixture("MockTracePDAS")[0]) == fixture("MockEndpointInfoPDAS1")


def test_realtime_list_known_answer(engine):
    from kmamiz_amd import RealtimeDataList

    got = RealtimeDataList(fixture("MockBaseRlData1")).toCombinedRealtimeData().toJSON()
    exp = fixture("MockBaseCrlData1")  # RealtimeDataList.test.ts:10-13, cv 0.17888543819998
    assert len(got) == 1
    for k in ("combined", "latestTimestamp", "avgReplica", "status", "uniqueEndpointName"):
        assert got[0][k] == exp[0][k]
    assert got[0]["latency"] == exp[0]["latency"]


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
@pytest.mark.parametrize("rule", ["rt", "tag"])
def test_fixture_stats_vs_oracle(engine, fx, rule):
    traces = fixture(fx)
    if fx != "MockTrace":
        traces = [traces]
    ours, ref = _run_both(traces)
    reps = [{"uniqueServiceName": "details\tbook\tv1", "replicas": 3}]
    if rule == "rt":
        got = ours.toRealTimeData(reps).toCombinedRealtimeData().toJSON()
        exp = ref.toRealTimeData(reps).toCombinedRealtimeData().toJSON()
    else:
        got = ours.combineLogsToRealtimeData([], reps).toCombinedRealtimeData().toJSON()
        exp = ref.combineLogsToRealtimeData([], reps).toCombinedRealtimeData().toJSON()
    _stats_equal(got, O.strip_undef(exp))


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_fixture_dependencies_vs_oracle(engine, fx):
    traces = fixture(fx)
    if fx != "MockTrace":
        traces = [traces]
    ours, ref = _run_both(traces)
    got = ours.toEndpointDependencies()
    exp = ref.toEndpointDependencies()
    assert got.toJSON() == O.strip_undef(exp.toJSON())
    # the worker's merge + the cache's trim (RealtimeWorkerImpl.ts:67-70)
    from kmamiz_amd import EndpointDependencies

    g2 = EndpointDependencies([]).combineWith(ours.toEndpointDependencies()).trim().toJSON()
    e2 = O.EndpointDependencies([]).combineWith(ref.toEndpointDependencies()).trim().toJSON()
    assert g2 == O.strip_undef(e2)
    # service-level tail
    gd = EndpointDependencies(g2)
    od = O.EndpointDependencies(O.strip_undef(e2))
    assert gd.toServiceInstability() == od.toServiceInstability()
    assert gd.toServiceCoupling() == od.toServiceCoupling()
    assert gd.toServiceEndpointCohesion() == od.toServiceEndpointCohesion()
    assert gd.toChordData() == od.toChordData()


# ---------------------------------------------------------------------------
# randomized messy batches vs the Python oracle
# ---------------------------------------------------------------------------
NAMES = [
    "a.ns1.svc.cluster.local:80/x",
    "b.ns1.svc.cluster.local:9080/*",
    "c.ns2.svc.c2:80/y",
    "istio-ingressgateway",  # no ".svc." -> tag fallback in ToEndpointInfo
    "dsvc.ns3.svc:81/z",
    "e.svc.cluster.local/q",
]
URLS = ["http://a:80/x", "http://b/y?q=1", "https://10.0.0.1:8443/z#f", "c.ns2.svc.c2/p", "http://e"]


def messy_batch(rng: random.Random, n_traces: int, pool: int):
    ids = [f"{rng.getrandbits(64):016x}" for _ in range(pool)] + ["", "not-hex", "0000000000000000"]
    traces = []
    ts = 1646208338000000
    for _ in range(n_traces):
        tr = []
        for _ in range(rng.randint(0, 7)):
            s = {
                "traceId": "t",
                "id": rng.choice(ids),
                "kind": rng.choice(["SERVER", "SERVER", "CLIENT", "CLIENT", "PRODUCER"]),
                "name": rng.choice(NAMES),
                "timestamp": ts + rng.randint(0, 10**7),
                "duration": rng.randint(0, 10**6),
                "tags": {
                    "http.method": rng.choice(["GET", "POST"]),
                    "http.url": rng.choice(URLS),
                    "http.status_code": rng.choice(["200", "404", "500", "200 "]),
                    "istio.canonical_service": rng.choice(["a", "b", "c"]),
                    "istio.namespace": rng.choice(["ns1", "ns2"]),
                    "istio.mesh_id": "cluster.local",
                },
            }
            if rng.random() < 0.8:
                s["tags"]["istio.canonical_revision"] = rng.choice(["v1", "v2", "latest"])
            if rng.random() < 0.9:
                s["parentId"] = rng.choice(ids)
            tr.append(s)
        traces.append(tr)
    return traces


@pytest.mark.parametrize("seed", range(40))
def test_messy_batches_vs_oracle(engine, seed):
    from kmamiz_amd import CycleError, Traces

    rng = random.Random(seed)
    traces = messy_batch(rng, rng.randint(0, 12), rng.choice([4, 8, 32]))
    ref = O.Traces(traces)
    try:
        exp_deps = O.strip_undef(ref.toEndpointDependencies(max_depth=10000).toJSON())
    except RuntimeError:
        with pytest.raises(CycleError):
            Traces(traces, engine=engine).toEndpointDependencies().toJSON()
        return
    ours = Traces(traces, engine=engine)
    assert ours.toEndpointDependencies().toJSON() == exp_deps
    # the service tail at scale over the same batch (kmz_tail_run) vs the
    # oracle's tail of the reduced graph (duplicate ids, non-SERVER ancestors,
    # tag-fallback identities)
    from test_tail import _compare

    red = O.strip_undef(O.EndpointDependencies([]).combineWith(O.EndpointDependencies(exp_deps)).trim().toJSON())
    _compare(ours.toEndpointDependencies().service_tail(), O.EndpointDependencies(red))
    for rule in ("rt", "tag"):
        try:
            exp = (ref.toRealTimeData() if rule == "rt" else ref.combineLogsToRealtimeData([])).toCombinedRealtimeData()
        except TypeError:
            with pytest.raises(TypeError):
                ours.toRealTimeData().toCombinedRealtimeData()
            continue
        got = (ours.toRealTimeData() if rule == "rt" else ours.combineLogsToRealtimeData([])).toCombinedRealtimeData()
        _stats_equal(got.toJSON(), O.strip_undef(exp.toJSON()))


def test_empty_batch(engine):
    from kmamiz_amd import Traces

    t = Traces([], engine=engine)
    assert t.toEndpointDependencies().toJSON() == []
    tail = t.toEndpointDependencies().service_tail()
    assert tail.instability() == [] and tail.coupling() == [] and tail.cohesion() == []
    assert t.toRealTimeData().toCombinedRealtimeData().toJSON() == []


def test_cycle_is_reported(engine):
    from kmamiz_amd import CycleError, Traces

    a = {"id": "00000000000000aa", "parentId": "00000000000000bb", "kind": "SERVER", "name": "a.b.svc.c:1/x",
         "timestamp": 1, "duration": 1, "tags": {"http.url": "http://a/x"}}
    b = {**a, "id": "00000000000000bb", "parentId": "00000000000000aa"}
    with pytest.raises(CycleError):
        Traces([[a, b]], engine=engine).toEndpointDependencies()


# ---------------------------------------------------------------------------
# synthetic configs vs the C oracle
# ---------------------------------------------------------------------------
def _compare_synth(engine, batch, table, odeps=None):
    from kmamiz_amd import _lib as L

    engine.load(batch, table)
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    g = engine.groups()
    o = c_oracle.stats(batch, table.tag_ep, table.n_tag_ep, table.n_status)
    assert np.array_equal(g["combined"], o["combined"])
    used = o["combined"] > 0
    assert np.array_equal(g["latest_timestamp"][used], o["latest_timestamp"][used])
    assert np.array_equal(g["first"][used], o["first"][used])
    np.testing.assert_allclose(g["mean"][used], o["mean"][used], rtol=REL, atol=0)
    np.testing.assert_allclose(g["cv"][used], o["cv"][used], rtol=REL, atol=1e-13)
    keys = engine.triples()
    ep = engine.endpoints()
    info = engine.info()
    okeys, oep, ocnt = odeps or c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    assert np.array_equal(keys, okeys)
    assert np.array_equal(ep["has_row"].astype(bool), oep["has_row"])
    assert np.array_equal(ep["first_row"][oep["has_row"]], oep["first"][oep["has_row"]])
    assert np.array_equal(ep["external"][oep["has_row"]].astype(bool), oep["external"][oep["has_row"]])
    seen = ep["last_ts"] != np.iinfo(np.int64).min
    last = np.where(seen, np.maximum(ep["last_ts"] / 1000.0, 0.0), 0.0)
    assert np.array_equal(last, oep["last"])
    assert info["n_rows"] == ocnt["rows"]
    assert info["n_relations"] == ocnt["relations"]
    assert info["max_depth"] == ocnt["max_depth"]
    return info


@pytest.mark.parametrize("config,ntr", [(2, 30000), (3, 4000), (3, 40000), (3, 366000), (5, 2000), (5, 20000)])
def test_synthetic_vs_c_oracle(engine, config, ntr):
    from kmamiz_amd import synth

    batch, off = synth.host_batch(config, 0, ntr)
    info = _compare_synth(engine, batch, synth.shape_table(config))
    assert info["n_dups"] == 0


@pytest.mark.parametrize("ntr", [4000, 366000])
def test_wide_durations_vs_c_oracle(engine, ntr):
    """K3's packed accumulators (k3_reduce<PACK>) take durations < 2^20 us;
    wider ones (up to 2^32 - 1) take the rare split path: both against the C
    oracle on the mesh (partitioned K3), at 1e5 and 1e7 spans."""
    from kmamiz_amd import synth
    from kmamiz_amd.engine import SpanBatch

    batch, _ = synth.host_batch(3, 0, ntr)
    rng = np.random.default_rng(11)
    d = batch.duration.astype(np.uint64)
    wide = rng.random(len(d)) < 0.05
    d[wide] = rng.integers(1 << 20, 1 << 32, int(wide.sum()), dtype=np.uint64)
    d[rng.random(len(d)) < 0.001] = (1 << 32) - 1
    b2 = SpanBatch(batch.span_id, batch.parent_id, batch.kind, batch.shape, batch.status,
                   d.astype(batch.duration.dtype), batch.timestamp, batch.index_base)
    _compare_synth(engine, b2, synth.shape_table(3))


@pytest.mark.parametrize("ntr", [3000, 40000])
def test_chain_elements_by_shape_with_shared_endpoints(engine, ntr):
    """k4_tile8 interns chains over shapes when the dependency table maps
    every shape into range (kmz_walk.hip): exact whatever the table, only
    fewer repeats where shapes share an endpoint.  Here every mesh endpoint
    gets a second shape (s + n and s map to endpoint s) and a third of the
    spans move to it; rows, relations, edge keys and endpoints equal the C
    oracle and the same run with chain elements by endpoint (KMZ_ABLATE2 bit
    11); the shape chains outnumber the endpoint chains.  (Fresh engines with
    chain interning forced and the fused kernel off, so that k4_tile8 runs at
    both sizes.)"""
    from kmamiz_amd import Engine
    from kmamiz_amd import synth
    from kmamiz_amd.engine import ShapeTable, SpanBatch

    batch, _ = synth.host_batch(3, 0, ntr)
    t = synth.shape_table(3)
    n = len(t.dep_ep)
    rng = np.random.default_rng(5)
    shape = batch.shape.copy()
    shape[rng.random(len(shape)) < 1 / 3] += np.uint32(n)
    two = lambda x: np.concatenate([np.asarray(x, np.uint32)] * 2)  # noqa: E731
    table = ShapeTable(two(t.rt_ep), two(t.tag_ep), two(t.dep_ep), t.n_rt_ep, t.n_tag_ep, t.n_dep_ep, t.n_status)
    b2 = SpanBatch(batch.span_id, batch.parent_id, batch.kind, shape, batch.status, batch.duration, batch.timestamp,
                   batch.index_base)
    out = []
    for bits2 in (1 << 4, (1 << 4) | (1 << 11)):
        os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"] = str(1 << 29), str(bits2)
        try:
            e = Engine(0)
        finally:
            del os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"]
        try:
            info = _compare_synth(e, b2, table)
            out.append((info, e.triples().copy(), e.endpoints().tobytes()))
        finally:
            e.close()
    (by_shape, k1, p1), (by_ep, k2, p2) = out
    assert np.array_equal(k1, k2) and p1 == p2
    assert by_shape["path"] & 32 and by_ep["path"] & 32  # (k4_tile8 both times)
    assert by_shape["n_chains"] > by_ep["n_chains"] > 0


@pytest.mark.parametrize("config,ntr,variant", [(2, 30000, "plain"), (3, 4000, "plain"), (3, 40000, "plain"),
                                                (3, 40000, "by_endpoint"), (3, 20000, "other_kinds"),
                                                (5, 2000, "plain"), (5, 20000, "plain"), (5, 6000, "other_kinds")])
def test_tile9_equals_tile8_and_oracle(config, ntr, variant):
    """k4_tile9 (element hashes in LDS, sentinel-terminated walks, kmz_walk.hip)
    against k4_tile8 (KMZ_ABLATE2 bit 22) and the C oracle: the same rows,
    relations, depths, edge keys, endpoints and interned chains.  Variants:
    chain elements by endpoint (KMZ_ABLATE2 bit 11: the gathered ids), and
    5 % of the spans turned into kind-0 spans (neither SERVER nor CLIENT: the
    walk's lastUsage branch, Traces.ts:192-208).  Chain interning forced and
    the fused kernel off, so that the tile kernels run at every size."""
    from kmamiz_amd import Engine
    from kmamiz_amd import synth
    from kmamiz_amd.engine import SpanBatch

    batch, _ = synth.host_batch(config, 0, ntr)
    table = synth.shape_table(config)
    if variant == "other_kinds":
        kind = batch.kind.copy()
        rng = np.random.default_rng(9)
        kind[(rng.random(len(kind)) < 0.05) & (kind == 1)] = 0
        batch = SpanBatch(batch.span_id, batch.parent_id, kind, batch.shape, batch.status, batch.duration,
                          batch.timestamp, batch.index_base)
    odeps = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    base2 = (1 << 4) | ((1 << 11) if variant == "by_endpoint" else 0)
    out = []
    for bits2 in (base2, base2 | (1 << 22)):
        os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"] = str(1 << 29), str(bits2)
        try:
            e = Engine(0)
        finally:
            del os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"]
        try:
            info = _compare_synth(e, batch, table, odeps)
            out.append((info, e.triples().copy(), e.endpoints().tobytes()))
        finally:
            e.close()
    (i9, k9, p9), (i8, k8, p8) = out
    assert i9["path"] & 96 == 96 and i8["path"] & 96 == 32  # k4_tile9, then k4_tile8
    assert np.array_equal(k9, k8) and p9 == p8
    assert i9["n_chains"] == i8["n_chains"] > 0


def test_chain_elements_by_endpoint_when_a_shape_is_out_of_range(engine):
    """A dependency table with an entry past n_dep (a shape no span uses) keeps
    the walk on endpoint elements (gathered per slot): same results as the
    C oracle."""
    from kmamiz_amd import synth
    from kmamiz_amd.engine import ShapeTable

    batch, _ = synth.host_batch(3, 0, 3000)
    t = synth.shape_table(3)
    dep = np.concatenate([np.asarray(t.dep_ep, np.uint32), np.array([t.n_dep_ep + 7], np.uint32)])
    ext = lambda x: np.concatenate([np.asarray(x, np.uint32), np.zeros(1, np.uint32)])  # noqa: E731
    table = ShapeTable(ext(t.rt_ep), ext(t.tag_ep), dep, t.n_rt_ep, t.n_tag_ep, t.n_dep_ep, t.n_status)
    _compare_synth(engine, batch, table)


def test_synthetic_shard_base_vs_c_oracle(engine):
    from kmamiz_amd import synth

    batch, off = synth.host_batch(3, 1000, 2500)
    assert batch.index_base == synth.count_spans(3, 0, 1000)
    _compare_synth(engine, batch, synth.shape_table(3))


def test_device_generation_equals_host(engine):
    """kmz_synth_load (device) produces the same batch as kmz_synth_host."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    for config, (t0, t1) in ((2, (5, 20000)), (3, (17, 3000)), (5, (11, 2000))):
        batch, _ = synth.host_batch(config, t0, t1)
        table = synth.shape_table(config)
        engine.load(batch, table)
        engine.run(L.RUN_STATS_RT | L.RUN_DEPS)
        a = (engine.groups(), engine.triples(), engine.endpoints(), engine.info())
        n = engine.load_synthetic(config, synth.SEED, t0, t1)
        assert n == len(batch)
        engine.run(L.RUN_STATS_RT | L.RUN_DEPS)
        b = (engine.groups(), engine.triples(), engine.endpoints(), engine.info())
        assert a[0].tobytes() == b[0].tobytes()
        assert np.array_equal(a[1], b[1])
        assert a[2].tobytes() == b[2].tobytes()
        assert _info_results(a[3]) == _info_results(b[3])


def _info_results(info):
    """kmz_info without the fields that say which K4 mode ran (chain interning
    or direct enumeration: the same results, different diagnostics)."""
    return {k: v for k, v in info.items() if k not in ("n_chains", "path")}


@pytest.mark.parametrize("config,ntr", [(2, 136000)])
def test_full_size_properties(engine, config, ntr):
    """Config 2 at its BASELINE size (1M spans): conservation + idempotence."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    n = engine.load_synthetic(config, synth.SEED, 0, ntr)
    assert n > 990000
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    g1, k1, e1, i1 = engine.groups(), engine.triples(), engine.endpoints(), engine.info()
    assert int(g1["combined"].sum()) == i1["n_server"] == i1["n_rows"]  # unique ids: every SERVER is a row
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    assert engine.groups().tobytes() == g1.tobytes()
    assert np.array_equal(engine.triples(), k1)
    # Bookinfo shape: exactly these (anc, desc, distance) edges
    from kmamiz_amd import decode_triples

    a, d, dist, on = decode_triples(k1)
    edges = set(zip(a.tolist(), d.tolist(), dist.tolist(), on.tolist()))
    assert edges == {(0, 1, 1, True), (0, 2, 1, True), (0, 3, 1, True), (0, 4, 1, True), (3, 5, 1, True),
                     (4, 5, 1, True), (0, 5, 2, True)}
    # kmz_fetch (one synchronisation) returns the same three result sets
    g2, k2, e2 = engine.fetch()
    assert g2.tobytes() == g1.tobytes()
    assert np.array_equal(np.sort(k2), k1)
    assert e2.tobytes() == e1.tobytes()


def test_hot_descendant_falls_back_to_global_edge_set(engine):
    """One endpoint with > 6144 distinct (ancestor, distance) edges overflows the
    LDS edge set of the tile path; the engine must fall back, not drop edges."""
    from kmamiz_amd import Traces

    traces = []
    for k in range(7000):
        base = f"{k + 1:012x}"
        tags = lambda svc: {"http.url": f"http://{svc}/x", "http.method": "GET", "istio.canonical_revision": "v1",
                            "http.status_code": "200"}
        traces.append([
            {"id": base + "0001", "kind": "SERVER", "name": f"a{k}.ns.svc.cluster.local:80/x", "timestamp": 1 + k,
             "duration": 10, "tags": tags(f"a{k}")},
            {"id": base + "0002", "parentId": base + "0001", "kind": "CLIENT", "name": "x.ns.svc.cluster.local:80/x",
             "timestamp": 2 + k, "duration": 5, "tags": tags("x")},
            {"id": base + "0003", "parentId": base + "0002", "kind": "SERVER", "name": "x.ns.svc.cluster.local:80/x",
             "timestamp": 3 + k, "duration": 4, "tags": tags("x")},
        ])
    got = Traces(traces, engine=engine).toEndpointDependencies()
    keys, _ = got.reduced()
    assert len(keys) == 7000
    exp = O.strip_undef(O.Traces(traces).toEndpointDependencies().toJSON())
    assert got.toJSON() == exp


# ---------------------------------------------------------------------------
# K1' window join: far parents, repeated ids far apart, CLIENT chains that
# leave the window (kmz_join.hip)
# ---------------------------------------------------------------------------
def _permuted(batch, perm):
    from kmamiz_amd.engine import SpanBatch

    return SpanBatch(batch.span_id[perm], batch.parent_id[perm], batch.kind[perm], batch.shape[perm],
                     batch.status[perm], batch.duration[perm], batch.timestamp[perm], batch.index_base)


@pytest.mark.parametrize("frac", [1.0, 0.02])
def test_far_parents_vs_c_oracle(engine, frac):
    """Spans moved far from their trace (all of them, or 2%): parents outside
    the LDS window go through the MISS semi-join and PEND chains."""
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(3, 0, 3000)
    n = len(batch)
    rng = np.random.default_rng(7)
    perm = np.arange(n)
    sel = np.flatnonzero(rng.random(n) < frac)
    perm[sel] = perm[rng.permutation(sel)]
    info = _compare_synth(engine, _permuted(batch, perm), synth.shape_table(3))
    assert info["path"] & 1  # window join (ids unique)


@pytest.mark.parametrize("where", ["far", "near"])
def test_repeated_id_falls_back_to_span_table(engine, where):
    """A span id repeated anywhere in the batch voids the window answers: the
    certificate must catch it and the global Map rule must apply."""
    from kmamiz_amd import synth

    batch, off = synth.host_batch(3, 0, 3000)
    n = len(batch)
    # i and j in different traces (no cycle): far apart, or in one LDS window
    i, j = (10, n - 10) if where == "far" else (int(off[200]), int(off[201]) + 1)
    batch.span_id[j] = batch.span_id[i]
    info = _compare_synth(engine, batch, synth.shape_table(3))
    assert info["n_dups"] == 1
    assert not (info["path"] & 1)


def test_window_join_matches_span_table(engine):
    """Same batch through both resolve paths (KMZ_ABLATE bit 32 forces the table)."""
    import os

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    def run(e):
        e.load_synthetic(3, synth.SEED, 0, 20000)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_SPAN_LINKS)
        cp, rp = e.span_links()
        return cp, rp, e.triples(), e.endpoints(), e.info()

    a = run(engine)
    os.environ["KMZ_ABLATE"] = "32"
    try:
        e2 = Engine(0)
    finally:
        del os.environ["KMZ_ABLATE"]
    try:
        b = run(e2)
    finally:
        e2.close()
    assert a[4]["path"] & 3 == 3 and b[4]["path"] & 3 == 2  # (bit 4: which K4 mode ran)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3].tobytes() == b[3].tobytes()
    assert _info_results(a[4]) == _info_results(b[4])


WIDE_CERT_BINS = 64  # KMZ_ABLATE2: the certificate's pass 1 in 2^8 bins (default past ~10^8 ids) at any size


@pytest.mark.parametrize("repeat", [False, True])
def test_wide_certificate_bins(engine, repeat):
    """The certificate with 2^8 pass-1 bins (k_join_window<8>, k_cert_split's
    binary-searched tile runs: the layout batches past ~10^8 ids take) proves
    a clean mesh batch unique -- the window answers stand, results equal the
    default plan's -- and catches one span id repeated far apart."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(3, 0, 20000)
    table = synth.shape_table(3)
    if repeat:
        batch.span_id[len(batch) - 7] = batch.span_id[5]

    def run(e):
        e.load(batch, table)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        return e.triples(), e.endpoints(), e.groups(), e.info()

    wide = _engine_with2(0, WIDE_CERT_BINS)
    try:
        a = run(wide)
    finally:
        wide.close()
    b = run(engine)
    assert bool(a[3]["path"] & 1) == (not repeat) and bool(b[3]["path"] & 1) == (not repeat)
    assert np.array_equal(a[0], b[0]) and a[1].tobytes() == b[1].tobytes() and a[2].tobytes() == b[2].tobytes()
    assert _info_results(a[3]) == _info_results(b[3])
    if repeat:
        assert a[3]["n_dups"] == 1


SEPARATE_JOIN_WALK = 16  # KMZ_ABLATE2: k_join_window + k4_chain instead of the fused k_join_chain
FUSED_ANY_SIZE = 32      # KMZ_ABLATE2: the fused k_join_chain at any batch size


@pytest.mark.parametrize("case", ["mesh", "power", "far", "messy"])
def test_fused_join_walk_equals_two_kernels(engine, case):
    """The fused join + chain walk (kmz_fuse.hip: one LDS window for the parent
    join, the contraction and the walk; halo spans resolved in-window, the rest
    pending) gives the same span links, edge keys, endpoints and counts as
    k_join_window followed by k4_chain, on the mesh, config 5 (interning
    forced), a batch with 5 % of its spans moved far from their traces (MISS
    parents, PEND chains, pending ancestries) and messy batches."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.engine import SpanBatch

    if case in ("mesh", "power"):
        cfg = 3 if case == "mesh" else 5
        batch, _ = synth.host_batch(cfg, 0, 8000)
        table = synth.shape_table(cfg)
    elif case == "far":
        batch, _ = synth.host_batch(3, 0, 6000)
        n = len(batch)
        rng = np.random.default_rng(11)
        perm = np.arange(n)
        sel = np.flatnonzero(rng.random(n) < 0.05)
        perm[sel] = perm[rng.permutation(sel)]
        batch = _permuted(batch, perm)
        table = synth.shape_table(3)

    def run(e):
        if case == "messy":
            out = []
            from kmamiz_amd import CycleError, Traces

            for seed in range(12):
                rng = random.Random(1000 + seed)
                traces = messy_batch(rng, rng.randint(4, 40), rng.choice([8, 64, 4096, 4096]))
                try:
                    out.append((Traces(traces, engine=e).toEndpointDependencies().toJSON(), e.info()["path"]))
                except CycleError:  # (random parent ids can close a loop: both paths must refuse it)
                    out.append(("cycle", 0))
            return out
        e.load(batch, table)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_SPAN_LINKS)
        cp, rp = e.span_links()
        return cp, rp, e.triples(), e.endpoints(), e.info(), e.groups()

    sep = _engine_with2(1 << 29, SEPARATE_JOIN_WALK)  # (bit 29: chain interning on config 5 too)
    fused = _engine_with2(1 << 29, FUSED_ANY_SIZE)
    try:
        a, b = run(fused), run(sep)
    finally:
        sep.close()
        fused.close()
    if case == "messy":
        assert [x[0] for x in a] == [x[0] for x in b]
        assert any(x[1] & 16 for x in a) and not any(x[1] & 16 for x in b)
        return
    assert a[4]["path"] & 16 and not b[4]["path"] & 16 and a[4]["path"] & 3 == 3
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3].tobytes() == b[3].tobytes() and a[5].tobytes() == b[5].tobytes()
    assert _info_results(a[4]) == _info_results(b[4])
    keys, _, _ = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    assert np.array_equal(a[2], keys)


# ---------------------------------------------------------------------------
# K4 chain interning: hash collisions, deep chains (kmz_chain.hip)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("separate", [False, True])
def test_sig_collision_is_detected_and_retried(engine, separate):
    """KMZ_ABLATE bit 24 truncates the ancestry sigs to 4 bits on the first
    seed: different chains share sigs, the exact entry checks raise F_SIG, and
    the run repeats with another seed.  The result must equal a normal run --
    in the fused join + walk (this batch's default) and in k4_chain."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    def run(e):
        e.load_synthetic(3, synth.SEED, 0, 20000)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        return e.triples(), e.endpoints(), e.info()

    a = run(engine)
    e2 = _engine_with2(1 << 24, 16 if separate else 0)  # (KMZ_ABLATE2 bit 4: the two kernels)
    try:
        b = run(e2)
    finally:
        e2.close()
    assert np.array_equal(a[0], b[0])
    assert a[1].tobytes() == b[1].tobytes()
    assert _info_results(a[2]) == _info_results(b[2])


@pytest.mark.parametrize("config,ntr,knob2", [(2, 30000, 0), (3, 4000, 16), (5, 20000, 0), (3, 20000, 0)])
def test_gather_table_kept_across_runs(config, ntr, knob2):
    """The walk's per-shape gather table (k_chain_etab) is built once per shape
    table and seed and kept by later runs of the same engine (kmz_api.hip
    etab_cached): repeated runs of one loaded batch -- the fused join + walk
    (config 2), k4_chain (KMZ_ABLATE2 bit 4 at 4000 traces), config 5's
    direct walk -- equal the C oracle every time; after a reload with another
    config's shape table the table is rebuilt; under the collision knob the
    retried seed's table is the one kept."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    def check(e, cfg):
        batch, _ = synth.host_batch(cfg, 0, ntr)
        table = synth.shape_table(cfg)
        okeys, _, ocnt = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
        e.load_synthetic(cfg, synth.SEED, 0, ntr)
        for _ in range(3):
            e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
            assert np.array_equal(np.sort(e.triples()), np.sort(okeys))
            assert e.info()["n_rows"] == ocnt["rows"]

    other = 5 if config != 5 else 2
    for knob in (0, 1 << 24):
        e = _engine_with2(knob, knob2)
        try:
            check(e, config)
            check(e, other)  # another shape table on the same engine
            check(e, config)
        finally:
            e.close()


SPIN_TINY_DEFER = 1 << 10  # KMZ_ABLATE: 4 deferred chain checks per workgroup (in-place chain_put waits)
SPIN_NO_WAIT = 1 << 11     # KMZ_ABLATE: every chain-table wait "runs out" at once (F_SPIN)
FORCE_INTERNING = 1 << 29  # KMZ_ABLATE: K4 chain interning even where auto mode would enumerate


@pytest.mark.parametrize("separate", [False, True])
@pytest.mark.parametrize("knob", [SPIN_TINY_DEFER, SPIN_NO_WAIT, SPIN_TINY_DEFER | SPIN_NO_WAIT])
def test_chain_waits_never_drop_results(knob, separate):
    """The chain-table waits of kmz_chain.hip (a leader whose workgroup's
    deferred list is full, k_chain_settle's deferred checks, k4_chain_pend)
    on config 5 with chain interning, where a fresh table makes workgroups
    race on the same new chains.  A tiny deferred list forces the in-place
    waits that once hung config 5; a zero wait bound makes every wait run out,
    which must raise F_SPIN and redo the run on the exact walk (path bit 3),
    never drop a row, an ancestor's timestamp or a check.  Both equal the C
    oracle (Traces.ts:128-143, 192-208).  The batch (1.4e6 spans) takes the
    fused join + walk; ``separate``: k_join_window + k4_chain."""
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(5, 0, 20000)
    table = synth.shape_table(5)
    odeps = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    e = _engine_with2(knob | FORCE_INTERNING, 16 if separate else 0)
    try:
        for run in range(2):  # a fresh chain table, then a cleared one
            info = _compare_synth(e, batch, table, odeps)
            if knob & SPIN_NO_WAIT and run == 0:
                assert info["path"] & 8, "no chain-table wait ran out: the knob did not reach the waits"
            if not knob & SPIN_NO_WAIT:
                assert not info["path"] & 8  # (the waits finish normally)
    finally:
        e.close()


def test_spin_exhaustion_on_the_pending_path():
    """A 300-deep chain (unique ids: the window join and k4_chain) always
    takes k4_chain_pend, whose chain_put wait runs out at once under the zero
    bound: F_SPIN, and the exact walk gives the oracle's order-exact rows."""
    from kmamiz_amd import Traces

    front = [_deep_span(100000, "SERVER", None, "front")]
    deep = _deep_trace(300)
    e = _engine_with(SPIN_NO_WAIT | FORCE_INTERNING)
    try:
        got = Traces([front, deep], engine=e).toEndpointDependencies().toJSON()
        info = e.info()
        assert info["path"] & 1 and info["path"] & 8, info["path"]
    finally:
        e.close()
    assert got == O.strip_undef(O.Traces([front, deep]).toEndpointDependencies(max_depth=10000).toJSON())


def _deep_span(i, kind, parent, svc):
    tags = {"http.url": f"http://{svc}/x", "http.method": "GET", "istio.canonical_revision": "v1",
            "http.status_code": "200"}
    d = {"id": f"{i + 1:016x}", "kind": kind, "name": f"{svc}.ns.svc.cluster.local:80/x", "timestamp": 1000 + i,
         "duration": 10 + i % 7, "tags": tags}
    if parent is not None:
        d["parentId"] = f"{parent + 1:016x}"
    return d


def _deep_trace(levels):
    trace, prev, i = [], None, 0
    for level in range(levels):
        svc = f"s{level % 5}"
        if prev is not None:
            trace.append(_deep_span(i, "CLIENT", prev, svc))
            i += 1
            prev = i - 1
        trace.append(_deep_span(i, "SERVER", prev, svc))
        prev = i
        i += 1
    return trace


def test_deep_chain_takes_the_pending_path(engine):
    """A 300-deep SERVER/CLIENT chain is deeper than the LDS window and
    WIN_DEPTH: its spans hash over the global contracted parents."""
    from kmamiz_amd import Traces

    def span(i, kind, parent, svc):
        tags = {"http.url": f"http://{svc}/x", "http.method": "GET", "istio.canonical_revision": "v1",
                "http.status_code": "200"}
        d = {"id": f"{i + 1:016x}", "kind": kind, "name": f"{svc}.ns.svc.cluster.local:80/x", "timestamp": 1000 + i,
             "duration": 10 + i % 7, "tags": tags}
        if parent is not None:
            d["parentId"] = f"{parent + 1:016x}"
        return d

    trace, prev, i = [], None, 0
    for level in range(300):
        svc = f"s{level % 5}"
        if prev is not None:
            trace.append(span(i, "CLIENT", prev, svc))
            i += 1
            prev = i - 1
        trace.append(span(i, "SERVER", prev, svc))
        prev = i
        i += 1
    # a short normal trace in front, so the deep one also crosses tiles
    ours = Traces([trace[:1], trace], engine=engine)
    exp = O.strip_undef(O.Traces([trace[:1], trace]).toEndpointDependencies(max_depth=10000).toJSON())
    assert ours.toEndpointDependencies().toJSON() == exp


def test_merge_triples_is_the_union_of_shards(engine):
    """kmz_merge_triples: shard B's edge keys unioned into shard A's device set
    equal the edge set of one run over both shards; a union that outgrows the
    set (many foreign keys, host memory) takes the fresh-table path."""
    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    F = L.RUN_STATS_TAG | L.RUN_DEPS
    engine.load_synthetic(3, synth.SEED, 0, 4000)
    engine.run(F)
    full = engine.triples()
    b = Engine(0)
    try:
        b.load_synthetic(3, synth.SEED, 2000, 4000)
        b.run(F)
        kb = b.triples()
    finally:
        b.close()
    engine.load_synthetic(3, synth.SEED, 0, 2000)
    engine.run(F)
    ka = engine.triples()
    assert len(ka) < len(full) and len(kb) < len(full)
    pad = np.concatenate([kb, np.zeros(17, np.uint64)])  # zeros: padding, skipped
    engine.merge_triples(pad.ctypes.data, len(pad), False)
    assert np.array_equal(engine.triples(), full)
    assert engine.info()["n_triples"] == len(full)
    rng = np.random.default_rng(3)
    foreign = np.unique(rng.integers(1, 2**62, size=300000, dtype=np.uint64))
    engine.merge_triples(foreign.ctypes.data, len(foreign), False)
    assert np.array_equal(engine.triples(), np.union1d(full, foreign))


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_fixture_historical_data_vs_oracle(engine, fx):
    """The whole worker step of ServiceOperator.ts:153-160 on the fixtures:
    GPU stats + GPU dependency graph -> service dependencies ->
    CombinedRealtimeDataList.toHistoricalData (host)."""
    traces = fixture(fx)
    if fx != "MockTrace":
        traces = [traces]
    ours, ref = _run_both(traces)
    reps = [{"uniqueServiceName": "details\tbook\tv1", "replicas": 3}]
    sdep = ours.toEndpointDependencies().toServiceDependencies()
    got = ours.combineLogsToRealtimeData([], reps).toCombinedRealtimeData().toHistoricalData(sdep, reps)
    rsdep = ref.toEndpointDependencies().toServiceDependencies()
    exp = ref.combineLogsToRealtimeData([], reps).toCombinedRealtimeData().toHistoricalData(rsdep, reps)
    exp = O.strip_undef(exp)
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        assert g["date"] == e["date"]
        assert len(g["services"]) == len(e["services"])
        for gs, es in zip(g["services"], e["services"]):
            for k in ("service", "namespace", "version", "requests", "requestErrors", "serverErrors",
                      "uniqueServiceName", "date"):
                assert gs.get(k) == es.get(k), k
            assert ("risk" in gs) == ("risk" in es)
            if "risk" in es:
                assert gs["risk"] == pytest.approx(es["risk"], rel=REL, abs=1e-13)
            assert gs["latencyMean"] == pytest.approx(es["latencyMean"], rel=REL, abs=0)
            assert gs["latencyCV"] == pytest.approx(es["latencyCV"], rel=REL, abs=1e-13)
            assert [x["uniqueEndpointName"] for x in gs["endpoints"]] == [x["uniqueEndpointName"]
                                                                           for x in es["endpoints"]]


@pytest.mark.parametrize("src", ["MockTracePDAS", "MockTrace", "MockData2_traces", "mesh"])
def test_from_json_equals_object_ingest(engine, src):
    """Traces.from_json (native JSON parser) gives the
    same realtime rows, combined stats and dependency graph as Traces over
    the parsed objects."""
    import json

    from kmamiz_amd import Traces, synth

    if src == "mesh":
        batch, off = synth.host_batch(3, 0, 2000)
        traces = synth.to_traces(3, batch, off)
    else:
        traces = fixture(src)
        if src != "MockTrace":
            traces = [traces]
    data = json.dumps(traces).encode()
    a, b = Traces.from_json(data, engine=engine), Traces(traces, engine=engine)
    assert a.toRealTimeData().toJSON() == b.toRealTimeData().toJSON()
    assert (a.combineLogsToRealtimeData([]).toCombinedRealtimeData().toJSON()
            == b.combineLogsToRealtimeData([]).toCombinedRealtimeData().toJSON())
    assert a.toEndpointDependencies().toJSON() == b.toEndpointDependencies().toJSON()


@pytest.mark.parametrize("knob", [1 << 30, (1 << 30) | (1 << 28)])
def test_key_staging_paths_equal(engine, knob):
    """K4's staged edge keys reach the edge set through k_key_part +
    k_key_slice, or in place when a workgroup's staging overflows (KMZ_ABLATE
    bit 30: 256 slots; the staging then grows run by run), with chain
    interning or direct enumeration (bit 28).  Same graph either way."""
    import os

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    def run(e):
        e.load_synthetic(5, synth.SEED, 0, 20000)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        return e.triples(), e.endpoints(), e.info()

    a = run(engine)
    os.environ["KMZ_ABLATE"] = str(knob)
    try:
        e2 = Engine(0)
    finally:
        del os.environ["KMZ_ABLATE"]
    try:
        for _ in range(3):  # overflow, then grown staging
            b = run(e2)
            assert np.array_equal(a[0], b[0])
            assert a[1].tobytes() == b[1].tobytes()
            skip = ("flags", "n_chains", "path")  # (which K4 mode ran: diagnostics, not results)
            assert {k: v for k, v in a[2].items() if k not in skip} == {k: v for k, v in b[2].items() if k not in skip}
    finally:
        e2.close()


def _engine_with(knob):
    import os

    from kmamiz_amd import Engine

    os.environ["KMZ_ABLATE"] = str(knob)
    try:
        return Engine(0)
    finally:
        del os.environ["KMZ_ABLATE"]


WIDE_KEYS = 1        # KMZ_ABLATE2: direct enumeration stages 8-byte keys (no compact 4-byte keys)
BIG_EDGE_SET = 2     # KMZ_ABLATE2: the edge set starts at 2^20 slots (compact staging from the first run)


def _engine_with2(knob, knob2):
    import os

    from kmamiz_amd import Engine

    os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"] = str(knob), str(knob2)
    try:
        return Engine(0)
    finally:
        del os.environ["KMZ_ABLATE"], os.environ["KMZ_ABLATE2"]


def test_compact_key_staging_equals_wide_keys():
    """Direct enumeration's 4-byte staged keys (x38 residuals below the slice
    bits, kmz_common.h) and its 8-byte keys give the same edge set and
    endpoints on config 5, equal to the C oracle's keys."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    def run(e):
        e.load_synthetic(5, synth.SEED, 0, 20000)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        return e.triples(), e.endpoints(), e.info()

    out = []
    for knob2 in (BIG_EDGE_SET, BIG_EDGE_SET | WIDE_KEYS):
        e = _engine_with2(1 << 28, knob2)
        try:
            for _ in range(2):
                r = run(e)
            assert r[2]["path"] & 4  # direct enumeration
            out.append(r)
        finally:
            e.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1].tobytes() == out[1][1].tobytes()
    batch, _ = synth.host_batch(5, 0, 20000)
    table = synth.shape_table(5)
    keys, _, _ = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    assert np.array_equal(np.sort(out[0][0]), np.sort(keys))


def test_compact_staging_with_distances_past_32():
    """A 40-deep SERVER/CLIENT chain inside one LDS window: direct enumeration
    with compact staging inserts its keys of distance >= 32 in place (they have
    no 38-bit code); the rows equal the oracle's, order-exact."""
    from kmamiz_amd import Traces

    front = [_deep_span(100000, "SERVER", None, "front")]
    deep = _deep_trace(40)
    e = _engine_with2(1 << 28, BIG_EDGE_SET)
    try:
        got = Traces([front, deep], engine=e).toEndpointDependencies().toJSON()
        assert e.info()["path"] & 4
    finally:
        e.close()
    assert got == O.strip_undef(O.Traces([front, deep]).toEndpointDependencies(max_depth=10000).toJSON())


K3_FIXED_SLICES = 1 << 14  # KMZ_ABLATE: K3 reduce with S fixed slices per partition (no record-balanced items)
K3_UNPACKED = 1 << 15      # KMZ_ABLATE: the balanced K3 reduce with unpacked accumulators in every item


@pytest.mark.parametrize("config,ntr", [(5, 20000), (3, 40000)])
def test_k3_reduce_variants_equal(engine, config, ntr):
    """The record-balanced K3 reduce (items sized by each partition's records:
    config 5's hot partitions hold ~6x the mean), the fixed-slice reduce and
    the balanced one with unpacked accumulators give byte-identical group
    partials and groups, equal to the C oracle's combined groups."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from oracle import c_oracle

    def run(e):
        n = e.load_synthetic(config, synth.SEED, 0, ntr)
        e.run(L.RUN_STATS_TAG)
        gw = e.partials_words(L.PART_GROUPS)
        g = np.zeros(gw, np.uint64)
        e.export_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
        return n, g, e.groups()

    n, pa, ga = run(engine)
    assert n > 64 * 2048  # past the one-slice small-batch path
    for knob in (K3_FIXED_SLICES, K3_UNPACKED):
        e2 = _engine_with(knob)
        try:
            _, pb, gb = run(e2)
        finally:
            e2.close()
        assert pa.tobytes() == pb.tobytes(), knob
        assert ga.tobytes() == gb.tobytes(), knob
    batch, _ = synth.host_batch(config, 0, ntr)
    table = synth.shape_table(config)
    ref = c_oracle.stats(batch, table.tag_ep, table.n_tag_ep, table.n_status)
    assert np.array_equal(ga["combined"], ref["combined"])
    used = ref["combined"] > 0
    assert np.array_equal(ga["first"][used], ref["first"][used])
    assert np.array_equal(ga["latest_timestamp"][used], ref["latest_timestamp"][used])
    np.testing.assert_allclose(ga["mean"][used], ref["mean"][used], rtol=REL, atol=0)


@pytest.fixture(scope="module")
def direct_engine():
    """An engine whose K4 always enumerates directly (KMZ_ABLATE bit 28: every
    row stages all its keys, no chain table)."""
    e = _engine_with(1 << 28)
    yield e
    e.close()


@pytest.mark.parametrize("config,ntr", [(2, 30000), (3, 4000), (3, 40000), (5, 2000), (5, 20000)])
def test_direct_enumeration_vs_c_oracle(direct_engine, config, ntr):
    from kmamiz_amd import synth

    batch, off = synth.host_batch(config, 0, ntr)
    for _ in range(2):  # the second run reuses the edge set, buckets and staging
        info = _compare_synth(direct_engine, batch, synth.shape_table(config))
        assert info["path"] & 4 and info["n_chains"] == 0


@pytest.mark.parametrize("seed", range(0, 40, 3))
def test_direct_enumeration_messy_batches(direct_engine, seed):
    test_messy_batches_vs_oracle(direct_engine, seed)


def test_direct_enumeration_deep_chain(direct_engine):
    test_deep_chain_takes_the_pending_path(direct_engine)


def test_k4_mode_follows_chain_reuse(engine):
    """Auto mode: config 5 (most rows start a new chain) switches to direct
    enumeration after an interning run; config 3 (chains repeat; a small
    batch) stays interning.  The graph is the same either way."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    e = _engine_with(0)
    try:
        for config, ntr, want in ((5, 20000, 4), (3, 20000, 0)):
            e.load_synthetic(config, synth.SEED, 0, ntr)
            runs = []
            for _ in range(3):
                e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
                runs.append((e.triples(), e.endpoints(), e.info()))
            # (the first kmz_run interns; a retry inside it -- the edge set
            # grown -- may already enumerate)
            assert runs[1][2]["path"] & 4 == want and runs[2][2]["path"] & 4 == want
            assert (runs[2][2]["n_chains"] > 0) == (want == 0)
            for t, ep, _ in runs[1:]:
                assert np.array_equal(t, runs[0][0]) and ep.tobytes() == runs[0][1].tobytes()
    finally:
        e.close()


@pytest.mark.parametrize("seed", range(6))
def test_side_stream_run_equals_separate_runs(engine, seed):
    """A stats + dependency run of a small batch uses the side stream (K3 and
    the certificate beside the join and the walk); with repeated span ids the
    certificate fails and the run is redone on the table path.  Either way the
    results equal a stats-only run followed by a dependency-only run (both
    serial)."""
    from kmamiz_amd import CycleError
    from kmamiz_amd import _lib as L
    from kmamiz_amd.ingest import ingest_traces

    rng = random.Random(1000 + seed)
    traces = messy_batch(rng, 60, rng.choice([8, 64, 4096]))
    batch, d, _ = ingest_traces(traces)
    engine.load(batch, d.shape_table())
    engine._loaded_token = None
    try:
        engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    except CycleError:
        return
    g1, k1, e1 = engine.groups(), engine.triples(), engine.endpoints()
    engine.run(L.RUN_STATS_TAG)
    g2 = engine.groups()
    engine.run(L.RUN_DEPS)
    k2, e2 = engine.triples(), engine.endpoints()
    assert g1.tobytes() == g2.tobytes()
    assert np.array_equal(k1, k2)
    assert e1.tobytes() == e2.tobytes()


def test_certificate_at_scale_finds_one_repeated_id(engine):
    """At 10^7 spans the certificate has 4096 sub-bins, more than the
    persistent check kernel has workgroups, so each workgroup checks many
    sub-bins over one LDS set.  A clean batch must pass (window path); the
    same batch with one span id repeated far away must fail it and take the
    table path, with the reference's duplicate-id semantics."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(3, 0, 370000)
    assert len(batch) > 10_000_000
    table = synth.shape_table(3)
    engine.load(batch, table)
    engine._loaded_token = None
    engine.run(L.RUN_DEPS)
    info = engine.info()
    assert info["path"] & 1 and info["n_dups"] == 0
    rng = np.random.default_rng(7)
    for _ in range(5):  # one repeated id at a time, in different sub-bins
        i, j = int(rng.integers(0, len(batch) // 2)), int(rng.integers(len(batch) // 2, len(batch)))
        keep = batch.span_id[j].copy()
        batch.span_id[j] = batch.span_id[i]
        engine.load(batch, table)
        engine._loaded_token = None
        engine.run(L.RUN_DEPS)
        info = engine.info()
        batch.span_id[j] = keep
        assert not (info["path"] & 1), "the certificate missed a repeated span id"
        assert info["n_dups"] == 1


@pytest.mark.parametrize("pattern", ["sequential", "strided", "high"])
def test_structured_span_ids_pass_the_certificate(engine, pattern):
    """Span ids with structure (1, 2, 3, ... or multiples of 2^20) must spread
    over the certificate's bins, sub-bins and check buckets like random ones:
    the window path holds (no overflow into the table path) and the results
    equal the C oracle.  Ids that vary only in their top bits (multiples of
    2^43) may overflow the check's buckets: then the exact table path runs,
    with the same results."""
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(3, 0, 40000)
    n = len(batch)
    order = np.argsort(batch.span_id, kind="stable")
    shift = {"sequential": 0, "strided": 20, "high": 43}[pattern]
    new = np.arange(1, n + 1, dtype=np.uint64) << np.uint64(shift)
    remap = np.empty(n, dtype=np.uint64)
    remap[order] = new
    pos = np.searchsorted(batch.span_id, batch.parent_id, sorter=order)
    pos = np.minimum(pos, n - 1)
    found = (batch.parent_id != 0) & (batch.span_id[order[pos]] == batch.parent_id)
    batch.parent_id[:] = np.where(found, remap[order[pos]], batch.parent_id)
    batch.span_id[:] = remap
    info = _compare_synth(engine, batch, synth.shape_table(3))
    assert info["n_dups"] == 0
    if pattern != "high":
        assert info["path"] & 1


def test_certificate_massively_repeated_id(engine):
    """One span id repeated 70 000 times puts more than 2^16 ids into one
    certificate sub-bin (far past its capacity): the certificate must fail
    (never a silent window answer) and the run must equal the C oracle on the
    table path."""
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(3, 0, 40000)
    rng = np.random.default_rng(5)
    # leaves (span ids no one points at), so that every parent stays resolvable
    parents = set(int(p) for p in batch.parent_id if p)
    cand = np.array([i for i in range(len(batch)) if int(batch.span_id[i]) not in parents])
    sel = rng.choice(cand, 70000, replace=False)
    batch.span_id[sel] = batch.span_id[sel[0]]
    info = _compare_synth(engine, batch, synth.shape_table(3))
    assert not (info["path"] & 1)
    assert info["n_dups"] > 0


def _ids_of_hashes(h):
    """Span ids whose kmz_common.h id_hash are the given uint64 values (its
    inverse: undo the xorshift by 29, then the odd multiplier)."""
    h = np.asarray(h, dtype=np.uint64)
    x = h ^ (h >> np.uint64(29)) ^ (h >> np.uint64(58))
    return x * np.uint64(pow(0x9E3779B97F4A7C15, -1, 1 << 64))


@pytest.mark.parametrize("group", [2, 12])
def test_certificate_fingerprint_collisions_are_not_repeats(engine, group):
    """The check compares 19-bit fingerprints of the ids in one bucket and
    reads the ids back only on a fingerprint hit.  Groups of distinct ids
    whose hashes agree on every bit but one in the middle (same sub-bin,
    bucket and fingerprint) must pass the certificate; with 12 a group also
    overflows its bucket's 8 slots.  Then one group with a real repeat fails
    it."""
    from kmamiz_amd import synth
    from kmamiz_amd import dist as kdist

    batch, _ = synth.host_batch(3, 0, 40000)
    parents = set(int(p) for p in batch.parent_id if p)
    cand = np.array([i for i in range(len(batch)) if int(batch.span_id[i]) not in parents])
    rng = np.random.default_rng(11 + group)
    sel = rng.choice(cand, 600 - 600 % group, replace=False).reshape(-1, group)
    base = rng.integers(1, 1 << 63, size=len(sel), dtype=np.uint64)
    for g, b in zip(sel, base):
        hs = b ^ (np.arange(group, dtype=np.uint64) << np.uint64(32))  # bits 32..35: outside every field
        batch.span_id[g] = _ids_of_hashes(hs)
    assert np.array_equal(kdist.id_hash_np(batch.span_id[sel[0]]), base[0] ^ (np.arange(group, dtype=np.uint64) << np.uint64(32)))
    assert len(np.unique(batch.span_id)) == len(batch)
    info = _compare_synth(engine, batch, synth.shape_table(3))
    assert info["path"] & 1 and info["n_dups"] == 0
    batch.span_id[sel[3][-1]] = batch.span_id[sel[3][0]]
    engine._loaded_token = None
    info = _compare_synth(engine, batch, synth.shape_table(3))
    assert not (info["path"] & 1)
    assert info["n_dups"] == 1


# ---------------------------------------------------------------------------
# traceId sharding: device shard generation + index map
# ---------------------------------------------------------------------------
def _host_shard(config, t0, t1, world, rank):
    """The traces of [t0, t1) with kmz_trace_shard(traceId) == rank, generated
    on the host, with the index-map runs of their global positions."""
    from kmamiz_amd import SpanBatch, synth
    from kmamiz_amd.shard import trace_shard

    batch, off = synth.host_batch(config, t0, t1)
    sel, ls, gs, loc = [], [], [], 0
    for t in range(t1 - t0):
        if trace_shard(f"{(t0 + t) * 0x9E3779B97F4A7C15 % (1 << 128):032x}", world) != rank:
            continue
        a, b = int(off[t]), int(off[t + 1])
        sel.append(np.arange(a, b))
        ls.append(loc)
        gs.append(batch.index_base + a)
        loc += b - a
    idx = np.concatenate(sel) if sel else np.zeros(0, np.int64)
    cols = {f: getattr(batch, f)[idx] for f in ("span_id", "parent_id", "kind", "shape", "status", "duration",
                                                 "timestamp")}
    return SpanBatch(index_base=0, **cols), np.array(ls or [0], np.uint64), np.array(gs or [0], np.uint64)


@pytest.mark.parametrize("config,t0,t1,world", [(3, 0, 3000, 3), (5, 7, 1500, 2), (2, 0, 20000, 4)])
def test_shard_generation_and_index_map(engine, config, t0, t1, world):
    """kmz_synth_load_shard == the host selection of the same traces through
    kmz_set_index_map; the shards' partials, summed / max'ed / min'ed as
    merge_all does, finalise to the single run over [t0, t1) bit for bit."""
    from kmamiz_amd import Engine, synth
    from kmamiz_amd import _lib as L

    table = synth.shape_table(config)
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    parts = []
    total = 0
    for rank in range(world):
        n = engine.load_synthetic_shard(config, synth.SEED, t0, t1, world, rank)
        engine.run(flags)
        dev = engine.fetch()
        dev = (dev[0].copy(), np.sort(dev[1]), dev[2])
        hb, ls, gs = _host_shard(config, t0, t1, world, rank)
        assert n == len(hb)
        total += n
        engine.load(hb, table)
        engine.set_index_map(ls, gs)
        engine.run(flags)
        host = engine.fetch()
        host = (host[0].copy(), host[1].copy(), host[2].copy())
        _check_fetch_used(engine, host)  # (the compacted groups remapped to global indices too)
        assert dev[0].tobytes() == host[0].tobytes()
        assert np.array_equal(dev[1], np.sort(host[1]))
        assert dev[2].tobytes() == host[2].tobytes()
        gw, ew, tw = (engine.partials_words(w) for w in (L.PART_GROUPS, L.PART_ENDPOINTS, L.PART_TRIPLES))
        g, e, k = np.zeros(gw, np.uint64), np.zeros(ew, np.uint64), np.zeros(max(1, tw), np.uint64)
        engine.export_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
        engine.export_partials(L.PART_ENDPOINTS, e.ctypes.data, ew, False)
        engine.export_partials(L.PART_TRIPLES, k.ctypes.data, tw, False)
        parts.append((g, e, k[:tw]))
    G, E = len(parts[0][0]) // 6, len(parts[0][1]) // 2
    g = parts[0][0].copy()
    e = parts[0][1].copy()
    for pg, pe, _ in parts[1:]:
        g[: 4 * G] += pg[: 4 * G]
        g[4 * G: 5 * G] = np.maximum(g[4 * G: 5 * G], pg[4 * G: 5 * G])
        g[5 * G:] = np.minimum(g[5 * G:], pg[5 * G:])
        e[:E] = np.maximum(e[:E], pe[:E])
        e[E:] = np.minimum(e[E:], pe[E:])
    keys = np.unique(np.concatenate([k for _, _, k in parts]))
    n = engine.load_synthetic(config, synth.SEED, t0, t1)
    assert n == total
    engine.run(flags)
    whole = engine.fetch()
    assert np.array_equal(np.sort(whole[1]), keys)
    gw, ew = engine.partials_words(L.PART_GROUPS), engine.partials_words(L.PART_ENDPOINTS)
    wg, we = np.zeros(gw, np.uint64), np.zeros(ew, np.uint64)
    engine.export_partials(L.PART_GROUPS, wg.ctypes.data, gw, False)
    engine.export_partials(L.PART_ENDPOINTS, we.ctypes.data, ew, False)
    assert np.array_equal(canon_limbs(wg), canon_limbs(g))
    assert np.array_equal(we, e)


def _check_fetch_used(engine, dense):
    """kmz_fetch_used == the dense fetch's used groups (ascending ids), the
    same edge keys and endpoints."""
    g, t, e = dense
    ids, gu, tu, eu = engine.fetch_used()
    used = np.nonzero(g["combined"] > 0)[0]
    assert np.array_equal(ids.astype(np.int64), used)
    assert gu.tobytes() == g[used].tobytes()
    assert np.array_equal(np.sort(tu), np.sort(t))
    assert eu.tobytes() == e.tobytes()


@pytest.mark.parametrize("config,ntr", [(2, 2500), (3, 2500), (5, 2500), (3, 40000), (5, 20000), (3, 370000)])
def test_fetch_used_equals_dense_fetch(engine, config, ntr):
    """The used groups compacted on the device (k_finalize's per-chunk counts
    + k_used_scatter) after a run, and again after kmz_finalize (the merge
    path, whose count is read from the device)."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    engine.load_synthetic(config, synth.SEED, 0, ntr)
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    d = engine.fetch()
    d = (d[0].copy(), d[1].copy(), d[2].copy())
    assert (d[0]["combined"] > 0).sum() > 0
    _check_fetch_used(engine, d)
    gw = engine.partials_words(L.PART_GROUPS)
    g = np.zeros(gw, np.uint64)
    engine.export_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
    g[: gw // 6] = 0  # every group unused but those set again below: the compaction follows the import
    g[0] = 3
    engine.import_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
    engine.finalize()
    d2 = engine.fetch()
    d2 = (d2[0].copy(), d2[1].copy(), d2[2].copy())
    assert (d2[0]["combined"] > 0).sum() == 1
    _check_fetch_used(engine, d2)


def canon_limbs(g):
    """Group partials with their sum of squared durations in canonical limbs
    (S2 = s2a + 2^32 s2b, s2a < 2^32): summed partials (a merge) may carry
    low-limb sums past 2^32, which finalise to the same S2."""
    G = len(g) // 6
    g = g.copy()
    a = g[2 * G: 3 * G].copy()
    g[2 * G: 3 * G] = a & np.uint64(0xFFFFFFFF)
    g[3 * G: 4 * G] += a >> np.uint64(32)
    return g


def test_headline_size_config3_properties(engine):
    """Config 3 at its BASELINE size (1e8 spans, beyond the oracle): every
    SERVER span is one row and one group member; a second run is byte-equal;
    the edge set / groups / endpoints equal the merge of two traceId shards of
    the same batch (kmz_synth_load_shard + the index map)."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    ntr = 3657845  # bench.py's config-3 batch (100 071 364 spans)
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    n = engine.load_synthetic(3, synth.SEED, 0, ntr)
    assert n > 1e8
    engine.run(flags)
    i1 = engine.info()
    g1, k1, e1 = (x.copy() for x in engine.fetch())
    k1.sort()
    assert int(g1["combined"].sum()) == i1["n_server"] == i1["n_rows"]
    assert i1["n_dups"] == 0 and i1["max_depth"] == 7  # 8 levels: 7 hops to the root service
    # every endpoint with a row is first used by its first row; external rows are roots' children
    assert np.all(e1["first_row"][e1["has_row"] == 1] < n)
    engine.run(flags)
    g2, k2, e2 = engine.fetch()
    assert g2.tobytes() == g1.tobytes() and e2.tobytes() == e1.tobytes()
    assert np.array_equal(np.sort(k2), k1)
    # two shards by traceId, merged as merge_all does
    G = len(g1)
    parts = []
    for rank in range(2):
        engine.load_synthetic_shard(3, synth.SEED, 0, ntr, 2, rank)
        engine.run(flags)
        gw, ew, tw = (engine.partials_words(w) for w in (L.PART_GROUPS, L.PART_ENDPOINTS, L.PART_TRIPLES))
        g, e, k = np.zeros(gw, np.uint64), np.zeros(ew, np.uint64), np.zeros(max(1, tw), np.uint64)
        engine.export_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
        engine.export_partials(L.PART_ENDPOINTS, e.ctypes.data, ew, False)
        engine.export_partials(L.PART_TRIPLES, k.ctypes.data, tw, False)
        parts.append((g, e, k[:tw]))
    (ga, ea, ka), (gb, eb, kb) = parts
    E = len(ea) // 2
    g = np.concatenate([ga[:4 * G] + gb[:4 * G], np.maximum(ga[4 * G:5 * G], gb[4 * G:5 * G]),
                        np.minimum(ga[5 * G:], gb[5 * G:])])
    e = np.concatenate([np.maximum(ea[:E], eb[:E]), np.minimum(ea[E:], eb[E:])])
    from kmamiz_amd import finalize_host

    assert finalize_host(g, G).tobytes() == g1.tobytes()
    assert np.array_equal(e[E:] >> np.uint64(1), np.where(e1["has_row"] == 1, e1["first_row"], e[E:] >> np.uint64(1)))
    assert np.array_equal(np.union1d(ka, kb), k1)


def test_config4_size_on_one_gpu():
    """Config 4's whole batch (1e9 mesh spans, 35 GB of columns) on one GPU:
    one pass, then the same traces as 8 traceId shards (kmz_synth_load_shard,
    SURVEY.md 8e: shard = h(traceId) mod 8) merged with merge_all's
    arithmetic (sums of the integer moments, max timestamps, min first
    indices, the union of the edge keys).  Groups, endpoints and edge keys
    must be bit-identical; every SERVER span is one row and one group member
    (the bulk batch of Initializer.ts:40-101, at 10^4 x its 10^5 traces)."""
    from kmamiz_amd import Engine, finalize_host
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    ntr = 36578450  # bench.py --spans 1e9
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    eng = Engine(0)
    try:
        n = eng.load_synthetic(3, synth.SEED, 0, ntr)
        assert n > 9.9e8
        eng.run(flags)
        i1 = eng.info()
        g1, k1, e1 = (x.copy() for x in eng.fetch())
        k1.sort()
        assert int(g1["combined"].sum()) == i1["n_server"] == i1["n_rows"]
        assert i1["n_dups"] == 0 and i1["max_depth"] == 7 and i1["path"] & 3 == 3
        assert np.all(e1["first_row"][e1["has_row"] == 1] < n)
        G = len(g1)
        world = 8
        acc = None
        keys = []
        n_sum = 0
        for rank in range(world):
            n_sum += eng.load_synthetic_shard(3, synth.SEED, 0, ntr, world, rank)
            eng.run(flags)
            gw, ew, tw = (eng.partials_words(w) for w in (L.PART_GROUPS, L.PART_ENDPOINTS, L.PART_TRIPLES))
            g, e, k = np.zeros(gw, np.uint64), np.zeros(ew, np.uint64), np.zeros(max(1, tw), np.uint64)
            eng.export_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
            eng.export_partials(L.PART_ENDPOINTS, e.ctypes.data, ew, False)
            eng.export_partials(L.PART_TRIPLES, k.ctypes.data, tw, False)
            keys.append(k[:tw])
            if acc is None:
                acc = [g, e]
                continue
            ga, ea = acc
            E = len(ea) // 2
            acc = [np.concatenate([ga[:4 * G] + g[:4 * G], np.maximum(ga[4 * G:5 * G], g[4 * G:5 * G]),
                                   np.minimum(ga[5 * G:], g[5 * G:])]),
                   np.concatenate([np.maximum(ea[:E], e[:E]), np.minimum(ea[E:], e[E:])])]
    finally:
        eng.close()
    assert n_sum == n
    g, e = acc
    E = len(e) // 2
    assert finalize_host(g, G).tobytes() == g1.tobytes()
    assert np.array_equal(e[E:] >> np.uint64(1), np.where(e1["has_row"] == 1, e1["first_row"], e[E:] >> np.uint64(1)))
    assert np.array_equal((e[:E] ^ np.uint64(1 << 63)).view(np.int64)[e1["has_row"] == 1],
                          e1["last_ts"][e1["has_row"] == 1])
    assert np.array_equal(np.unique(np.concatenate(keys)), k1)


def test_headline_config5_vs_c_oracle_and_tail():
    """Config 5 at 1e7 spans: groups, edges and endpoints vs the C oracle, and
    the service tail kernel vs the numpy restatement over the ORACLE's edge
    keys and endpoint records (so the tail is pinned to the oracle at scale)."""
    from test_tail import _tail_np

    from kmamiz_amd import Engine, synth
    from kmamiz_amd.tail import maps_for_synth, run_tail

    batch, _ = synth.host_batch(5, 0, 175000)
    assert len(batch) > 9.9e6
    table = synth.shape_table(5)
    e = Engine(0)
    try:
        odeps = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
        okeys, oep, _ = odeps
        _compare_synth(e, batch, table, odeps)  # groups / edges / endpoints vs the C oracle
        maps = maps_for_synth(5)
        tail = run_tail(e, maps, e.endpoints())
        first = np.where(oep["has_row"], oep["first"], np.iinfo(np.uint64).max).astype(np.uint64)
        ref = _tail_np(okeys, maps, oep["has_row"], first)
        for f in tail.details.dtype.names:
            assert np.array_equal(tail.details[f], ref.details[f]), f
        for f in tail.pairs.dtype.names:
            assert np.array_equal(tail.pairs[f], ref.pairs[f]), f
        assert np.array_equal(tail.gateway, ref.gateway)
        assert np.array_equal(tail.total, ref.total)
        # (columns 6 / 7 are the device's per-service rows and gateway flag,
        # compared above as total / gateway; the restatement derives those
        # from the endpoint records instead)
        assert np.array_equal(tail.stats[:, :6], ref.stats[:, :6])
        assert tail.instability() == ref.instability()
        assert tail.coupling() == ref.coupling()
        mt, mr = tail.metrics(), ref.metrics()
        for k in mt:
            np.testing.assert_allclose(np.asarray(mt[k], dtype=float), np.asarray(mr[k], dtype=float), rtol=REL)
    finally:
        e.close()


# ---------------------------------------------------------------------------
# hipGraph replay of small-batch runs (kmz_api.hip run_enqueue_graphed)
# ---------------------------------------------------------------------------
GRAPH_OFF = 1 << 23  # KMZ_ABLATE2: no run graphs (KMZ_HIPGRAPH=0)


def _run_results(e, flags):
    e.run(flags)
    g, k, ep = e.fetch()
    return g.tobytes(), np.sort(k).tobytes(), ep.tobytes(), _info_results(e.info())


@pytest.mark.parametrize("config,ntr", [(2, 2500), (3, 2500), (5, 2500), (5, 40000)])
def test_graph_replay_equals_direct_runs(config, ntr):
    """Production-tick batches (2 500 traces, RealtimeWorkerImpl.ts:31-35):
    runs replayed from a captured hipGraph give the results of runs enqueued
    one launch at a time, run after run, also when the loaded data change
    under the same launch sequence (same size, other durations / timestamps)."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(config, 0, ntr)
    table = synth.shape_table(config)
    other = batch.__class__(**{f: (lambda v: v.copy() if isinstance(v, np.ndarray) else v)(getattr(batch, f))
                               for f in batch.__dataclass_fields__})
    other.duration = other.duration[::-1].copy()
    other.timestamp = other.timestamp + 7
    on, off = _engine_with(0), _engine_with2(0, GRAPH_OFF)  # (graphs on by default)
    try:
        for flags in (L.RUN_STATS_TAG | L.RUN_DEPS, L.RUN_STATS_RT | L.RUN_DEPS | L.RUN_SPAN_LINKS):
            for b in (batch, other, batch):
                on.load(b, table)
                off.load(b, table)
                exp = _run_results(off, flags)
                for _ in range(4):
                    assert _run_results(on, flags) == exp
        assert on.graph_stats()[0] > 0 and off.graph_stats() == (0, 0)
    finally:
        on.close()
        off.close()


def test_pipelined_fetch_equals_fetch(engine):
    """kmz_fetch_begin / _end (bench.py's loop: one batch's results cross PCIe
    while the next batch's kernels run) return what kmz_fetch returns for each
    batch, although the next run overwrites the device results before _end."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    ranges = ((0, 3000), (3000, 5200))
    want = []
    for a, b in ranges:
        engine.load_synthetic(synth.MESH, synth.SEED, a, b)
        engine.run(flags)
        g, k, e = engine.fetch()
        want.append((g.copy(), np.sort(k), e.copy()))
    assert want[0][0].tobytes() != want[1][0].tobytes()
    engine.load_synthetic(synth.MESH, synth.SEED, *ranges[0])
    engine.run(flags)
    engine.fetch_begin()
    engine.load_synthetic(synth.MESH, synth.SEED, *ranges[1])
    engine.run(flags)  # (overwrites the first batch's device results)

    def same(got, i):
        g, k, e = got
        wg, wk, we = want[i]
        assert g.tobytes() == wg.tobytes()
        assert np.array_equal(np.sort(k), wk)
        assert e.tobytes() == we.tobytes()

    same(engine.fetch_end(), 0)
    first = engine.fetch_begin()
    engine.run(flags)  # a run while the second batch's copies are in flight
    engine.fetch_begin()  # (a _begin ends the open fetch first)
    same(first, 1)
    same(engine.fetch_end(), 1)
    assert engine.fetch_end() is None
    # without keys (the service tail's fetch) and without deps
    engine.fetch_begin(keys=False)
    g, k, e = engine.fetch_end()
    assert k is None and g.tobytes() == want[1][0].tobytes() and e.tobytes() == want[1][2].tobytes()


def test_run_begin_end_equals_run(engine):
    """kmz_run_begin / _end (host work between the two overlaps the run's
    kernels) give kmz_run's results; any other call while the run is open is
    refused, and so is an _end without a _begin."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    engine.load_synthetic(synth.MESH, synth.SEED, 0, 4000)
    engine.run(flags)
    g, k, e = engine.fetch()
    want = (g.copy(), np.sort(k), e.copy(), engine.info())
    engine.run_begin(flags)
    with pytest.raises(Exception, match="run is open"):
        engine.info()
    with pytest.raises(Exception, match="run is open"):
        engine.fetch()
    with pytest.raises(Exception):
        engine.run_begin(flags)
    engine.run_end()
    g, k, e = engine.fetch()
    assert g.tobytes() == want[0].tobytes() and np.array_equal(np.sort(k), want[1]) and e.tobytes() == want[2].tobytes()
    assert engine.info() == want[3]
    with pytest.raises(Exception, match="without kmz_run_begin"):
        engine.run_end()


def test_fetch_begin_pageable_and_runtime_copies(engine):
    """kmz_fetch_begin into pageable host arrays (the runtime's copies, not
    k_copy_out's pinned path) returns kmz_fetch's result sets."""
    import ctypes as C

    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    engine.load_synthetic(synth.MESH, synth.SEED, 100, 2600)
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    wg, wk, we = engine.fetch()
    wg, wk, we = wg.copy(), np.sort(wk), we.copy()
    g = np.empty(len(wg), dtype=L.GROUP_DTYPE)
    k = np.empty(len(wk), dtype=np.uint64)
    e = np.empty(len(we), dtype=L.ENDPOINT_DTYPE)
    n = C.c_uint64()
    lib = L.lib()
    L.check(engine.ctx, lib.kmz_fetch_begin(engine.ctx, L.ptr(g), len(g), L.ptr(k), len(k), C.byref(n), L.ptr(e),
                                            len(e)))
    L.check(engine.ctx, lib.kmz_fetch_end(engine.ctx))
    assert n.value == len(wk)
    assert g.tobytes() == wg.tobytes() and np.array_equal(np.sort(k), wk) and e.tobytes() == we.tobytes()
