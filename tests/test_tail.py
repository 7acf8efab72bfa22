"""Service-level tail at scale: kmz_tail_run + the host
finish (kmamiz_amd/tail.py) against the Python oracle's tail over the reduced
form ``EndpointDependencies([]).combineWith(deps).trim()``
(EndpointDependencies.ts:369-657, RiskAnalyzer.ts:10-248).

* CPU: a numpy restatement of the kernel's reduction over the C oracle's edge
  keys feeds the same host finish (checks the edge-key -> link-detail algebra);
* GPU: the kernel through the C ABI, on the reference fixtures, synthetic
  configs 2/3/5, with and without a label map.
"""
import math

import numpy as np
import pytest

from conftest import fixture
from oracle import kmz_oracle as O

REL = 1e-9


def _oracle(traces, label_map=None, replicas=None):
    ref = O.Traces(traces)
    red = O.EndpointDependencies([]).combineWith(ref.toEndpointDependencies()).trim().toJSON()
    od = O.EndpointDependencies(O.strip_undef(red))
    if label_map is not None:
        od = O.EndpointDependencies(od.label(label_map))
    data = ref.toRealTimeData(replicas).toCombinedRealtimeData().toJSON()
    data = [d for d in O.strip_undef(data) if d.get("uniqueServiceName") is not None]
    risk = O.strip_undef(O.RiskAnalyzer.RealtimeRisk(data, od.toServiceDependencies(), replicas or []))
    return od, data, risk


def _compare(tail, od, data=None, risk=None):
    exp_i = od.toServiceInstability()
    assert tail.instability() == exp_i
    assert tail.coupling() == od.toServiceCoupling()
    got_c, exp_c = tail.cohesion(), od.toServiceEndpointCohesion()
    assert [c["uniqueServiceName"] for c in got_c] == [c["uniqueServiceName"] for c in exp_c]
    for g, e in zip(got_c, exp_c):
        assert g["totalEndpoints"] == e["totalEndpoints"]
        key = lambda c: c["uniqueServiceName"]  # noqa: E731
        assert sorted(g["consumers"], key=key) == sorted(e["consumers"], key=key)
        assert g["endpointUsageCohesion"] == pytest.approx(e["endpointUsageCohesion"], rel=REL)
    # relying factor / ACS through the compact service-deps form
    from kmamiz_amd import risk as R

    sd = od.toServiceDependencies()
    comp = tail.service_deps_compact()
    assert [s["uniqueServiceName"] for s in comp] == [s["uniqueServiceName"] for s in sd]
    assert R.absolute_criticality(comp) == R.absolute_criticality(sd)
    for a, b in zip(R.relying_factor(comp), R.relying_factor(sd)):
        assert a["uniqueServiceName"] == b["uniqueServiceName"]
        assert a["factor"] == pytest.approx(b["factor"], rel=REL)
    if risk is not None:
        from kmamiz_amd.tail import realtime_risk_arrays

        names = list(dict.fromkeys(d["uniqueServiceName"] for d in data))
        ids = {u: i for i, u in enumerate(names)}
        got = realtime_risk_arrays(tail, np.array([ids[d["uniqueServiceName"]] for d in data]), names,
                                   np.array([d["combined"] for d in data]),
                                   np.array([d["latency"]["cv"] for d in data]),
                                   np.array([str(d["status"]).startswith("5") for d in data]))
        assert [r["uniqueServiceName"] for r in got] == [r["uniqueServiceName"] for r in risk]
        for g, e in zip(got, risk):
            for k in ("risk", "impact", "probability", "norm"):
                assert (k in g) == (k in e)
                if k in g:
                    assert g[k] == pytest.approx(e[k], rel=REL, abs=1e-15), k


# ---------------------------------------------------------------------------
# CPU: numpy restatement of k_tail_links over the C oracle's edge keys
# ---------------------------------------------------------------------------
from oracle.tail_np import tail_np as _tail_np  # noqa: E402


@pytest.mark.parametrize("config,ntr", [(2, 300), (3, 120), (5, 150)])
def test_tail_restatement_vs_oracle_cpu(config, ntr):
    from kmamiz_amd import synth
    from kmamiz_amd.tail import maps_for_synth
    from oracle import c_oracle

    batch, off = synth.host_batch(config, 0, ntr)
    table = synth.shape_table(config)
    keys, oep, _ = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    first = np.where(oep["has_row"], oep["first"], np.iinfo(np.uint64).max).astype(np.uint64)
    tail = _tail_np(keys, maps_for_synth(config), oep["has_row"], first)
    od, data, risk = _oracle(synth.to_traces(config, batch, off))
    _compare(tail, od, data, risk)
    m = tail.metrics()
    coh = {c["uniqueServiceName"]: c for c in od.toServiceEndpointCohesion()}
    for i, c in enumerate(tail.coupling()):
        assert m["acs"][i] == c["acs"]
        assert m["cohesion"][i] == pytest.approx(coh[c["uniqueServiceName"]]["endpointUsageCohesion"], rel=REL)
    assert list(m["instability"]) == [x["instability"] for x in od.toServiceInstability()]


# ---------------------------------------------------------------------------
# GPU: the kernel through the C ABI
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("fx", ["MockTrace", "MockTracePDAS", "MockData2_traces"])
def test_tail_fixtures_gpu(engine, fx):
    from kmamiz_amd import Traces

    traces = fixture(fx)
    if fx != "MockTrace":
        traces = [traces]
    tail = Traces(traces, engine=engine).toEndpointDependencies().service_tail()
    od, data, risk = _oracle(traces)
    _compare(tail, od, data, risk)


@pytest.mark.gpu
@pytest.mark.parametrize("config,ntr", [(2, 2000), (3, 300), (5, 400)])
def test_tail_synthetic_gpu(engine, config, ntr):
    from kmamiz_amd import Traces, synth

    batch, off = synth.host_batch(config, 0, ntr)
    traces = synth.to_traces(config, batch, off)
    tail = Traces(traces, engine=engine).toEndpointDependencies().service_tail()
    od, data, risk = _oracle(traces)
    _compare(tail, od, data, risk)


@pytest.mark.gpu
def test_tail_label_map_gpu(engine):
    """Labels collapse or split link keys (EndpointDependencies.ts:419-421)."""
    from kmamiz_amd import Traces, synth

    batch, off = synth.host_batch(3, 0, 200)
    traces = synth.to_traces(3, batch, off)
    names = sorted({s["name"] for t in traces for s in t})
    deps = Traces(traces, engine=engine).toEndpointDependencies()
    lm = {}
    for r in deps.toJSON():
        u = r["endpoint"]["uniqueEndpointName"]
        lm.setdefault(u, "/api/L%d" % (len(lm) % 3))
    assert names
    tail = deps.service_tail(lm)
    od, _, _ = _oracle(traces, label_map=lm)
    _compare(tail, od)


@pytest.mark.gpu
def test_tail_full_size_matches_restatement(engine):
    """Config 5 at 2e6 spans on the device: the kernel equals the numpy
    restatement over the engine's own edge keys (a size the oracle cannot
    reach)."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.tail import maps_for_synth, run_tail

    engine.load_synthetic(5, synth.SEED, 0, 60000)
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    maps = maps_for_synth(5)
    ep = engine.endpoints()
    tail = run_tail(engine, maps, ep)
    ref = _tail_np(engine.triples(), maps, ep["has_row"], ep["first_row"])
    for f in tail.details.dtype.names:
        assert np.array_equal(tail.details[f], ref.details[f]), f
    for f in tail.pairs.dtype.names:
        assert np.array_equal(tail.pairs[f], ref.pairs[f]), f
    assert np.array_equal(tail.gateway, ref.gateway)
    # rows / gateway / first row per service: computed on the device (slots 6, 7
    # and kmz_tail_service_first) = derived on the host from the endpoints
    assert np.array_equal(tail.total, ref.total)
    assert np.array_equal(tail.services, ref.services)
    assert np.array_equal(tail.stats[:, :6], ref.stats[:, :6])
    nd = min(tail.by_dist.shape[1], ref.by_dist.shape[1])
    assert np.array_equal(tail.by_dist[:, :nd], ref.by_dist[:, :nd])
    assert not tail.by_dist[:, nd:].any() and not ref.by_dist[:, nd:].any()
    assert tail.instability() == ref.instability()
    assert tail.coupling() == ref.coupling()


def test_risk_arrays_row_order_free():
    """realtime_risk_arrays with ``first`` gives the same answer on shuffled rows."""
    from kmamiz_amd import synth
    from kmamiz_amd.tail import maps_for_synth, realtime_risk_arrays
    from oracle import c_oracle

    batch, off = synth.host_batch(5, 0, 150)
    table = synth.shape_table(5)
    keys, oep, _ = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    first = np.where(oep["has_row"], oep["first"], np.iinfo(np.uint64).max).astype(np.uint64)
    tail = _tail_np(keys, maps_for_synth(5), oep["has_row"], first)
    od, data, risk = _oracle(synth.to_traces(5, batch, off))
    names = list(dict.fromkeys(d["uniqueServiceName"] for d in data))
    ids = {u: i for i, u in enumerate(names)}
    perm = np.random.default_rng(1).permutation(len(data))
    rows = [data[i] for i in perm]
    got = realtime_risk_arrays(tail, np.array([ids[d["uniqueServiceName"]] for d in rows]), names,
                               np.array([d["combined"] for d in rows]), np.array([d["latency"]["cv"] for d in rows]),
                               np.array([str(d["status"]).startswith("5") for d in rows]),
                               first=perm.astype(np.uint64))
    assert [r["uniqueServiceName"] for r in got] == [r["uniqueServiceName"] for r in risk]
    for g, e in zip(got, risk):
        assert g["risk"] == pytest.approx(e["risk"], rel=REL, abs=1e-15)


@pytest.mark.gpu
def test_service_tail_reuses_the_dependency_run(engine):
    """service_tail() reads the edge set the dependency run left in HBM (no
    second kmz_run); after another run on the engine it runs the dependency
    pass again, with the same result."""
    from kmamiz_amd import Traces, synth

    batch, off = synth.host_batch(3, 0, 300)
    traces = synth.to_traces(3, batch, off)
    t = Traces(traces, engine=engine)
    deps = t.toEndpointDependencies()
    g = engine.gen
    a = deps.service_tail()
    assert engine.gen == g  # no run in between: reused
    t.toRealTimeData().toCombinedRealtimeData().toJSON()  # a stats run on the same engine
    assert engine.gen != g
    b = deps.service_tail()
    assert a.instability() == b.instability() and a.coupling() == b.coupling()
    assert a.cohesion() == b.cohesion()


def test_service_sums_grid_equals_row_sums():
    """service_sums_grid (the bench's per-endpoint pre-reduction over the group
    grid) = service_sums over the used rows: same service order, sums within
    1e-12 (reassociated), counts exact."""
    from kmamiz_amd.tail import service_sums, service_sums_grid

    rng = np.random.default_rng(7)
    n_ep, n_st, n_sid = 3000, 3, 97
    comb = rng.integers(0, 40, (n_ep, n_st)).astype(np.uint64)
    comb[rng.random((n_ep, n_st)) < 0.3] = 0
    cv = np.where(comb > 0, rng.random((n_ep, n_st)) * 2, 0.0)
    first = rng.permutation(n_ep * n_st).astype(np.uint64).reshape(n_ep, n_st)
    ep_sid = rng.integers(0, n_sid, n_ep)
    st5 = np.array([False, False, True])
    used = np.nonzero(comb.reshape(-1) > 0)[0]
    a = service_sums(ep_sid[used // n_st], n_sid, comb.reshape(-1)[used], cv.reshape(-1)[used], st5[used % n_st],
                     first.reshape(-1)[used])
    b = service_sums_grid(comb.reshape(-1), cv.reshape(-1), first.reshape(-1), st5, ep_sid, n_sid)
    assert np.array_equal(a[0], b[0])
    assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
    np.testing.assert_allclose(a[1], b[1], rtol=1e-12)


def _same(a, b):
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    return a == pytest.approx(b, rel=REL, abs=1e-15)


def test_risk_with_a_zero_count_service_follows_js():
    """A service whose combined rows all count 0: its latency CV metric and
    error rate are 0/0 = NaN in JS, Math.max/Math.min then give NaN, and
    `probability || MINIMUM_PROB` / `impact || 0` replace NaN
    (RiskAnalyzer.ts:10-49, 87-122; Normalizer.ts:17-64).  Both host paths
    (row dicts in risk.py, columns in tail.py) equal the oracle."""
    import math as _m  # noqa: F401

    from kmamiz_amd import risk as R
    from kmamiz_amd import synth
    from kmamiz_amd.tail import maps_for_synth, realtime_risk_arrays
    from oracle import c_oracle

    batch, off = synth.host_batch(5, 0, 150)
    table = synth.shape_table(5)
    keys, oep, _ = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
    first = np.where(oep["has_row"], oep["first"], np.iinfo(np.uint64).max).astype(np.uint64)
    tail = _tail_np(keys, maps_for_synth(5), oep["has_row"], first)
    od, data, _ = _oracle(synth.to_traces(5, batch, off))
    zero = data[len(data) // 2]["uniqueServiceName"]
    data = [dict(d, combined=0) if d["uniqueServiceName"] == zero else d for d in data]
    sdeps = od.toServiceDependencies()
    exp = O.strip_undef(O.RiskAnalyzer.RealtimeRisk(data, sdeps, []))
    assert any(isinstance(e["risk"], float) and math.isnan(e["risk"]) for e in exp) or any(
        e["uniqueServiceName"] == zero for e in exp)
    got_rows = R.realtime_risk(data, sdeps, [])
    names = list(dict.fromkeys(d["uniqueServiceName"] for d in data))
    ids = {u: i for i, u in enumerate(names)}
    got_cols = realtime_risk_arrays(tail, np.array([ids[d["uniqueServiceName"]] for d in data]), names,
                                    np.array([d["combined"] for d in data]),
                                    np.array([d["latency"]["cv"] for d in data]),
                                    np.array([str(d["status"]).startswith("5") for d in data]))
    for got in (got_rows, got_cols):
        assert [r["uniqueServiceName"] for r in got] == [r["uniqueServiceName"] for r in exp]
        for g, e in zip(got, exp):
            for k in ("risk", "impact", "probability", "norm"):
                assert (k in g) == (k in e), k
                if k in g:
                    assert _same(g[k], e[k]), (k, g[k], e[k])


@pytest.mark.gpu
def test_service_tail_after_a_json_parse_on_the_engine(engine):
    """kmz_json_parse overwrites the engine's columns and drops its run (also
    when it refuses the input); service_tail() must notice (Engine.gen) and
    run the dependency pass again instead of failing with KMZ_E_STATE."""
    import json

    from kmamiz_amd import Traces, synth

    batch, off = synth.host_batch(3, 0, 300)
    traces = synth.to_traces(3, batch, off)
    deps = Traces(traces, engine=engine).toEndpointDependencies()
    a = deps.service_tail()
    other, ooff = synth.host_batch(2, 0, 50)
    engine.json_parse(json.dumps(synth.to_traces(2, other, ooff)).encode())
    b = deps.service_tail()
    assert a.instability() == b.instability() and a.coupling() == b.coupling()
    engine.json_parse(b"not json")  # refused (E_UNSUPPORTED): still a new generation
    c = deps.service_tail()
    assert a.instability() == c.instability()


def _synth_service_map(config):
    """Per stats (tag) endpoint of a synthetic config: its service id (by
    uniqueServiceName) and the service names, as bench.py builds them."""
    from kmamiz_amd import synth
    from kmamiz_amd.ingest import SHAPE_TAGS, UNDEFINED, tag_identity

    n_shapes, n_status, _ = synth.describe(config)
    sid_of, names = {}, []
    sid = np.zeros(n_shapes, dtype=np.int64)
    for sh in range(n_shapes):
        name, tags = synth.shape_tags(config, sh)
        usn = tag_identity((name,) + tuple(tags.get(t, UNDEFINED) for t in SHAPE_TAGS))["uniqueServiceName"]
        sid[sh] = sid_of.setdefault(usn, len(names))
        if sid[sh] == len(names):
            names.append(usn)
    is5 = np.array([str(x).startswith("5") for x in synth.STATUSES[:n_status]], dtype=bool)
    return sid, names, is5


@pytest.mark.gpu
@pytest.mark.parametrize("config,ntr", [(5, 60000), (3, 3000), (2, 2000)])
def test_service_sums_on_device_equal_row_sums(engine, config, ntr):
    """kmz_service_sums (RiskAnalyzer.RealtimeRisk's per-service sums on the
    device) = tail.service_sums over the fetched used groups: same service
    order, counts exact, and sum(cv * combined) bit-equal (both add in
    ascending group order); the realtime risk from either is identical."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.tail import maps_for_synth, realtime_risk_from_sums, run_tail, service_sums

    sid, names, is5 = _synth_service_map(config)
    n_status = len(is5)
    engine.load_synthetic(config, synth.SEED, 0, ntr)
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    g = engine.groups()
    engine.set_service_map(sid, len(names), is5)
    dev = engine.service_sums()
    used = np.nonzero(g["combined"] > 0)[0]
    host = service_sums(sid[used // n_status], len(names), g["combined"][used], g["cv"][used], is5[used % n_status],
                        g["first"][used])
    assert np.array_equal(dev[0], host[0])
    for a, b in zip(dev[1:], host[1:]):
        assert a.tobytes() == b.tobytes()
    tail = run_tail(engine, maps_for_synth(config))
    ra = realtime_risk_from_sums(tail, names, *dev)
    rb = realtime_risk_from_sums(tail, names, *host)
    for k in ra:
        assert ra[k].tobytes() == rb[k].tobytes(), k


@pytest.mark.gpu
@pytest.mark.parametrize("config,ntr", [(5, 60000), (3, 3000)])
def test_tail_and_sums_in_halves_equal_the_synchronous_calls(engine, config, ntr):
    """kmz_tail_begin / _end and kmz_service_sums_begin / _end (the bench's
    order: both enqueued right after the run, the fetch in between, the next
    run begun before _end) give what kmz_tail_run and kmz_service_sums give:
    another (smaller) batch loaded and run behind the open tail does not
    reach it."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.tail import maps_for_synth, run_tail, tail_begin, tail_end

    sid, names, is5 = _synth_service_map(config)
    maps = maps_for_synth(config)
    engine.load_synthetic(config, synth.SEED, 0, ntr)
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    engine.set_service_map(sid, len(names), is5)
    a = run_tail(engine, maps)
    sa = engine.service_sums()
    tail_begin(engine, maps)
    engine.service_sums_begin()
    g, t, e = engine.fetch(keys=False)
    engine.load_synthetic(config, synth.SEED + 1, 0, ntr // 2)
    engine.run_begin(L.RUN_STATS_TAG | L.RUN_DEPS)
    b = tail_end(engine, maps)
    sb = engine.service_sums_end()
    engine.run_end()
    assert a.stats.tobytes() == b.stats.tobytes()
    assert a.by_dist.tobytes() == b.by_dist.tobytes()
    assert (a.n_details, a.n_pairs) == (b.n_details, b.n_pairs)
    for x, y in zip(sa, sb):
        assert x.tobytes() == y.tobytes()
    ma, mb = a.metrics(), b.metrics()
    assert ma.keys() == mb.keys()
    for k in ma:
        assert np.asarray(ma[k]).tobytes() == np.asarray(mb[k]).tobytes(), k
