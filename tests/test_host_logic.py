"""Host-side logic of the product (no GPU): ingest/identities, the tail views,
the cross-window merges; and the C oracle pinned against the Python oracle."""
import random

import numpy as np
import pytest

from conftest import fixture
from oracle import c_oracle
from oracle import kmz_oracle as O

URLS = [
    "http://example.com:8080/test/test",
    "https://192.168.1.1/test#123",
    "service.test.svc.cluster.local:80/test/endpoint",
    "reviews.book.svc.cluster.local:9080/*",
    "a.b.svc:1/x",
    "e.svc.cluster.local/q",
    "dsvc.ns3.svc:81/z",
    "istio-ingressgateway",
    "HTTP://UPPER:80/x",
    "x://",
    "",
    "::://a",
    "http://h:12a/b",
    "svc.svc.svc",
    "a\nb.svc.c",
]


@pytest.mark.parametrize("url", URLS)
@pytest.mark.parametrize("service", [False, True])
def test_explode_url_matches_oracle(url, service):
    from kmamiz_amd import ingest

    def norm(v):
        return [None if (x is O.UNDEF or x is ingest.UNDEFINED) else x for x in v]

    assert norm(ingest.explode_url(url, service)) == norm(O.explode_url(url, service))


def _traces_of(fx):
    t = fixture(fx)
    return t if fx == "MockTrace" else [t]


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_endpoint_info_matches_oracle(fx):
    from kmamiz_amd import Traces

    for tr in _traces_of(fx):
        for s in tr:
            assert Traces.ToEndpointInfo(s) == O.strip_undef(O.Traces.ToEndpointInfo(s))


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_ingest_identities(fx):
    """Per-shape identities equal the oracle's per-span strings."""
    from kmamiz_amd.ingest import ingest_traces

    traces = _traces_of(fx)
    batch, d, flat = ingest_traces(traces)
    rl = O.strip_undef(O.Traces(traces).toRealTimeData().toJSON())
    srv = [i for i, s in enumerate(flat) if s["kind"] == "SERVER"]
    for row, i in zip(rl, srv):
        f = d.shape_ident["rt"][batch.shape[i]].fields
        assert f["uniqueEndpointName"] == row["uniqueEndpointName"]
        assert d.ep_names["rt"][d.shape_ep["rt"][batch.shape[i]]] == row["uniqueEndpointName"]
    for i, s in enumerate(flat):
        assert int(batch.span_id[i]) == int(s["id"], 16)
        assert int(batch.duration[i]) == s["duration"]


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_c_oracle_matches_python_oracle(fx):
    """The C restatement (used at scale) agrees with the Python one (pinned by
    the reference fixtures) through the product ingest."""
    from kmamiz_amd.ingest import ingest_traces

    traces = _traces_of(fx)
    batch, d, flat = ingest_traces(traces)
    tab = d.shape_table()
    st = c_oracle.stats(batch, tab.tag_ep, tab.n_tag_ep, tab.n_status)
    exp = O.strip_undef(O.Traces(traces).combineLogsToRealtimeData([]).toCombinedRealtimeData().toJSON())
    used = np.nonzero(st["combined"])[0]
    got = sorted(
        (d.ep_names["tag"][g // tab.n_status], d.statuses[g % tab.n_status], int(st["combined"][g]),
         float(st["mean"][g]), float(st["cv"][g]), int(st["latest_timestamp"][g]))
        for g in used
    )
    want = sorted((c["uniqueEndpointName"], c["status"], c["combined"], c["latency"]["mean"], c["latency"]["cv"],
                   c["latestTimestamp"]) for c in exp)
    assert got == want
    keys, ep, cnt = c_oracle.deps(batch, tab.dep_ep, tab.n_dep_ep)
    deps = O.strip_undef(O.Traces(traces).toEndpointDependencies().toJSON())
    assert cnt["rows"] == len(deps)
    assert cnt["relations"] == sum(len(x["dependingBy"]) for x in deps)
    names = d.ep_names["dep"]
    triples = set()
    for x in deps:
        for b in x["dependingBy"]:
            triples.add((b["endpoint"]["uniqueEndpointName"], x["endpoint"]["uniqueEndpointName"], b["distance"]))
    got_t = {(names[int(k >> 40)], names[int((k >> 16) & 0xFFFFFF)], int((k >> 1) & 0x7FFF)) for k in keys.tolist()}
    assert got_t == triples
    for x in deps:
        e = names.index(x["endpoint"]["uniqueEndpointName"])
        assert ep["last"][e] == x["lastUsageTimestamp"]


def test_product_combine_with_matches_oracle():
    from kmamiz_amd import CombinedRealtimeDataList

    a, b = fixture("MockBaseCrlData1"), fixture("MockBaseCrlData2")
    got = CombinedRealtimeDataList([dict(x) for x in a]).combineWith(CombinedRealtimeDataList([dict(x) for x in b]))
    exp = O.CombinedRealtimeDataList([dict(x) for x in a]).combineWith(O.CombinedRealtimeDataList([dict(x) for x in b]))
    g, e = got.toJSON()[0], O.strip_undef(exp.toJSON())[0]
    assert g == e


def test_product_combine_with_random():
    from kmamiz_amd import CombinedRealtimeDataList

    rng = random.Random(3)
    for _ in range(50):
        def rows():
            return [
                {"uniqueEndpointName": f"s\tn\tv\tGET\t/{rng.randint(0, 3)}", "uniqueServiceName": "s\tn\tv",
                 "status": rng.choice(["200", "500"]), "combined": rng.randint(1, 50),
                 "latestTimestamp": rng.randint(0, 10**9), "avgReplica": rng.choice([1, 2, None]),
                 "latency": {"mean": rng.uniform(0.01, 5000), "cv": rng.uniform(0, 3)}}
                for _ in range(rng.randint(0, 6))
            ]
        a, b = rows(), rows()
        for r in a + b:
            if r["avgReplica"] is None:
                del r["avgReplica"]
        import copy

        got = CombinedRealtimeDataList(copy.deepcopy(a)).combineWith(CombinedRealtimeDataList(copy.deepcopy(b)))
        exp = O.CombinedRealtimeDataList(copy.deepcopy(a)).combineWith(O.CombinedRealtimeDataList(copy.deepcopy(b)))
        assert got.toJSON() == O.strip_undef(exp.toJSON())


@pytest.mark.parametrize("fx", ["MockEndpointDependenciesPDAS"])
def test_product_tail_matches_oracle(fx):
    from kmamiz_amd import EndpointDependencies

    deps = fixture(fx)
    ours, ref = EndpointDependencies(deps), O.EndpointDependencies(deps)
    assert len(ours.toServiceDependencies()) == 3
    assert ours.toServiceInstability() == ref.toServiceInstability()
    assert ours.toServiceCoupling() == ref.toServiceCoupling()
    assert ours.toServiceEndpointCohesion() == ref.toServiceEndpointCohesion()
    assert ours.toChordData() == ref.toChordData()
    g = ours.toGraphData()
    assert len(g["nodes"]) == 7 and len(g["links"]) == 6
    assert ours.trim().toJSON() == O.strip_undef(ref.trim().toJSON())
    # merge of the list with itself: unchanged rows, no duplicate nested entries
    m = EndpointDependencies([]).combineWith(EndpointDependencies(fixture(fx))).toJSON()
    e = O.EndpointDependencies([]).combineWith(O.EndpointDependencies(fixture(fx))).toJSON()
    assert m == O.strip_undef(e)


def test_product_risk_matches_oracle():
    from kmamiz_amd import EndpointDependencies, risk

    deps = EndpointDependencies(fixture("MockEndpointDependenciesPDAS"))
    sdeps = deps.toServiceDependencies()
    data = [
        {"uniqueServiceName": s["uniqueServiceName"], "status": st, "combined": n, "latency": {"mean": 3.0, "cv": cv}}
        for s, st, n, cv in zip(sdeps, ["200", "500", "200"], [10, 3, 7], [0.2, 1.4, 0.0])
    ]
    reps = [{"uniqueServiceName": sdeps[0]["uniqueServiceName"], "replicas": 2}]
    got = risk.realtime_risk(data, sdeps, reps)
    exp = O.RiskAnalyzer.RealtimeRisk(data, O.EndpointDependencies(fixture("MockEndpointDependenciesPDAS"))
                                      .toServiceDependencies(), reps)
    assert [(r["uniqueServiceName"], r["norm"], r["risk"]) for r in got] == \
           [(r["uniqueServiceName"], r["norm"], r["risk"]) for r in exp]
    assert risk.Normalizer.Strategy.BetweenFixedNumber([1, 2, 3]) == [0.1, 0.55, 1]
    assert risk.Normalizer.Strategy.Linear([1, 2, 3]) == [0.4, 0.7, 1]


# ---------------------------------------------------------------------------
# CombinedRealtimeDataList.toHistoricalData
# ---------------------------------------------------------------------------
def _fx(name):
    import json
    import os

    return json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", f"{name}.json")))


def test_historical_data_oracle_matches_reference_fixture():
    """CombinedRealtimeDataList.test.ts:14-18 (MockHistoricalData)."""
    from oracle import kmz_oracle as O

    got = O.CombinedRealtimeDataList(_fx("MockBaseCrlData1")).toHistoricalData(_fx("MockDependencies"),
                                                                               _fx("MockReplicas"))
    assert got == _fx("MockHistoricalData")


def test_historical_data_mirror_matches_reference_fixture():
    from kmamiz_amd.classes import CombinedRealtimeDataList

    got = CombinedRealtimeDataList(_fx("MockBaseCrlData1")).toHistoricalData(_fx("MockDependencies"),
                                                                             _fx("MockReplicas"))
    assert got == _fx("MockHistoricalData")


def test_historical_data_mirror_matches_oracle_on_many_minutes():
    """Rows spread over several minutes and services, with 4xx/5xx statuses and
    a missing mean: the mirror and the oracle agree exactly."""
    import copy
    import random

    from kmamiz_amd.classes import CombinedRealtimeDataList
    from oracle import kmz_oracle as O

    rng = random.Random(5)
    base = _fx("MockBaseCrlData1")[0]
    rows = []
    for i in range(300):
        r = copy.deepcopy(base)
        svc = f"s{rng.randrange(6)}"
        r["service"], r["uniqueServiceName"] = svc, f"{svc}\tns\tlatest"
        r["uniqueEndpointName"] = f"{svc}\tns\tlatest\tGET\thttp://{svc}/api/{rng.randrange(4)}"
        r["status"] = rng.choice(["200", "404", "500", "201"])
        r["combined"] = rng.randrange(1, 50)
        r["latestTimestamp"] = (1700000000000 + rng.randrange(0, 5 * 60000)) * 1000 + rng.randrange(1000)
        r["latency"] = {"mean": rng.random() * 100, "cv": rng.random()}
        if i % 37 == 0:
            del r["latency"]["mean"]
        rows.append(r)
    deps = _fx("MockDependencies")
    exp = O.CombinedRealtimeDataList(copy.deepcopy(rows)).toHistoricalData(deps, _fx("MockReplicas"))
    got = CombinedRealtimeDataList(copy.deepcopy(rows)).toHistoricalData(deps, _fx("MockReplicas"))
    assert len(got) >= 5  # (the range starts 20 s into a minute)
    assert got == exp


@pytest.mark.parametrize("config,ntr", [(2, 3000), (3, 800), (5, 600)])
def test_openmp_baseline_matches_sequential_oracle(config, ntr):
    """oracle/kmz_cpu_omp.c (bench.py's all-core cpu_baseline) computes the
    same results as the sequential C oracle: integers exactly, latency
    statistics within the north_star's 1e-9."""
    from kmamiz_amd import synth
    from oracle import c_oracle

    b, _ = synth.host_batch(config, 5, 5 + ntr)
    t = synth.shape_table(config)
    o = c_oracle.stats(b, t.tag_ep, t.n_tag_ep, t.n_status)
    p = c_oracle.omp_stats(b, t.tag_ep, t.n_tag_ep, t.n_status)
    for k in ("combined", "first", "latest_timestamp"):
        assert np.array_equal(o[k], p[k]), k
    used = o["combined"] > 0
    np.testing.assert_allclose(p["mean"][used], o["mean"][used], rtol=1e-9, atol=0)
    np.testing.assert_allclose(p["cv"][used], o["cv"][used], rtol=1e-9, atol=1e-13)
    k1, e1, c1 = c_oracle.deps(b, t.dep_ep, t.n_dep_ep)
    k2, e2, c2 = c_oracle.omp_deps(b, t.dep_ep, t.n_dep_ep)
    assert np.array_equal(k1, k2) and c1 == c2
    for k in e1:
        assert np.array_equal(e1[k], e2[k]), k
