"""Config 1's Bookinfo dependency graph pinned on the reference's own fixture.

``MockEndpointDependencies`` (/root/reference/tests/MockData.ts:3169-3579,
extracted as data by tests/golden/extract_mockdata.py) holds the deduplicated
Bookinfo dependency rows of ``MockTrace`` (MockData.ts:11).  No reference test
reads it, and it predates the current row schema:

* its endpoints carry ``labelName`` and ``timestamp: 0`` (the current
  TEndpointInfo has neither a label nor a per-row timestamp of 0),
* its rows have no ``lastUsageTimestamp`` / ``isDependedByExternal``
  (TEndpointDependency.ts adds them),
* productpage's ``dependingOn`` list is in another order (below).

Its schema-independent content -- per row the endpoint's
``uniqueEndpointName`` and the (``uniqueEndpointName``, ``distance``,
``type``) entries of ``dependingBy`` / ``dependingOn`` -- is what
``EndpointDependencies([]).combineWith(new Traces(MockTrace)
.toEndpointDependencies()).trim()`` must give (EndpointDependencies.ts:
91-112, 499-563; Traces.ts:112-211).  Checked for the oracle here (CPU) and for
the engine's drop-in classes on the GPU: the same six rows in the same order,
the same entries, every list in the same order except productpage's
``dependingOn``.  That one list is (fixture) reviews v1, reviews v3, details
v1, reviews v2, ratings v1 at distance 2, against (current code, oracle and
engine) ratings v1 at distance 2, reviews v2, details v1, reviews v3, reviews
v1 -- the order the current TS code gives (oracle and engine agree).  No
reference test compares the fixture with the code, so nothing ever held its
list order to it.  The oracle itself is pinned on the reference's jest
answers for the PDAS fixtures (tests/test_oracle_goldens.py).
"""
import pytest

from conftest import fixture
from oracle import kmz_oracle as O

PRODUCTPAGE = "productpage\tbook\tv1\tGET\thttp://192.168.39.24:31629/productpage"


def _content(rows):
    """[(endpoint, [dependingBy (name, distance, type)], [dependingOn ...])] in order."""
    ent = lambda xs: [(x["endpoint"]["uniqueEndpointName"], x["distance"], x["type"]) for x in xs]  # noqa: E731
    return [(r["endpoint"]["uniqueEndpointName"], ent(r["dependingBy"]), ent(r["dependingOn"])) for r in rows]


def _check_against_fixture(rows):
    fx = fixture("MockEndpointDependencies")
    got, exp = _content(rows), _content(fx)
    assert [g[0] for g in got] == [e[0] for e in exp]  # the same rows, in the same order
    for (name, gby, gon), (_, eby, eon) in zip(got, exp):
        assert gby == eby, name
        assert sorted(gon) == sorted(eon), name  # the same entries
        if name != PRODUCTPAGE:
            assert gon == eon, name
    pp = [g for g in got if g[0] == PRODUCTPAGE][0][2]
    assert [(n.split("\t")[0] + " " + n.split("\t")[2], d) for n, d, _ in pp] == [
        ("ratings v1", 2), ("reviews v2", 1), ("details v1", 1), ("reviews v3", 1), ("reviews v1", 1)]
    # the endpoint objects agree field for field except the old schema's
    # labelName and its timestamp 0; the rows carry the current fields
    for r, f in zip(rows, fx):
        e, fe = r["endpoint"], f["endpoint"]
        assert {k: v for k, v in e.items() if k != "timestamp"} == {
            k: v for k, v in fe.items() if k not in ("labelName", "timestamp")}
        assert fe["timestamp"] == 0 and "labelName" in fe
        assert set(r) - set(f) == {"lastUsageTimestamp", "isDependedByExternal"}


def test_oracle_graph_equals_reference_fixture():
    red = O.EndpointDependencies([]).combineWith(O.Traces(fixture("MockTrace")).toEndpointDependencies()).trim()
    _check_against_fixture(O.strip_undef(red.toJSON()))


@pytest.mark.gpu
def test_engine_graph_equals_reference_fixture(engine):
    from kmamiz_amd import Traces

    got = Traces(fixture("MockTrace"), engine=engine).toEndpointDependencies().toReduced().toJSON()
    _check_against_fixture(got)
