"""GPU parity of the reduced graph's entry order (kmz_order.hip,
KMZ_RUN_DEP_ORDER) and of the cache merges fed by it.

* kmz_get_dep_entries == the C oracle's oracle_dep_entries, record for record
  (bit-exact: keys, rows, positions, spans, timestamps, shapes), on the
  reference fixtures, mixed and messy batches (repeated ids: the span-table
  path), synthetic configs 2/3/5, and a non-contiguous shard (index map);
* the drop-in classes: Traces.toEndpointDependencies().toReduced() equals
  EndpointDependencies([]).combineWith(...).trim() of the Python oracle, and a
  cache fed window by window equals the oracle's ticks.
"""
import copy

import numpy as np
import pytest

from conftest import fixture
from oracle import c_oracle
from oracle import kmz_oracle as O
from shard_util import mixed_traces
from test_cache import _messy, _ticks

pytestmark = pytest.mark.gpu

FIELDS = ("key", "row", "span", "pos", "ts", "shape")


def _sorted(e):
    return e[np.argsort(e["key"], kind="stable")]


def _same_entries(got, exp):
    got = _sorted(got)
    assert len(got) == len(exp)
    for f in FIELDS:
        assert np.array_equal(got[f], exp[f]), f


def _check_batch(engine, batch, table):
    from kmamiz_amd import _lib as L

    engine.load(batch, table)
    engine.run(L.RUN_DEPS | L.RUN_DEP_ORDER)
    got, rts, rsh = engine.dep_entries()
    exp, ets, esh = c_oracle.dep_entries(batch, table.dep_ep, table.n_dep_ep)
    _same_entries(got, exp)
    has = engine.endpoints()["has_row"] != 0
    assert np.array_equal(rts[has], ets[has]) and np.array_equal(rsh[has], esh[has])
    assert np.all(rsh[~has] == L.NONE32) and np.all(rts[~has] == np.iinfo(np.int64).min)
    return engine.info()


@pytest.mark.parametrize("which", ["MockTrace", "MockTracePDAS", "mixed", "messy1", "messy2"])
def test_entries_vs_c_oracle_objects(engine, which):
    from kmamiz_amd.ingest import ingest_traces

    traces = {"MockTrace": lambda: fixture("MockTrace"), "MockTracePDAS": lambda: [fixture("MockTracePDAS")],
              "mixed": lambda: mixed_traces(300), "messy1": lambda: _messy(11, 300),
              "messy2": lambda: _messy(12, 2000)}[which]()
    batch, d, _ = ingest_traces(traces)
    info = _check_batch(engine, batch, d.shape_table())
    if which.startswith("messy"):
        assert info["n_dups"] > 0  # the span-table path (k_row_value maps positions to spans)


@pytest.mark.parametrize("config,ntr", [(2, 30000), (3, 40000), (3, 200000), (5, 4000)])
def test_entries_vs_c_oracle_synthetic(engine, config, ntr):
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(config, 0, ntr)
    info = _check_batch(engine, batch, synth.shape_table(config))
    assert info["n_dups"] == 0 and info["path"] & 2  # chain-interning path


def test_entries_of_a_shard_are_global(engine):
    """A non-contiguous shard (kmz_set_index_map): rows, spans and positions
    come back as global flatten indices; per key, the record with the smallest
    row over the shards is the whole batch's record (a row and all its
    descendants live in one trace, so in one shard)."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.cache import merge_shard_entries
    from test_gpu_parity import _host_shard

    config, t0, t1, world = 3, 5, 6000, 3
    table = synth.shape_table(config)
    parts = []
    for rank in range(world):
        hb, ls, gs = _host_shard(config, t0, t1, world, rank)
        engine.load(hb, table)
        engine.set_index_map(ls, gs)
        engine.run(L.RUN_DEPS | L.RUN_DEP_ORDER)
        parts.append((engine.dep_entries(), engine.endpoints()))
    whole, _ = synth.host_batch(config, t0, t1)
    exp, ets, esh = c_oracle.dep_entries(whole, table.dep_ep, table.n_dep_ep)
    ents, rts, rsh = merge_shard_entries([(e, r, s, ep["first_row"]) for (e, r, s), ep in parts])
    _same_entries(ents, exp)
    ok = rsh != L.NONE32
    assert np.array_equal(rts[ok], ets[ok]) and np.array_equal(rsh[ok], esh[ok])


@pytest.mark.parametrize("fx", ["MockTrace", "MockTracePDAS"])
def test_to_reduced_equals_oracle(engine, fx):
    from kmamiz_amd import Traces

    traces = fixture(fx) if fx == "MockTrace" else [fixture(fx)]
    got = Traces(traces, engine=engine).toEndpointDependencies().toReduced().toJSON()
    exp = O.EndpointDependencies([]).combineWith(O.Traces(traces).toEndpointDependencies()).trim().toJSON()
    assert got == O.strip_undef(exp)


def test_gpu_windows_feed_the_cache(engine):
    """The worker tick (RealtimeWorkerImpl.ts:67-70: no cache yet -> newDep
    itself, per row; then existingDep.combineWith(newDep)) + CEndpointDependencies
    .setData (trim) over four windows computed on the GPU, and
    CCombinedRealtimeData.setData of the windows' combined rows, against the
    oracle's ticks."""
    from kmamiz_amd import Traces
    from kmamiz_amd.cache import CCombinedRealtimeData, CEndpointDependencies, ReducedDependencies, worker_dependencies

    traces = mixed_traces(240) + _messy(7, 80)
    deps, comb = CEndpointDependencies(), CCombinedRealtimeData()
    odeps = ocomb = None
    for k, w in enumerate(_ticks(traces, [0, 40, 95, 150, len(traces)])):
        t = Traces(copy.deepcopy(w), engine=engine)
        win = t.toEndpointDependencies()
        existing = deps.getData()
        # the worker gets existingDep as JSON (ServiceOperator.ts:290-298)
        deps.setData(worker_dependencies(ReducedDependencies.from_json(existing.toJSON()) if existing else None,
                                         win))
        comb.setData(t.combineLogsToRealtimeData([]).toCombinedRealtimeData())
        newdep = O.Traces(copy.deepcopy(w)).toEndpointDependencies()
        odeps = (O.EndpointDependencies(copy.deepcopy(odeps)).combineWith(newdep) if odeps is not None
                 else newdep).trim().toJSON()
        assert deps.getData().toJSON() == O.strip_undef(odeps), k
        upd = O.strip_undef(O.Traces(copy.deepcopy(w)).combineLogsToRealtimeData([], None)
                            .toCombinedRealtimeData().toJSON())
        f = [r for r in upd if O.truthy(O.get(r, "service"))]
        ocomb = O.strip_undef((O.CombinedRealtimeDataList(copy.deepcopy(ocomb)).combineWith(
            O.CombinedRealtimeDataList(f)) if ocomb is not None else O.CombinedRealtimeDataList(f)).toJSON())
        got = comb.getData().toJSON()
        assert len(got) == len(ocomb)
        for a, b in zip(got, ocomb):
            for key in ("uniqueEndpointName", "status", "combined", "latestTimestamp", "service", "namespace"):
                assert a.get(key) == b.get(key), (k, key)
            for key in ("mean", "cv"):  # window stats: engine vs sequential Welford (north_star 1e-9)
                assert a["latency"][key] == pytest.approx(b["latency"][key], rel=1e-9, abs=1e-13)
