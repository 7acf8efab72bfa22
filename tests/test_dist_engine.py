"""The bench's multi-GPU merge sequence on real engines: two ranks (gloo, CPU
tensors) share the one GPU, each runs its traceId shard, and the partials and
edge keys merge through kmamiz_amd.dist.merge_all (kmz_partials_copy, kmz_merge_triples,
kmz_finalize).  Both ranks must end with the single-engine result over the
whole batch, bit for bit -- including the service tail run on the merged edge
set (kmz_tail_run: the north_star's "edge sets merge ... before the
service-level instability, coupling/cohesion and risk computation")."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd import Engine
        from kmamiz_amd import _lib as L
        from kmamiz_amd import dist as kdist
        from kmamiz_amd import synth

        e = Engine(0)
        cut = [0, 1500, 4000]
        e.load_synthetic(synth.MESH, synth.SEED, cut[rank], cut[rank + 1])
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        gw, ew, tw = (e.partials_words(w) for w in (L.PART_GROUPS, L.PART_ENDPOINTS, L.PART_TRIPLES))
        g = torch.zeros(gw, dtype=torch.int64)
        ep = torch.zeros(ew, dtype=torch.int64)
        t = torch.zeros(max(1, tw), dtype=torch.int64)
        e.export_partials(L.PART_GROUPS, g.data_ptr(), gw, False)
        e.export_partials(L.PART_ENDPOINTS, ep.data_ptr(), ew, False)
        e.export_partials(L.PART_TRIPLES, t.data_ptr(), tw, False)
        kdist.merge_all(g, gw // 6, ep, ew // 2, t[:tw], engine=e)  # bench.py's three-collective merge
        e.import_partials(L.PART_GROUPS, g.data_ptr(), gw, False)
        e.import_partials(L.PART_ENDPOINTS, ep.data_ptr(), ew, False)
        e.finalize()
        groups, keys, eps = e.fetch()
        from kmamiz_amd.tail import maps_for_synth, run_tail

        tl = run_tail(e, maps_for_synth(synth.MESH), eps)
        q.put((rank, groups.tobytes(), np.sort(keys).tobytes(), eps.tobytes(),
               (tl.stats.tobytes(), tl.by_dist.tobytes(), tl.gateway.tobytes(), tl.services.tobytes())))
        e.close()
    except Exception as ex:  # surfaced by the parent
        q.put((rank, "error", repr(ex), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_merge_equals_single_engine():
    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=150) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
    e = Engine(0)
    try:
        e.load_synthetic(synth.MESH, synth.SEED, 0, 4000)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        g, k, ep = e.fetch()
        exp = (g.tobytes(), np.sort(k).tobytes(), ep.tobytes())
        from kmamiz_amd.tail import maps_for_synth, run_tail

        tl = run_tail(e, maps_for_synth(synth.MESH), ep)
        exp_tail = (tl.stats.tobytes(), tl.by_dist.tobytes(), tl.gateway.tobytes(), tl.services.tobytes())
    finally:
        e.close()
    for r in res:
        assert r[1] == exp[0]
        assert r[2] == exp[1]
        assert r[3] == exp[2]
        assert r[4] == exp_tail


def _crossing_batches(case, world, t0=0):
    """Per rank: the host batch of its traces, with the span-id map crossing
    shards as ``case`` says -- "parent": rank 1 has a span whose parentId is a
    span of rank 0's shard; "repeat": the last rank reuses one span id of rank
    0's shard (a leaf SERVER span: no parent link crosses); "inner": the last
    rank repeats one of its own span ids (its run takes the span-table path);
    "none": clean shards.  ``t0``: the batch's first trace (a batch after the
    first starts at a global flatten position > 0)."""
    from kmamiz_amd import synth

    ntr = 900 if case != "parent" else 700
    cut = [ntr * r // world for r in range(world + 1)] if case != "parent" else [0, 300, 700][: world + 1]
    cut = [t0 + c for c in cut]
    out = []
    b0, _ = synth.host_batch(synth.MESH, cut[0], cut[1])
    for rank in range(world):
        batch, _ = synth.host_batch(synth.MESH, cut[rank], cut[rank + 1])
        if case == "parent" and rank == 1:
            roots = np.nonzero(batch.parent_id == 0)[0]
            batch.parent_id[roots[3]] = b0.span_id[10]  # a parent on the other shard
        if case in ("repeat", "inner") and rank == world - 1:
            # the last leaf SERVER span takes the id of another trace's span
            # (an id of the leaf's own ancestry would make the global map's
            # parent chain a cycle, which the reference never leaves)
            kids = set(batch.parent_id.tolist())
            leaf = next(i for i in range(len(batch) - 1, -1, -1)
                        if batch.kind[i] == 1 and int(batch.span_id[i]) not in kids)
            batch.span_id[leaf] = b0.span_id[len(b0) - 1] if case == "repeat" else batch.span_id[0]
        out.append(batch)
    return out


def _crossing_worker(rank, world, port, q, case, exact, t0=0, no_cert=False):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd import Engine
        from kmamiz_amd import _lib as L
        from kmamiz_amd import dist as kdist
        from kmamiz_amd import synth

        batch = _crossing_batches(case, world, t0)[rank]
        e = Engine(0)
        e.load(batch, synth.shape_table(synth.MESH))
        # (no_cert: the run skips its own certificate, merge_all's id guard
        # covers every shard's ids -- a repeat inside one shard included)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS | (L.RUN_NO_CERT if no_cert else 0))
        gw, ew, tw = (e.partials_words(w) for w in (L.PART_GROUPS, L.PART_ENDPOINTS, L.PART_TRIPLES))
        g = torch.zeros(gw, dtype=torch.int64)
        ep = torch.zeros(ew, dtype=torch.int64)
        t = torch.zeros(max(1, tw), dtype=torch.int64)
        e.export_partials(L.PART_GROUPS, g.data_ptr(), gw, False)
        e.export_partials(L.PART_ENDPOINTS, ep.data_ptr(), ew, False)
        e.export_partials(L.PART_TRIPLES, t.data_ptr(), tw, False)
        try:
            kdist.merge_all(g, gw // 6, ep, ew // 2, t[:tw], engine=e, exact=exact)
        except kdist.ShardingError:
            q.put((rank, "refused", None, None, None))
            return
        e.import_partials(L.PART_GROUPS, g.data_ptr(), gw, False)
        e.import_partials(L.PART_ENDPOINTS, ep.data_ptr(), ew, False)
        e.finalize()
        groups, keys, eps = e.fetch()
        q.put((rank, "merged", groups.tobytes(), np.sort(keys).tobytes(), eps.tobytes()))
        e.close()
    except Exception:  # surfaced by the parent
        import traceback

        q.put((rank, traceback.format_exc(), None, None, None))
    finally:
        dist.destroy_process_group()


def _run_crossing(case, world, exact=True, t0=0, no_cert=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_crossing_worker, args=(r, world, port, q, case, exact, t0, no_cert))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=150) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    return res


def _whole_batch_expected(case, world, t0=0):
    """One engine over the whole batch (the reference's single global span
    map), and the C oracle's edge keys and endpoints of the same batch."""
    from kmamiz_amd import Engine, SpanBatch
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from oracle import c_oracle

    parts = _crossing_batches(case, world, t0)
    cols = {f: np.concatenate([getattr(b, f) for b in parts]) for f in ("span_id", "parent_id", "kind", "shape",
                                                                      "status", "duration", "timestamp")}
    whole = SpanBatch(index_base=parts[0].index_base, **cols)
    table = synth.shape_table(synth.MESH)
    e = Engine(0)
    try:
        e.load(whole, table)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        g, k, ep = e.fetch()
        exp = (g.tobytes(), np.sort(k).tobytes(), ep.tobytes())
    finally:
        e.close()
    okeys, oep, _ = c_oracle.deps(whole, table.dep_ep, table.n_dep_ep)
    return exp, okeys, oep


@pytest.mark.gpu
@pytest.mark.parametrize("case,world,t0,no_cert", [("parent", 2, 0, False), ("repeat", 2, 0, False),
                                                  ("repeat", 3, 0, False), ("inner", 2, 0, False),
                                                  ("repeat", 2, 1000, False), ("parent", 2, 500, False),
                                                  ("inner", 2, 0, True), ("repeat", 3, 0, True),
                                                  ("none", 2, 0, True)])
def test_crossing_shards_merge_exactly(case, world, t0, no_cert):
    """SURVEY.md 8e / Traces.ts:117-143: the reference keys ONE Map by span id
    over the whole batch, so a parent in another shard, an id in two shards or
    an id repeated inside one shard changes rows and edges that per-shard runs
    cannot see.  merge_all's guards find it on every rank and the merge stays
    exact (one unsharded dependency pass on rank 0, broadcast): every rank ends
    with the single-engine result over the whole batch, bit for bit, whose
    edges and endpoints equal the C oracle's.  ``t0`` > 0: a batch that does
    not start at global position 0 (the first rows stay global).  ``no_cert``:
    the runs skip their own uniqueness certificate (KMZ_RUN_NO_CERT, the
    multi-GPU bench's setting) and the id guard alone finds the repeat --
    inside one shard too, whose window-join result it replaces."""
    res = _run_crossing(case, world, t0=t0, no_cert=no_cert)
    assert [r[1] for r in res] == ["merged"] * world, [r[1] for r in res]
    exp, okeys, oep = _whole_batch_expected(case, world, t0)
    assert np.array_equal(np.frombuffer(exp[1], np.uint64), okeys)
    from kmamiz_amd import _lib as L

    eps = np.frombuffer(exp[2], L.ENDPOINT_DTYPE)
    assert np.array_equal(eps["has_row"] != 0, oep["has_row"])
    assert np.array_equal(eps["first_row"][oep["has_row"]], oep["first"][oep["has_row"]])
    for r in res:
        assert r[2] == exp[0]
        assert r[3] == exp[1]
        assert r[4] == exp[2]


@pytest.mark.gpu
def test_crossing_shards_refused_without_exact():
    """exact=False keeps the old contract: every rank raises ShardingError
    (and a clean batch merges either way)."""
    assert [r[1] for r in _run_crossing("parent", 2, exact=False)] == ["refused"] * 2
    assert [r[1] for r in _run_crossing("repeat", 3, exact=False)] == ["refused"] * 3
    assert [r[1] for r in _run_crossing("none", 2, exact=False)] == ["merged"] * 2


# ---------------------------------------------------------------------------
# traceId sharding with different JSON shards (SURVEY.md 8e, config 4's merge)
# ---------------------------------------------------------------------------
def _json_shard_worker(rank, world, port, q, n_mesh):
    import json

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_util import endpoints_by_name, groups_by_name, mixed_traces

        from kmamiz_amd import Engine
        from kmamiz_amd import _lib as L
        from kmamiz_amd.ingest import ingest_json
        from kmamiz_amd.shard import gather_names, run_sharded, shard_traces

        plan = shard_traces(mixed_traces(n_mesh), world)[rank]
        batch, d = ingest_json(json.dumps(plan.traces).encode())  # this rank's own Zipkin response bytes
        e = Engine(0)
        r1 = run_sharded(e, batch, d, plan.local_start, plan.global_start, L.RUN_STATS_TAG | L.RUN_DEPS)
        r2 = run_sharded(e, batch, d, plan.local_start, plan.global_start, L.RUN_STATS_RT)
        tag, rt, dep = (gather_names(r1.tables, d, x) for x in ("tag", "rt", "dep"))
        from shard_util import _edges

        q.put((rank, groups_by_name(r1.groups, tag, r1.tables.statuses), _edges(r1.keys, dep),
               endpoints_by_name(r1.endpoints, dep), groups_by_name(r2.groups, rt, r2.tables.statuses),
               len(d.shapes), len(batch)))
        e.close()
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_json_shards_merge_equals_c_oracle(world):
    """Config 4's merge on real engines: each rank parses its own JSON shard
    (different shape sets), ids are made global by shard.exchange_tables, first
    indices by the index map; the merged groups (both identity rules), edges
    and endpoints equal the C oracle over the whole batch, on every rank."""
    from shard_util import assert_groups_equal, mixed_traces, oracle_by_name

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_json_shard_worker, args=(r, world, port, q, 400)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=150) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
    traces = mixed_traces(400)
    exp_g, exp_k, exp_e = oracle_by_name(traces, "tag")
    exp_rt, _, _ = oracle_by_name(traces, "rt")
    assert len({r[5] for r in res}) > 1  # the shards' shape tables differ
    assert sum(r[6] for r in res) == sum(len(t) for t in traces)
    for r in res:
        assert_groups_equal(r[1], exp_g)
        assert r[2] == exp_k
        assert r[3] == exp_e
        assert_groups_equal(r[4], exp_rt)
