"""Multi-rank merge (kmamiz_amd.dist) with world_size 2 on gloo/CPU.

Each rank takes half of the traces of a synthetic batch (whole traces, global
indices via index_base), forms the engine's partial layout for its shard, and
merges through the same functions the GPU path uses over RCCL.  The merged
result must equal the single-batch oracle exactly (integers) / within 1e-9,
and so must the service tail computed over the merged edge set (its kernel's
numpy restatement, tests/test_tail.py, pinned there against the oracle)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

U64 = np.uint64


def shard_partials(batch, ep_of_shape, n_ep, n_status, dep_ep, n_dep, gidx=None):
    """Engine partial layout for one shard (test-side restatement of K3/K4's
    accumulators: integer moments, biased max timestamp, min first index).
    gidx: global flatten index of every local span (default index_base + i)."""
    G = n_ep * n_status
    if gidx is None:
        gidx = np.arange(len(batch), dtype=np.int64) + batch.index_base
    p = np.zeros(6 * G, dtype=U64)
    p[4 * G : 5 * G] = 0
    p[5 * G :] = U64(0xFFFFFFFFFFFFFFFF)
    srv = np.nonzero(batch.kind == 1)[0]
    g = ep_of_shape[batch.shape[srv]].astype(np.int64) * n_status + batch.status[srv]
    d = batch.duration[srv].astype(U64)
    dd = d * d
    np.add.at(p, g, U64(1))
    np.add.at(p, G + g, d)
    np.add.at(p, 2 * G + g, dd & U64(0xFFFFFFFF))
    np.add.at(p, 3 * G + g, dd >> U64(32))
    tsx = batch.timestamp[srv].astype(np.int64).view(U64) ^ U64(1 << 63)
    np.maximum.at(p, 4 * G + g, tsx)
    np.minimum.at(p, 5 * G + g, gidx[srv].astype(U64))
    # endpoint partials: rows = SERVER spans (unique ids in the synthetic data)
    e = np.zeros(2 * n_dep, dtype=U64)
    e[n_dep:] = U64(0xFFFFFFFFFFFFFFFF)
    es = dep_ep[batch.shape[srv]].astype(np.int64)
    np.maximum.at(e, es, tsx)
    idx = {int(s): i for i, s in enumerate(batch.span_id.tolist())}
    ext = np.array([0 if (batch.parent_id[i] and batch.kind[idx[int(batch.parent_id[i])]] == 2 and
                          batch.parent_id[idx[int(batch.parent_id[i])]] != 0) else 1 for i in srv], dtype=U64)
    np.minimum.at(e, n_dep + es, (gidx[srv].astype(U64) << U64(1)) | (U64(1) - ext))
    return p, e


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd import dist as kdist
        from kmamiz_amd import finalize_host, synth
        from oracle import c_oracle

        cfg, ntr = synth.MESH, 600
        table = synth.shape_table(cfg)
        cut = [0, 250, ntr]
        batch, _ = synth.host_batch(cfg, cut[rank], cut[rank + 1])
        p, e = shard_partials(batch, table.tag_ep, table.n_tag_ep, table.n_status, table.dep_ep, table.n_dep_ep)
        keys, _, _ = c_oracle.deps(batch, table.dep_ep, table.n_dep_ep)
        G = table.n_tag_ep * table.n_status
        pt = torch.from_numpy(p.view(np.int64).copy())
        et = torch.from_numpy(e.view(np.int64).copy())
        kt = torch.from_numpy(keys.view(np.int64).copy())
        # the fused three-collective merge (bench.py) equals the separate ones
        pf, ef = pt.clone(), et.clone()
        fused_keys = kdist.merge_all(pf, G, ef, table.n_dep_ep, kt)
        kdist.merge_group_partials(pt, G)
        kdist.merge_endpoint_partials(et, table.n_dep_ep)
        merged_keys = kdist.merge_edge_keys(kt)
        fused_ok = bool(torch.equal(pf, pt) and torch.equal(ef, et) and torch.equal(fused_keys, merged_keys))
        if rank == 0:
            full, _ = synth.host_batch(cfg, 0, ntr)
            assert fused_ok
            groups = finalize_host(pt.numpy().view(U64), G)
            o = c_oracle.stats(full, table.tag_ep, table.n_tag_ep, table.n_status)
            ok = bool(np.array_equal(groups["combined"], o["combined"]))
            used = o["combined"] > 0
            ok &= bool(np.array_equal(groups["latest_timestamp"][used], o["latest_timestamp"][used]))
            ok &= bool(np.array_equal(groups["first"][used], o["first"][used]))
            ok &= bool(np.allclose(groups["mean"][used], o["mean"][used], rtol=1e-9, atol=0))
            ok &= bool(np.allclose(groups["cv"][used], o["cv"][used], rtol=1e-9, atol=1e-13))
            okeys, oep, _ = c_oracle.deps(full, table.dep_ep, table.n_dep_ep)
            ok &= bool(np.array_equal(np.sort(merged_keys.numpy().view(U64)), okeys))
            ev = et.numpy().view(U64)
            E = table.n_dep_ep
            has = ev[E:] != U64(0xFFFFFFFFFFFFFFFF)
            ok &= bool(np.array_equal(has, oep["has_row"]))
            ok &= bool(np.array_equal(ev[E:][has] >> U64(1), oep["first"][has]))
            ok &= bool(np.array_equal((ev[E:][has] & U64(1)) == 0, oep["external"][has]))
            # the service tail over the merged edge set = over the single batch
            from test_tail import _tail_np

            from kmamiz_amd.tail import maps_for_synth

            maps = maps_for_synth(cfg)
            first = np.where(has, ev[E:] >> U64(1), U64(0xFFFFFFFFFFFFFFFF))
            got = _tail_np(np.sort(merged_keys.numpy().view(U64)), maps, has, first)
            ofirst = np.where(oep["has_row"], oep["first"], np.iinfo(np.uint64).max).astype(U64)
            exp = _tail_np(okeys, maps, oep["has_row"], ofirst)
            ok &= bool(np.array_equal(got.stats, exp.stats) and np.array_equal(got.by_dist, exp.by_dist))
            ok &= bool(np.array_equal(got.gateway, exp.gateway) and np.array_equal(got.services, exp.services))
            ok &= got.instability() == exp.instability() and got.coupling() == exp.coupling()
            q.put(ok)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_merge_equals_single_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


# ---------------------------------------------------------------------------
# sharding guards: ids repeated across shards, and
# ranks that disagree on the partials' sizes
# ---------------------------------------------------------------------------
def _guard_worker(rank, world, port, q, case):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd import dist as kdist
        from kmamiz_amd import synth

        ntr = 300
        cut = [ntr * r // world for r in range(world + 1)]
        batch, _ = synth.host_batch(synth.MESH, cut[rank], cut[rank + 1])
        ids = batch.span_id.copy()
        if case == "repeat" and rank == world - 1:
            first, _ = synth.host_batch(synth.MESH, 0, 1)
            ids[len(ids) // 2] = first.span_id[1]  # one id of rank 0's shard, far from it here
        if case in ("clean", "repeat"):
            try:
                kdist.check_repeated_ids(span_ids=ids)
                q.put((rank, "passed"))
            except kdist.ShardingError:
                q.put((rank, "refused"))
        elif case == "internal":  # rank 0's shard repeats an id inside itself (the span-table path)
            class _Eng:
                def unresolved_parents(self):
                    from kmamiz_amd._lib import KmzError

                    if rank == 0:
                        raise KmzError(-9, "span-table path")
                    return 0

            p = torch.zeros(6 * 3, dtype=torch.int64)
            try:
                kdist.merge_all(p, 3, torch.zeros(4, dtype=torch.int64), 2, torch.ones(2, dtype=torch.int64),
                                engine=_Eng(), check_ids=False, exact=False)
                q.put((rank, "merged"))
            except kdist.ShardingError:
                q.put((rank, "refused"))
        else:  # "sizes": rank 1 holds one group more -- refused before any size-dependent collective
            G = 3 + (rank == 1)
            p = torch.zeros(6 * G, dtype=torch.int64)
            e = torch.zeros(4, dtype=torch.int64)
            k = torch.ones(2, dtype=torch.int64)
            try:
                kdist.merge_all(p, G, e, 2, k)
                q.put((rank, "merged"))
            except kdist.ShardingError:
                q.put((rank, "refused"))
    except Exception as ex:  # surfaced by the parent
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def _run_guard(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    return [r[1] for r in res]


@pytest.mark.parametrize("world", [2, 3])
def test_span_id_repeated_across_shards_is_refused(world):
    """The reference's span map is global (Traces.ts:117-123): one id in two
    shards is one row there.  Routing the hashed ids to their owner rank and
    checking each owner's values finds it on every rank; a clean batch passes."""
    assert _run_guard(world, "clean") == ["passed"] * world
    assert _run_guard(world, "repeat") == ["refused"] * world


def test_ranks_with_different_sizes_are_refused():
    assert _run_guard(2, "sizes") == ["refused"] * 2


@pytest.mark.parametrize("world", [2, 3])
def test_one_rank_on_the_span_table_path_refuses_every_rank(world):
    """a shard with an id repeated inside it is known to every rank
    through the agreement all-reduce, so no rank waits in a collective the
    refusing rank never joins: with exact=False every rank raises (the exact
    merge of such shards runs on real engines: test_dist_engine.py)."""
    assert _run_guard(world, "internal") == ["refused"] * world


def test_route_ids_np_partitions_by_owner():
    from kmamiz_amd import dist as kdist

    rng = np.random.default_rng(7)
    ids = rng.integers(1, 2**63, size=5000, dtype=np.uint64)
    for world in (1, 2, 3, 8):
        h, c = kdist.route_ids_np(ids, world)
        assert c.sum() == len(ids) and len(c) == world
        own = kdist.id_owner_np(h, world)
        assert np.all(np.diff(own.astype(np.int64)) >= 0)  # grouped by owner, in rank order
        assert np.array_equal(np.sort(h), np.sort(kdist.id_hash_np(ids)))
    # id_hash is a bijection: distinct ids give distinct hashes
    assert len(np.unique(kdist.id_hash_np(np.arange(1, 100001, dtype=np.uint64)))) == 100000
