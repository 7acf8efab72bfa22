"""traceId sharding on the CPU (gloo): kmz_trace_shard, shard_traces, the
global id exchange (shard.exchange_tables) and merge_all's digest guard.

Each rank ingests a different Zipkin JSON shard through the native parser
(kmz_parse_zipkin), so the ranks have different local shape / endpoint /
status tables; the merged partials (a numpy restatement of the engine's
accumulators, indexed by the exchanged global ids, first indices through the
shard's index map) must equal the C oracle over the whole batch, compared by
endpoint and status strings."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shard_util import U64, _edges, assert_groups_equal, mixed_traces, oracle_by_name, status_key

# ---------------------------------------------------------------------------
# single process
# ---------------------------------------------------------------------------


def test_trace_shard_parses_hex_ids():
    from kmamiz_amd import _lib as L
    from kmamiz_amd.shard import trace_shard

    lib = L.lib()
    # 32-digit and 16-digit canonical ids hash by value: a 16-digit id and its
    # zero-padded 32-digit form are the same number
    for tid in ("4a5e59b938fc2484", "00000000000000000000000000000001"):
        assert trace_shard(tid, 8) == trace_shard(tid.rjust(32, "0"), 8)
    assert trace_shard("anything", 1) == 0
    # non-hex strings hash by their bytes: stable, in range
    for w in (2, 3, 8):
        vals = [trace_shard(f"trace-{i}", w) for i in range(2000)]
        assert set(vals) == set(range(w))
        assert vals == [trace_shard(f"trace-{i}", w) for i in range(2000)]
        counts = np.bincount(vals, minlength=w)
        assert counts.min() > 2000 / w * 0.8  # roughly uniform
    # undefined / non-string traceIds use their JS template string
    assert trace_shard(None, 4) == int(lib.kmz_trace_shard(b"null", 4, 4))


def test_shard_traces_partitions_in_order():
    from kmamiz_amd.shard import shard_traces

    traces = mixed_traces(120)
    flat = [s for t in traces for s in t]
    for world in (1, 2, 3, 4):
        plans = shard_traces(traces, world)
        assert sum(len(p.traces) for p in plans) == len(traces)
        for p in plans:
            local = [s for t in p.traces for s in t]
            for k, t in enumerate(p.traces):
                ls, gs = int(p.local_start[k]), int(p.global_start[k])
                for j, s in enumerate(t):  # the run maps local -> global flatten index
                    assert local[ls + j] is s and flat[gs + j] is s


def _map_index(ls, gs, n):
    """numpy restatement of kmz_set_index_map's map for every local index."""
    x = np.arange(n, dtype=np.int64)
    k = np.searchsorted(ls.astype(np.int64), x, side="right") - 1
    return gs.astype(np.int64)[k] + (x - ls.astype(np.int64)[k])


def _ep_partials(batch, dep_ep, n_dep, gidx):
    """Endpoint partials of the engine (unique span ids): per dependency
    endpoint max(ts ^ 2^63) over rows and their non-CLIENT ancestors, and
    min(first_row << 1 | !external) over rows (Traces.ts:117-208)."""
    e = np.zeros(2 * n_dep, dtype=U64)
    e[n_dep:] = U64(0xFFFFFFFFFFFFFFFF)
    idx = {int(s): i for i, s in enumerate(batch.span_id.tolist())}
    tsx = batch.timestamp.astype(np.int64).view(U64) ^ U64(1 << 63)
    for i in np.nonzero(batch.kind == 1)[0].tolist():
        ep = int(dep_ep[batch.shape[i]])
        e[ep] = max(e[ep], tsx[i])
        p, ext = int(batch.parent_id[i]), 1
        while p:
            j = idx.get(p)
            if j is None:
                break
            if batch.kind[j] != 2:
                ext = 0
                a = int(dep_ep[batch.shape[j]])
                e[a] = max(e[a], tsx[j])
            p = int(batch.parent_id[j])
        e[n_dep + ep] = min(e[n_dep + ep], (U64(gidx[i]) << U64(1)) | U64(1 - ext))
    return e


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
    return sorted(res, key=lambda r: r[0])


def _merge_worker(rank, world, port, q, n_mesh):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_dist_gloo import shard_partials

        from kmamiz_amd import dist as kdist
        from kmamiz_amd import finalize_host
        from kmamiz_amd.ingest import ingest_json
        from kmamiz_amd.shard import exchange_tables, gather_names, shard_traces
        from oracle import c_oracle

        traces = mixed_traces(n_mesh)
        plan = shard_traces(traces, world)[rank]
        batch, d = ingest_json(json.dumps(plan.traces).encode())
        gt = exchange_tables(d)
        table = gt.shape_table(d)
        b = gt.remap_batch(batch)
        gidx = _map_index(plan.local_start, plan.global_start, len(b))
        p, _ = shard_partials(b, table.tag_ep, table.n_tag_ep, table.n_status, table.dep_ep, table.n_dep_ep, gidx)
        e = _ep_partials(b, table.dep_ep, table.n_dep_ep, gidx)
        keys, _, _ = c_oracle.deps(b, table.dep_ep, table.n_dep_ep)
        G = table.n_tag_ep * table.n_status
        pt = torch.from_numpy(p.view(np.int64).copy())
        et = torch.from_numpy(e.view(np.int64).copy())
        kt = torch.from_numpy(keys.view(np.int64).copy())
        merged = kdist.merge_all(pt, G, et, table.n_dep_ep, kt, digest=gt.digest)
        groups = finalize_host(pt.numpy().view(U64), G)
        tag_names = gather_names(gt, d, "tag")
        dep_names = gather_names(gt, d, "dep")
        from shard_util import groups_by_name

        got_g = groups_by_name(groups, tag_names, gt.statuses)
        got_k = _edges(np.sort(merged.numpy().view(U64)), dep_names)
        ev = et.numpy().view(U64)
        E = table.n_dep_ep
        got_e = {}
        for x in range(E):
            has = ev[E + x] != U64(0xFFFFFFFFFFFFFFFF)
            last = max(float(np.int64((ev[x] ^ U64(1 << 63)).view(np.int64))) / 1000.0, 0.0) if ev[x] else 0.0
            if has or last:
                got_e[dep_names[x]] = (bool(has), int(ev[E + x] >> U64(1)) if has else -1,
                                       bool((ev[E + x] & U64(1)) == 0) if has else False, last)
        q.put((rank, got_g, got_k, got_e, len(d.shapes), gt.digest))
    except Exception as ex:  # surfaced by the parent
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_json_merge_equals_whole_batch_oracle(world):
    res = _spawn(_merge_worker, world, 160)
    for r in res:
        assert r[1] != "error", r[2]
    traces = mixed_traces(160)
    exp_g, exp_k, exp_e = oracle_by_name(traces)
    # the ranks' local tables really differ (different shape sets)
    assert len({r[4] for r in res}) > 1
    assert len({r[5] for r in res}) == 1  # one digest
    for r in res:
        assert_groups_equal(r[1], exp_g)
        assert r[2] == exp_k
        assert r[3] == exp_e


def _digest_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd import dist as kdist

        p = torch.zeros(12, dtype=torch.int64)
        e = torch.zeros(4, dtype=torch.int64)
        k = torch.tensor([5, 7], dtype=torch.int64)
        try:
            kdist.merge_all(p, 2, e, 2, k, digest=1234 + rank)
            q.put((rank, "merged"))
        except kdist.ShardingError:
            q.put((rank, "refused"))
    finally:
        dist.destroy_process_group()


def test_mismatched_id_tables_are_refused():
    assert [r[1] for r in _spawn(_digest_worker, 2)] == ["refused", "refused"]


def _tables_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd.ingest import Dictionary
        from kmamiz_amd.shard import exchange_tables, gather_names

        d = Dictionary()
        # overlapping, differently ordered shape sets per rank; one poisoned shape
        names = [f"s{(rank * 3 + i) % 7}.ns.svc.cluster.local:80/p" for i in range(5)]
        if rank == 1:
            names.append(123)  # not a string: every identity rule raises lazily
        for nm in names:
            d.shape_id(nm, {"http.method": "GET", "http.url": f"http://{nm}"})
        for v in (["200", "500"] if rank == 0 else ["404", "200", 200]):
            d.status_id(v)
        gt = exchange_tables(d)
        names = gather_names(gt, d, "dep")
        q.put((rank, names, [str(x) for x in gt.statuses], gt.digest, {r: sorted(gt.poison[r]) for r in ("rt", "tag", "dep")},
               [d.ep_names["dep"][e] == names[g] for e, g in enumerate(gt.ep_map["dep"])]))
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None, None))
    finally:
        dist.destroy_process_group()


def test_exchange_tables_agree_across_ranks():
    res = _spawn(_tables_worker, 3)
    for r in res:
        assert r[1] != "error", r[2]
    assert res[0][1] == res[1][1] == res[2][1]
    assert res[0][2] == res[1][2] == res[2][2]
    assert res[0][3] == res[1][3] == res[2][3]
    assert res[0][4] == res[1][4] == res[2][4]
    names = res[0][1]
    assert len([n for n in names if n is not None]) == len({n for n in names if n is not None}) == 7
    assert sum(n is None for n in names) == 1  # rank 1's poisoned shape
    # statuses: "200" (str) and 200 (number) are different group keys
    assert sorted(res[0][2]) == sorted(["200", "500", "404", "200"])
    for r in res:
        assert all(r[5])  # every local id maps to its own string
