"""Helpers of the traceId-sharding tests (test_shard.py, test_dist_engine.py):
a mixed Trace[][] batch and result views keyed by endpoint / status strings,
so shards with different local id tables compare with one whole-batch run."""
import json

import numpy as np

from conftest import fixture

U64 = np.uint64


def mixed_traces(n_mesh=300):
    """Synthetic mesh traces with the reference's Bookinfo and PDAS fixtures
    in between: shards see different shape sets and statuses."""
    from kmamiz_amd import synth

    b, off = synth.host_batch(synth.MESH, 0, n_mesh)
    mesh = synth.to_traces(synth.MESH, b, off)
    # a few 404/500 only in the fixtures' part, and an extra status string
    book = json.loads(json.dumps(fixture("MockTrace")))
    for i, t in enumerate(book):
        for s in t:
            if s.get("kind") == "SERVER" and i % 3 == 1:
                s.setdefault("tags", {})["http.status_code"] = "503"
    return mesh[: n_mesh // 2] + book + mesh[n_mesh // 2:] + [fixture("MockTracePDAS")]


def status_key(v):
    from kmamiz_amd.shard import _status_key

    return _status_key(v)


def oracle_by_name(traces, rule="tag"):
    """The C oracle over the whole batch (object ingest), keyed by strings."""
    from kmamiz_amd.ingest import ingest_traces
    from oracle import c_oracle

    batch, d, _ = ingest_traces(traces)
    t = d.shape_table()
    ep_of = t.tag_ep if rule == "tag" else t.rt_ep
    n_ep = t.n_tag_ep if rule == "tag" else t.n_rt_ep
    o = c_oracle.stats(batch, ep_of, n_ep, t.n_status)
    groups = {}
    for g in np.nonzero(o["combined"] > 0)[0].tolist():
        e, s = divmod(g, t.n_status)
        groups[(d.ep_names[rule][e], status_key(d.statuses[s]))] = (
            int(o["combined"][g]), int(o["first"][g]), int(o["latest_timestamp"][g]), float(o["mean"][g]),
            float(o["cv"][g]))
    keys, oep, _ = c_oracle.deps(batch, t.dep_ep, t.n_dep_ep)
    names = d.ep_names["dep"]
    edges = _edges(keys, names)
    eps = {}
    for e in range(t.n_dep_ep):
        if oep["has_row"][e] or oep["last"][e] != 0:
            eps[names[e]] = (bool(oep["has_row"][e]), int(oep["first"][e]) if oep["has_row"][e] else -1,
                             bool(oep["external"][e]) if oep["has_row"][e] else False, float(oep["last"][e]))
    return groups, edges, eps


def _edges(keys, names):
    k = np.asarray(keys, dtype=U64)
    a = (k >> U64(40)).astype(np.int64)
    d = ((k >> U64(16)) & U64(0xFFFFFF)).astype(np.int64)
    dist = ((k >> U64(1)) & U64(0x7FFF)).astype(np.int64)
    on = (k & U64(1)).astype(bool)
    return {(names[x], names[y], int(z), bool(w)) for x, y, z, w in zip(a.tolist(), d.tolist(), dist.tolist(),
                                                                        on.tolist())}


def groups_by_name(groups, ep_names, statuses):
    n_status = max(1, len(statuses))
    out = {}
    for g in np.nonzero(groups["combined"] > 0)[0].tolist():
        e, s = divmod(g, n_status)
        r = groups[g]
        out[(ep_names[e], status_key(statuses[s]))] = (int(r["combined"]), int(r["first"]),
                                                       int(r["latest_timestamp"]), float(r["mean"]), float(r["cv"]))
    return out


def endpoints_by_name(eps, names):
    out = {}
    for e in range(len(eps)):
        lt = int(eps["last_ts"][e])
        last = max(lt / 1000.0, 0.0) if lt != np.iinfo(np.int64).min else 0.0
        has = bool(eps["has_row"][e])
        if has or last != 0:
            out[names[e]] = (has, int(eps["first_row"][e]) if has else -1, bool(eps["external"][e]) if has else False,
                             last)
    return out


def assert_groups_equal(got, exp, rel=1e-9):
    assert set(got) == set(exp)
    for k, v in exp.items():
        g = got[k]
        assert g[:3] == v[:3], (k, g, v)
        assert abs(g[3] - v[3]) <= rel * abs(v[3]), (k, g, v)
        assert abs(g[4] - v[4]) <= rel * abs(v[4]) + 1e-13, (k, g, v)
