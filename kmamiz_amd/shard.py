"""Sharding a batch by traceId over the GPUs of one node.

The reference runs the whole path in one process over one ``Trace[][]``
(``new Traces(traces)``, Traces.ts:17-21).  Here rank r of G owns the traces
whose ``shard(t[0].traceId) == r`` (``kmz_trace_shard``; the reference keys a
trace by ``t[0].traceId``, RealtimeWorkerImpl.ts:17-27), keeps them in their
global order, and runs the whole pipeline on them.  Three things make the
merged result equal to the single-process one:

* global flatten indices: each rank's index map (``kmz_set_index_map``) turns
  its local indices into positions of ``this._traces.flat()`` (Traces.ts:29),
  so first-occurrence order (RealtimeDataList.ts:23-45, Traces.ts:117-127)
  survives the merge;
* global dense ids: endpoints (per identity rule) and status strings are keyed
  by their strings (``uniqueEndpointName``, RealtimeDataList.ts:23-27;
  ``Traces.ts:35,78,226-238``).  Each rank hashes its distinct keys, the ranks
  all-gather the 64-bit hashes (a tensor collective: RCCL or gloo), and every
  rank assigns the same dense ids in first-occurrence order over the ranks.  A
  second, independent 64-bit hash per key is all-reduced per id: two different
  strings behind one id would differ there, and the batch is refused;
* the merge itself (:func:`kmamiz_amd.dist.merge_all`), guarded by a digest of
  the id tables every rank used.
"""
from __future__ import annotations

import hashlib
import json
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .engine import Engine, ShapeTable, SpanBatch
from .ingest import UNDEFINED, Dictionary, tpl

RULES = ("rt", "tag", "dep")
_MASK62 = (1 << 62) - 1


def trace_shard(trace_id, world: int) -> int:
    """kmz_trace_shard of a traceId value (JS template string of it)."""
    s = tpl(trace_id).encode("utf-8", "surrogatepass") if not isinstance(trace_id, str) else trace_id.encode(
        "utf-8", "surrogatepass")
    return int(L.lib().kmz_trace_shard(s, len(s), world))


def _trace_key(trace) -> object:
    return trace[0].get("traceId", UNDEFINED) if len(trace) else ""


@dataclass
class ShardPlan:
    """One rank's part of a Trace[][]: its traces in global order and the
    local/global flatten start of each (the kmz_set_index_map runs)."""

    traces: list
    local_start: np.ndarray
    global_start: np.ndarray


def shard_traces(traces: Sequence[Sequence[dict]], world: int) -> List[ShardPlan]:
    plans = [ShardPlan([], [], []) for _ in range(world)]
    local = [0] * world
    g = 0
    for t in traces:
        r = trace_shard(_trace_key(t), world)
        p = plans[r]
        p.local_start.append(local[r])
        p.global_start.append(g)
        p.traces.append(t)
        local[r] += len(t)
        g += len(t)
    for p in plans:
        p.local_start = np.asarray(p.local_start or [0], dtype=np.uint64)
        p.global_start = np.asarray(p.global_start or [0], dtype=np.uint64)
    return plans


def _hash2(key: str) -> Tuple[int, int]:
    d = hashlib.blake2b(key.encode("utf-8", "surrogatepass"), digest_size=16).digest()
    return int.from_bytes(d[:8], "little") & _MASK62, int.from_bytes(d[8:], "little") & _MASK62


def _status_key(v) -> str:
    return json.dumps([type(v).__name__, None if v is UNDEFINED else v])


@dataclass
class GlobalTables:
    """Dense ids every rank agreed on (see the module docstring)."""

    ep_map: Dict[str, np.ndarray]  # rule -> local endpoint id -> global id
    n_ep: Dict[str, int]
    status_map: np.ndarray  # local status id -> global id
    statuses: list  # global status id -> value (every rank knows them all)
    owner: Dict[str, np.ndarray]  # rule -> global id -> first rank that has it
    local_of: Dict[str, Dict[int, int]]  # rule -> global id -> local id (ids this rank has)
    poison: Dict[str, set]  # rule -> global ids whose identity raises in the reference
    digest: int  # 62-bit digest of the tables (merge_all's guard)
    rank: int

    def shape_table(self, d: Dictionary) -> ShapeTable:
        return ShapeTable(self.ep_map["rt"][np.asarray(d.shape_ep["rt"], dtype=np.int64)],
                          self.ep_map["tag"][np.asarray(d.shape_ep["tag"], dtype=np.int64)],
                          self.ep_map["dep"][np.asarray(d.shape_ep["dep"], dtype=np.int64)],
                          self.n_ep["rt"], self.n_ep["tag"], self.n_ep["dep"], max(1, len(self.statuses)))

    def remap_batch(self, b: SpanBatch) -> SpanBatch:
        st = self.status_map[b.status.astype(np.int64)] if len(b) else b.status
        return SpanBatch(b.span_id, b.parent_id, b.kind, b.shape, st.astype(np.uint16), b.duration, b.timestamp, 0)


def _keys_of(d: Dictionary, rank: int) -> Tuple[Dict[str, List[str]], List[str]]:
    eps = {}
    for rule in RULES:
        eps[rule] = [n if n is not None else f"\x00poison\x00{rank}\x00{e}" for e, n in enumerate(d.ep_names[rule])]
    return eps, [_status_key(v) for v in d.statuses]


def exchange_tables(d: Dictionary, device=None, group=None) -> GlobalTables:
    """Collective: every rank of the default (or given) process group calls it
    with its own Dictionary.  ``device``: where the collective tensors live
    (a CUDA device for RCCL, None / cpu for gloo)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = torch.device(device) if device is not None else torch.device("cpu")
    eps, sts = _keys_of(d, rank)
    lists = [eps[r] for r in RULES] + [sts]
    h = [np.array([_hash2(k) for k in lst], dtype=np.int64).reshape(-1, 2) for lst in lists]
    sizes = torch.tensor([len(x) for x in h], dtype=torch.int64, device=dev)
    if world > 1:
        allsz = torch.empty(world * 4, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allsz, sizes, group=group)
        allsz = allsz.cpu().numpy().reshape(world, 4)
    else:
        allsz = sizes.cpu().numpy().reshape(1, 4)
    m = int(allsz.sum(axis=1).max())
    mine = np.zeros(max(1, m), dtype=np.int64)
    cat = np.concatenate([x[:, 0] for x in h]) if m else np.zeros(0, np.int64)
    mine[: len(cat)] = cat
    if world > 1:
        t = torch.from_numpy(mine).to(dev)
        allh = torch.empty(world * len(mine), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allh, t, group=group)
        allh = allh.cpu().numpy().reshape(world, len(mine))
    else:
        allh = mine.reshape(1, -1)
    # per list: global ids in first-occurrence order over (rank, local position)
    maps, n_of, owners, uniq_of = [], [], [], []
    for j in range(4):
        parts, rk = [], []
        for r in range(world):
            off = int(allsz[r, :j].sum())
            parts.append(allh[r, off:off + int(allsz[r, j])])
            rk.append(np.full(int(allsz[r, j]), r, dtype=np.int64))
        flat = np.concatenate(parts) if parts else np.zeros(0, np.int64)
        ranks = np.concatenate(rk) if rk else np.zeros(0, np.int64)
        u, first = np.unique(flat, return_index=True)
        order = np.argsort(first, kind="stable")  # global id = rank of first occurrence
        gid_of_u = np.empty(len(u), dtype=np.int64)
        gid_of_u[order] = np.arange(len(u))
        uniq_of.append((u, gid_of_u))
        mh = h[j][:, 0]
        maps.append(gid_of_u[np.searchsorted(u, mh)] if len(mh) else np.zeros(0, np.int64))
        n_of.append(len(u))
        owners.append(ranks[first[order]])
    # exact check: the second hash of every key agrees across ranks per id
    tot = sum(n_of)
    hi = np.full(tot, -1, dtype=np.int64)
    lo = np.full(tot, -(1 << 62), dtype=np.int64)
    base = 0
    for j in range(4):
        hi[base + maps[j]] = h[j][:, 1]
        lo[base + maps[j]] = -h[j][:, 1]
        base += n_of[j]
    chk = np.concatenate([hi, lo])
    if world > 1 and tot:
        ct = torch.from_numpy(chk).to(dev)
        dist.all_reduce(ct, op=dist.ReduceOp.MAX, group=group)
        chk = ct.cpu().numpy()
    if not np.array_equal(chk[:tot], -chk[tot:]):
        raise HashCollision("two distinct endpoint/status strings share a 64-bit hash: run unsharded")
    # statuses: every rank needs their values (group ids are endpoint * n_status + status)
    st_vals = _gather_statuses(d, maps[3], n_of[3], world, group)
    digest = int.from_bytes(hashlib.blake2b(np.concatenate([u for u, _ in uniq_of] +
                                                           [np.array(n_of, dtype=np.int64)]).tobytes(),
                                            digest_size=8).digest(), "little") & _MASK62
    poison = {}
    for j, rule in enumerate(RULES):
        poison[rule] = {int(maps[j][e]) for e in d.poison[rule]}
    # poison ids of other ranks: their keys start with a NUL, which no
    # uniqueEndpointName does; every rank learns them from the owners' lists
    poison_all = _allgather_obj({rule: sorted(poison[rule]) for rule in RULES}, world, group)
    for p in poison_all:
        for rule in RULES:
            poison[rule].update(p[rule])
    return GlobalTables(
        ep_map={rule: maps[j].astype(np.uint32) for j, rule in enumerate(RULES)},
        n_ep={rule: n_of[j] for j, rule in enumerate(RULES)},
        status_map=maps[3].astype(np.uint16),
        statuses=st_vals,
        owner={rule: owners[j] for j, rule in enumerate(RULES)},
        local_of={rule: {int(g): e for e, g in enumerate(maps[j].tolist())} for j, rule in enumerate(RULES)},
        poison=poison,
        digest=digest,
        rank=rank,
    )


class HashCollision(RuntimeError):
    pass


def gather_names(gt: GlobalTables, d: Dictionary, rule: str, group=None) -> list:
    """Collective: the uniqueEndpointName of every global id of ``rule``
    (None for ids whose identity raises), assembled from the ranks that have
    them.  For materialising results on any rank."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    mine = {int(g): d.ep_names[rule][e] for e, g in enumerate(gt.ep_map[rule].tolist())}
    out: list = [None] * gt.n_ep[rule]
    for part in _allgather_obj(mine, world, group):
        for g, n in part.items():
            if out[g] is None:
                out[g] = n
    return out


def _allgather_obj(obj, world, group):
    import torch.distributed as dist

    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj, group=group)
    return out


def _gather_statuses(d: Dictionary, gmap: np.ndarray, n: int, world: int, group) -> list:
    vals: list = [None] * n
    have = [False] * n
    for lst in _allgather_obj([(int(g), _status_key(v)) for g, v in zip(gmap.tolist(), d.statuses)], world, group):
        for g, k in lst:
            if not have[g]:
                t, v = json.loads(k)
                vals[g] = UNDEFINED if t == "_Undef" else v
                have[g] = True
    return vals


@dataclass
class ShardResult:
    """The merged results every rank holds after :func:`run_sharded`."""

    tables: GlobalTables
    groups: Optional[np.ndarray]  # kmz_group records, [n_ep * n_status] of the stats rule
    keys: Optional[np.ndarray]  # sorted unique edge keys (global dep ids)
    endpoints: Optional[np.ndarray]  # kmz_endpoint records per global dep id
    rule: Optional[str]


def run_sharded(engine: Engine, batch: SpanBatch, d: Dictionary, local_start, global_start, flags: int,
                group=None, tensor_device=None) -> ShardResult:
    """One rank's part of the sharded hot path: global ids, load, run, merge.
    Every rank returns the merged result of the whole batch.  The collective
    tensors live on the GPU under RCCL and on the CPU under gloo (or where
    ``tensor_device`` says)."""
    import torch
    import torch.distributed as dist

    from . import dist as kdist

    backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
    if tensor_device is not None:
        dev = torch.device(tensor_device)
    else:
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    gt = exchange_tables(d, dev, group)
    engine.load(gt.remap_batch(batch), gt.shape_table(d))
    engine.set_index_map(local_start, global_start)
    engine.run(flags)
    stats = bool(flags & (L.RUN_STATS_RT | L.RUN_STATS_TAG))
    deps = bool(flags & L.RUN_DEPS)
    on_dev = dev.type == "cuda"
    g = e = t = None
    gw = engine.partials_words(L.PART_GROUPS) if stats else 0
    ew = engine.partials_words(L.PART_ENDPOINTS) if deps else 0
    tw = engine.partials_words(L.PART_TRIPLES) if deps else 0
    g = torch.zeros(max(1, gw), dtype=torch.int64, device=dev)
    e = torch.zeros(max(1, ew), dtype=torch.int64, device=dev)
    t = torch.zeros(max(1, tw), dtype=torch.int64, device=dev)
    if stats:
        engine.export_partials(L.PART_GROUPS, g.data_ptr(), gw, on_dev)
    if deps:
        engine.export_partials(L.PART_ENDPOINTS, e.data_ptr(), ew, on_dev)
        engine.export_partials(L.PART_TRIPLES, t.data_ptr(), tw, on_dev)
    kdist.merge_all(g[:gw], gw // 6, e[:ew], ew // 2, t[:tw], engine=engine if deps else None, digest=gt.digest,
                    group=group)
    if stats:
        engine.import_partials(L.PART_GROUPS, g.data_ptr(), gw, on_dev)
        engine.finalize()
    if deps:
        engine.import_partials(L.PART_ENDPOINTS, e.data_ptr(), ew, on_dev)
    groups, keys, eps = engine.fetch(groups=stats, deps=deps)
    rule = "rt" if flags & L.RUN_STATS_RT else ("tag" if stats else None)
    res = ShardResult(gt, groups.copy() if stats else None, np.sort(keys) if deps else None, eps, rule)
    _check_poison(res, d)
    return res


def _check_poison(res: ShardResult, d: Dictionary):
    """The reference throws (Utils.ts:90) when it evaluates an identity that
    cannot be built; the sharded run raises once such an id is used."""
    gt = res.tables
    n_status = max(1, len(gt.statuses))
    used = []
    if res.groups is not None and gt.poison[res.rule]:
        ep = np.nonzero(res.groups["combined"] > 0)[0] // n_status
        used += [(res.rule, int(x)) for x in np.intersect1d(ep, sorted(gt.poison[res.rule]))]
    if res.endpoints is not None and gt.poison["dep"]:
        pe = np.array(sorted(gt.poison["dep"]), dtype=np.int64)
        if np.any(res.endpoints["has_row"][pe]) or np.any(np.isin((res.keys >> np.uint64(40)).astype(np.int64), pe)):
            used.append(("dep", int(pe[0])))
    for rule, gid in used:
        loc = gt.local_of[rule].get(gid)
        if loc is not None and loc in d.poison[rule]:
            for sh, ep in enumerate(d.shape_ep[rule]):
                if ep == loc:
                    raise d.shape_ident[rule][sh].error
        raise TypeError("Cannot read properties of undefined (reading 'match')")
