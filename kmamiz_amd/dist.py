"""Multi-GPU merge of traceId-sharded batches.

Each rank runs the whole pipeline on its own shard (whole traces, global
flatten indices via ``index_base``); no span crosses a GPU.  The per-rank
partials then merge with collectives over the default process group:

* group partials    [count, sum d, sum lo32(d^2), sum hi32(d^2)]  all_reduce SUM
                    [max timestamp]                                all_reduce MAX
                    [min first index]                              all_reduce MIN
* endpoint partials [max timestamp] MAX, [min first_row<<1|!external] MIN
* guards            a fixed-size agreement all-reduce (id tables, sizes), the
                    unresolved-parent exchange and the cross-shard repeated
                    span-id check (an all-to-all of hashed ids by owner rank)
* edge keys         size all_reduce MAX, padded all_gather, then a union:
                    into the engine's own device edge set (kmz_merge_triples,
                    ``merge_edge_keys_into``) or ``torch.unique`` (CPU tensors)

Integer moments make the merge exact: the merged groups are bit-identical to a
single-GPU run over the whole batch (the reference's pooled-variance formula,
CombinedRealtimeDataList.ts:278-315, is not needed for this).

Works with any backend: ``nccl`` (RCCL over xGMI) on device tensors in
production, ``gloo`` on CPU tensors in the tests.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

_BIAS = -(1 << 63)  # flips the sign bit: u64 order <-> i64 order
_I64_MAX = (1 << 63) - 1


def _engine_reads(engine, t: torch.Tensor) -> None:
    """Before the engine reads a device tensor that torch (or a collective on
    torch's stream) produced: wait for torch's stream unless the engine
    launches on that same stream."""
    if t.is_cuda and getattr(engine, "stream", None) != torch.cuda.current_stream(t.device).cuda_stream:
        torch.cuda.current_stream(t.device).synchronize()


def _as_signed_order(x: torch.Tensor) -> torch.Tensor:
    return torch.bitwise_xor(x, torch.tensor(_BIAS, dtype=torch.int64, device=x.device))


def merge_group_partials(p: torch.Tensor, n_groups: int) -> torch.Tensor:
    """In-place merge of a [6 * G] int64 view of the u64 group partials."""
    G = n_groups
    if dist.get_world_size() == 1 or G == 0:
        return p
    dist.all_reduce(p[: 4 * G], op=dist.ReduceOp.SUM)  # modular: exact for u64
    ts = _as_signed_order(p[4 * G : 5 * G])
    dist.all_reduce(ts, op=dist.ReduceOp.MAX)
    p[4 * G : 5 * G] = _as_signed_order(ts)
    first = p[5 * G :]
    first = torch.where(first == -1, torch.full_like(first, _I64_MAX), first)
    dist.all_reduce(first, op=dist.ReduceOp.MIN)
    p[5 * G :] = torch.where(first == _I64_MAX, torch.full_like(first, -1), first)
    return p


def merge_endpoint_partials(e: torch.Tensor, n_ep: int) -> torch.Tensor:
    """In-place merge of a [2 * E] int64 view of the endpoint partials."""
    if dist.get_world_size() == 1 or n_ep == 0:
        return e
    ts = _as_signed_order(e[:n_ep])
    dist.all_reduce(ts, op=dist.ReduceOp.MAX)
    e[:n_ep] = _as_signed_order(ts)
    f = e[n_ep:]
    f = torch.where(f == -1, torch.full_like(f, _I64_MAX), f)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    e[n_ep:] = torch.where(f == _I64_MAX, torch.full_like(f, -1), f)
    return e


def merge_all(p: torch.Tensor, n_groups: int, e: torch.Tensor, n_ep: int, keys: torch.Tensor, engine=None,
              digest: int = 0, group=None, check_ids: bool = True, exact: bool = True):
    """The whole per-step merge: one fixed-size MAX all-reduce that makes the
    ranks agree (group/endpoint counts, the id-table digest, the unresolved
    parent count) before any size-dependent collective, the sharding guards,
    then one SUM all-reduce of the group moments, one MAX all-reduce that
    carries every max field and every min field negated (min x = -max -x in
    signed order) plus the edge-key count, and one all-gather of the padded
    keys.  Same results as merge_group_partials + merge_endpoint_partials +
    merge_edge_keys(_into); returns the merged keys when ``engine`` is None.

    The same collective calls run on device tensors (RCCL) and on CPU tensors
    (gloo), so the CPU tests exercise the production sequence.  ``digest``:
    a digest of the endpoint/status id tables this rank's partials are indexed
    by (shard.exchange_tables); ranks that disagree raise ShardingError.
    ``check_ids`` (with an engine): the cross-shard repeated-span-id guard
    (check_repeated_ids) before the merge; an IdGuard started before the run
    is finished here instead."""
    world = dist.get_world_size(group)
    if world == 1:
        return None if engine is not None else torch.unique(keys)
    G, E = n_groups, n_ep
    dev = p.device
    # agreement first: every later collective's size depends on G and E
    # (ranks that disagree would hang RCCL or fail inside gloo before a clear
    # error); the sharding guard's count rides along
    # (a shard on the span-table path is refused on every rank, not just on
    # its own: a local raise would leave the others blocked in this all-reduce)
    refused = None
    try:
        nu = _unresolved(engine) if engine is not None else 0
    except ShardingError as err:
        nu, refused = 0, err
    dg = int(digest) & ((1 << 62) - 1)
    agree = torch.tensor([G, -G, E, -E, dg, -dg, nu, 1 if refused else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(agree, op=dist.ReduceOp.MAX, group=group)
    a = agree.tolist()
    if a[0] != -a[1] or a[2] != -a[3] or a[4] != -a[5]:
        if isinstance(check_ids, IdGuard):
            check_ids.abandon()
        raise ShardingError("ranks merged partials over different endpoint/status id tables "
                            "(assign global ids with shard.exchange_tables)")
    # the sharding guards: a span-id map that crosses shards (an id repeated
    # inside a shard or across shards, a parent in another shard) makes the
    # per-shard dependency results differ from the reference's global Map
    # (Traces.ts:117-143).  With an engine the merge stays exact: the whole
    # batch's dependency pass is re-run on one rank (_unsharded_deps); without
    # one, or with ``exact=False``, every rank raises ShardingError.
    crossed = bool(a[7])
    if crossed and isinstance(check_ids, IdGuard):
        check_ids.abandon()  # its exchange was posted before the run: drain it on every rank
    if not crossed and a[6] > 0:
        try:
            crossed = _check_shards(engine, nu, int(a[6]), dev, group, raise_=not exact)
        except ShardingError:
            if isinstance(check_ids, IdGuard):
                check_ids.abandon()
            raise
        if crossed and isinstance(check_ids, IdGuard):
            check_ids.abandon()  # posted before the run: drained before the exact merge's collectives
    if not crossed:
        if isinstance(check_ids, IdGuard):  # started before the run: its exchange overlapped it
            crossed = check_ids.finish(raise_=not exact)
        elif engine is not None and check_ids:
            crossed = IdGuard(engine, dev, group).start().finish(raise_=not exact)
    if crossed and (engine is None or not exact):
        raise refused or ShardingError("another rank's shard has repeated span ids: sharding is not exact, "
                                       "run unsharded")
    if crossed:
        # the stats are exact per shard (realtime rows keep repeated ids,
        # Traces.ts:28-31) and merge as usual; the dependency results come
        # from one pass over the whole batch
        if G:
            _merge_groups_only(p, G, group)
        _unsharded_deps(engine, e, E, dev, group)
        return None
    if G:
        dist.all_reduce(p[: 4 * G], op=dist.ReduceOp.SUM, group=group)  # modular: exact for u64
    ming = p[5 * G : 6 * G]
    mine = e[E : 2 * E]
    mx = torch.cat([
        _as_signed_order(p[4 * G : 5 * G]),
        _as_signed_order(e[:E]),
        -torch.where(ming == -1, torch.full_like(ming, _I64_MAX), ming),
        -torch.where(mine == -1, torch.full_like(mine, _I64_MAX), mine),
        torch.tensor([keys.numel()], dtype=torch.int64, device=dev),
    ])
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    nk = int(mx[-1].item())
    p[4 * G : 5 * G] = _as_signed_order(mx[:G])
    e[:E] = _as_signed_order(mx[G : G + E])
    fg = -mx[G + E : 2 * G + E]
    fe = -mx[2 * G + E : 2 * G + 2 * E]
    p[5 * G : 6 * G] = torch.where(fg == _I64_MAX, torch.full_like(fg, -1), fg)
    e[E : 2 * E] = torch.where(fe == _I64_MAX, torch.full_like(fe, -1), fe)
    allk = _gather_padded(keys, nk, world, group)
    if engine is not None:
        _engine_reads(engine, allk)
        engine.merge_triples(allk.data_ptr(), allk.numel(), keys.is_cuda)
        return None
    u = torch.unique(allk)
    return u[u != 0]


# ---- cross-shard repeated span ids -------------------------------------------
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def id_hash_np(ids: np.ndarray) -> np.ndarray:
    """kmz_common.h id_hash (the certificate's bijection) over uint64 ids."""
    with np.errstate(over="ignore"):
        x = ids.astype(np.uint64) * _GOLD
    return x ^ (x >> np.uint64(29))


def id_owner_np(h: np.ndarray, world: int) -> np.ndarray:
    """kmz_common.h id_owner: the owner rank of each hashed id."""
    return ((h >> np.uint64(32)) * np.uint64(world)) >> np.uint64(32)


def route_ids_np(span_ids: np.ndarray, world: int):
    """Host mirror of kmz_route_ids: (hashes grouped by owner, counts)."""
    h = id_hash_np(np.asarray(span_ids, dtype=np.uint64))
    own = id_owner_np(h, world).astype(np.int64)
    order = np.argsort(own, kind="stable")
    return h[order], np.bincount(own, minlength=world).astype(np.int64)


# agreed fixed-segment size of IdGuard's exchange per (group, world): set on
# every rank from the same all-reduced maximum in IdGuard.finish; each entry
# keeps its group object (IdGuard._seg_size)
_ID_SEG: dict = {}
# per device: the stream IdGuard's certificate runs on (it waits for the
# exchange there, beside the rank's own run)
_GUARD_STREAMS: dict = {}


def _guard_stream(dev: torch.device):
    s = _GUARD_STREAMS.get(dev.index)
    if s is None:
        s = _GUARD_STREAMS[dev.index] = torch.cuda.Stream(dev)
    return s


class IdGuard:
    """The cross-shard repeated-span-id check (check_repeated_ids) split in
    two, so that its all-to-all overlaps the run.

    ``start()`` routes this rank's id hashes and posts the exchange.  Once the
    ranks have agreed on a segment size (the previous finish()), the routing
    writes fixed segments (kmz_route_ids_fixed: each owner's count, then its
    values) and the exchange is an all-to-all of equal segments, so start()
    only enqueues: no counts exchange and no stream synchronisation before the
    run (under RCCL the all-to-all is posted on device tensors behind the
    routing; under gloo, CPU-only, the copy and the exchange wait for
    finish()).  The first call, and any step whose segment overflowed on some
    rank, use the exact protocol: the counts all-to-all, then the values with
    those split sizes.  Under RCCL with fixed segments start() also enqueues
    the uniqueness certificate over the segments as they arrive
    (kmz_id_repeats_seg_begin) on a stream of its own that waits for the
    exchange, so the check runs beside this rank's run too; ``finish()`` waits
    for its verdict (elsewhere it runs the certificate over what this rank
    received: kmz_id_repeats_seg_* or kmz_id_repeats) and agrees on the
    verdict and the next segment size in one MAX all-reduce, raising
    ShardingError on a repeat.

    Every span id of every shard, the owner's own included, is routed and
    checked, so a repeat inside one shard is found too: a run covered by a
    guard may skip its own certificate (KMZ_RUN_NO_CERT).

    ``start(fold=True)`` (RCCL, fixed segments) instead arms the routing into
    the next run (kmz_route_ids_join: the run's join writes the segments from
    the id hashes it bins anyway, no pass of its own); the caller runs
    ``post()`` after ``run_begin``, which posts the exchange on the guard's
    stream behind the join (kmz_route_wait) and the certificate behind it,
    both beside the rest of the run."""

    def __init__(self, engine=None, dev=None, group=None, span_ids: Optional[np.ndarray] = None, *,
                 world: Optional[int] = None, backend: Optional[str] = None):
        # (world / backend: given only by a single-process test that stands in
        # for the collectives, _a2a and _agree; otherwise the group's)
        self.engine, self.group, self.span_ids = engine, group, span_ids
        self.world = world if world is not None else dist.get_world_size(group)
        backend = backend if backend is not None else dist.get_backend(group)
        # device tensors under RCCL; host tensors under gloo (its all-to-all is CPU-only)
        self.on_dev = (engine is not None and dev is not None and torch.device(dev).type == "cuda"
                       and backend == "nccl")
        self.dev = torch.device(dev) if self.on_dev else torch.device("cpu")
        # (gloo with the engine on a GPU: the routing is still enqueued on the device)
        self.route_dev = (torch.device(dev) if engine is not None and dev is not None
                          and torch.device(dev).type == "cuda" else None)
        self.gobj = group if group is not None or world is not None else dist.distributed_c10d._get_default_group()
        self.work = self.fixed = self.pending = None
        self.seg_open = False  # kmz_id_repeats_seg_begin enqueued, not yet ended
        self.armed = False  # start(fold=True): routing armed into the next run, exchange not yet posted
        self.in_join = None  # post(): whether the run's join wrote the segments (else its fallback pass)

    # the guard's collectives (a single-process test overrides both)
    def _a2a(self, out, inp, out_splits=None, in_splits=None, async_op=False):
        return dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits,
                                      group=self.group, async_op=async_op)

    def _agree(self, flag: torch.Tensor) -> None:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)

    def _seg_size(self) -> Optional[int]:
        """The segment size every rank agreed on in this group's last finish(),
        or None (no finish() yet: the counts protocol).  The entry holds the
        group object itself and is used only while that very object is the
        group, so a destroyed group whose id() a new group reuses, or a
        re-initialised default group, starts over with the counts protocol on
        every rank (ranks that disagreed here would post different
        all-to-alls and hang under RCCL)."""
        e = _ID_SEG.get((id(self.gobj), self.world))
        return e[1] if e is not None and e[0] is self.gobj else None

    def start(self, fold: bool = False) -> "IdGuard":
        if self.world == 1:
            return self
        seg = self._seg_size() if self.engine is not None else None
        if seg is not None and fold and self.on_dev:
            # the run routes (kmz_route_ids_join); post() exchanges after run_begin
            self.fixed = seg
            self.send = torch.empty(self.world * seg, dtype=torch.int64, device=self.route_dev)
            self.recv = torch.empty_like(self.send)
            self.engine.route_ids_join(self.world, seg, self.send.data_ptr())
            self.armed = True
            return self
        if seg is not None:
            self.fixed = seg
            if self.route_dev is not None:  # enqueued on the engine's stream, no wait
                send = torch.empty(self.world * seg, dtype=torch.int64, device=self.route_dev)
                self.engine.route_ids_fixed(self.world, seg, send.data_ptr(), True)
                if self.on_dev and getattr(self.engine, "stream", None) != torch.cuda.current_stream(
                        self.route_dev).cuda_stream:
                    # (the exchange is ordered behind torch's stream: an engine
                    # on a stream of its own is waited for here; the bench's
                    # engine runs on torch's stream and needs no wait)
                    self.engine.sync()
            else:
                send = torch.empty(self.world * seg, dtype=torch.int64)
                self.engine.route_ids_fixed(self.world, seg, send.data_ptr(), False)
            if self.on_dev:
                self.recv = torch.empty_like(send)
                self.send = send
                self.work = self._a2a(self.recv, send, async_op=True)
                # the certificate over the segments as they arrive, on the
                # guard's stream behind the exchange (no host wait): it runs
                # beside this rank's run, finish() reads its verdict
                gs = _guard_stream(self.route_dev)
                with torch.cuda.stream(gs):
                    self.work.wait()
                self.recv.record_stream(gs)
                try:
                    self.engine.id_repeats_seg_begin(self.recv.data_ptr(), self.world, seg, gs.cuda_stream)
                    self.seg_open = True
                except Exception:  # noqa: BLE001 (the certificate cannot take it: finish() checks by compaction)
                    self.seg_open = False
            else:
                self.pending = send  # (gloo: copied and exchanged in finish)
            return self
        return self._start_counts()

    def post(self) -> "IdGuard":
        """After run_begin of the run start(fold=True) armed: the exchange on
        the guard's stream once the run's join has written the segments, and
        the certificate over what arrives, both beside the rest of the run
        (every rank posts it, in the same order as its other collectives)."""
        if not self.armed:
            return self
        self.armed = False
        gs = _guard_stream(self.route_dev)
        self.in_join = self.engine.route_wait(gs.cuda_stream)
        with torch.cuda.stream(gs):
            self.work = self._a2a(self.recv, self.send, async_op=True)
            self.work.wait()
        self.send.record_stream(gs)
        self.recv.record_stream(gs)
        try:
            self.engine.id_repeats_seg_begin(self.recv.data_ptr(), self.world, self.fixed, gs.cuda_stream)
            self.seg_open = True
        except Exception:  # noqa: BLE001 (the certificate cannot take it: finish() checks by compaction)
            self.seg_open = False
        return self

    def _start_counts(self) -> "IdGuard":
        """The exact protocol: counts first, then the values with those splits."""
        self.fixed = None
        if self.engine is not None:
            n = int(self.engine.n)
            send = torch.empty(max(1, n), dtype=torch.int64, device=self.dev)
            counts = self.engine.route_ids(self.world, send.data_ptr(), n, self.on_dev)
            send = send[:n]
        else:
            h, c = route_ids_np(self.span_ids, self.world)
            send = torch.from_numpy(h.view(np.int64).copy())
            counts = c.tolist()
        cnt = torch.tensor(counts, dtype=torch.int64, device=self.dev)
        rcnt = torch.empty_like(cnt)
        self._a2a(rcnt, cnt)
        rc = rcnt.tolist()
        self.recv = torch.empty(max(1, sum(rc)), dtype=torch.int64, device=self.dev)
        self.m = sum(rc)
        self.maxc = max(rc) if rc else 0
        self.send = send  # (kept alive until the exchange is done)
        self.work = self._a2a(self.recv[: self.m], send, rc, counts, async_op=True)
        return self

    def abandon(self) -> None:
        """Wait for a posted exchange without checking it (every rank calls
        this when the merge is refused before the guard's verdict)."""
        if self.armed:  # (its exchange is still every rank's to post)
            self.post()
        if self.seg_open:  # (its certificate reads the received segments: wait for it)
            self.seg_open = False
            self.engine.id_repeats_seg_end()
        if self.work is not None:
            self.work.wait()
        if self.pending is not None:  # (gloo, fixed segments: the exchange every rank still posts)
            if self.route_dev is not None:
                self.engine.sync()
            send = self.pending.cpu()
            self._a2a(torch.empty_like(send), send)
        self.work = self.send = self.recv = self.pending = None

    def _received(self):
        """-> (this rank's received values, the largest count any source sent
        it, whether some source's segment overflowed)."""
        if self.fixed is None:
            self.work.wait()
            return self.recv[: self.m], self.maxc, False
        seg = self.fixed
        if self.pending is not None:
            if self.route_dev is not None:
                self.engine.sync()  # (the routing ran on the engine's stream, not torch's)
            send = self.pending.cpu()
            self.pending = None
            self.recv = torch.empty_like(send)
            self._a2a(self.recv, send)
        else:
            self.work.wait()
        r = self.recv.view(self.world, seg)
        cnt = r[:, 0]
        maxc = int(cnt.max().item())
        if maxc >= seg:
            return None, maxc, True
        keep = torch.arange(seg - 1, device=r.device)[None, :] < cnt[:, None]
        return r[:, 1:][keep], maxc, False

    def _seg_verdict(self):
        """Fixed segments, engine on a GPU: the certificate over the segments
        as received (kmz_id_repeats_seg_*; under gloo the exchange runs here on
        the host and the segments go to the device first).  -> (repeated, the
        largest count any source sent, whether a segment overflowed)."""
        seg = self.fixed
        if not self.seg_open:
            self.engine.sync()  # (the routing ran on the engine's stream)
            send = self.pending.cpu()
            self.pending = None
            recv = torch.empty_like(send)
            self._a2a(recv, send)
            self.recv = recv.to(self.route_dev)
            try:
                self.engine.id_repeats_seg_begin(self.recv.data_ptr(), self.world, seg,
                                                 torch.cuda.current_stream(self.route_dev).cuda_stream)
                self.seg_open = True
            except Exception:  # noqa: BLE001 (the certificate cannot take it: compaction below, and every rank still agrees)
                self.seg_open = False
        if self.seg_open:
            self.seg_open = False
            rep, maxc = self.engine.id_repeats_seg_end()
        else:
            rep, maxc = None, int(self.recv.view(self.world, seg)[:, 0].max().item())
        over = maxc >= seg
        if rep is None and not over:  # the certificate could not decide: compact and check on the host
            r = self.recv.view(self.world, seg)
            keep = torch.arange(seg - 1, device=r.device)[None, :] < r[:, :1]
            v = r[:, 1:][keep]
            rep = bool(v.numel()) and torch.unique(v).numel() != v.numel()
        return rep, maxc, over

    def finish(self, raise_: bool = True) -> bool:
        """-> True when some span id is in two shards (ShardingError instead
        with ``raise_``)."""
        if self.world == 1:
            return False
        if self.armed:
            self.post()
        if self.work is None and self.pending is None and not self.seg_open:
            self.start()
        if (self.fixed is not None and self.engine is not None and self.route_dev is not None
                and (self.seg_open or self.pending is not None)):
            rep, maxc, over = self._seg_verdict()
        else:
            recv, maxc, over = self._received()
            rep = None
            if not over:
                if self.on_dev:
                    torch.cuda.current_stream(self.dev).synchronize()  # (the engine's stream may not be torch's)
                if self.engine is not None and recv.numel():
                    rep = self.engine.id_repeats(recv.data_ptr(), recv.numel(), self.on_dev)
                if rep is None:  # host check (no engine, or the certificate could not decide)
                    rep = bool(recv.numel()) and torch.unique(recv).numel() != recv.numel()
        # one MAX all-reduce: the verdict, any overflow, the largest count (the
        # next step's segment size, the same on every rank)
        flag = torch.tensor([1 if rep else 0, 1 if over else 0, maxc], dtype=torch.int64, device=self.dev)
        self._agree(flag)
        f = flag.tolist()
        self.work = self.send = self.recv = None
        if self.engine is not None:
            _ID_SEG[(id(self.gobj), self.world)] = (self.gobj, int(f[2] * 1.125) + 1025)
        if f[1]:  # a segment overflowed somewhere: this step exactly, every rank
            self._start_counts()
            return self.finish(raise_)
        if f[0] and raise_:
            raise ShardingError("a span id occurs in two shards: the reference's global span map would merge them "
                                "(Traces.ts:117-123); run unsharded")
        return bool(f[0])


def check_repeated_ids(engine=None, dev=None, group=None, span_ids: Optional[np.ndarray] = None) -> None:
    """Raise ShardingError if a span id occurs in two shards.

    The reference keys one Map by span id over the whole batch
    (Traces.ts:117-123): an id seen twice is one row (its last value at its
    first position), which per-shard runs cannot reproduce when the two
    occurrences sit in different shards.  Each rank routes the hashes of its
    span ids (a bijection: equal hashes are equal ids) to the rank that owns
    that hash range (kmz_route_ids), one all-to-all delivers them, and each
    owner runs the uniqueness certificate over what it received
    (kmz_id_repeats); a shard's own ids are unique already (its own
    certificate, or the span-table path that _unresolved refuses).  Cost per
    span: 8 bytes over the all-to-all and ~40 bytes of HBM traffic on its
    owner.  ``span_ids`` (no engine): the same protocol on the host (numpy
    hashes, a sort for the check), for CPU tensors under gloo.  IdGuard splits
    it around the run."""
    IdGuard(engine, dev, group, span_ids).start().finish()


def _gather_padded(x: torch.Tensor, m: int, world: int, group=None) -> torch.Tensor:
    """All-gather of every rank's int64 list, each padded with 0 to m."""
    pad = torch.zeros(max(1, m), dtype=torch.int64, device=x.device)
    pad[: x.numel()] = x
    out = torch.empty(pad.numel() * world, dtype=torch.int64, device=x.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    if x.is_cuda:
        torch.cuda.current_stream(x.device).synchronize()  # the engine's stream may not be torch's
    return out


class ShardingError(RuntimeError):
    """A parent link crosses shards: the sharded result would differ from the
    reference's global span map (Traces.ts:117-123); run unsharded."""


def _unresolved(engine) -> int:
    from ._lib import KmzError

    try:
        return engine.unresolved_parents()
    except KmzError as e:
        if e.code == -9:  # KMZ_E_UNSUPPORTED: the span-table path (repeated span ids in a shard)
            raise ShardingError("repeated span ids in a shard: sharding is not exact, run unsharded") from e
        raise


def _check_shards(engine, nu: int, mu: int, dev, group=None, raise_: bool = True) -> bool:
    """Exchange the unresolved parent ids (padded to the largest list) and
    count, on every rank, how many of them are span ids of its own shard.
    -> True when some are (ShardingError instead with ``raise_``)."""
    mine = torch.zeros(mu, dtype=torch.int64, device=dev)
    if nu:
        engine.unresolved_parents(mine.data_ptr(), mu, mine.is_cuda)
    allu = _gather_padded(mine, mu, dist.get_world_size(group), group)
    _engine_reads(engine, allu)
    found = torch.tensor([engine.count_ids(allu.data_ptr(), allu.numel(), allu.is_cuda)], dtype=torch.int64,
                         device=dev)
    dist.all_reduce(found, op=dist.ReduceOp.SUM, group=group)
    if int(found.item()) and raise_:
        raise ShardingError(f"{int(found.item())} parent ids of one shard are spans of another: shard by whole traces")
    return bool(int(found.item()))


def _merge_groups_only(p: torch.Tensor, G: int, group=None) -> None:
    """merge_group_partials on ``group``: SUM of the moments, MAX / MIN fields."""
    dist.all_reduce(p[: 4 * G], op=dist.ReduceOp.SUM, group=group)
    ts = _as_signed_order(p[4 * G : 5 * G])
    dist.all_reduce(ts, op=dist.ReduceOp.MAX, group=group)
    p[4 * G : 5 * G] = _as_signed_order(ts)
    first = p[5 * G :]
    first = torch.where(first == -1, torch.full_like(first, _I64_MAX), first)
    dist.all_reduce(first, op=dist.ReduceOp.MIN, group=group)
    p[5 * G :] = torch.where(first == _I64_MAX, torch.full_like(first, -1), first)


def _bcast(t: torch.Tensor, dev, group=None) -> torch.Tensor:
    """Broadcast a host tensor from rank 0 on ``dev``'s backend (device
    tensors under RCCL); returns it on the host."""
    if dev.type == "cpu":
        dist.broadcast(t, group=group, group_src=0)
        return t
    d = t.to(dev)
    dist.broadcast(d, group=group, group_src=0)
    return d.cpu()


def _unsharded_deps(engine, e: torch.Tensor, E: int, dev, group=None) -> None:
    """The exact merge of shards whose span-id map crosses shards: rank 0
    gathers every shard's columns (placed at their global flatten positions,
    kmz_get_global_index) and shape tables, runs the dependency pass of the
    whole batch on a second context of its GPU -- the reference's one global
    Map (Traces.ts:117-143) -- and broadcasts its endpoint partials and edge
    keys, which replace every rank's own (``e`` in place; the engine's edge
    set by kmz_set_triples).  Cost: the batch's columns (35 B/span) to rank 0
    and one unsharded dependency pass there, only when a guard fires."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    try:
        b = engine.spans()
        tab = engine.shape_table()
        mine = {"gidx": engine.global_index(), "sid": b.span_id, "pid": b.parent_id, "kind": b.kind,
                "shape": b.shape, "status": b.status, "dur": b.duration, "ts": b.timestamp,
                "tab": (np.asarray(tab.rt_ep, np.uint32), np.asarray(tab.tag_ep, np.uint32),
                        np.asarray(tab.dep_ep, np.uint32), int(tab.n_rt_ep), int(tab.n_tag_ep), int(tab.n_dep_ep),
                        int(tab.n_status))}
    except Exception as ex:  # noqa: BLE001 (a shard that cannot send its columns fails the pass on rank 0)
        mine = {"error": f"rank {rank}: {ex}"}
    # only rank 0 needs the columns: gather, not all-gather (an all-gather
    # would copy every shard to every rank)
    parts = [None] * world if rank == 0 else None
    dist.gather_object(mine, parts, group=group, group_dst=0)
    del mine
    W = 2 * E  # endpoint partial words: [max ts] E, [min first row] E
    # endpoint partials, the key count, then a status word: rank 0 reports its
    # own failure through the broadcast every rank waits in, so that no rank is
    # left blocked when rank 0 raises (an error on rank 0 -> ShardingError on all)
    head = torch.zeros(W + 2, dtype=torch.int64)
    keys2 = np.zeros(0, np.uint64)
    err = None
    if rank == 0:
        try:
            bad = [x["error"] for x in parts if "error" in x]
            if bad:
                raise ShardingError("; ".join(bad))
            keys2 = _unsharded_pass(parts, head, W)
        except Exception as ex:  # noqa: BLE001 (re-raised below, on every rank)
            err = ex
            head.zero_()
            head[W + 1] = 1
        parts = None
    head = _bcast(head, dev, group)
    if int(head[W + 1].item()):
        if err is not None:
            raise ShardingError(f"the unsharded dependency pass failed on rank 0: {err}") from err
        raise ShardingError("the unsharded dependency pass failed on rank 0")
    nk = int(head[W].item())
    kt = torch.zeros(max(1, nk), dtype=torch.int64)
    if rank == 0 and nk:
        kt[:nk] = torch.from_numpy(keys2.view(np.int64))
    kt = _bcast(kt, dev, group)
    e[:W] = head[:W].to(e.device)
    kh = np.ascontiguousarray(kt[:nk].numpy().view(np.uint64))
    engine.set_triples(kh.ctypes.data, nk, False)


def _unsharded_pass(parts, head: torch.Tensor, W: int) -> np.ndarray:
    """Rank 0's half of _unsharded_deps: place every shard's spans at their
    global flatten positions (relative to the batch's first position, which
    is not 0 for any batch after the first), run the dependency pass of the
    whole batch on a second engine context, write its endpoint partials and
    key count into ``head`` and return the keys."""
    from . import _lib as L
    from .engine import Engine, ShapeTable, SpanBatch

    N = sum(len(x["gidx"]) for x in parts)
    nonempty = [np.asarray(x["gidx"], np.int64) for x in parts if len(x["gidx"])]
    base = min(int(g.min()) for g in nonempty) if nonempty else 0
    top = max(int(g.max()) for g in nonempty) + 1 if nonempty else 0
    if top - base != N:  # the shards together must be one contiguous batch
        raise ShardingError(f"the shards' global positions span [{base}, {top}) for {N} spans")
    cols = {k: np.zeros(N, dt) for k, dt in (("sid", np.uint64), ("pid", np.uint64), ("kind", np.uint8),
                                              ("shape", np.uint32), ("status", np.uint16), ("dur", np.uint32),
                                              ("ts", np.int64))}
    filled = np.zeros(N, np.bool_)
    soff, tabs = 0, []
    for x in parts:  # shard r's shape s is shape soff_r + s of the whole batch
        g = np.asarray(x["gidx"], np.int64) - base
        filled[g] = True
        for k in cols:
            cols[k][g] = np.asarray(x[k]) + (np.uint32(soff) if k == "shape" else 0)
        tabs.append(x["tab"])
        soff += len(x["tab"][2])
    if not filled.all():
        raise ShardingError("two shards claim the same global position")
    table = ShapeTable(*(np.concatenate([t[j] for t in tabs]) for j in range(3)),
                       *(max(t[j] for t in tabs) for j in range(3, 7)))
    # index_base = the batch's first global position: first rows stay global
    whole = SpanBatch(cols["sid"], cols["pid"], cols["kind"], cols["shape"], cols["status"], cols["dur"],
                      cols["ts"], base)
    del cols
    e2 = Engine(torch.cuda.current_device())
    try:
        e2.load(whole, table)
        e2.run(L.RUN_DEPS)
        ew = e2.partials_words(L.PART_ENDPOINTS)
        ep2 = np.zeros(max(1, ew), np.uint64)
        e2.export_partials(L.PART_ENDPOINTS, ep2.ctypes.data, ew, False)
        keys2 = np.asarray(e2.triples(sort=False), np.uint64)
    finally:
        e2.close()
    if ew != W:
        raise ShardingError(f"the unsharded pass has {ew // 2} endpoints, the shards {W // 2}")
    head[:W] = torch.from_numpy(ep2[:W].view(np.int64))
    head[W] = len(keys2)
    return keys2


def merge_edge_keys(keys: torch.Tensor, group=None) -> torch.Tensor:
    """Union of every rank's unique edge keys (int64 view, keys are > 0)."""
    if dist.get_world_size(group) == 1:
        return torch.unique(keys)
    n = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
    allk = torch.unique(_gather_padded(keys, int(n.item()), dist.get_world_size(group), group))
    return allk[allk != 0]


def merge_edge_keys_into(engine, keys: torch.Tensor, group=None) -> None:
    """Union every rank's edge keys into ``engine``'s device edge set
    (kmz_merge_triples: hash inserts into the run's set, no sort).  ``keys``:
    this rank's unique keys, int64 view, on the engine's GPU (RCCL) or on the
    CPU (gloo)."""
    if dist.get_world_size(group) == 1:
        return
    n = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
    allk = _gather_padded(keys, int(n.item()), dist.get_world_size(group), group)
    engine.merge_triples(allk.data_ptr(), allk.numel(), keys.is_cuda)
