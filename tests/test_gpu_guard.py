"""The cross-shard repeated-span-id guard on the GPU (kmz_guard.hip
kmz_route_ids, the certificate's kmz_id_repeats) against its host mirror
(kmamiz_amd.dist.route_ids_np) and a sort.  The reference's span map is global
(Traces.ts:117-123): an id in two shards must make the sharded run refuse."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("device", [False, True])
def test_route_ids_equals_host_mirror(engine, world, device):
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 3000)
    engine.load(batch, synth.shape_table(synth.MESH))
    n = len(batch)
    out = torch.zeros(n, dtype=torch.int64, device="cuda" if device else "cpu")
    counts = engine.route_ids(world, out.data_ptr(), n, device)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    h, c = kdist.route_ids_np(batch.span_id, world)
    assert counts == c.tolist()
    o = 0
    for r in range(world):  # each owner's segment holds exactly its hashes (order inside is free)
        assert np.array_equal(np.sort(got[o : o + counts[r]]), np.sort(h[o : o + counts[r]]))
        o += counts[r]


@pytest.mark.parametrize("m", [2, 1000, 1 << 20, 3_000_000])
def test_id_repeats_finds_one_repeat(engine, m):
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 20)
    engine.load(batch, synth.shape_table(synth.MESH))  # (any loaded batch: the check reads only its input)
    rng = np.random.default_rng(m)
    v = np.unique(rng.integers(1, 2**64 - 1, size=m + m // 8 + 8, dtype=np.uint64))[:m]
    rng.shuffle(v)
    assert len(v) == m
    assert engine.id_repeats(v.ctypes.data, m, False) is False
    w = v.copy()
    w[m - 1] = w[m // 3]
    assert engine.id_repeats(w.ctypes.data, m, False) is True
    d = torch.from_numpy(w.view(np.int64)).cuda()
    torch.cuda.synchronize()
    assert engine.id_repeats(d.data_ptr(), m, True) is True


def test_id_repeats_past_1e8_values(engine):
    """1.5e8 values: the certificate's split runs in rounds (2^10 sub-bins,
    k_cert_split_r); distinct values pass, one repeat is found."""
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 20)
    engine.load(batch, synth.shape_table(synth.MESH))
    m = 150_000_000
    v = torch.arange(1, m + 1, dtype=torch.int64, device="cuda") * 0x2545F4914F6CDD1D  # odd: distinct mod 2^64
    torch.cuda.synchronize()
    assert engine.id_repeats(v.data_ptr(), m, True) is False
    v[m - 7] = v[12345]
    torch.cuda.synchronize()
    assert engine.id_repeats(v.data_ptr(), m, True) is True
    del v
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("device", [False, True])
def test_route_ids_fixed_equals_host_mirror(engine, world, device):
    """kmz_route_ids_fixed: segment r = [count_r, its hashes] (word 0 the true
    count even past the segment: an overflowed segment says so)."""
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 3000)
    engine.load(batch, synth.shape_table(synth.MESH))
    h, c = kdist.route_ids_np(batch.span_id, world)
    for seg in (int(c.max()) + 1 + 7, max(2, int(c.max()) // 2)):
        out = torch.zeros(world * seg, dtype=torch.int64, device="cuda" if device else "cpu")
        engine.route_ids_fixed(world, seg, out.data_ptr(), device)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64).reshape(world, seg)
        assert got[:, 0].tolist() == c.tolist()
        o = 0
        for r in range(world):
            k = min(int(c[r]), seg - 1)
            mine = h[o : o + int(c[r])]
            if k == int(c[r]):  # complete segment: exactly its hashes
                assert np.array_equal(np.sort(got[r, 1 : 1 + k]), np.sort(mine))
            else:  # overflowed: a subset of them
                assert np.isin(got[r, 1:], mine).all()
            o += int(c[r])


@pytest.mark.parametrize("world,ntr,in_join", [(2, 3000, True), (3, 3000, True), (8, 3000, True), (64, 3000, True),
                                               (65, 3000, False), (8, 40000, False), (8, 370000, True)])
def test_route_in_join_equals_route_fixed(engine, world, ntr, in_join):
    """kmz_route_ids_join: the run's join writes kmz_route_ids_fixed's
    segments (word 0 the true count, then exactly the owner's hashes; a
    subset past an overflowed segment) when the owners fit its pass-1 bins
    (64 at these sizes), else the run's fallback pass does (world 65; the
    fused join + walk at 40 000 traces); the run's results are those of a run
    without routing; the arming is one-shot.  (The fused case on an engine of
    its own with chain interning forced, KMZ_ABLATE bit 29: the shared
    engine may have switched this shape table to direct enumeration, which
    takes the window join.)"""
    if ntr == 40000:
        own = _engine_ablate(1 << 29)
        try:
            _route_in_join_case(own, world, ntr, in_join)
        finally:
            own.close()
        return
    _route_in_join_case(engine, world, ntr, in_join)


def _engine_ablate(ablate):
    import os

    from kmamiz_amd import Engine

    old = os.environ.get("KMZ_ABLATE")
    os.environ["KMZ_ABLATE"] = str(ablate)
    try:
        return Engine(0)
    finally:
        if old is None:
            del os.environ["KMZ_ABLATE"]
        else:
            os.environ["KMZ_ABLATE"] = old


def _route_in_join_case(engine, world, ntr, in_join):
    from kmamiz_amd import _lib as L
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, ntr)
    engine.load(batch, synth.shape_table(synth.MESH))
    flags = L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_NO_CERT
    engine.run(flags)
    g0, k0 = engine.groups().tobytes(), engine.triples().copy()
    h, c = kdist.route_ids_np(batch.span_id, world)
    for seg in (int(c.max()) + 1 + 7, max(2, int(c.max()) // 2)):
        out = torch.zeros(world * seg, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        engine.route_ids_join(world, seg, out.data_ptr())
        engine.run(flags)
        assert engine.route_wait(0) is in_join
        torch.cuda.synchronize()
        assert engine.groups().tobytes() == g0
        assert np.array_equal(engine.triples(), k0)
        got = out.cpu().numpy().view(np.uint64).reshape(world, seg)
        assert got[:, 0].tolist() == c.tolist()
        o = 0
        for r in range(world):
            k = min(int(c[r]), seg - 1)
            mine = h[o : o + int(c[r])]
            if k == int(c[r]):
                assert np.array_equal(np.sort(got[r, 1 : 1 + k]), np.sort(mine))
            else:
                assert np.isin(got[r, 1:], mine).all()
            o += int(c[r])
    # one-shot: the next run routes nothing
    engine.run(flags)
    with pytest.raises(Exception):
        engine.route_wait(0)


def _guard_worker(rank, world, port, q, dev_kind):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kmamiz_amd import Engine
        from kmamiz_amd import dist as kdist
        from kmamiz_amd import synth

        e = Engine(0)
        dev = torch.device("cuda", 0) if dev_kind == "cuda" else torch.device("cpu")
        cut = [0, 400, 900, 1300][: world + 1]
        b0, _ = synth.host_batch(synth.MESH, cut[0], cut[1])
        out = []
        # steps: clean (exact protocol, first), clean (fixed segments), a
        # repeat across shards (fixed), clean with a forced tiny segment
        # (overflow -> the exact protocol, same step), a repeat after it
        for step, (rep, tiny) in enumerate([(False, False), (False, False), (True, False), (False, True),
                                            (True, False)]):
            batch, _ = synth.host_batch(synth.MESH, cut[rank], cut[rank + 1])
            if rep and rank == world - 1:
                batch.span_id[len(batch) - 1] = b0.span_id[5]
            e.load(batch, synth.shape_table(synth.MESH))
            g = kdist.IdGuard(e, dev)
            if tiny:  # (the agreed size, forced: the entry keeps its group object)
                kdist._ID_SEG[(id(g.gobj), world)] = (g.gobj, 4)
            g.start()
            fixed = g.fixed is not None
            got = g.finish(raise_=False)
            out.append((fixed, got))
        q.put((rank, out))
        e.close()
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dev_kind", [(2, "cpu"), (3, "cuda")])
def test_id_guard_fixed_segments_over_steps(world, dev_kind):
    """IdGuard across steps (dist.py): the first step exchanges counts, later
    ones fixed segments with no host round trip in start(); a repeat across
    shards is found either way, and a step whose segment overflows (forced
    here) is redone exactly on every rank."""
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_guard_worker, args=(r, world, port, q, dev_kind)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=200) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert isinstance(r[1], list), r[1]
        fixed = [x[0] for x in r[1]]
        found = [x[1] for x in r[1]]
        assert fixed == [False, True, True, True, True]
        assert found == [False, False, True, False, True]


@pytest.mark.parametrize("world", [1, 2, 8])
def test_id_repeats_seg_over_received_segments(engine, world):
    """kmz_id_repeats_seg_begin/_end over fixed segments as an all-to-all
    delivers them (count word, values, stale words past the count), enqueued
    on a stream of its own: distinct values pass, one repeat inside a segment
    or across two is found, an overflowed segment reports its count."""
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 3000)
    engine.load(batch, synth.shape_table(synth.MESH))
    h, c = kdist.route_ids_np(batch.span_id, world)
    seg = int(c.max()) + 1 + 4100  # slack past a pass-1 tile: short and empty tiles in every segment
    out = torch.full((world * seg,), -1, dtype=torch.int64, device="cuda")  # stale words: never read
    engine.route_ids_fixed(world, seg, out.data_ptr(), True)
    torch.cuda.synchronize()
    gs = torch.cuda.Stream()

    def verdict(buf, s):
        torch.cuda.synchronize()
        engine.id_repeats_seg_begin(buf.data_ptr(), world, s, gs.cuda_stream)
        return engine.id_repeats_seg_end()

    assert verdict(out, seg) == (False, int(c.max()))
    r = out.view(world, seg)
    last = world - 1
    k = int(c[last])
    save = r[last, k].item()
    r[last, k] = r[last, 1]  # inside the last segment
    assert verdict(out, seg) == (True, int(c.max()))
    r[last, k] = save
    if world > 1:
        r[last, k] = r[0, 1]  # across segments (two sources sent one value)
        assert verdict(out, seg) == (True, int(c.max()))
        r[last, k] = save
    assert verdict(out, seg) == (False, int(c.max()))
    small = max(2, int(c.max()) // 2)  # overflowed: the count says so
    o2 = torch.zeros(world * small, dtype=torch.int64, device="cuda")
    engine.route_ids_fixed(world, small, o2.data_ptr(), True)
    rep, maxc = verdict(o2, small)
    assert maxc == int(c.max()) and maxc >= small


def test_no_cert_run_equals_certified_run(engine):
    """KMZ_RUN_NO_CERT (a run covered by the multi-GPU id guard) changes no
    result on a batch with unique ids."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 4000)
    engine.load(batch, synth.shape_table(synth.MESH))
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    g0, k0, e0 = engine.fetch()
    engine.run(L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_NO_CERT)
    g1, k1, e1 = engine.fetch()
    assert g0.tobytes() == g1.tobytes()
    assert np.array_equal(np.sort(k0), np.sort(k1))
    assert e0.tobytes() == e1.tobytes()


class _LoopGuard:
    """IdGuard's RCCL branch (dist.py IdGuard.start: device routing, the
    all-to-all posted behind it, the segment certificate on the guard's stream
    waiting for the exchange) on one process: the all-to-all is stood in for
    by a copy of the routed segments on a stream of its own -- optionally
    appending the first value of segment ``inject[0]`` to segment
    ``inject[1]``, as if another source had sent it too -- and the MAX
    all-reduce by the identity.  Built as a subclass at call time (the module
    imports torch.distributed lazily)."""

    @staticmethod
    def make(engine, inject=None):
        from kmamiz_amd import dist as kdist

        class G(kdist.IdGuard):
            def __init__(self):
                super().__init__(engine, torch.device("cuda", 0), world=2, backend="nccl")
                self.inject = inject
                self.xs = torch.cuda.Stream()

            def _a2a(self, out, inp, out_splits=None, in_splits=None, async_op=False):
                self.xs.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.xs):
                    out.copy_(inp)  # (identity: this rank's segments stand in for what the sources sent)
                    if self.inject is not None and out_splits is None and self.fixed is not None:
                        r = out.view(self.world, self.fixed)
                        a, b = self.inject
                        pos = (r[b, 0] + 1).clamp(max=self.fixed - 1).view(1)
                        r[b].index_copy_(0, pos, r[a, 1].view(1))
                        r[b, 0] += 1
                ev = torch.cuda.Event()
                ev.record(self.xs)
                inp.record_stream(self.xs)
                out.record_stream(self.xs)

                class Work:
                    def wait(self):
                        torch.cuda.current_stream().wait_event(ev)

                w = Work()
                if not async_op:
                    w.wait()
                return w

            def _agree(self, flag):
                pass

        return G()


@pytest.mark.parametrize("fold,ntr,in_join", [(False, 3000, None), (True, 3000, True), (True, 40000, False)])
def test_id_guard_device_wiring_single_process(fold, ntr, in_join):
    """the RCCL branch of IdGuard.start/finish as the multi-GPU
    bench wires it (one explicit stream for torch and the engine, the run
    without its own certificate beside the guard), on one process: the first
    step exchanges counts, later ones fixed segments whose certificate is
    enqueued on the guard stream (seg_open); a repeat inside the shard and one
    across two sources' segments are found, clean steps pass, and when
    kmz_id_repeats_seg_begin fails start() falls back to finish()'s
    compaction check with the same verdicts.  With ``fold`` the routing rides
    in the run (kmz_route_ids_join) and post() exchanges after run_begin: in
    the join at 3000 traces (~8e4 spans, the window join), by the fallback
    pass at 40 000 (~1.1e6 spans: the fused join + walk)."""
    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    import os

    stream = torch.cuda.Stream()
    prev = torch.cuda.current_stream()
    torch.cuda.set_stream(stream)
    old = os.environ.get("KMZ_ABLATE")
    if ntr == 40000:  # (chain interning forced: the fused join + walk, whose routing is the fallback pass)
        os.environ["KMZ_ABLATE"] = str(1 << 29)
    try:
        e = Engine(0, stream=stream.cuda_stream)
    finally:
        if old is None:
            os.environ.pop("KMZ_ABLATE", None)
        else:
            os.environ["KMZ_ABLATE"] = old
    try:
        table = synth.shape_table(synth.MESH)
        kdist._ID_SEG.pop((id(None), 2), None)  # (this process's stand-in group: no agreed size yet)
        clean, _ = synth.host_batch(synth.MESH, 0, ntr)
        rep_in, _ = synth.host_batch(synth.MESH, 0, ntr)
        rep_in.span_id[len(rep_in) - 1] = rep_in.span_id[5]

        def step(batch, inject=None, fail_seg=False):
            e.load(batch, table)
            g = _LoopGuard.make(e, inject)
            if fail_seg:
                def boom(*a, **k):
                    raise RuntimeError("KMZ_E_UNSUPPORTED (test)")
                e.id_repeats_seg_begin = boom
            try:
                g.start(fold=fold)
                e.run_begin(L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_NO_CERT)  # beside the guard, as the bench runs
                armed = g.armed
                g.post()
                e.run_end()
                if armed:
                    assert g.in_join is in_join
                else:
                    assert not fold or g.fixed is None
                opened = g.seg_open
                fixed = g.fixed is not None
                got = g.finish(raise_=False)
            finally:
                if fail_seg:
                    del e.id_repeats_seg_begin
            return fixed, opened, got

        assert step(clean) == (False, False, False)  # first step: counts protocol
        assert step(clean) == (True, True, False)  # fixed segments, certificate on the guard stream
        assert step(rep_in) == (True, True, True)  # a repeat inside this shard
        assert step(clean, inject=(0, 1)) == (True, True, True)  # one value from two sources
        assert step(clean, inject=(1, 0)) == (True, True, True)
        assert step(clean) == (True, True, False)
        # kmz_id_repeats_seg_begin failing: start() leaves it closed, finish() compacts
        assert step(clean, fail_seg=True) == (True, False, False)
        assert step(rep_in, fail_seg=True) == (True, False, True)
        assert step(clean, inject=(0, 1), fail_seg=True) == (True, False, True)
        assert step(clean) == (True, True, False)
    finally:
        e.close()
        torch.cuda.set_stream(prev)
