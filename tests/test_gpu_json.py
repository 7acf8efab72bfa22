"""K1 on the GPU (kmz_json_parse, kmz_json.hip): the device parse of Zipkin
Trace[][] JSON equals the host fast path (kmz_parse_zipkin, kmz_ingest.cpp)
column for column, raw shape for raw shape, and declines (KMZ_E_UNSUPPORTED)
exactly where the host path does; the engine's results from a device-parsed
batch equal those of the host-parsed one."""
import ctypes as C
import json

import numpy as np
import pytest

from conftest import fixture
from shard_util import mixed_traces

pytestmark = pytest.mark.gpu


def _host_raw(data: bytes):
    """kmz_parse_zipkin's raw output (shape / status ids in first-occurrence
    order of the raw slices), or None."""
    from kmamiz_amd import _lib as L

    out = C.POINTER(L.ZipkinBatch)()
    rc = L.lib().kmz_parse_zipkin(data, len(data), 0, C.byref(out))
    if rc == L.E_UNSUPPORTED:
        return None
    L.check(None, rc)
    try:
        b = out.contents
        n = int(b.n)

        def col(ptr, dt):
            return np.ctypeslib.as_array(ptr, shape=(max(1, n),))[:n].astype(dt, copy=True)

        ns, nt = int(b.n_shapes), int(b.n_statuses)
        return dict(
            span_id=col(b.span_id, np.uint64), parent_id=col(b.parent_id, np.uint64), kind=col(b.kind, np.uint8),
            shape=col(b.shape, np.uint32), status=col(b.status, np.uint32), duration=col(b.duration, np.uint32),
            timestamp=col(b.timestamp, np.int64),
            sf=np.ctypeslib.as_array(b.shape_fields, shape=(max(1, ns) * 14,))[: ns * 14].reshape(-1, 2).copy(),
            tf=np.ctypeslib.as_array(b.status_fields, shape=(max(1, nt) * 2,))[: nt * 2].reshape(-1, 2).copy())
    finally:
        L.lib().kmz_zipkin_free(out)


def _device_raw(engine, data: bytes):
    from kmamiz_amd import ShapeTable

    r = engine.json_parse(data)
    if r is None:
        return None
    n, ns, nt = r
    sf, tf = engine.json_fields(ns, nt)
    ids = np.arange(max(ns, 1), dtype=np.uint32)
    table = ShapeTable(ids, ids, ids, max(ns, 1), max(ns, 1), max(ns, 1), max(nt, 1))
    engine.json_load(np.arange(ns, dtype=np.uint32), np.arange(nt, dtype=np.uint32), table, 0, n=n)
    b = engine.spans()
    return dict(span_id=b.span_id, parent_id=b.parent_id, kind=b.kind, shape=b.shape, status=b.status.astype(np.uint32),
                duration=b.duration, timestamp=b.timestamp, sf=sf, tf=tf)


def _same(engine, data: bytes):
    h = _host_raw(data)
    d = _device_raw(engine, data)
    assert (h is None) == (d is None), "host and device disagree on the fast path's domain"
    if h is None:
        return None
    for k in h:
        assert np.array_equal(h[k], d[k]), k
    return h


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_fixtures(engine, fx):
    t = fixture(fx)
    if fx != "MockTrace":  # (one trace each)
        t = [t]
    assert _same(engine, json.dumps(t).encode()) is not None


@pytest.mark.parametrize("config,ntr", [(2, 30000), (3, 20000), (5, 3000)])
def test_synthetic(engine, config, ntr):
    from kmamiz_amd import synth

    b, off = synth.host_batch(config, 0, ntr)
    data = json.dumps(synth.to_traces(config, b, off)).encode()
    h = _same(engine, data)
    assert len(h["span_id"]) == len(b)


def test_mixed_pretty_escaped_and_falsy(engine):
    t = mixed_traces(200)
    t[3][0]["name"] = 'say "hi" \\ there é中'
    t[5][0]["parentId"] = ""
    t[6][0]["tags"] = None
    t[7][0].pop("parentId", None)
    t[8][0]["tags"]["x"] = "]], [[ {\"a\": [1, 2]} }}" * 50
    _same(engine, json.dumps(t).encode())
    _same(engine, json.dumps(t, indent=2).replace("/", "\\/").encode())
    _same(engine, json.dumps(t, separators=(" , ", " :  ")).encode())
    # a long string full of structural characters across many 64-byte chunks
    t[9][0]["tags"]["y"] = "]], [[" * 200_000
    _same(engine, json.dumps(t).encode())


@pytest.mark.parametrize("mutate", ["upper_id", "float_duration", "escaped_key", "string_tags", "zero_parent",
                                    "missing_id", "not_nested", "escaped_kind", "empty_span"])
def test_fallbacks_agree(engine, mutate):
    t = [fixture("MockTracePDAS")]
    s = t[0][1]
    data = None
    if mutate == "upper_id":
        s["id"] = "ABCDEF0123456789"
    elif mutate == "float_duration":
        s["duration"] = 1.5
    elif mutate == "escaped_key":
        data = json.dumps(t).replace('"kind"', '"\\u006bind"', 1).encode()
    elif mutate == "escaped_kind":
        data = json.dumps(t).replace('"SERVER"', '"SERV\\u0045R"', 1).encode()
    elif mutate == "string_tags":
        s["tags"] = "x"
    elif mutate == "zero_parent":
        s["parentId"] = "0" * 16
    elif mutate == "missing_id":
        del s["id"]
    elif mutate == "not_nested":
        t = t[0]
    elif mutate == "empty_span":
        t[0].append({})
    assert _same(engine, data if data is not None else json.dumps(t).encode()) is None


@pytest.mark.parametrize("text", [b"{}", b"[{}]", b'[["a"]]', b"[[1]]", b"[[{}{}]]", b"[[],]", b"[,[]]", b"[[]] x",
                                  b"[[]", b"[[]]]", b'["x"]', b"", b"   ", b"[[\\]]", b"[[{\"a\":\"\\\"}]]"])
def test_structure_errors_agree(engine, text):
    assert _same(engine, text) is None


def test_structure_with_spans(engine):
    sp = json.dumps(fixture("MockTracePDAS")[0])
    for text in ["[[%s %s]]" % (sp, sp), "[[%s,]]" % sp, "[[%s],]" % sp, "[[%s]] ]" % sp, "[[,%s]]" % sp,
                 "[[%s]][[%s]]" % (sp, sp), "[[%s] [%s]]" % (sp, sp)]:
        assert _same(engine, text.encode()) is None, text
    for text in ["[[%s , %s]]" % (sp, sp), " [ [ ] , [ %s ] ] " % sp, "[[%s],[],[%s]]" % (sp, sp)]:
        assert _same(engine, text.encode()) is not None, text


@pytest.mark.parametrize("text", [b"[]", b" [ ] \n", b"[[]]", b"[[], []]"])
def test_empty(engine, text):
    h = _same(engine, text)
    assert len(h["span_id"]) == 0


def test_many_distinct_shapes_grow_the_table(engine):
    """> 2^19 distinct shapes: the interning table fills, grows, and the spans
    are parsed again."""
    n = 600_000
    spans = ",".join('{"id":"%016x","kind":"SERVER","name":"svc.ns.svc.cluster.local:80/e%d",'
                     '"timestamp":%d,"duration":5,"tags":{"http.status_code":"200"}}' % (i + 1, i, 1000 + i)
                     for i in range(n))
    data = ("[[" + spans + "]]").encode()
    h = _same(engine, data)
    assert len(h["sf"]) == 7 * n


def test_device_ingest_runs_like_host_ingest(engine):
    """ingest_json_device + kmz_run == ingest_json + kmz_load + kmz_run."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.ingest import ingest_json, ingest_json_device

    b, off = synth.host_batch(3, 0, 5000)
    traces = synth.to_traces(3, b, off) + mixed_traces(100)
    data = json.dumps(traces).encode()
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    batch, d1 = ingest_json(data)
    engine.load(batch, d1.shape_table())
    engine.run(flags)
    g1, k1, e1 = (np.array(x, copy=True) for x in engine.fetch())
    d2, n = ingest_json_device(engine, data)
    assert n == len(batch) and d2.shapes == d1.shapes and d2.statuses == d1.statuses
    engine.run(flags)
    g2, k2, e2 = engine.fetch()
    assert g1.tobytes() == g2.tobytes()
    assert np.array_equal(np.sort(k1), np.sort(k2))
    assert e1.tobytes() == e2.tobytes()


def test_device_ingest_remembers_identities(engine):
    """DeviceIngest over overlapping windows: each window's batch equals the
    host parse of the same bytes (shapes compared by content), the second
    window finds its repeated shapes in kmz_json_known, and kmz_json_forget
    clears them."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth
    from kmamiz_amd.ingest import DeviceIngest, ingest_json

    b, off = synth.host_batch(3, 0, 6000)
    tr = synth.to_traces(3, b, off)
    windows = [tr[:3000] + mixed_traces(40), tr[2000:5000], tr[4000:] + mixed_traces(80)]
    di = DeviceIngest(engine)
    for k, w in enumerate(windows):
        data = json.dumps(w).encode()
        if k == 1:
            r = engine.json_parse(data)
            ks, kt = engine.json_known(r[1], r[2])
            assert (ks != L.NONE32).sum() > 0 and (ks == L.NONE32).sum() > 0
        n = di.ingest(data)
        hb, hd = ingest_json(data)
        got = engine.spans()
        assert n == len(hb)
        for f in ("span_id", "parent_id", "kind", "duration", "timestamp"):
            assert np.array_equal(getattr(got, f), getattr(hb, f)), f
        assert [di.d.shapes[i] for i in got.shape] == [hd.shapes[i] for i in hb.shape]
        assert [di.d.statuses[i] for i in got.status] == [hd.statuses[i] for i in hb.status]
    r = engine.json_parse(json.dumps(windows[0]).encode())
    assert (engine.json_known(r[1], r[2])[0] != L.NONE32).all()
    L.check(engine.ctx, L.lib().kmz_json_forget(engine.ctx))
    assert (engine.json_known(r[1], r[2])[0] == L.NONE32).all()
