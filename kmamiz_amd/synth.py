"""Synthetic Zipkin workloads of BASELINE.json (configs 2, 3 and 5).

The same C generator (``kmz_synth.h``) runs on the device
(``Engine.load_synthetic``) and on the host (:func:`host_batch`), so tests can
regenerate any trace range on the CPU bit for bit.  Shape strings follow the
Istio naming the reference sees (``<svc>.<ns>.svc.cluster.local:<port>/...``,
compare tests/MockData.ts:11-3168).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Tuple

import numpy as np

from . import _lib as L
from .engine import ShapeTable, SpanBatch

BOOKINFO, MESH, POWER = L.SYNTH_BOOKINFO, L.SYNTH_MESH, L.SYNTH_POWER
SEED = 0x4B4D414D495A  # "KMAMIZ"
STATUSES = ["200", "404", "500"]

_BOOK = [
    ("productpage", "v1", "productpage.book.svc.cluster.local:9080/productpage", "http://192.168.39.24:31629/productpage"),
    ("details", "v1", "details.book.svc.cluster.local:9080/*", "http://details:9080/details/0"),
    ("reviews", "v1", "reviews.book.svc.cluster.local:9080/*", "http://reviews:9080/reviews/0"),
    ("reviews", "v2", "reviews.book.svc.cluster.local:9080/*", "http://reviews:9080/reviews/0"),
    ("reviews", "v3", "reviews.book.svc.cluster.local:9080/*", "http://reviews:9080/reviews/0"),
    ("ratings", "v1", "ratings.book.svc.cluster.local:9080/*", "http://ratings:9080/ratings/0"),
]


def describe(config: int):
    d = L.SynthDesc()
    L.check(None, L.lib().kmz_synth_describe(config, C.byref(d)))
    return d.n_shapes, d.n_status, d.n_endpoints


def shape_tags(config: int, shape: int) -> Tuple[str, dict]:
    """(name, tags) of one synthetic shape."""
    if config == BOOKINFO:
        svc, ver, name, url = _BOOK[shape]
        ns = "book"
        method = "GET"
    else:
        s, k = divmod(shape, 40)
        svc, ns, ver = f"s{s:04d}", f"ns{s % 10:02d}", f"v{1 + s % 2}"
        method = "GET" if k % 2 == 0 else "POST"
        name = f"{svc}.{ns}.svc.cluster.local:80/api/e{k:02d}"
        url = f"http://{svc}.{ns}.svc.cluster.local:80/api/e{k:02d}"
    return name, {
        "http.method": method,
        "http.url": url,
        "istio.canonical_revision": ver,
        "istio.canonical_service": svc,
        "istio.namespace": ns,
        "istio.mesh_id": "cluster.local",
    }


def shape_table(config: int) -> ShapeTable:
    n_shapes, n_status, n_ep = describe(config)
    ids = np.arange(n_shapes, dtype=np.uint32)
    return ShapeTable(ids, ids, ids, n_ep, n_ep, n_ep, n_status)


def dictionary(config: int):
    """The host Dictionary of a synthetic config's shapes and statuses, interned
    in id order (so its endpoint ids are the device tables' identity ids)."""
    from .ingest import Dictionary

    n_shapes, n_status, _ = describe(config)
    d = Dictionary()
    for s in range(n_shapes):
        assert d.shape_id(*shape_tags(config, s)) == s
    for st in STATUSES[:n_status]:
        d.status_id(st)
    for rule in ("rt", "tag", "dep"):
        if d.shape_ep[rule] != list(range(n_shapes)):
            raise ValueError(f"synthetic config {config}: {rule} endpoints are not one per shape")
    return d


def table_digest(config: int) -> int:
    """Digest of a synthetic config's id tables (merge_all's guard): every
    rank of a synthetic run indexes its partials by the same static tables."""
    import hashlib

    n_shapes, n_status, n_ep = describe(config)
    h = hashlib.blake2b(f"kmz-synth:{config}:{n_shapes}:{n_status}:{n_ep}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & ((1 << 62) - 1)


def count_spans(config: int, trace_begin: int, trace_end: int, seed: int = SEED) -> int:
    n = C.c_uint64()
    L.check(
        None,
        L.lib().kmz_synth_host(config, seed, trace_begin, trace_end, 0, *([None] * 8), C.byref(n)),
    )
    return n.value


def host_batch(config: int, trace_begin: int, trace_end: int, seed: int = SEED):
    """-> (SpanBatch, trace offsets) generated on the host."""
    lib = L.lib()
    n = count_spans(config, trace_begin, trace_end, seed)
    cols = dict(
        span_id=np.zeros(n, np.uint64),
        parent_id=np.zeros(n, np.uint64),
        kind=np.zeros(n, np.uint8),
        shape=np.zeros(n, np.uint32),
        status=np.zeros(n, np.uint16),
        duration=np.zeros(n, np.uint32),
        timestamp=np.zeros(n, np.int64),
    )
    off = np.zeros(trace_end - trace_begin + 1, np.uint64)
    got = C.c_uint64()
    L.check(
        None,
        lib.kmz_synth_host(
            config, seed, trace_begin, trace_end, n,
            L.ptr(cols["span_id"]), L.ptr(cols["parent_id"]), L.ptr(cols["kind"]), L.ptr(cols["shape"]),
            L.ptr(cols["status"]), L.ptr(cols["duration"]), L.ptr(cols["timestamp"]), L.ptr(off), C.byref(got),
        ),
    )
    base = count_spans(config, 0, trace_begin, seed) if trace_begin else 0
    return SpanBatch(index_base=base, **cols), off


def to_traces(config: int, batch: SpanBatch, off: np.ndarray, trace_begin: int = 0) -> List[List[dict]]:
    """Render a host batch as Zipkin ``Trace[][]`` JSON objects."""
    kinds = {1: "SERVER", 2: "CLIENT"}
    out = []
    cache = {}
    for t in range(len(off) - 1):
        spans = []
        tid = f"{(trace_begin + t) * 0x9E3779B97F4A7C15 % (1 << 128):032x}"
        for i in range(int(off[t]), int(off[t + 1])):
            sh = int(batch.shape[i])
            if sh not in cache:
                cache[sh] = shape_tags(config, sh)
            name, tags = cache[sh]
            sp = {
                "traceId": tid,
                "id": f"{int(batch.span_id[i]):016x}",
                "kind": kinds.get(int(batch.kind[i]), "PRODUCER"),
                "name": name,
                "timestamp": int(batch.timestamp[i]),
                "duration": int(batch.duration[i]),
                "tags": {**tags, "http.status_code": STATUSES[int(batch.status[i])]},
            }
            if batch.parent_id[i]:
                sp["parentId"] = f"{int(batch.parent_id[i]):016x}"
            spans.append(sp)
        out.append(spans)
    return out
