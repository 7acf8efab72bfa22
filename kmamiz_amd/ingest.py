"""Host ingest: ``Trace[][]`` (Zipkin JSON) -> columnar :class:`SpanBatch` plus
the string dictionaries the engine's integer ids point into.

Per span only ids, kinds, integers and a tuple of strings are touched; the
string work the reference does per span (three ``ExplodeUrl`` regexes per
SERVER span, five per ``ToEndpointInfo`` call: Traces.ts:32,145-183,
Utils.ts:83-106) is done once per DISTINCT shape here.

Identity rules restated from the reference:
* ``toRealTimeData`` (Traces.ts:32-46): service/namespace from
  ``ExplodeUrl(name, true)`` without fallback (missing -> "undefined" inside
  the template strings), version = raw ``istio.canonical_revision``.
* ``combineLogsToRealtimeData`` (Traces.ts:73-99): istio tags.
* ``ToEndpointInfo`` (Traces.ts:213-241): tag fallback when the name lacks
  ".svc.", version ``|| "NONE"``, port ``|| "80"`` (a present port keeps its
  colon), clusterName from the name or ``istio.mesh_id``.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ._lib import KIND_CLIENT, KIND_OTHER, KIND_SERVER
from .engine import ShapeTable, SpanBatch


class _Undef:
    __slots__ = ()

    def __repr__(self):
        return "undefined"

    def __bool__(self):
        return False


UNDEFINED = _Undef()

# JS RegExp '.' excludes line terminators
_ANY = "[^\n\r  ]"
_SCHEME = re.compile("[a-z]+://")
_URL = re.compile("://([^:/]*)([:0-9]*)(" + _ANY + "*)")
_SVC = re.compile("(" + _ANY + "*)" + _ANY + r"svc\.*(" + _ANY + "*)")


def tpl(v) -> str:
    """``${v}`` of a JS template literal for the values a Trace can hold."""
    if v is UNDEFINED:
        return "undefined"
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer() and abs(v) < 1e21:
        return str(int(v))
    return str(v)


def js_truthy(v) -> bool:
    return not (v is UNDEFINED or v is None or v is False or v == "" or
                (isinstance(v, (int, float)) and (v == 0 or v != v)))  # (NaN is falsy)


def explode_url(url, service: bool = False) -> List[Any]:
    """``Utils.ExplodeUrl`` (Utils.ts:83-106): [host, port, path(, service,
    namespace, clusterName)].  Raises TypeError where the reference does."""
    if not isinstance(url, str):
        raise TypeError(f"Cannot read properties of {tpl(url)} (reading 'search')")
    s = url if _SCHEME.search(url) else "://" + url
    m = _URL.search(s)
    parts: List[Any] = [m.group(1), m.group(2), m.group(3)] if m else [UNDEFINED, UNDEFINED, UNDEFINED]
    if service:
        host = parts[0]
        if host is UNDEFINED:
            raise TypeError("Cannot read properties of undefined (reading 'match')")
        sm = _SVC.search(host)
        if sm and sm.group(1):
            full = sm.group(1)
            cut = full.rfind(".")
            parts.append(full[:cut] if cut >= 0 else full[:-1])
            parts.append(full[cut + 1 :])
            parts.append(sm.group(2) or "cluster.local")
    return parts


def _nth(a, i):
    return a[i] if i < len(a) else UNDEFINED


_HEX = re.compile(r"\A[0-9a-f]{16}\Z")

# fields of a span that any output of the path can read (besides ids/ints)
SHAPE_TAGS = (
    "http.method",
    "http.url",
    "istio.canonical_revision",
    "istio.canonical_service",
    "istio.namespace",
    "istio.mesh_id",
)


class Identity:
    """Identity of one shape under one of the three rules (or the error the
    reference would raise when it evaluates it)."""

    __slots__ = ("fields", "error")

    def __init__(self, fields=None, error=None):
        self.fields = fields
        self.error = error


# The identity rules are pure functions of a shape, and a realtime worker sees
# the same endpoints batch after batch: their results are kept across batches
# (read-only Identity objects, keyed by the typed shape tuple).
_IDENT_CACHE: Dict[Tuple, Tuple] = {}
_IDENT_CACHE_MAX = 1 << 20


class Dictionary:
    """Interned strings of one batch: shapes, statuses, endpoint names."""

    def __init__(self):
        self.shapes: List[Tuple] = []  # (name, *SHAPE_TAGS)
        self.shape_index: Dict[Tuple, int] = {}
        self.statuses: List[Any] = []
        self.status_index: Dict[Tuple, int] = {}
        # per identity rule: endpoint name list + index + per-shape id + per-shape Identity
        self.ep_names = {"rt": [], "tag": [], "dep": []}
        self.ep_index = {"rt": {}, "tag": {}, "dep": {}}
        self.shape_ep = {"rt": [], "tag": [], "dep": []}
        self.shape_ident = {"rt": [], "tag": [], "dep": []}
        self.poison = {"rt": set(), "tag": set(), "dep": set()}

    # -- interning --------------------------------------------------------------
    def shape_id(self, name, tags: dict) -> int:
        key = (name,) + tuple(tags.get(t, UNDEFINED) if isinstance(tags, dict) else UNDEFINED for t in SHAPE_TAGS)
        hk = tuple((type(x).__name__, x if x is not UNDEFINED else None) for x in key)
        i = self.shape_index.get(hk)
        if i is None:
            i = len(self.shapes)
            self.shape_index[hk] = i
            self.shapes.append(key)
            self._add_identities(key, hk)
        return i

    def status_id(self, v) -> int:
        hk = (type(v).__name__, v if v is not UNDEFINED else None)
        i = self.status_index.get(hk)
        if i is None:
            i = len(self.statuses)
            self.status_index[hk] = i
            self.statuses.append(v)
        return i

    def _ep(self, rule: str, ident: Identity) -> int:
        if ident.error is not None:
            eid = len(self.ep_names[rule])
            self.ep_names[rule].append(None)
            self.poison[rule].add(eid)
            return eid
        name = ident.fields["uniqueEndpointName"]
        eid = self.ep_index[rule].get(name)
        if eid is None:
            eid = len(self.ep_names[rule])
            self.ep_index[rule][name] = eid
            self.ep_names[rule].append(name)
        return eid

    def _add_identities(self, key: Tuple, hk: Tuple):
        idents = _IDENT_CACHE.get(hk)
        if idents is None:
            idents = []
            for fn in (rt_identity, tag_identity, dep_identity):
                try:
                    idents.append(Identity(fn(key)))
                except TypeError as e:  # reference raises when it evaluates this shape
                    idents.append(Identity(error=e))
            if len(_IDENT_CACHE) >= _IDENT_CACHE_MAX:
                _IDENT_CACHE.clear()
            _IDENT_CACHE[hk] = idents = tuple(idents)
        for rule, ident in zip(("rt", "tag", "dep"), idents):
            self.shape_ident[rule].append(ident)
            self.shape_ep[rule].append(self._ep(rule, ident))

    def shape_table(self) -> ShapeTable:
        return ShapeTable(
            np.array(self.shape_ep["rt"], dtype=np.uint32),
            np.array(self.shape_ep["tag"], dtype=np.uint32),
            np.array(self.shape_ep["dep"], dtype=np.uint32),
            len(self.ep_names["rt"]),
            len(self.ep_names["tag"]),
            len(self.ep_names["dep"]),
            max(1, len(self.statuses)),
        )


def _tags(key):
    return dict(zip(SHAPE_TAGS, key[1:]))


def rt_identity(key) -> dict:
    """Traces.ts:32-35 (+ the row fields of 36-46)."""
    name = key[0]
    t = _tags(key)
    if not isinstance(name, str):
        raise TypeError("name is not a string")
    ex = explode_url(name, True)
    svc, ns = _nth(ex, 3), _nth(ex, 4)
    version, method = t["istio.canonical_revision"], t["http.method"]
    usn = f"{tpl(svc)}\t{tpl(ns)}\t{tpl(version)}"
    return {
        "service": svc,
        "namespace": ns,
        "version": version,
        "method": method,
        "uniqueServiceName": usn,
        "uniqueEndpointName": f"{usn}\t{tpl(method)}\t{tpl(t['http.url'])}",
    }


def tag_identity(key) -> dict:
    """Traces.ts:73-99."""
    t = _tags(key)
    svc, ns, version = t["istio.canonical_service"], t["istio.namespace"], t["istio.canonical_revision"]
    usn = f"{tpl(svc)}\t{tpl(ns)}\t{tpl(version)}"
    return {
        "service": svc,
        "namespace": ns,
        "version": version,
        "method": t["http.method"],
        "uniqueServiceName": usn,
        "uniqueEndpointName": f"{usn}\t{tpl(t['http.method'])}\t{tpl(t['http.url'])}",
    }


def dep_identity(key) -> dict:
    """Traces.ts:213-241 without the per-span timestamp."""
    name = key[0]
    t = _tags(key)
    host, port, path = explode_url(t["http.url"])[:3]
    if not isinstance(name, str):
        raise TypeError("name is not a string")
    ex = explode_url(name, True)
    svc, ns, cluster = _nth(ex, 3), _nth(ex, 4), _nth(ex, 5)
    if ".svc." not in name:
        svc, ns, cluster = t["istio.canonical_service"], t["istio.namespace"], t["istio.mesh_id"]
    rev = t["istio.canonical_revision"]
    version = rev if js_truthy(rev) else "NONE"
    usn = f"{tpl(svc)}\t{tpl(ns)}\t{tpl(version)}"
    return {
        "version": version,
        "service": svc,
        "namespace": ns,
        "url": t["http.url"],
        "host": host,
        "path": path,
        "port": port if js_truthy(port) else "80",
        "clusterName": cluster,
        "method": t["http.method"],
        "uniqueServiceName": usn,
        "uniqueEndpointName": f"{usn}\t{tpl(t['http.method'])}\t{tpl(t['http.url'])}",
    }


class IdMapper:
    """Span id strings -> u64.  Canonical Zipkin ids (16 lowercase hex, not all
    zero) map to their value; anything else (including a missing id, which JS
    keys as ``undefined``) gets a dictionary value that collides with no
    canonical id of the batch.  Equal JS keys <=> equal u64."""

    def __init__(self):
        self.other: Dict[Tuple, int] = {}
        self.pending: List[Tuple[np.ndarray, int, Tuple]] = []
        self.canonical = set()

    def key(self, v) -> Tuple:
        return (type(v).__name__, v if v is not UNDEFINED else None)

    def canon(self, v) -> int:
        if isinstance(v, str) and _HEX.match(v):
            x = int(v, 16)
            if x:
                self.canonical.add(x)
                return x
        return -1

    def assign_others(self):
        nxt = 1
        vals = {}
        for k in self.other:
            while nxt in self.canonical:
                nxt += 1
            vals[k] = nxt
            nxt += 1
        return vals


def ingest_traces(traces: Sequence[Sequence[dict]], index_base: int = 0):
    """Trace[][] -> (SpanBatch, Dictionary, flat list of span dicts)."""
    flat = [s for t in traces for s in t]
    n = len(flat)
    sid = np.zeros(n, dtype=np.uint64)
    pid = np.zeros(n, dtype=np.uint64)
    kind = np.zeros(n, dtype=np.uint8)
    shape = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.uint16)
    dur = np.zeros(n, dtype=np.uint32)
    ts = np.zeros(n, dtype=np.int64)
    d = Dictionary()
    ids = IdMapper()
    sid_other, pid_other = [], []
    for i, s in enumerate(flat):
        v = s.get("id", UNDEFINED)
        c = ids.canon(v)
        if c >= 0:
            sid[i] = c
        else:
            ids.other.setdefault(ids.key(v), None)
            sid_other.append((i, ids.key(v)))
        p = s.get("parentId", UNDEFINED)
        if js_truthy(p):
            c = ids.canon(p)
            if c >= 0:
                pid[i] = c
            else:
                ids.other.setdefault(ids.key(p), None)
                pid_other.append((i, ids.key(p)))
        k = s.get("kind", UNDEFINED)
        kind[i] = KIND_SERVER if k == "SERVER" else (KIND_CLIENT if k == "CLIENT" else KIND_OTHER)
        tags = s.get("tags", {}) or {}
        shape[i] = d.shape_id(s.get("name", UNDEFINED), tags)
        status[i] = d.status_id(tags.get("http.status_code", UNDEFINED))
        du, t = s.get("duration", UNDEFINED), s.get("timestamp", UNDEFINED)
        if not (isinstance(du, (int, float)) and float(du).is_integer() and 0 <= du < 2**32):
            raise ValueError(f"span {i}: duration {du!r} is not an integer number of microseconds in [0, 2^32)")
        if not (isinstance(t, (int, float)) and float(t).is_integer() and abs(t) < 2**63):
            raise ValueError(f"span {i}: timestamp {t!r} is not an integer number of microseconds")
        dur[i] = int(du)
        ts[i] = int(t)
    if len(d.statuses) > 65535:
        raise ValueError("more than 65535 distinct status strings")
    if ids.other:
        vals = ids.assign_others()
        for i, k in sid_other:
            sid[i] = vals[k]
        for i, k in pid_other:
            pid[i] = vals[k]
    batch = SpanBatch(sid, pid, kind, shape, status, dur, ts, index_base)
    return batch, d, flat


def ingest_rows(rows: Sequence[dict]):
    """TRealtimeData[] -> a SERVER-only batch whose shapes are the rows' own
    uniqueEndpointName (RealtimeDataList.ts:23-27 groups on it)."""
    n = len(rows)
    d = Dictionary()
    kind = np.full(n, KIND_SERVER, dtype=np.uint8)
    shape = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.uint16)
    dur = np.zeros(n, dtype=np.uint32)
    ts = np.zeros(n, dtype=np.int64)
    names: Dict[str, int] = {}
    first_row: List[int] = []
    for i, r in enumerate(rows):
        uen = r["uniqueEndpointName"]
        e = names.get(uen)
        if e is None:
            e = names[uen] = len(first_row)
            first_row.append(i)
        shape[i] = e
        status[i] = d.status_id(r.get("status", UNDEFINED))
        lat = r["latency"]
        us = lat * 1000
        if not (float(us).is_integer() and 0 <= us < 2**32 and us / 1000 == lat):
            raise ValueError(f"row {i}: latency {lat!r} ms is not an exact number of microseconds")
        dur[i] = int(us)
        t = r["timestamp"]
        if not float(t).is_integer():
            raise ValueError(f"row {i}: timestamp {t!r} is not an integer")
        ts[i] = int(t)
    eps = np.arange(len(first_row), dtype=np.uint32)
    table = ShapeTable(eps, eps, eps, len(first_row), len(first_row), len(first_row), max(1, len(d.statuses)))
    n_ids = np.arange(1, n + 1, dtype=np.uint64)
    batch = SpanBatch(n_ids, np.zeros(n, np.uint64), kind, shape, status, dur, ts, 0)
    return batch, table, d, first_row


def dictionary_from_fields(data: bytes, sf: np.ndarray, tf: np.ndarray, d: Optional["Dictionary"] = None):
    """The Dictionary of a parsed batch from its raw shape / status slices
    ([n*7, 2] and [n, 2] (offset, length) into ``data``): the identity rules run
    once per distinct shape, on one json.loads of all slices.  ``d``: intern
    into an existing Dictionary.  -> (Dictionary, raw shape -> shape id, raw
    status -> status id)."""
    import json

    from . import _lib as L

    ns, nt = len(sf) // 7, len(tf)
    fields = np.concatenate([sf.reshape(-1, 2), tf.reshape(-1, 2)]).tolist()
    present = [ln != L.JSON_ABSENT for _, ln in fields]
    dec = iter(json.loads(b"[" + b",".join(data[o:o + ln] for (o, ln), p in zip(fields, present) if p) + b"]"))
    vals = [next(dec) if p else UNDEFINED for p in present]
    d = d if d is not None else Dictionary()
    smap = np.zeros(max(1, ns), dtype=np.uint32)
    for i in range(ns):
        v = vals[7 * i:7 * i + 7]
        tags = {t: x for t, x in zip(SHAPE_TAGS, v[1:]) if x is not UNDEFINED}
        smap[i] = d.shape_id(v[0], tags)
    tmap = np.zeros(max(1, nt), dtype=np.uint32)
    for i in range(nt):
        tmap[i] = d.status_id(vals[7 * ns + i])
    if len(d.statuses) > 65535:
        raise ValueError("more than 65535 distinct status strings")
    return d, smap, tmap


class DeviceIngest:
    """Zipkin JSON -> the engine's batch with K1 on the GPU, for a realtime
    worker that parses a window every 5 s: the Dictionary persists across
    batches and the context remembers each raw shape's id (kmz_json_known), so
    the identity rules run once per shape ever seen, not once per window."""

    def __init__(self, eng):
        from . import _lib as L

        self.eng = eng
        self.d = Dictionary()
        # one identity space per context: ids remembered for another
        # dictionary would index this one wrongly
        L.check(eng.ctx, L.lib().kmz_json_forget(eng.ctx))

    def ingest(self, data: bytes, index_base: int = 0, ptr: Optional[int] = None) -> Optional[int]:
        """-> the batch's span count, or None outside the fast path (nothing
        loaded).  ``ptr``: the same bytes in pinned host memory (faster H2D)."""
        from . import _lib as L

        r = self.eng.json_parse(data) if ptr is None else self.eng.json_parse(ptr=ptr, length=len(data))
        if r is None:
            return None
        n, ns, nt = r
        ks, kt = self.eng.json_known(ns, nt)
        new_s, new_t = np.nonzero(ks == L.NONE32)[0], np.nonzero(kt == L.NONE32)[0]
        if len(new_s) or len(new_t):
            sf, tf = self.eng.json_fields(ns, nt)
            _, sm, tm = dictionary_from_fields(data, sf.reshape(ns, 7, 2)[new_s].reshape(-1, 2), tf[new_t], self.d)
            ks[new_s] = sm[: len(new_s)]
            kt[new_t] = tm[: len(new_t)]
        self.eng.json_load(ks, kt, self.d.shape_table(), index_base, n=n)
        return n


def ingest_json_device(eng, data: bytes, index_base: int = 0):
    """Zipkin Trace[][] JSON bytes parsed on the GPU (kmz_json_parse, K1) and
    loaded as the engine's batch: -> (Dictionary, n_spans), or None when the
    batch is outside the fast path (nothing loaded; parse on the host)."""
    from . import _lib as L

    r = eng.json_parse(data)
    if r is None:
        return None
    n, ns, nt = r
    sf, tf = eng.json_fields(ns, nt)
    d, smap, tmap = dictionary_from_fields(data, sf, tf)
    L.check(eng.ctx, L.lib().kmz_json_forget(eng.ctx))  # (a fresh dictionary: a fresh identity space)
    eng.json_load(smap[:ns], tmap[:nt], d.shape_table(), index_base, n=n)
    return d, n


def ingest_json(data: bytes, index_base: int = 0, threads: int = 0):
    """Zipkin Trace[][] JSON bytes -> (SpanBatch, Dictionary) through the native
    parser (kmz_parse_zipkin), or None when the batch is
    outside its fast path (the caller then parses it the general way).  The
    identity rules run once per distinct shape, on json.loads of the raw
    field slices the parser returns."""
    import ctypes as C
    import json

    from . import _lib as L

    out = C.POINTER(L.ZipkinBatch)()
    rc = L.lib().kmz_parse_zipkin(data, len(data), threads, C.byref(out))
    if rc == L.E_UNSUPPORTED:
        return None
    L.check(None, rc)
    try:
        b = out.contents
        n = int(b.n)

        def col(ptr, dtype):
            return np.ctypeslib.as_array(ptr, shape=(max(1, n),))[:n].astype(dtype, copy=True)

        sid, pid = col(b.span_id, np.uint64), col(b.parent_id, np.uint64)
        kind, dur, ts = col(b.kind, np.uint8), col(b.duration, np.uint32), col(b.timestamp, np.int64)
        shp, sts = col(b.shape, np.uint32), col(b.status, np.uint32)
        ns, nt = int(b.n_shapes), int(b.n_statuses)
        sf = np.ctypeslib.as_array(b.shape_fields, shape=(max(1, ns) * 14,))[: ns * 14].reshape(ns * 7, 2)
        tf = np.ctypeslib.as_array(b.status_fields, shape=(max(1, nt) * 2,))[: nt * 2].reshape(nt, 2)
        d, smap, tmap = dictionary_from_fields(data, sf, tf)
    finally:
        L.lib().kmz_zipkin_free(out)
    batch = SpanBatch(sid, pid, kind, smap[shp] if n else shp, (tmap[sts] if n else sts).astype(np.uint16), dur,
                      ts, index_base)
    return batch, d
