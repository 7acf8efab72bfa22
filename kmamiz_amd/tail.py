"""Service-level tail at scale (SURVEY.md 8a row a8, config 5's "service
risk/instability/coupling recompute").

The engine's ``kmz_tail_run`` (kmz_tail.hip) turns the run's reduced edge set
into the link-detail counters of ``EndpointDependencies.toServiceDependencies``
(EndpointDependencies.ts:369-470) and the distance-1 consumer pairs of
``toServiceEndpointCohesion`` (565-612).  This module interns the strings the
kernels need (:class:`TailMaps`) and finishes the service metrics on the host
over those few rows (:class:`ServiceTail`):

* ``toServiceInstability``       EndpointDependencies.ts:614-641
* ``toServiceCoupling``          EndpointDependencies.ts:643-657 via
                                 RiskAnalyzer.AbsoluteCriticalityOfServices (RiskAnalyzer.ts:145-169)
* ``toServiceEndpointCohesion``  EndpointDependencies.ts:565-612
* ``realtime_risk``              RiskAnalyzer.RealtimeRisk (RiskAnalyzer.ts:10-49)

Parity is defined on the reduced form, ``new EndpointDependencies([])
.combineWith(deps).trim()``: services come in first-row order, every count is
exact, fp64 metrics are within 1e-9 relative (summation order differs from the
TS link order), and list members whose order the TS takes from per-row
iteration (cohesion consumers) are compared as sets.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib as L
from .ingest import UNDEFINED, tpl


def _split3(usn: str):
    return (usn.split("\t") + [UNDEFINED] * 3)[:3]


class TailMaps:
    """Interned ids of the dependency endpoints (one per ``dep`` endpoint id).

    ``fields[e]`` is endpoint e's TEndpointInfo fields (``uniqueServiceName``,
    ``method``, ``uniqueEndpointName``) or None for an id no row uses;
    ``label_map`` is the host's uniqueEndpointName -> labelName map
    (EndpointDependencies.label(), EndpointDependencies.ts:114-153), unlabeled
    endpoints get the string "undefined" as in the TS."""

    def __init__(self, fields: Sequence[Optional[dict]], label_map: Optional[Dict[str, str]] = None):
        svc_idx: Dict[str, int] = {}
        cls_idx: Dict[str, int] = {}
        lsvc_idx: Dict[str, int] = {}
        self.svc = np.zeros(len(fields), dtype=np.uint32)
        self.cls = np.zeros(len(fields), dtype=np.uint32)
        lsvc_of_cls: List[int] = []
        for e, f in enumerate(fields):
            if f is None:
                usn, method, uen = "", UNDEFINED, ""
            else:
                usn, method, uen = f["uniqueServiceName"], f.get("method", UNDEFINED), f["uniqueEndpointName"]
            label = label_map.get(uen) if label_map else None
            self.svc[e] = svc_idx.setdefault(usn, len(svc_idx))
            ck = f"{usn}\t{tpl(method)}\t{tpl(label if label is not None else UNDEFINED)}"
            c = cls_idx.get(ck)
            if c is None:
                c = cls_idx[ck] = len(cls_idx)
                # the key is re-split on tabs in the TS: the linked service is its first three fields
                lsvc_of_cls.append(lsvc_idx.setdefault("\t".join(usn.split("\t")[:3]), len(lsvc_idx)))
            self.cls[e] = c
        self.lsvc = np.array(lsvc_of_cls, dtype=np.uint32)
        self.svc_names = list(svc_idx)
        self.lsvc_names = list(lsvc_idx)
        self.n_ep = len(fields)

    def rank(self, kind: str) -> np.ndarray:
        """Rank of every service name in RiskAnalyzer's sort orders, cached:
        ``locale`` (localeCompare, RiskAnalyzer.ts:63-70) or ``code`` (the
        default Array.sort code-unit order, RiskAnalyzer.ts:72)."""
        cache = self.__dict__.setdefault("_ranks", {})
        if kind not in cache:
            from .risk import _collation_key

            key = _collation_key if kind == "locale" else (lambda x: x)
            order = sorted(range(len(self.svc_names)), key=lambda i: key(self.svc_names[i]))
            r = np.empty(len(order), dtype=np.int64)
            r[order] = np.arange(len(order))
            cache[kind] = r
        return cache[kind]

    def c_struct(self) -> L.TailMap:
        return L.TailMap(L.ptr(self.svc), L.ptr(self.cls), L.ptr(self.lsvc), self.n_ep, len(self.svc_names),
                         len(self.lsvc), len(self.lsvc_names))


def maps_from_dictionary(d, label_map: Optional[Dict[str, str]] = None) -> TailMaps:
    """TailMaps of an ingested batch (ingest.Dictionary's ``dep`` identities)."""
    fields: List[Optional[dict]] = [None] * len(d.ep_names["dep"])
    for s, ident in enumerate(d.shape_ident["dep"]):
        if ident.error is None:
            fields[d.shape_ep["dep"][s]] = ident.fields
    return TailMaps(fields, label_map)


def maps_for_synth(config: int, label_map: Optional[Dict[str, str]] = None) -> TailMaps:
    """TailMaps of a synthetic config (shape id = endpoint id)."""
    from . import synth
    from .ingest import SHAPE_TAGS, dep_identity

    n_shapes, _, _ = synth.describe(config)
    fields = []
    for sh in range(n_shapes):
        name, tags = synth.shape_tags(config, sh)
        fields.append(dep_identity((name,) + tuple(tags.get(t, UNDEFINED) for t in SHAPE_TAGS)))
    return TailMaps(fields, label_map)


def run_tail(eng, maps: TailMaps, endpoints: Optional[np.ndarray] = None) -> "ServiceTail":
    """kmz_tail_run over the engine's current edge set (after a dependency run
    and any multi-GPU merge).  Only the per-service counters come back to the
    host (one read-back: the link counters, each service's rows, gateway flag
    and first row); the link details and cohesion pairs are copied when a list
    output needs them.  ``endpoints`` is no longer needed (kept for callers
    that pass it)."""
    tail_begin(eng, maps)
    return tail_end(eng, maps)


def tail_begin(eng, maps: TailMaps) -> None:
    """run_tail's first half: the tail enqueued on the engine's stream
    (kmz_tail_begin); the host is free until ``tail_end``."""
    lib = L.lib()
    if getattr(eng, "_tail_maps", None) is not maps:
        m = maps.c_struct()
        L.check(eng.ctx, lib.kmz_tail_map_set(eng.ctx, C.byref(m)))
        eng._tail_maps = maps
    L.check(eng.ctx, lib.kmz_tail_begin(eng.ctx))


def tail_end(eng, maps: TailMaps) -> "ServiceTail":
    """Waits for ``tail_begin``'s tail: run_tail's result."""
    lib = L.lib()
    nd, npairs = C.c_uint64(), C.c_uint64()
    L.check(eng.ctx, lib.kmz_tail_end(eng.ctx, C.byref(nd), C.byref(npairs)))
    n_svc = len(maps.svc_names)
    nd_, npairs_ = nd.value, npairs.value
    dist = C.c_uint32()
    L.check(eng.ctx, lib.kmz_tail_service_stats(eng.ctx, None, 0, None, 0, C.byref(dist)))
    stats = np.empty((n_svc, 8), dtype=np.uint32)
    by_dist = np.empty((n_svc, dist.value), dtype=np.uint32)
    L.check(eng.ctx, lib.kmz_tail_service_stats(eng.ctx, L.ptr(stats), stats.size, L.ptr(by_dist), by_dist.size,
                                                  C.byref(dist)))
    first = np.empty(n_svc, dtype=np.uint64)
    L.check(eng.ctx, lib.kmz_tail_service_first(eng.ctx, L.ptr(first), n_svc))
    rows = (stats[:, 6], stats[:, 7] != 0, first)

    def fetch():
        det = np.empty(nd_, dtype=L.TAIL_DETAIL_DTYPE)
        pairs = np.empty(npairs_, dtype=L.TAIL_PAIR_DTYPE)
        L.check(eng.ctx, lib.kmz_tail_get(eng.ctx, L.ptr(det), len(det), L.ptr(pairs), len(pairs), None, 0))
        return det, pairs

    if dist.value == 0:  # a distance beyond the dense relying table: sum the details instead
        det, pairs = fetch()
        t = ServiceTail.from_details(maps, det, pairs, None, None, rows=rows)
    else:
        t = ServiceTail(maps, stats, by_dist, None, None, fetch, rows=rows)
    t.n_details, t.n_pairs = nd_, npairs_
    return t


def _by(n, idx, w=None):
    return np.bincount(np.asarray(idx, dtype=np.int64), weights=w, minlength=n)


class ServiceTail:
    """Service metrics of the reduced dependency graph.

    ``stats[svc]`` are kmz_tail_service_stats' counters (linked services with
    dependingBy / dependingOn, distance-1 AIS/ADS details, cohesion consumers
    and consumes), ``by_dist[svc, d]`` the dependingBy sums per distance."""

    def __init__(self, maps: TailMaps, stats: np.ndarray, by_dist: np.ndarray, hasin: Optional[np.ndarray],
                 endpoints: Optional[np.ndarray], fetch=None, details: Optional[np.ndarray] = None,
                 pairs: Optional[np.ndarray] = None, rows=None):
        """``rows`` = (endpoints with a row, gateway, first row) per service as
        kmz_tail_run computes them on the device; else they are derived here
        from ``endpoints`` (kmz_endpoint records) and ``hasin``."""
        self.maps = maps
        self.stats = stats.astype(np.int64)
        self.by_dist = by_dist
        self._fetch = fetch
        self._details, self._pairs = details, pairs
        n_svc = len(maps.svc_names)
        if rows is not None:
            total, gw, first = rows
            self.total = np.asarray(total, dtype=np.int64)
            self.gateway = np.asarray(gw, dtype=bool)
            first = np.asarray(first, dtype=np.uint64)
        else:
            r = np.nonzero(endpoints["has_row"] != 0)[0]
            rsvc = maps.svc[r].astype(np.int64)
            first = np.full(n_svc, np.iinfo(np.uint64).max, dtype=np.uint64)
            np.minimum.at(first, rsvc, endpoints["first_row"][r])
            self.total = np.bincount(rsvc, minlength=n_svc)
            gw = np.zeros(n_svc, dtype=bool)
            gw[rsvc[hasin[r] == 0]] = True
            self.gateway = gw
        present = np.nonzero(self.total > 0)[0]
        self.services = present[np.argsort(first[present], kind="stable")]  # first-row order (EndpointDependencies.ts:372-384)

    @classmethod
    def from_details(cls, maps: TailMaps, details: np.ndarray, pairs: np.ndarray, hasin: Optional[np.ndarray],
                     endpoints: Optional[np.ndarray], rows=None) -> "ServiceTail":
        """The same counters summed from the link details and pairs (the path
        for distances beyond the dense table, and the CPU restatement's)."""
        n = len(maps.svc_names)
        d = details
        stats = np.zeros((n, 8), dtype=np.int64)
        key = d["svc"].astype(np.int64) * (1 << 24) + d["lsvc"]
        uk, inv = np.unique(key, return_inverse=True)
        by = np.bincount(inv, weights=d["depending_by"], minlength=len(uk))
        on = np.bincount(inv, weights=d["depending_on"], minlength=len(uk))
        s = uk >> 24
        stats[:, 0] = _by(n, s, by > 0)
        stats[:, 1] = _by(n, s, on > 0)
        one = d["distance"] == 1
        stats[:, 2] = _by(n, d["svc"][one], d["depending_by"][one] > 0)
        stats[:, 3] = _by(n, d["svc"][one], d["depending_on"][one] > 0)
        stats[:, 4] = _by(n, pairs["svc"])
        stats[:, 5] = _by(n, pairs["svc"], pairs["consumes"])
        nd = int(d["distance"].max()) + 1 if len(d) else 1
        by_dist = np.zeros((n, nd), dtype=np.int64)
        np.add.at(by_dist, (d["svc"].astype(np.int64), d["distance"].astype(np.int64)), d["depending_by"])
        return cls(maps, stats, by_dist, hasin, endpoints, None, details, pairs, rows=rows)

    # -- lists (copied from the device on demand) ----------------------------------
    def _lists(self):
        if self._details is None:
            det, pairs = self._fetch()
            self._details, self._pairs = det, pairs
        return self._details, self._pairs

    @property
    def details(self) -> np.ndarray:
        d = self._lists()[0]
        return d[np.lexsort((d["distance"], d["lsvc"], d["svc"]))]

    @property
    def pairs(self) -> np.ndarray:
        p = self._lists()[1]
        return p[np.lexsort((p["consumer"], p["svc"]))]

    # -- per service (svc id) ----------------------------------------------------
    def _acs(self):
        return self.stats[:, 2] + self.gateway, self.stats[:, 3]

    def relying_factor(self) -> np.ndarray:
        """RiskAnalyzer.ts:124-137: sum of dependingBy / distance (+1 gateway)."""
        bd = self.by_dist
        if bd.shape[1] <= 1:
            return self.gateway.astype(np.float64)
        return (bd[:, 1:] / np.arange(1, bd.shape[1], dtype=np.float64)).sum(axis=1) + self.gateway

    def instability(self) -> List[dict]:
        """EndpointDependencies.ts:614-641."""
        out = []
        for v in self.services.tolist():
            usn = self.maps.svc_names[v]
            sv, ns, ver = _split3(usn)
            b, o = int(self.stats[v, 0]), int(self.stats[v, 1])
            out.append({"uniqueServiceName": usn, "name": f"{tpl(sv)}.{tpl(ns)} ({tpl(ver)})", "dependingBy": b,
                        "dependingOn": o, "instability": 0 if o + b == 0 else o / (o + b)})
        return out

    def coupling(self) -> List[dict]:
        """EndpointDependencies.ts:643-657 (RiskAnalyzer.ts:145-169)."""
        ais, ads = self._acs()
        out = []
        for v in self.services.tolist():
            usn = self.maps.svc_names[v]
            s, n, ver = (usn.split("\t") + ["undefined"] * 3)[:3]
            out.append({"uniqueServiceName": usn, "name": f"{s}.{n} ({ver})", "ais": int(ais[v]), "ads": int(ads[v]),
                        "acs": int(ais[v] * ads[v])})
        return out

    def cohesion(self) -> List[dict]:
        """EndpointDependencies.ts:565-612 (consumer lists from the pairs)."""
        p = self.pairs
        starts = np.searchsorted(p["svc"], self.services)
        ends = np.searchsorted(p["svc"], self.services, side="right")
        out = []
        for v, a, b in zip(self.services.tolist(), starts.tolist(), ends.tolist()):
            tot = int(self.total[v])
            consumers = [{"uniqueServiceName": self.maps.svc_names[int(c)], "consumes": int(k)}
                         for c, k in zip(p["consumer"][a:b], p["consumes"][a:b])]
            coh = 0
            if tot and consumers:
                acc = 0
                for c in consumers:
                    acc = acc + c["consumes"] / tot
                coh = acc / len(consumers)
            out.append({"uniqueServiceName": self.maps.svc_names[v], "totalEndpoints": tot, "consumers": consumers,
                        "endpointUsageCohesion": coh})
        return out

    def metrics(self) -> Dict[str, np.ndarray]:
        """Every per-service scalar at once, as arrays over ``self.services``
        (no list output: nothing but the counters crosses from the device)."""
        st = self.stats
        nby, non = st[:, 0], st[:, 1]
        tot = nby + non
        inst = np.divide(non, tot, out=np.zeros(len(tot)), where=tot > 0)
        ais, ads = self._acs()
        ncons, cons = st[:, 4], st[:, 5]
        coh = np.divide(cons / np.maximum(self.total, 1), ncons, out=np.zeros(len(tot)),
                        where=(ncons > 0) & (self.total > 0))
        v = self.services
        return {"depending_by": nby[v], "depending_on": non[v], "instability": inst[v], "ais": ais[v],
                "ads": ads[v], "acs": (ais * ads)[v], "relying": self.relying_factor()[v], "cohesion": coh[v],
                "total_endpoints": self.total[v]}

    def service_deps_compact(self) -> List[dict]:
        """What RiskAnalyzer reads from toServiceDependencies(): per service its
        link details and whether it is a gateway (risk.py accepts this form)."""
        d = self.details
        starts = np.searchsorted(d["svc"], self.services)
        ends = np.searchsorted(d["svc"], self.services, side="right")
        out = []
        for v, a, b in zip(self.services.tolist(), starts.tolist(), ends.tolist()):
            dets = [{"distance": int(x["distance"]), "count": int(x["count"]), "dependingBy": int(x["depending_by"]),
                     "dependingOn": int(x["depending_on"])} for x in d[a:b]]
            out.append({"uniqueServiceName": self.maps.svc_names[v], "links": [{"details": dets}],
                        "gateway": bool(self.gateway[v])})
        return out


# -- risk over column arrays (RiskAnalyzer.ts:10-122, 171-248) -------------------
def _js_max(a: np.ndarray) -> float:
    """Math.max(...a): NaN if any element is NaN, -Infinity for no elements."""
    if not len(a):
        return -math.inf
    return float(a.max())  # (numpy's max propagates NaN, as Math.max does)


def _js_min(a: np.ndarray) -> float:
    if not len(a):
        return math.inf
    return float(a.min())


def _fixed_ratio(a: np.ndarray) -> np.ndarray:
    """Normalizer.Strategy.FixedRatio (Normalizer.ts:45-52) on an array."""
    hi = _js_max(a)
    return a if hi == 0 else a / hi


def _linear(a: np.ndarray, minimum: float = 0.1) -> np.ndarray:
    """Normalizer.Strategy.Linear (Normalizer.ts:54-64) on an array."""
    if minimum >= 1:
        return a
    return _fixed_ratio(a) * (1 - minimum) + minimum


def service_sums(data_sid: np.ndarray, n_sid: int, combined: np.ndarray, cv: np.ndarray, is_5xx: np.ndarray,
                 first: Optional[np.ndarray] = None):
    """Per service of the combined rows (RiskAnalyzer.ts:18, 228-248): the
    services in first-occurrence order (``first``: each row's first span
    index; else row order) and, in that order, sum(cv * combined),
    sum(combined) and sum(combined of 5xx rows)."""
    sid = np.asarray(data_sid, dtype=np.int64)
    if first is None:
        uniq, pos = np.unique(sid, return_index=True)
        order_ids = uniq[np.argsort(pos, kind="stable")]
    else:
        mn = np.full(n_sid, np.iinfo(np.uint64).max, dtype=np.uint64)
        np.minimum.at(mn, sid, np.asarray(first, dtype=np.uint64))
        uniq = np.nonzero(mn != np.iinfo(np.uint64).max)[0]
        order_ids = uniq[np.argsort(mn[uniq], kind="stable")]
    remap = np.full(n_sid, -1, dtype=np.int64)
    remap[order_ids] = np.arange(len(order_ids))
    r = remap[sid]
    k = len(order_ids)
    comb = np.asarray(combined, dtype=np.float64)
    wsum = np.bincount(r, weights=np.asarray(cv, dtype=np.float64) * comb, minlength=k)
    cnt = np.bincount(r, weights=comb, minlength=k)
    err = np.bincount(r, weights=comb * np.asarray(is_5xx, dtype=bool), minlength=k)
    return order_ids, wsum, cnt, err


def service_sums_grid(combined: np.ndarray, cv: np.ndarray, first: np.ndarray, status_5xx: np.ndarray,
                      ep_sid: np.ndarray, n_sid: int):
    """``service_sums`` over the engine's group grid (endpoint-major, one column
    per status; unused groups have combined == 0): summed per endpoint first,
    then per service (the fp64 sums reassociate, within the 1e-9 of the
    parity tests), without gathering the used rows."""
    n_st = len(status_5xx)
    comb = np.asarray(combined, dtype=np.float64).reshape(-1, n_st)
    w_ep = (np.asarray(cv, dtype=np.float64).reshape(-1, n_st) * comb).sum(axis=1)
    c_ep = comb.sum(axis=1)
    e_ep = comb[:, np.asarray(status_5xx, dtype=bool)].sum(axis=1)
    big = np.iinfo(np.uint64).max
    f_ep = np.where(comb > 0, np.asarray(first, dtype=np.uint64).reshape(-1, n_st), big).min(axis=1)
    has = c_ep > 0
    sid = np.asarray(ep_sid, dtype=np.int64)[has]
    mn = np.full(n_sid, big, dtype=np.uint64)
    np.minimum.at(mn, sid, f_ep[has])
    uniq = np.nonzero(mn != big)[0]
    order_ids = uniq[np.argsort(mn[uniq], kind="stable")]
    remap = np.full(n_sid, -1, dtype=np.int64)
    remap[order_ids] = np.arange(len(order_ids))
    r = remap[sid]
    k = len(order_ids)
    return (order_ids, np.bincount(r, weights=w_ep[has], minlength=k), np.bincount(r, weights=c_ep[has], minlength=k),
            np.bincount(r, weights=e_ep[has], minlength=k))


def realtime_risk_columns(tail: ServiceTail, data_sid: np.ndarray, sid_names: Sequence[str], combined: np.ndarray,
                          cv: np.ndarray, is_5xx: np.ndarray, replicas: Optional[List[dict]] = None,
                          first: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
    """RiskAnalyzer.RealtimeRisk over the combined rows as columns:
    ``data_sid[i]`` indexes ``sid_names`` (row i's uniqueServiceName).  Rows
    are in toCombinedRealtimeData order, or in any order with ``first`` (each
    row's first span index), which orders services by first occurrence
    (RiskAnalyzer.ts:18).  Same fp64 operations, in the same order, as
    ``risk.realtime_risk`` (which takes row dicts and the full service
    dependencies), as numpy columns: ``sid`` (service ids in output order),
    ``risk``, ``impact``, ``probability``, ``norm`` (one element when every
    risk is equal, Normalizer.ts:22)."""
    return realtime_risk_from_sums(tail, sid_names, *service_sums(data_sid, len(sid_names), combined, cv, is_5xx, first),
                                   replicas=replicas)


def realtime_risk_from_sums(tail: ServiceTail, sid_names: Sequence[str], order_ids: np.ndarray, wsum: np.ndarray,
                            cnt: np.ndarray, err: np.ndarray, replicas: Optional[List[dict]] = None):
    """The rest of ``realtime_risk_columns`` from ``service_sums``."""
    from .cache import to_precise
    from .risk import MINIMUM_PROB as MP

    k = len(order_ids)
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.where(cnt != 0, wsum / np.where(cnt != 0, cnt, 1.0), math.nan)
        # SigmoidAdj (Normalizer.ts:32-41): the libm exp of risk.py (math.exp),
        # element by element, in one call (kmz_host_exp)
        z = 2 * math.log(3)
        arg = np.ascontiguousarray(-z * (rel - 1.5), dtype=np.float64)
        ex = np.empty_like(arg)
        L.lib().kmz_host_exp(L.ptr(arg), L.ptr(ex), len(arg))
        rel_norm = to_precise(1 / (1 + ex))
        total = float(cnt.sum())
        npro = (cnt / total) * (1 - MP) + MP
        nerr = (err / cnt) * (1 - MP) + MP
    base = _linear(npro * nerr, MP)
    prob = (rel_norm * np.where(base < MP, MP, base)) * (1 - MP) + MP
    # impact (RiskAnalyzer.ts:51-85): factors sorted by localeCompare, zipped
    # with the names in code-unit order
    sv = tail.services
    rf = tail.relying_factor()[sv].astype(np.float64)
    ais, ads = tail._acs()
    acs = (ais * ads)[sv].astype(np.float64)
    # (the present services rarely change between ticks: their two orders are
    # kept on the maps for the last set seen)
    memo = tail.maps.__dict__.setdefault("_order_memo", {})
    sk = sv.tobytes()
    if memo.get("key") != sk:
        memo.clear()
        memo["key"] = sk
        memo["orders"] = (np.argsort(tail.maps.rank("locale")[sv], kind="stable"),
                          sv[np.argsort(tail.maps.rank("code")[sv], kind="stable")])
    by_locale, by_code = memo["orders"]
    raw = _fixed_ratio(rf[by_locale]) + _fixed_ratio(acs[by_locale])
    if replicas:
        rep = {}
        for x in replicas:
            rep.setdefault(x["uniqueServiceName"], x.get("replicas"))
        names = tail.maps.svc_names
        raw = raw / np.array([rep.get(names[v]) or 1 for v in by_code.tolist()], dtype=np.float64)
    ni = _linear(raw)
    # service id (sid_names) -> tail service id, through the names (cached on
    # the maps, which outlive the per-run tails), then -> position in code-unit order
    cache = tail.maps.__dict__.setdefault("_sid_to_svc", {})
    key = (id(sid_names), len(sid_names))
    if key not in cache:
        at = {u: v for v, u in enumerate(tail.maps.svc_names)}
        cache.clear()
        cache[key] = (sid_names, np.array([at.get(u, -1) for u in sid_names], dtype=np.int64))
    code_pos = np.full(len(tail.maps.svc_names) + 1, -1, dtype=np.int64)
    code_pos[by_code] = np.arange(len(by_code))
    at_sid = code_pos[cache[key][1][order_ids]]  # (index -1 -> the sentinel: `imp.get(usn) || 0` below)
    im = np.where(at_sid >= 0, ni[np.maximum(at_sid, 0)] if len(ni) else 0.0, 0.0)
    im = np.where(np.isnan(im), 0.0, im)  # `impact || 0` (NaN is falsy)
    p = np.where((prob == 0) | np.isnan(prob), MP, prob)  # `probability || MINIMUM_PROB`
    risk = im * p
    hi, lo = _js_max(risk), _js_min(risk)
    norm = np.array([0.1]) if hi - lo == 0 else ((risk - lo) / (hi - lo)) * 0.9 + 0.1
    return {"sid": order_ids, "risk": risk, "impact": im, "probability": p, "norm": norm}


def realtime_risk_arrays(tail: ServiceTail, data_sid: np.ndarray, sid_names: Sequence[str], combined: np.ndarray,
                         cv: np.ndarray, is_5xx: np.ndarray, replicas: Optional[List[dict]] = None,
                         first: Optional[np.ndarray] = None) -> List[dict]:
    """``realtime_risk_columns`` as RiskAnalyzer.RealtimeRisk's row objects."""
    c = realtime_risk_columns(tail, data_sid, sid_names, combined, cv, is_5xx, replicas, first)
    norm = c["norm"].tolist()
    out = []
    for i, (v, rk, im, p) in enumerate(zip(c["sid"].tolist(), c["risk"].tolist(), c["impact"].tolist(),
                                           c["probability"].tolist())):
        usn = sid_names[v]
        s, n, ver = (usn.split("\t") + [None] * 3)[:3]
        x = {"uniqueServiceName": usn, "service": s, "namespace": n, "version": ver, "risk": rk, "impact": im,
             "probability": p}
        if i < len(norm):
            x["norm"] = norm[i]
        out.append(x)
    return out
