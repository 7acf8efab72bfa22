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


def run_tail(eng, maps: TailMaps, endpoints: np.ndarray) -> "ServiceTail":
    """kmz_tail_run over the engine's current edge set (after a dependency run
    and any multi-GPU merge), then the host finish."""
    lib = L.lib()
    if getattr(eng, "_tail_maps", None) is not maps:
        m = maps.c_struct()
        L.check(eng.ctx, lib.kmz_tail_map_set(eng.ctx, C.byref(m)))
        eng._tail_maps = maps
    nd, npairs = C.c_uint64(), C.c_uint64()
    L.check(eng.ctx, lib.kmz_tail_run(eng.ctx, C.byref(nd), C.byref(npairs)))
    det = np.empty(nd.value, dtype=L.TAIL_DETAIL_DTYPE)
    pairs = np.empty(npairs.value, dtype=L.TAIL_PAIR_DTYPE)
    hasin = np.empty(maps.n_ep, dtype=np.uint8)
    L.check(eng.ctx, lib.kmz_tail_get(eng.ctx, L.ptr(det), len(det), L.ptr(pairs), len(pairs), L.ptr(hasin),
                                      len(hasin)))
    return ServiceTail(maps, det, pairs, hasin, endpoints)


class ServiceTail:
    """Service metrics of the reduced dependency graph."""

    def __init__(self, maps: TailMaps, details: np.ndarray, pairs: np.ndarray, hasin: np.ndarray,
                 endpoints: np.ndarray):
        self.maps = maps
        order = np.lexsort((details["distance"], details["lsvc"], details["svc"]))
        self.details = details[order]
        self.pairs = pairs[np.lexsort((pairs["consumer"], pairs["svc"]))]
        n_svc = len(maps.svc_names)
        rows = np.nonzero(endpoints["has_row"] != 0)[0]
        rsvc = maps.svc[rows].astype(np.int64)
        first = np.full(n_svc, np.iinfo(np.uint64).max, dtype=np.uint64)
        np.minimum.at(first, rsvc, endpoints["first_row"][rows])
        self.total = np.bincount(rsvc, minlength=n_svc)
        gw = np.zeros(n_svc, dtype=bool)
        gw[rsvc[hasin[rows] == 0]] = True
        self.gateway = gw
        present = np.nonzero(self.total > 0)[0]
        self.services = present[np.argsort(first[present], kind="stable")]  # first-row order (EndpointDependencies.ts:372-384)

    # -- per service (svc id) ----------------------------------------------------
    def _link_sides(self):
        """(svc, lsvc) -> (sum dependingBy, sum dependingOn) over distances."""
        d = self.details
        key = d["svc"].astype(np.int64) * (1 << 24) + d["lsvc"]
        uk, inv = np.unique(key, return_inverse=True)
        by = np.bincount(inv, weights=d["depending_by"], minlength=len(uk))
        on = np.bincount(inv, weights=d["depending_on"], minlength=len(uk))
        return (uk >> 24).astype(np.int64), by, on

    def instability(self) -> List[dict]:
        """EndpointDependencies.ts:614-641."""
        n_svc = len(self.maps.svc_names)
        s, by, on = self._link_sides()
        nby = np.bincount(s, weights=(by > 0), minlength=n_svc).astype(np.int64)
        non = np.bincount(s, weights=(on > 0), minlength=n_svc).astype(np.int64)
        out = []
        for v in self.services.tolist():
            usn = self.maps.svc_names[v]
            sv, ns, ver = _split3(usn)
            b, o = int(nby[v]), int(non[v])
            out.append({"uniqueServiceName": usn, "name": f"{tpl(sv)}.{tpl(ns)} ({tpl(ver)})", "dependingBy": b,
                        "dependingOn": o, "instability": 0 if o + b == 0 else o / (o + b)})
        return out

    def _acs(self):
        n_svc = len(self.maps.svc_names)
        d = self.details[self.details["distance"] == 1]
        s = d["svc"].astype(np.int64)
        ais = np.bincount(s, weights=d["depending_by"] > 0, minlength=n_svc).astype(np.int64) + self.gateway
        ads = np.bincount(s, weights=d["depending_on"] > 0, minlength=n_svc).astype(np.int64)
        return ais, ads

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

    def relying_factor(self) -> np.ndarray:
        """RiskAnalyzer.ts:124-137: sum of dependingBy / distance (+1 gateway)."""
        d = self.details
        f = np.zeros(len(self.maps.svc_names), dtype=np.float64)
        np.add.at(f, d["svc"].astype(np.int64), d["depending_by"] / d["distance"])
        return f + self.gateway

    def cohesion(self) -> List[dict]:
        """EndpointDependencies.ts:565-612."""
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
        (instability counts, AIS/ADS/ACS, relying factor, cohesion); the
        cohesion mean is summed in consumer-id order."""
        n_svc = len(self.maps.svc_names)
        s, by, on = self._link_sides()
        nby = np.bincount(s, weights=(by > 0), minlength=n_svc)
        non = np.bincount(s, weights=(on > 0), minlength=n_svc)
        tot = nby + non
        inst = np.divide(non, tot, out=np.zeros(n_svc), where=tot > 0)
        ais, ads = self._acs()
        p = self.pairs
        ps = p["svc"].astype(np.int64)
        share = p["consumes"] / np.maximum(self.total[ps], 1)
        ncons = np.bincount(ps, minlength=n_svc)
        coh = np.divide(np.bincount(ps, weights=share, minlength=n_svc), ncons, out=np.zeros(n_svc),
                        where=(ncons > 0) & (self.total > 0))
        v = self.services
        return {"depending_by": nby[v].astype(np.int64), "depending_on": non[v].astype(np.int64),
                "instability": inst[v], "ais": ais[v], "ads": ads[v], "acs": (ais * ads)[v],
                "relying": self.relying_factor()[v], "cohesion": coh[v], "total_endpoints": self.total[v]}

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
def realtime_risk_arrays(tail: ServiceTail, data_sid: np.ndarray, sid_names: Sequence[str], combined: np.ndarray,
                         cv: np.ndarray, is_5xx: np.ndarray, replicas: Optional[List[dict]] = None) -> List[dict]:
    """RiskAnalyzer.RealtimeRisk over the combined rows as columns (in row
    order): ``data_sid[i]`` indexes ``sid_names`` (the row's
    uniqueServiceName).  Same arithmetic as ``risk.realtime_risk``, which
    takes row dicts and the full service dependencies."""
    from .risk import MINIMUM_PROB, Normalizer, _collation_key

    sid = np.asarray(data_sid, dtype=np.int64)
    # services in first-occurrence order of their rows
    uniq, first = np.unique(sid, return_index=True)
    order_ids = uniq[np.argsort(first, kind="stable")]
    remap = np.full(len(sid_names), -1, dtype=np.int64)
    remap[order_ids] = np.arange(len(order_ids))
    r = remap[sid]
    k = len(order_ids)
    comb = np.asarray(combined, dtype=np.float64)
    # latency CV per service weighted by request count (RiskAnalyzer.ts:228-248)
    wsum = np.zeros(k)
    np.add.at(wsum, r, np.asarray(cv, dtype=np.float64) * comb)
    cnt = np.bincount(r, weights=comb, minlength=k)
    err = np.bincount(r, weights=comb * np.asarray(is_5xx, dtype=bool), minlength=k)
    rel_norm = Normalizer.Strategy.SigmoidAdj([wsum[i] / cnt[i] if cnt[i] else math.nan for i in range(k)])
    total = float(cnt.sum())
    npro = [(cnt[i] / total) * (1 - MINIMUM_PROB) + MINIMUM_PROB for i in range(k)]
    nerr = [(err[i] / cnt[i]) * (1 - MINIMUM_PROB) + MINIMUM_PROB for i in range(k)]
    base = Normalizer.Strategy.Linear([p * nerr[i] for i, p in enumerate(npro)], MINIMUM_PROB)
    prob = [(rel_norm[i] * (MINIMUM_PROB if base[i] < MINIMUM_PROB else base[i])) * (1 - MINIMUM_PROB) + MINIMUM_PROB
            for i in range(k)]
    # impact (RiskAnalyzer.ts:51-85)
    svc_names = [tail.maps.svc_names[v] for v in tail.services.tolist()]
    rf = tail.relying_factor()[tail.services]
    ais, ads = tail._acs()
    acs = (ais * ads)[tail.services]
    order = sorted(range(len(svc_names)), key=lambda i: _collation_key(svc_names[i]))
    nrf = Normalizer.Strategy.FixedRatio([float(rf[i]) for i in order])
    nacs = Normalizer.Strategy.FixedRatio([float(acs[i]) for i in order])
    rep = {}
    for x in replicas or []:
        rep.setdefault(x["uniqueServiceName"], x.get("replicas"))
    raw = []
    for i, usn in enumerate(sorted(svc_names)):
        div = rep.get(usn) or 1
        raw.append((usn, (nrf[i] + nacs[i]) / div))
    ni = Normalizer.Strategy.Linear([x[1] for x in raw])
    imp: Dict[str, float] = {}
    for i, (usn, _) in enumerate(raw):
        imp.setdefault(usn, ni[i])
    risks = []
    for i, v in enumerate(order_ids.tolist()):
        usn = sid_names[v]
        s, n, ver = (usn.split("\t") + [None] * 3)[:3]
        im = imp.get(usn) or 0
        p = prob[i] or MINIMUM_PROB
        risks.append({"uniqueServiceName": usn, "service": s, "namespace": n, "version": ver, "risk": im * p,
                      "impact": im, "probability": p})
    norm = Normalizer.Strategy.BetweenFixedNumber([x["risk"] for x in risks])
    return [{**x, **({"norm": norm[i]} if i < len(norm) else {})} for i, x in enumerate(risks)]
