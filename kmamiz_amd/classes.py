"""Drop-in mirror of the reference's hot-path classes, backed by the HIP engine.

Same class and method names as the TypeScript (src/classes/*.ts), same
argument meaning, same output objects (``toJSON()`` lists of plain dicts with
JS semantics: properties that would be ``undefined`` are absent).

* :class:`Traces`                   src/classes/Traces.ts:17-241
* :class:`RealtimeDataList`         src/classes/RealtimeDataList.ts:7-157
* :class:`CombinedRealtimeDataList` src/classes/CombinedRealtimeDataList.ts:16-333
* :class:`EndpointDependencies`     src/classes/EndpointDependencies.ts:17-658

The per-span work (join, contraction, traversal, reductions) runs on the GPU;
the host only interns strings per distinct shape, and turns the engine's
integer results back into objects (per group / per row, never per regex).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib as L
from . import settings
from .engine import Engine
from .envoy import merge, merge_string_body, object_to_interface_string, parse_request_response_body
from .ingest import (UNDEFINED, Dictionary, dep_identity, explode_url, ingest_json, ingest_rows, ingest_traces,
                     js_truthy, tpl)

_engines: Dict[int, Engine] = {}


def default_engine(device: int = 0) -> Engine:
    e = _engines.get(device)
    if e is None or e.ctx is None:
        e = _engines[device] = Engine(device)
        e._loaded_token = None
    return e


def _clean(d: dict) -> dict:
    return {k: v for k, v in d.items() if v is not UNDEFINED}


# ------------------------------------------------------------------------------
# Traces
# ------------------------------------------------------------------------------
class _LazyFlat:
    """The flattened span dicts of a Traces built from raw JSON, parsed only if
    a per-span object is ever materialised (small batches)."""

    def __init__(self, owner: "Traces"):
        self._owner = owner
        self._flat = None

    def _get(self):
        if self._flat is None:
            self._flat = [s for t in self._owner._traces for s in t]
        return self._flat

    def __getitem__(self, i):
        return self._get()[i]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())


class Traces:
    def __init__(self, traces, engine: Optional[Engine] = None):
        self._traces_v = traces
        self._raw = None
        self._engine = engine
        self._ingested = None

    @classmethod
    def from_json(cls, data: bytes, engine: Optional[Engine] = None, threads: int = 0) -> "Traces":
        """Traces of a raw Zipkin response (Trace[][] JSON bytes, as
        ZipkinService.ts:44-57 receives it): columns come from the native
        parser (kmz_parse_zipkin) without building span
        objects; the JSON is parsed into objects only if a per-span result is
        materialised, or if the batch is outside the parser's fast path."""
        t = cls(None, engine)
        t._raw = bytes(data)
        t._threads = threads
        return t

    @property
    def _traces(self):
        if self._traces_v is None and self._raw is not None:
            import json

            self._traces_v = json.loads(self._raw)
        return self._traces_v

    def toJSON(self):
        return self._traces

    # -- plumbing -------------------------------------------------------------
    def _ingest(self):
        if self._ingested is None:
            r = ingest_json(self._raw, threads=self._threads) if self._raw is not None else None
            self._ingested = (r[0], r[1], _LazyFlat(self)) if r is not None else ingest_traces(self._traces)
        return self._ingested

    def _load(self) -> Engine:
        batch, d, _ = self._ingest()
        eng = self._engine or default_engine()
        if getattr(eng, "_loaded_token", None) is not self:
            eng.load(batch, d.shape_table())
            eng._loaded_token = self
        return eng

    # -- realtime -------------------------------------------------------------
    def toRealTimeData(self, replicas=None) -> "RealtimeDataList":
        """Traces.ts:27-53 (rows stay on the device until toJSON())."""
        return RealtimeDataList(_native=(self, "rt", replicas))

    def combineLogsToRealtimeData(self, structuredLogs=(), replicas=None) -> "RealtimeDataList":
        """Traces.ts:55-106.  The stats come from the engine (K3); the Envoy-log
        join (59-84: per SERVER span the log of (traceId, id), or of (traceId,
        parentId) when that is missing or a fallback) only adds request /
        response bodies and content types, host-side."""
        logs = _log_map(structuredLogs)
        return RealtimeDataList(_native=(self, "tag", replicas, logs))

    def _span_log(self, logs, i: int):
        """The log entry the reference picks for flat span i (Traces.ts:80-84)."""
        if not logs:
            return None
        s = self._ingest()[2][i]
        lm = logs.get(s.get("traceId", UNDEFINED))
        log = lm.get(s.get("id", UNDEFINED)) if lm is not None else None
        # (a log object is truthy in JS even when empty)
        if (log is None or js_truthy(log.get("isFallback", UNDEFINED))) and js_truthy(s.get("parentId", UNDEFINED)):
            log = lm.get(s["parentId"]) if lm is not None else None
        return log

    def extractContainingNamespaces(self):
        """Traces.ts:108-110."""
        _, d, flat = self._ingest()
        return set(s.get("tags", {}).get("istio.namespace", None) for s in flat)

    # -- dependencies -----------------------------------------------------------
    def toEndpointDependencies(self) -> "EndpointDependencies":
        """Traces.ts:112-211 on the GPU; objects are materialised lazily."""
        eng = self._load()
        eng.run(L.RUN_DEPS | L.RUN_SPAN_LINKS | L.RUN_DEP_ORDER)
        return EndpointDependencies(_native=_DepResult(self, eng))

    @staticmethod
    def ToEndpointInfo(trace: dict) -> dict:
        """Traces.ts:213-241."""
        tags = trace.get("tags", {}) or {}
        from .ingest import SHAPE_TAGS

        key = (trace.get("name", UNDEFINED),) + tuple(tags.get(t, UNDEFINED) for t in SHAPE_TAGS)
        info = dict(dep_identity(key))
        info["timestamp"] = trace["timestamp"] / 1000
        return _clean(info)


def _log_map(structuredLogs):
    """traceId -> spanId -> TStructuredEnvoyLogTrace (Traces.ts:59-67); a log
    with no traces is skipped, the last entry of a spanId wins."""
    m: Dict = {}
    for l in structuredLogs or ():
        trs = l.get("traces", [])
        if len(trs) == 0:
            continue
        d = m.setdefault(trs[0]["traceId"], {})
        for t in trs:
            d[t["spanId"]] = t
    return m


def _log_fields(log) -> dict:
    """The body fields of a realtime row (Traces.ts:94-97)."""
    if log is None:
        return {}
    req, res = log.get("request"), log.get("response")
    if req is None or res is None:  # `log?.response.body` throws in the reference
        raise TypeError("Cannot read properties of undefined (reading 'body')")
    return {"responseBody": res.get("body", UNDEFINED), "responseContentType": res.get("contentType", UNDEFINED),
            "requestBody": req.get("body", UNDEFINED), "requestContentType": req.get("contentType", UNDEFINED)}


JSON_CT = "application/json"


def _replica_lookup(replicas, usn):
    if not replicas:
        return UNDEFINED
    for r in replicas:
        if r.get("uniqueServiceName") == usn:
            return r.get("replicas", UNDEFINED)
    return UNDEFINED


# ------------------------------------------------------------------------------
# RealtimeDataList
# ------------------------------------------------------------------------------
class RealtimeDataList:
    def __init__(self, realtimeData: Optional[List[dict]] = None, *, _native=None):
        self._rows = realtimeData
        self._native = _native  # (Traces, rule, replicas)

    def toJSON(self):
        if self._rows is None:
            self._rows = self._materialize_rows()
        return self._rows

    def getContainingNamespaces(self):
        return set(r.get("namespace") for r in self.toJSON())

    def _materialize_rows(self):
        traces, rule, replicas, logs = (tuple(self._native) + (None,))[:4]
        batch, d, flat = traces._ingest()
        out = []
        idx = np.nonzero(batch.kind == L.KIND_SERVER)[0]
        bad = [i for i in idx if d.shape_ident[rule][batch.shape[i]].error is not None]
        if bad:
            raise d.shape_ident[rule][batch.shape[bad[0]]].error
        for i in idx:
            f = d.shape_ident[rule][batch.shape[i]].fields
            s = flat[i]
            out.append(
                _clean(
                    {
                        "timestamp": s["timestamp"],
                        "service": f["service"],
                        "namespace": f["namespace"],
                        "version": f["version"],
                        "method": f["method"],
                        "latency": s["duration"] / 1000,
                        "status": s.get("tags", {}).get("http.status_code", UNDEFINED),
                        "uniqueServiceName": f["uniqueServiceName"],
                        "uniqueEndpointName": f["uniqueEndpointName"],
                        "replica": _replica_lookup(replicas, f["uniqueServiceName"]),
                        **_log_fields(traces._span_log(logs, int(i))),
                    }
                )
            )
        return out

    def toCombinedRealtimeData(self) -> "CombinedRealtimeDataList":
        """RealtimeDataList.ts:22-97 on the GPU (K3 + finalisation)."""
        if self._native is not None:
            traces, rule, replicas, logs = (tuple(self._native) + (None,))[:4]
            eng = traces._load()
            eng.run(L.RUN_STATS_RT if rule == "rt" else L.RUN_STATS_TAG)
            batch, d, _ = traces._ingest()
            return CombinedRealtimeDataList(_combine_native(_run_groups(eng), eng.index_base, batch, d, rule, replicas,
                                                            traces if logs else None, logs))
        rows = self._rows or []
        batch, table, d, first_row = ingest_rows(rows)
        eng = default_engine()
        eng.load(batch, table)
        eng._loaded_token = None
        eng.run(L.RUN_STATS_RT)
        return CombinedRealtimeDataList(_combine_rows(_run_groups(eng), rows, d, table.n_status))


class _UsedGroups:
    """The used groups of a run (kmz_fetch_used: ids ascending, their records),
    indexable by group id like the dense array."""

    def __init__(self, ids: np.ndarray, recs: np.ndarray):
        self.ids = np.asarray(ids, dtype=np.int64)
        self.recs = recs

    def __getitem__(self, g):
        return self.recs[int(np.searchsorted(self.ids, g))]


def _run_groups(eng):
    """The last stats run's groups: only the used ones where the engine
    compacts them (a small batch touches a few percent of the groups), else
    the dense array."""
    try:
        ids, recs, _, _ = eng.fetch_used(deps=False)
    except Exception:  # noqa: BLE001 (KMZ_E_UNSUPPORTED past 2^22 groups: the dense copy)
        return eng.groups()
    return _UsedGroups(ids.copy(), recs.copy())


def _ordered_groups(groups, n_status: int):
    """Used groups in toCombinedRealtimeData order: endpoints by first row,
    statuses by first row within the endpoint (RealtimeDataList.ts:24-45)."""
    if isinstance(groups, _UsedGroups):
        used, first = groups.ids, groups.recs["first"]
    else:
        used = np.nonzero(groups["combined"] > 0)[0]
        first = groups["first"][used]
    if len(used) == 0:
        return []
    ep = used // n_status
    ep_first = {}
    for e, f in zip(ep.tolist(), first.tolist()):
        if e not in ep_first or f < ep_first[e]:
            ep_first[e] = f
    order = sorted(range(len(used)), key=lambda k: (ep_first[int(ep[k])], int(first[k])))
    return [(int(used[k]), int(ep[k]), ep_first[int(ep[k])]) for k in order]


def _combine_native(groups, index_base, batch, d: Dictionary, rule, replicas, traces=None, logs=None):
    n_status = max(1, len(d.statuses))
    out = []
    # with Envoy logs: reduce() keeps the first row's content types
    # (RealtimeDataList.ts:53-67); bodies reach the output only for
    # application/json, where the reference also infers a schema with
    # json-to-ts (RealtimeDataList.ts:120-155) -- absent here, so refused
    firsts = rows_of = None
    if logs:
        firsts = {}
        srv = np.nonzero(batch.kind == L.KIND_SERVER)[0]
        gid = np.asarray(d.shape_ep[rule], dtype=np.int64)[batch.shape[srv]] * n_status + batch.status[srv]
        for i, g in zip(srv.tolist(), gid.tolist()):
            firsts.setdefault(g, i)
        # groups whose first row is application/json fold every row's bodies
        rows_of = {}
        for g, i in firsts.items():
            f = _log_fields(traces._span_log(logs, i))
            if JSON_CT in (f.get("requestContentType"), f.get("responseContentType")):
                rows_of[g] = []
        if rows_of:
            for i, g in zip(srv.tolist(), gid.tolist()):
                if g in rows_of:
                    rows_of[g].append(i)
    for g, e, ep_first in _ordered_groups(groups, n_status):
        if e in d.poison[rule]:
            # the reference throws while building the realtime rows (Utils.ts:90)
            i = int(ep_first - index_base)
            raise d.shape_ident[rule][batch.shape[i]].error
        rec = groups[g]
        f = d.shape_ident[rule][batch.shape[int(ep_first - index_base)]].fields
        n = int(rec["combined"])
        r = _replica_lookup(replicas, f["uniqueServiceName"])
        avg = UNDEFINED
        if js_truthy(r):
            avg = (r * n) / n if float(r).is_integer() else _seq_sum(r, n) / n
        out.append(
            _clean(
                {
                    "uniqueServiceName": f["uniqueServiceName"],
                    "uniqueEndpointName": f["uniqueEndpointName"],
                    "service": f["service"],
                    "namespace": f["namespace"],
                    "version": f["version"],
                    "method": f["method"],
                    "status": d.statuses[g % n_status],
                    "combined": n,
                    "avgReplica": avg,
                    "latestTimestamp": int(rec["latest_timestamp"]),
                    "latency": {"mean": float(rec["mean"]), "cv": float(rec["cv"])},
                    **_group_log_fields(traces, logs, firsts, rows_of, g),
                }
            )
        )
    return out


def _group_log_fields(traces, logs, firsts, rows_of, g) -> dict:
    """The group's content types (its first row's: the reduce starts from it,
    RealtimeDataList.ts:53-67) and, for application/json, the bodies folded
    with Utils.MergeStringBody over the group's rows in order, parsed, with
    their schemas (parseRequestResponseBody, RealtimeDataList.ts:120-155)."""
    if firsts is None:
        return {}
    f = _log_fields(traces._span_log(logs, firsts[g]))
    ct = {k: f[k] for k in ("requestContentType", "responseContentType") if f.get(k, UNDEFINED) is not UNDEFINED}
    if g not in rows_of:
        return ct
    req, res = f.get("requestBody", UNDEFINED), f.get("responseBody", UNDEFINED)
    for i in rows_of[g][1:]:
        fi = _log_fields(traces._span_log(logs, i))
        req = merge_string_body(req, fi.get("requestBody", UNDEFINED))
        res = merge_string_body(res, fi.get("responseBody", UNDEFINED))
    return {**ct, **parse_request_response_body({**ct, "requestBody": req, "responseBody": res})}


def _seq_sum(r, n):
    s = r
    for _ in range(n - 1):
        s += r
    return s


def _combine_rows(groups, rows, d: Dictionary, n_status):
    out = []
    # rows of each group in order (for the replica reduce, RealtimeDataList.ts:53-67)
    for g, e, ep_first in _ordered_groups(groups, n_status):
        rec = groups[g]
        sample = rows[ep_first]
        first = rows[int(rec["first"])]
        st = d.statuses[g % n_status]
        acc = first.get("replica", UNDEFINED)
        cts = (first.get("requestContentType", UNDEFINED), first.get("responseContentType", UNDEFINED))
        bodies = {}
        if js_truthy(acc) or JSON_CT in cts:
            uen = sample["uniqueEndpointName"]
            req, res = first.get("requestBody", UNDEFINED), first.get("responseBody", UNDEFINED)
            seen_first = False
            for r in rows:
                if r["uniqueEndpointName"] != uen or r.get("status", UNDEFINED) != st:
                    continue
                if not seen_first:
                    seen_first = True
                    continue
                cur = r.get("replica", UNDEFINED)
                if js_truthy(acc) and js_truthy(cur):
                    acc = acc + cur
                req = merge_string_body(req, r.get("requestBody", UNDEFINED))
                res = merge_string_body(res, r.get("responseBody", UNDEFINED))
            if JSON_CT in cts:
                bodies = parse_request_response_body({"requestContentType": cts[0], "responseContentType": cts[1],
                                                      "requestBody": req, "responseBody": res})
        n = int(rec["combined"])
        out.append(
            _clean(
                {
                    "uniqueServiceName": sample.get("uniqueServiceName", UNDEFINED),
                    "uniqueEndpointName": sample["uniqueEndpointName"],
                    "service": sample.get("service", UNDEFINED),
                    "namespace": sample.get("namespace", UNDEFINED),
                    "version": sample.get("version", UNDEFINED),
                    "method": sample.get("method", UNDEFINED),
                    "status": st,
                    "combined": n,
                    "avgReplica": acc / n if js_truthy(acc) else UNDEFINED,
                    "latestTimestamp": int(rec["latest_timestamp"]),
                    "latency": {"mean": float(rec["mean"]), "cv": float(rec["cv"])},
                    "requestContentType": first.get("requestContentType", UNDEFINED),
                    "responseContentType": first.get("responseContentType", UNDEFINED),
                    **bodies,
                }
            )
        )
    return out


# ------------------------------------------------------------------------------
# CombinedRealtimeDataList
# ------------------------------------------------------------------------------
def _decimal_shift(m1: float, m2: float) -> int:
    """CombinedRealtimeDataList.ts:322-332."""
    e1 = math.floor(math.log10(m1)) if m1 > 0 else 0
    e2 = math.floor(math.log10(m2)) if m2 > 0 else 0
    return math.floor((e1 + e2) / 2)


def _pooled(n1, m1, c1, n2, m2, c2):
    """CombinedRealtimeDataList.ts:278-315 (same operation order)."""
    scale = math.pow(10, _decimal_shift(m1, m2))
    a, b = m1 / scale, m2 / scale
    sa, sb = c1 * a, c2 * b
    tot = n1 + n2
    mt = (n1 * a + n2 * b) / tot
    da, db = a - mt, b - mt  # (x ** 2 is Math.pow(x, 2) = x * x in V8's fdlibm pow)
    pv = (n1 * (sa * sa) + n2 * (sb * sb) + n1 * (da * da) + n2 * (db * db)) / tot
    return mt * scale, (0 if mt == 0 else math.sqrt(pv) / mt)


def _to_precise(x: float) -> float:
    t = (x + 2.220446049250313e-16) * 1e14
    r = math.floor(t)
    if t - r >= 0.5:
        r += 1
    return float(r) / 1e14


class CombinedRealtimeDataList:
    def __init__(self, combinedRealtimeData: List[dict]):
        self._data = combinedRealtimeData

    def toJSON(self):
        return self._data

    def getContainingNamespaces(self):
        return set(r.get("namespace") for r in self._data)

    def adjustTimestamp(self, to):
        return CombinedRealtimeDataList([{**r, "latestTimestamp": to * 1000} for r in self._data])

    def combineWith(self, rlData: "CombinedRealtimeDataList") -> "CombinedRealtimeDataList":
        """CombinedRealtimeDataList.ts:183-263: group by endpoint+status, sum
        counts, max timestamps, Utils.Merge the bodies (+ their schemas), fold
        (n, mean, cv) pairwise in list order."""
        by_key: Dict[str, List[dict]] = {}
        for r in list(self._data) + list(rlData._data):
            by_key.setdefault(f"{r['uniqueEndpointName']}\t{tpl(r.get('status', UNDEFINED))}", []).append(r)
        out = []
        for grp in by_key.values():
            s = grp[0]
            total = sum(int(x["combined"]) for x in grp)
            latest = s["latestTimestamp"]
            avg = s.get("avgReplica", UNDEFINED)
            for x in grp[1:]:
                xa = x.get("avgReplica", UNDEFINED)
                if js_truthy(avg) and js_truthy(xa):
                    avg = avg + xa
                latest = max(latest, x["latestTimestamp"])
                # Utils.Merge of the parsed bodies (two absent ones merge to {}),
                # and the schema of a truthy result (CombinedRealtimeDataList.ts:212-223)
                for side in ("request", "response"):
                    b = merge(s.get(side + "Body", UNDEFINED), x.get(side + "Body", UNDEFINED))
                    s[side + "Body"] = b
                    if js_truthy(b):
                        s[side + "Schema"] = object_to_interface_string(b)
            if js_truthy(avg) and "avgReplica" in s:
                s["avgReplica"] = avg  # the reduce mutates group[0] (208-210)
            s["latestTimestamp"] = latest
            n, m, c = 0, 0.0, 0.0
            for x in grp:
                m, c = _pooled(n, m, c, x["combined"], x["latency"]["mean"], x["latency"]["cv"])
                n += x["combined"]
            out.append(
                _clean(
                    {
                        "uniqueEndpointName": s["uniqueEndpointName"],
                        "uniqueServiceName": s.get("uniqueServiceName", UNDEFINED),
                        "service": s.get("service", UNDEFINED),
                        "namespace": s.get("namespace", UNDEFINED),
                        "version": s.get("version", UNDEFINED),
                        "method": s.get("method", UNDEFINED),
                        "status": s.get("status", UNDEFINED),
                        "combined": total,
                        "requestContentType": s.get("requestContentType", UNDEFINED),
                        "responseContentType": s.get("responseContentType", UNDEFINED),
                        "latestTimestamp": latest,
                        "requestBody": s.get("requestBody", UNDEFINED),
                        "requestSchema": s.get("requestSchema", UNDEFINED),
                        "responseBody": s.get("responseBody", UNDEFINED),
                        "responseSchema": s.get("responseSchema", UNDEFINED),
                        "latency": {"mean": _to_precise(m), "cv": _to_precise(c)},
                    }
                )
            )
        return CombinedRealtimeDataList(out)

    def toHistoricalData(self, serviceDependencies: List[dict], replicas: Optional[List[dict]] = None,
                         labelMap: Optional[Dict[str, str]] = None) -> List[dict]:
        """CombinedRealtimeDataList.ts:26-150, host side:
        the combined rows (one per endpoint x status, already reduced on the
        GPU) are bucketed by the UTC minute of their latestTimestamp
        (Utils.BelongsToMinuteTimestamp, Utils.ts:135-141); each minute gets its
        endpoint and service summaries and RiskAnalyzer.RealtimeRisk
        (RiskAnalyzer.ts:10-49).  ``date`` is the ISO string of the JSON form."""
        import datetime

        from .risk import realtime_risk

        def minute(ts_ms: float) -> int:
            return (math.trunc(ts_ms) // 60000) * 60000  # Date truncates, the ISO minute floors

        def iso(ms: int) -> str:
            d = datetime.datetime(1970, 1, 1) + datetime.timedelta(milliseconds=ms)
            return d.strftime("%Y-%m-%dT%H:%M:%S.") + f"{ms % 1000:03d}Z"

        def mean_of(rows, ok) -> float:
            vals = [r["latency"]["mean"] for r in rows if ok(r["latency"].get("mean"))]
            if not vals:
                return 0
            acc = 0.0
            for v in vals:  # left-to-right, as Array.reduce
                acc += v
            m = acc / len(vals)
            return m if math.isfinite(m) else 0

        buckets: Dict[int, List[dict]] = {}
        for r in self._data:
            buckets.setdefault(minute(r["latestTimestamp"] / 1000), []).append(r)
        out = []
        for t, rows in buckets.items():
            risks = {x["uniqueServiceName"]: x for x in reversed(realtime_risk(rows, serviceDependencies, replicas or []))}
            by_ep: Dict[str, List[dict]] = {}
            by_svc: Dict[str, List[dict]] = {}
            for r in rows:
                by_ep.setdefault(r["uniqueEndpointName"], []).append(r)
                by_svc.setdefault(r["uniqueServiceName"], []).append(r)
            endpoints = []
            for uen, rs in by_ep.items():
                svc, ns, ver, method = (uen.split("\t") + [None] * 4)[:4]
                e = {
                    "latencyMean": mean_of(rs, lambda m: m is not None),
                    "latencyCV": max((r["latency"].get("cv") or 0) for r in rs),
                    "method": method,
                    "requestErrors": sum(r["combined"] for r in rs if str(r["status"]).startswith("4")),
                    "requests": sum(r["combined"] for r in rs),
                    "serverErrors": sum(r["combined"] for r in rs if str(r["status"]).startswith("5")),
                    "uniqueEndpointName": uen,
                    "uniqueServiceName": f"{svc}\t{ns}\t{ver}",
                }
                if labelMap and uen in labelMap:
                    e["labelName"] = labelMap[uen]
                endpoints.append(e)
            services = []
            for usn, rs in by_svc.items():
                svc, ns, ver = (usn.split("\t") + [None] * 3)[:3]
                mine = [e for e in endpoints if e["uniqueServiceName"] == usn]
                svc_info = {
                    "date": iso(t),
                    "endpoints": mine,
                    "service": svc,
                    "namespace": ns,
                    "version": ver,
                    "requests": sum(e["requests"] for e in mine),
                    "requestErrors": sum(e["requestErrors"] for e in mine),
                    "serverErrors": sum(e["serverErrors"] for e in mine),
                    "latencyMean": mean_of(rs, lambda m: isinstance(m, (int, float)) and math.isfinite(m)),
                    "latencyCV": max((r["latency"].get("cv") or 0) for r in rs),
                    "uniqueServiceName": usn,
                }
                if "norm" in risks[usn]:  # (BetweenFixedNumber of equal risks gives one value: Normalizer.ts:22)
                    svc_info["risk"] = risks[usn]["norm"]
                services.append(svc_info)
            out.append({"date": iso(t), "services": services})
        return out

    def extractEndpointDataType(self, *a, **k):
        raise NotImplementedError("endpoint schema inference is out of scope (SURVEY.md 2)")


# ------------------------------------------------------------------------------
# EndpointDependencies
# ------------------------------------------------------------------------------
class _DepResult:
    """Engine outputs of one toEndpointDependencies() call."""

    def __init__(self, traces: Traces, eng: Engine):
        batch, d, flat = traces._ingest()
        self.traces = traces
        self.batch, self.dict, self.flat = batch, d, flat
        self.cparent, self.rowpos = eng.span_links()
        self.endpoints = eng.endpoints()
        self.triples = eng.triples()
        self.info = eng.info()
        self.index_base = eng.index_base
        self.order = eng.dep_entries()
        self.eng, self.gen = eng, eng.gen  # (the engine still holds this run while its gen is unchanged)
        for e in d.poison["dep"]:
            if self.endpoints["has_row"][e] or np.any((self.triples >> np.uint64(40)) == np.uint64(e)):
                raise self._poison_error(e)

    def _poison_error(self, e):
        d, b = self.dict, self.batch
        for i in range(len(b)):
            if d.shape_ep["dep"][b.shape[i]] == e:
                return d.shape_ident["dep"][b.shape[i]].error
        return TypeError("ExplodeUrl failed")

    def reduced_graph(self, reg=None):
        """cache.ReducedDependencies of EndpointDependencies([]).combineWith(rows).trim()
        from the engine's entry order (kmz_get_dep_entries), no per-span work."""
        from .cache import ReducedDependencies

        entries, rts, rsh = self.order
        idents = self.dict.shape_ident["dep"]
        return ReducedDependencies.from_window(entries, rts, rsh, self.endpoints, self.dict.ep_names["dep"],
                                               lambda s: idents[s].fields, reg)

    def info_of(self, i: int) -> dict:
        f = self.dict.shape_ident["dep"][self.batch.shape[i]].fields
        return _clean({**f, "timestamp": self.flat[i]["timestamp"] / 1000})

    def materialize(self) -> List[dict]:
        """Exact per-row objects (Traces.ts:145-210) from the GPU links."""
        rp = self.rowpos
        rows = np.nonzero(rp != np.uint64(L.NONE64))[0]
        rows = rows[np.argsort(rp[rows], kind="stable")]
        cp = self.cparent
        d = self.dict
        dep_of = d.shape_ep["dep"]
        shape = self.batch.shape
        uppers = []
        lower: Dict[int, List] = {}
        for s in rows.tolist():
            chain = []
            q = int(cp[s])
            depth = 1
            while q != L.NONE32:
                chain.append((q, depth))
                lower.setdefault(q, []).append((s, depth))
                q = int(cp[q])
                depth += 1
            uppers.append(chain)
        last = self.endpoints["last_ts"]
        out = []
        for s, chain in zip(rows.tolist(), uppers):
            by = [{"endpoint": self.info_of(q), "distance": dist, "type": "CLIENT"} for q, dist in chain]
            seen: Dict[tuple, int] = {}
            on_keys: List[tuple] = []
            for t, dist in lower.get(s, []):
                k = (dep_of[shape[t]], dist)
                if k not in seen:
                    on_keys.append(k)
                seen[k] = t
            on = [{"endpoint": self.info_of(seen[k]), "distance": k[1], "type": "SERVER"} for k in on_keys]
            e = dep_of[shape[s]]
            lt = int(last[e])
            out.append(
                {
                    "endpoint": self.info_of(s),
                    "lastUsageTimestamp": max(0.0, lt / 1000) if lt != np.iinfo(np.int64).min else 0,
                    "isDependedByExternal": len(by) == 0,
                    "dependingBy": by,
                    "dependingOn": on,
                }
            )
        return out


class EndpointDependencies:
    def __init__(self, dependencies: Optional[List[dict]] = None, *, _native: Optional[_DepResult] = None):
        # the constructor's deprecation filter (EndpointDependencies.ts:40-74):
        # the identity unless DEPRECATED_ENDPOINT_THRESHOLD is set; the cutoff
        # is taken now (Date.now() in the constructor) and applied to an
        # engine result when its rows or reduced form are first built
        self._cutoff = settings.deprecated_cutoff()
        self._deps = settings.filter_out_deprecated(dependencies, self._cutoff) if dependencies is not None else None
        self._native = _native

    def _list(self) -> List[dict]:
        if self._deps is None:
            self._deps = settings.filter_out_deprecated(self._native.materialize(), self._cutoff)
        return self._deps

    def toJSON(self):
        return self._list()

    def reduced(self):
        """Scale form of the graph: sorted unique edge keys
        (anc_ep<<40|desc_ep<<16|distance<<1|on) + per-endpoint records."""
        if self._native is None:
            raise ValueError("reduced() needs an engine-backed result")
        keys, eps = self._native.triples, self._native.endpoints
        if self._cutoff != 0:  # the constructor's filter on the reduced form (EndpointDependencies.ts:44-74)
            lt = eps["last_ts"]
            last = np.where(lt == np.iinfo(np.int64).min, 0.0, np.maximum(0.0, lt / 1000))
            stale = (eps["has_row"] != 0) & (last < self._cutoff)
            if stale.any():
                a = (keys >> np.uint64(40)).astype(np.int64)
                d = ((keys >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.int64)
                keys = keys[~(stale[a] | stale[d])]
                eps = eps.copy()
                eps["has_row"][stale] = 0
        return keys, eps

    def service_tail(self, labelMap: Optional[Dict[str, str]] = None):
        """Scale form of the service-level tail (tail.ServiceTail) of the
        reduced graph ``EndpointDependencies([]).combineWith(self).trim()``,
        computed on the GPU from the edge keys (kmz_tail_run).

        Side effect with DEPRECATED_ENDPOINT_THRESHOLD set: the filtered edge
        keys and endpoint partials are written into the engine that holds the
        run (kmz_set_triples, kmz_partials_copy), so the engine no longer holds
        the unfiltered run.  Results already taken from the run (rows,
        reduced(), toReduced(): host copies) are unaffected; a later call that
        needs the device state -- another result's service_tail(), this one
        unfiltered included -- sees the moved ``gen`` and runs the batch's
        dependency pass again first (correct, at the cost of one pass).  Only
        the stale endpoints' first-row half is cleared: the tail reads rows
        (has_row, first row) and never a last-usage timestamp."""
        from .tail import maps_from_dictionary, run_tail

        if self._native is None:
            raise ValueError("service_tail() needs an engine-backed result")
        nat = self._native
        eng = nat.eng
        if eng.gen != nat.gen:  # the engine ran something else since: this batch's dependency pass again
            eng = nat.traces._load()
            eng.run(L.RUN_DEPS)
        if self._cutoff != 0:
            # DEPRECATED_ENDPOINT_THRESHOLD set: the tail of the constructor-
            # filtered graph (EndpointDependencies.ts:44-74).  The filtered edge
            # keys replace the run's edge set (kmz_set_triples) and the stale
            # endpoints lose their rows (first-row partial -> none), so the
            # kernels see exactly the kept rows; the engine no longer holds this
            # run afterwards (its gen moved: a later call runs the pass again).
            keys, eps = self.reduced()
            stale = (nat.endpoints["has_row"] != 0) & (eps["has_row"] == 0)
            if stale.any() or len(keys) != len(nat.triples):
                ew = eng.partials_words(L.PART_ENDPOINTS)
                part = np.zeros(max(1, ew), np.uint64)
                eng.export_partials(L.PART_ENDPOINTS, part.ctypes.data, ew, False)
                n_ep = ew // 2
                part[n_ep:][np.nonzero(stale[:n_ep])[0]] = np.uint64(L.NONE64)  # [min first row] half
                eng.import_partials(L.PART_ENDPOINTS, part.ctypes.data, ew, False)
                kh = np.ascontiguousarray(keys, dtype=np.uint64)
                eng.set_triples(kh.ctypes.data, len(kh), False)
        return run_tail(eng, maps_from_dictionary(nat.dict, labelMap), eng.endpoints())

    def toReduced(self, reg=None):
        """Columns of ``EndpointDependencies([]).combineWith(self).trim()``
        (cache.ReducedDependencies, the form the dependency cache keeps)."""
        from .cache import ReducedDependencies

        if self._native is not None and self._deps is None:
            return self._native.reduced_graph(reg).filtered(self._cutoff)
        return ReducedDependencies.from_json(self._list(), merge_rows=True, reg=reg)

    def trim(self):
        """EndpointDependencies.ts:91-112."""
        out = []
        for d in self._list():
            on = {f"{x['distance']}\t{x['endpoint']['uniqueEndpointName']}": x for x in d["dependingOn"]}
            by = {f"{x['distance']}\t{x['endpoint']['uniqueEndpointName']}": x for x in d["dependingBy"]}
            out.append({**d, "dependingBy": list(by.values()), "dependingOn": list(on.values())})
        return EndpointDependencies(out)

    def label(self, labelMap: Optional[Dict[str, str]] = None):
        """EndpointDependencies.ts:114-153; DataCache's LabelMapping is passed
        explicitly (``uniqueEndpointName -> label``)."""

        def lab(ep):
            v = labelMap.get(ep["uniqueEndpointName"]) if labelMap else None
            return _clean({**ep, "labelName": v if v is not None else UNDEFINED})

        return [
            {
                "endpoint": lab(d["endpoint"]),
                "isDependedByExternal": d["isDependedByExternal"],
                "lastUsageTimestamp": d["lastUsageTimestamp"],
                "dependingOn": [{**x, "endpoint": lab(x["endpoint"])} for x in d["dependingOn"]],
                "dependingBy": [{**x, "endpoint": lab(x["endpoint"])} for x in d["dependingBy"]],
            }
            for d in self._list()
        ]

    def combineWith(self, endpointDependencies: "EndpointDependencies") -> "EndpointDependencies":
        """EndpointDependencies.ts:499-542 (mutates the incoming rows as the TS does)."""

        def keyset(lst):
            return {f"{x['endpoint']['uniqueEndpointName']}\t{x['distance']}" for x in lst}

        acc: Dict[str, list] = {}
        for d in self._list():
            acc[d["endpoint"]["uniqueEndpointName"]] = [d, keyset(d["dependingBy"]), keyset(d["dependingOn"])]
        for d in endpointDependencies._list():
            name = d["endpoint"]["uniqueEndpointName"]
            slot = acc.get(name)
            if slot is None:
                acc[name] = [d, keyset(d["dependingBy"]), keyset(d["dependingOn"])]
                continue
            row, by, on = slot
            d["lastUsageTimestamp"] = max(d["lastUsageTimestamp"], row["lastUsageTimestamp"])
            for side, seen in (("dependingBy", by), ("dependingOn", on)):
                for x in d[side]:
                    k = f"{x['endpoint']['uniqueEndpointName']}\t{x['distance']}"
                    if k not in seen:
                        row[side].append(x)
                        seen.add(k)
        return EndpointDependencies([v[0] for v in acc.values()])

    # -- service-level tail (a8) ------------------------------------------------
    def toServiceDependencies(self):
        """EndpointDependencies.ts:369-470."""
        deps = self._list()
        by_service: Dict[str, List[dict]] = {}
        for d in deps:
            by_service.setdefault(d["endpoint"]["uniqueServiceName"], []).append(d)
        out = []
        for usn, rows in by_service.items():
            links = _service_links(rows)
            s, n, v = (usn.split("\t") + [UNDEFINED] * 3)[:3]
            out.append(
                {
                    "service": s,
                    "namespace": n,
                    "version": v,
                    "dependency": rows,
                    "links": [
                        {
                            **dict(zip(("service", "namespace", "version"), (lk.split("\t") + [UNDEFINED] * 3)[:3])),
                            **info,
                            "uniqueServiceName": lk,
                        }
                        for lk, info in links.items()
                    ],
                    "uniqueServiceName": usn,
                }
            )
        return out

    def toChordData(self):
        """EndpointDependencies.ts:472-497."""

        def nid(usn):
            s, n, v = (usn.split("\t") + ["undefined"] * 3)[:3]
            return f"{s}.{n} ({v})"

        links = [
            {"from": s["uniqueServiceName"], "to": l["uniqueServiceName"], "value": l["dependingOn"]}
            for s in self.toServiceDependencies()
            for l in s["links"]
            if l["dependingOn"] > 0
        ]
        nodes = list(dict.fromkeys(x for l in links for x in (l["from"], l["to"])))
        return {
            "nodes": [{"id": nid(x), "name": x} for x in nodes],
            "links": [{**l, "from": nid(l["from"]), "to": nid(l["to"])} for l in links],
        }

    def toServiceEndpointCohesion(self):
        """EndpointDependencies.ts:565-612."""
        by_service: Dict[str, List[dict]] = {}
        for d in self._list():
            by_service.setdefault(d["endpoint"]["uniqueServiceName"], []).append(d)
        out = []
        for usn, eps in by_service.items():
            used: Dict[str, Dict[str, None]] = {}
            for e in eps:
                for x in e["dependingBy"]:
                    if x["distance"] == 1:
                        used.setdefault(x["endpoint"]["uniqueServiceName"], {})[e["endpoint"]["uniqueEndpointName"]] = None
            consumers = [{"uniqueServiceName": k, "consumes": len(v)} for k, v in used.items()]
            coh = 0
            if eps and consumers:
                acc = 0
                for c in consumers:
                    acc = acc + c["consumes"] / len(eps)
                coh = acc / len(consumers)
            out.append(
                {"uniqueServiceName": usn, "totalEndpoints": len(eps), "consumers": consumers, "endpointUsageCohesion": coh}
            )
        return out

    def toServiceInstability(self):
        """EndpointDependencies.ts:614-641."""
        out = []
        for s in self.toServiceDependencies():
            by = sum(1 for l in s["links"] if l["dependingBy"] > 0)
            on = sum(1 for l in s["links"] if l["dependingOn"] > 0)
            out.append(
                {
                    "uniqueServiceName": s["uniqueServiceName"],
                    "name": f"{tpl(s['service'])}.{tpl(s['namespace'])} ({tpl(s['version'])})",
                    "dependingBy": by,
                    "dependingOn": on,
                    "instability": 0 if on + by == 0 else on / (on + by),
                }
            )
        return out

    def toServiceCoupling(self):
        """EndpointDependencies.ts:643-657 via RiskAnalyzer.AbsoluteCriticalityOfServices."""
        from .risk import absolute_criticality

        out = []
        for c in absolute_criticality(self.toServiceDependencies()):
            s, n, v = (c["uniqueServiceName"].split("\t") + ["undefined"] * 3)[:3]
            out.append(
                {
                    "uniqueServiceName": c["uniqueServiceName"],
                    "name": f"{s}.{n} ({v})",
                    "ais": c["ais"],
                    "ads": c["ads"],
                    "acs": c["factor"],
                }
            )
        return out

    def toGraphData(self):
        """EndpointDependencies.ts:157-265: base nodes and links (all Active:
        INACTIVE_ENDPOINT_THRESHOLD unset)."""
        by_service: Dict[str, List[dict]] = {}
        for d in self._list():
            by_service.setdefault(f"{tpl(d['endpoint'].get('service', UNDEFINED))}\t"
                                  f"{tpl(d['endpoint'].get('namespace', UNDEFINED))}", []).append(d)
        nodes = [{"id": "null", "group": "null", "name": "external requests", "usageStatus": "Active"}]
        links, have_node, have_link = [], set(), set()

        def nid(ep):
            return f"{ep['uniqueServiceName']}\t{tpl(ep.get('method', UNDEFINED))}\t{tpl(ep.get('labelName', UNDEFINED))}"

        def link(a, b):
            if f"{a}\t{b}" not in have_link:
                have_link.add(f"{a}\t{b}")
                links.append({"source": a, "target": b})

        for svc, eps in by_service.items():
            nodes.append({"id": svc, "group": svc, "name": svc.replace("\t", ".", 1), "usageStatus": "Active"})
            for e in eps:
                i = nid(e["endpoint"])
                if i not in have_node:
                    have_node.add(i)
                    nodes.append({"id": i, "group": svc, "usageStatus": "Active"})
                link(svc, i)
                for x in e["dependingOn"]:
                    if x["distance"] == 1:
                        link(i, nid(x["endpoint"]))
                if e["isDependedByExternal"]:
                    link("null", i)
        return {"nodes": nodes, "links": links}


def _service_links(rows: List[dict]) -> Dict[str, dict]:
    """EndpointDependencies.ts:412-470: distinct (service, method, label, type,
    distance) link keys, counted per linked service and distance."""
    keys: Dict[tuple, None] = {}
    for d in rows:
        for x in list(d["dependingOn"]) + list(d["dependingBy"]):
            ep = x["endpoint"]
            keys[(ep["uniqueServiceName"], tpl(ep.get("method", UNDEFINED)), tpl(ep.get("labelName", UNDEFINED)),
                  x["type"], x["distance"])] = None
    detail: Dict[str, Dict[int, dict]] = {}
    for usn, _, _, typ, dist in keys:
        # the key is re-split on tabs in the TS: a usn keeps its first 3 fields
        usn3 = "\t".join(usn.split("\t")[:3])
        slot = detail.setdefault(usn3, {}).setdefault(
            dist, {"count": 0, "dependingBy": 0, "dependingOn": 0, "distance": dist}
        )
        slot["count"] += 1
        slot["dependingBy"] += typ == "CLIENT"
        slot["dependingOn"] += typ == "SERVER"
    out = {}
    for usn, dm in detail.items():
        det = list(dm.values())
        out[usn] = {
            "details": det,
            "count": sum(x["count"] for x in det),
            "dependingBy": sum(x["dependingBy"] for x in det),
            "dependingOn": sum(x["dependingOn"] for x in det),
        }
    return out
