"""CPU ORACLE (test infrastructure only) -- pure-Python restatement of the
KMamiz trace-processing hot path with JavaScript semantics.

THIS IS NOT PRODUCT CODE.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker.

It restates, line for line in behaviour (not in code), the reference's
TypeScript on V8 builtins:

* ``src/utils/Utils.ts:83-106``    ExplodeUrl          -> explode_url
* ``src/utils/Utils.ts:311-313``   ToPrecise           -> to_precise
* ``src/classes/Traces.ts:27-241`` Traces              -> Traces
* ``src/classes/RealtimeDataList.ts:22-118``           -> RealtimeDataList
* ``src/classes/CombinedRealtimeDataList.ts:183-332``  -> CombinedRealtimeDataList
* ``src/classes/EndpointDependencies.ts:40-657``       -> EndpointDependencies
* ``src/utils/RiskAnalyzer.ts:10-248``                 -> RiskAnalyzer
* ``src/utils/Normalizer.ts:17-70``                    -> Normalizer
* ``src/classes/EnvoyLog.ts:7-149``, ``services/KubernetesService.ts:201-242``
                                                       -> EnvoyLogs, parse_envoy_logs
* ``src/utils/Utils.ts:14-75, 279-309`` (Merge, MergeStringBody,
  ObjectToInterfaceString without json-to-ts)          -> js_merge, merge_string_body,
                                                          object_to_interface_string

JS semantics reproduced:
* ``Map``/``Set`` keep the position of the first insertion and the value of the
  last ``set`` -- Python ``dict`` does exactly the same.
* ``undefined`` is the sentinel ``UNDEF``; it renders as ``"undefined"`` inside
  template strings and properties holding it are dropped by ``strip_undef``
  (Jest ``toEqual`` ignores them).
* ``Math.round`` rounds half toward +inf (``js_round``); all arithmetic is IEEE
  fp64 (CPython floats) with no contraction.
* JS regex ``.`` does not match line terminators.

Parity pinning: every known answer in the reference's jest suite for this
path is checked in ``tests/test_oracle_goldens.py``.

``String.prototype.localeCompare`` (used by ``RiskAnalyzer.Impact``,
``RiskAnalyzer.ts:57-60``) is restated as a three-level ICU-root key whose
tables come from the reference's own Node (tests/golden/locale_order.json);
it is pinned on that file's corpus (ASCII names, tabs, punctuation, case,
decomposable Latin accents).  Letters without a canonical decomposition
outside ASCII remain unpinned.
"""
from __future__ import annotations

import json
import math
import re
import time
from typing import Any, Dict, List, Optional


class _Undefined:
    __slots__ = ()

    def __repr__(self):
        return "undefined"

    def __bool__(self):
        return False


UNDEF = _Undefined()
EPSILON = 2.0 ** -52

# JS '.' == any char except line terminators
_DOT = "[^\n\r  ]"
_RE_SCHEME = re.compile(r"[a-z]+://")
_RE_URL = re.compile(r"://([^:/]*)([:0-9]*)(" + _DOT + r"*)")
_RE_SVC = re.compile(r"(" + _DOT + r"*)" + _DOT + r"svc[\.]*(" + _DOT + r"*)")


def js_str(v) -> str:
    """String conversion as done by a JS template literal."""
    if v is UNDEF:
        return "undefined"
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        if v == int(v) and abs(v) < 1e21:
            return str(int(v))
        return repr(v)
    return str(v)


def get(obj: dict, key: str):
    """Property read: missing -> undefined."""
    v = obj.get(key, UNDEF) if isinstance(obj, dict) else UNDEF
    return v


def truthy(v) -> bool:
    if v is UNDEF or v is None:
        return False
    if isinstance(v, float) and math.isnan(v):
        return False
    if isinstance(v, (dict, list)):
        return True  # every object is truthy in JS, {} and [] included
    return bool(v)


def js_round(x: float) -> float:
    """Math.round: nearest integer, ties toward +infinity (ECMA-262 21.3.2.28)."""
    if not math.isfinite(x):
        return x
    r = math.floor(x)
    if x - r >= 0.5:
        r += 1
    return float(r)


def belongs_to_minute(ts_ms: float) -> int:
    """Utils.BelongsToMinuteTimestamp (Utils.ts:135-141): new Date(ts) truncates
    the time value toward zero; the ISO string then names its UTC minute."""
    ms = math.trunc(ts_ms)
    return (ms // 60000) * 60000


def iso_minute(ms: int) -> str:
    """Date.prototype.toISOString of a whole-minute time value."""
    import datetime

    d = datetime.datetime(1970, 1, 1) + datetime.timedelta(milliseconds=ms)
    return d.strftime("%Y-%m-%dT%H:%M:%S.") + f"{ms % 1000:03d}Z"


def to_precise(num: float) -> float:
    """Utils.ToPrecise (Utils.ts:311-313)."""
    return js_round((num + EPSILON) * 1e14) / 1e14


def strip_undef(v):
    """Drop properties whose value is undefined (what Jest toEqual ignores)."""
    if isinstance(v, dict):
        return {k: strip_undef(x) for k, x in v.items() if x is not UNDEF}
    if isinstance(v, list):
        return [strip_undef(x) for x in v]
    return v


def js_max(values, start=None):
    """Math.max(...values) with -Infinity for the empty list."""
    m = -math.inf if start is None else start
    for v in values:
        if isinstance(v, float) and math.isnan(v):
            return math.nan
        if v > m:
            m = v
    return m


def js_min(values):
    m = math.inf
    for v in values:
        if isinstance(v, float) and math.isnan(v):
            return math.nan
        if v < m:
            m = v
    return m


# --------------------------------------------------------------------------
# Utils.ExplodeUrl  (src/utils/Utils.ts:83-106)
# --------------------------------------------------------------------------
def explode_url(url, is_service_url: bool = False) -> list:
    if not isinstance(url, str):
        # url.search on undefined -> TypeError (Utils.ts:84)
        raise TypeError("Cannot read property 'search' of undefined")
    if _RE_SCHEME.search(url) is None:
        url = "://" + url
    m = _RE_URL.search(url)
    if m:
        host, port, path = m.group(1), m.group(2), m.group(3)
    else:
        host = port = path = UNDEF
    out = [host, port, path]
    if is_service_url:
        if host is UNDEF:
            # host.match on undefined -> TypeError (Utils.ts:90)
            raise TypeError("Cannot read property 'match' of undefined")
        sm = _RE_SVC.search(host)
        full = sm.group(1) if sm else UNDEF
        cluster = sm.group(2) if sm else UNDEF
        if truthy(full):
            div = full.rfind(".")
            service = full[:div] if div >= 0 else full[:-1]
            namespace = full[div + 1 :]
            out += [service, namespace, cluster if truthy(cluster) else "cluster.local"]
    return out


def _at(arr: list, i: int):
    return arr[i] if i < len(arr) else UNDEF


# --------------------------------------------------------------------------
# Traces  (src/classes/Traces.ts)
# --------------------------------------------------------------------------
class Traces:
    def __init__(self, traces: List[List[dict]]):
        self._traces = traces

    def toJSON(self):
        return self._traces

    def _flat(self):
        for t in self._traces:
            for s in t:
                yield s

    @staticmethod
    def _find_replica(replicas, usn):
        # replicas?.find(r => r.uniqueServiceName === usn)?.replicas (Traces.ts:47-49)
        if replicas is None or replicas is UNDEF:
            return UNDEF
        for r in replicas:
            if get(r, "uniqueServiceName") == usn:
                return get(r, "replicas")
        return UNDEF

    def toRealTimeData(self, replicas=None):
        """Traces.ts:27-53."""
        out = []
        for t in self._flat():
            if get(t, "kind") != "SERVER":
                continue
            ex = explode_url(t["name"], True)
            service, namespace = _at(ex, 3), _at(ex, 4)
            tags = t.get("tags", {})
            version = get(tags, "istio.canonical_revision")
            method = get(tags, "http.method")
            usn = f"{js_str(service)}\t{js_str(namespace)}\t{js_str(version)}"
            out.append(
                {
                    "timestamp": t["timestamp"],
                    "service": service,
                    "namespace": namespace,
                    "version": version,
                    "method": method,
                    "latency": t["duration"] / 1000,
                    "status": get(tags, "http.status_code"),
                    "uniqueServiceName": usn,
                    "uniqueEndpointName": f"{usn}\t{js_str(method)}\t{js_str(get(tags, 'http.url'))}",
                    "replica": self._find_replica(replicas, usn),
                }
            )
        return RealtimeDataList(out)

    def combineLogsToRealtimeData(self, structuredLogs=(), replicas=None):
        """Traces.ts:55-106."""
        log_map: Dict[str, Dict[str, dict]] = {}
        for l in structuredLogs:
            trs = l.get("traces", [])
            if len(trs) == 0:
                continue
            trace_id = trs[0]["traceId"]
            if trace_id not in log_map:
                log_map[trace_id] = {}
            for t in trs:
                log_map[trace_id][t["spanId"]] = t
        out = []
        for tr in self._flat():
            if get(tr, "kind") != "SERVER":
                continue
            tags = tr.get("tags", {})
            service = get(tags, "istio.canonical_service")
            namespace = get(tags, "istio.namespace")
            version = get(tags, "istio.canonical_revision")
            method = get(tags, "http.method")
            status = get(tags, "http.status_code")
            usn = f"{js_str(service)}\t{js_str(namespace)}\t{js_str(version)}"
            lm = log_map.get(get(tr, "traceId"))
            log = lm.get(get(tr, "id"), UNDEF) if lm is not None else UNDEF
            if (not truthy(log) or truthy(get(log, "isFallback"))) and truthy(get(tr, "parentId")):
                log = lm.get(tr["parentId"], UNDEF) if lm is not None else UNDEF
            req = get(log, "request") if truthy(log) else UNDEF
            res = get(log, "response") if truthy(log) else UNDEF
            if truthy(log) and (res is UNDEF or res is None or req is UNDEF or req is None):
                # `log?.response.body` (Traces.ts:94-97): a log without request /
                # response throws a TypeError in the reference
                raise TypeError("Cannot read properties of undefined (reading 'body')")
            out.append(
                {
                    "timestamp": tr["timestamp"],
                    "service": service,
                    "namespace": namespace,
                    "version": version,
                    "method": method,
                    "latency": tr["duration"] / 1000,
                    "status": status,
                    "responseBody": get(res, "body") if truthy(res) else UNDEF,
                    "responseContentType": get(res, "contentType") if truthy(res) else UNDEF,
                    "requestBody": get(req, "body") if truthy(req) else UNDEF,
                    "requestContentType": get(req, "contentType") if truthy(req) else UNDEF,
                    "uniqueServiceName": usn,
                    "uniqueEndpointName": f"{usn}\t{js_str(get(tags, 'http.method'))}\t{js_str(get(tags, 'http.url'))}",
                    "replica": self._find_replica(replicas, usn),
                }
            )
        return RealtimeDataList(out)

    def extractContainingNamespaces(self):
        """Traces.ts:108-110."""
        return list(dict.fromkeys(get(t.get("tags", {}), "istio.namespace") for t in self._flat()))

    def toEndpointDependencies(self, max_depth: Optional[int] = None):
        """Traces.ts:112-211.

        ``max_depth`` only exists to turn the reference's endless loop on a
        cyclic parent chain into an exception.
        """
        span_map: Dict[Any, dict] = {}
        for span in self._flat():
            span_map[get(span, "id")] = {"span": span, "upper": {}, "lower": {}}
        filtered = [(sid, node) for sid, node in span_map.items() if get(node["span"], "kind") == "SERVER"]
        for span_id, node in filtered:
            span, upper = node["span"], node["upper"]
            parent_id = get(span, "parentId")
            depth = 1
            steps = 0
            while truthy(parent_id):
                steps += 1
                if max_depth is not None and steps > max_depth:
                    raise RuntimeError("cyclic parent chain")
                pnode = span_map.get(parent_id)
                if pnode is None:
                    break
                if get(pnode["span"], "kind") == "CLIENT":
                    parent_id = get(pnode["span"], "parentId")
                    continue
                upper[get(pnode["span"], "id")] = depth
                pnode["lower"][span_id] = depth
                parent_id = get(pnode["span"], "parentId")
                depth += 1

        deps = []
        for _, node in filtered:
            upper_map: Dict[str, dict] = {}
            for s, distance in node["upper"].items():
                ep = Traces.ToEndpointInfo(span_map[s]["span"])
                upper_map[f"{ep['uniqueEndpointName']}\t{js_str(distance)}"] = ep
            lower_map: Dict[str, dict] = {}
            for s, distance in node["lower"].items():
                ep = Traces.ToEndpointInfo(span_map[s]["span"])
                lower_map[f"{ep['uniqueEndpointName']}\t{js_str(distance)}"] = ep
            depending_by = [
                {"endpoint": ep, "distance": int(k.split("\t")[-1]), "type": "CLIENT"} for k, ep in upper_map.items()
            ]
            depending_on = [
                {"endpoint": ep, "distance": int(k.split("\t")[-1]), "type": "SERVER"} for k, ep in lower_map.items()
            ]
            deps.append(
                {
                    "endpoint": Traces.ToEndpointInfo(node["span"]),
                    "lastUsageTimestamp": 0,
                    "isDependedByExternal": len(depending_by) == 0,
                    "dependingBy": depending_by,
                    "dependingOn": depending_on,
                }
            )
        last_ts: Dict[str, float] = {}

        def upd(ep):
            name = ep["uniqueEndpointName"]
            last_ts[name] = js_max([ep["timestamp"]], start=last_ts.get(name, 0))

        for d in deps:
            upd(d["endpoint"])
            for x in d["dependingBy"]:
                upd(x["endpoint"])
            for x in d["dependingOn"]:
                upd(x["endpoint"])
        for d in deps:
            d["lastUsageTimestamp"] = last_ts.get(d["endpoint"]["uniqueEndpointName"], 0)
        return EndpointDependencies(deps)

    @staticmethod
    def ToEndpointInfo(trace: dict) -> dict:
        """Traces.ts:213-241."""
        tags = trace.get("tags", {})
        ex = explode_url(get(tags, "http.url"))
        host, port, path = ex[0], ex[1], ex[2]
        exs = explode_url(trace["name"], True)
        service, namespace, cluster = _at(exs, 3), _at(exs, 4), _at(exs, 5)
        if ".svc." not in trace["name"]:
            service = get(tags, "istio.canonical_service")
            namespace = get(tags, "istio.namespace")
            cluster = get(tags, "istio.mesh_id")
        rev = get(tags, "istio.canonical_revision")
        version = rev if truthy(rev) else "NONE"
        usn = f"{js_str(service)}\t{js_str(namespace)}\t{js_str(version)}"
        return {
            "version": version,
            "service": service,
            "namespace": namespace,
            "url": get(tags, "http.url"),
            "host": host,
            "path": path,
            "port": port if truthy(port) else "80",
            "clusterName": cluster,
            "method": get(tags, "http.method"),
            "uniqueServiceName": usn,
            "uniqueEndpointName": f"{usn}\t{js_str(get(tags, 'http.method'))}\t{js_str(get(tags, 'http.url'))}",
            "timestamp": trace["timestamp"] / 1000,
        }


# --------------------------------------------------------------------------
# RealtimeDataList  (src/classes/RealtimeDataList.ts)
# --------------------------------------------------------------------------
def welford_mean_cv(latencies: List[float]):
    """RealtimeDataList.ts:100-118 (sequential, fp64, no contraction)."""
    if len(latencies) == 0:
        return 0.0, 0.0
    mean = 0.0
    m2 = 0.0
    for i, x in enumerate(latencies):
        old = mean
        mean += (x - mean) / (i + 1)
        m2 += (x - mean) * (x - old)
    variance = m2 / len(latencies)
    std = math.sqrt(variance)
    cv = std / mean if mean != 0 else 0
    return mean, cv


class RealtimeDataList:
    def __init__(self, realtime_data: List[dict]):
        self._realtime_data = realtime_data

    def toJSON(self):
        return self._realtime_data

    def getContainingNamespaces(self):
        return list(dict.fromkeys(get(r, "namespace") for r in self._realtime_data))

    def toCombinedRealtimeData(self):
        """RealtimeDataList.ts:22-97 (trace-only subset: request/response
        bodies are carried through ``MergeStringBody``-free, schemas are out of
        scope -- SURVEY.md 8f item 3)."""
        by_name: Dict[str, List[dict]] = {}
        for r in self._realtime_data:
            by_name.setdefault(r["uniqueEndpointName"], []).append(r)
        combined = []
        for group in by_name.values():
            status_map: Dict[Any, List[dict]] = {}
            for r in group:
                status_map.setdefault(get(r, "status"), []).append(r)
            sample = group[0]
            base = {
                "uniqueServiceName": get(sample, "uniqueServiceName"),
                "uniqueEndpointName": get(sample, "uniqueEndpointName"),
                "service": get(sample, "service"),
                "namespace": get(sample, "namespace"),
                "version": get(sample, "version"),
                "method": get(sample, "method"),
            }
            for status, sub in status_map.items():
                mean, cv = welford_mean_cv([r["latency"] for r in sub])
                # reduce without an initial value, {...prev} spread (53-67)
                acc = dict(sub[0])
                for cur in sub[1:]:
                    acc = dict(acc)
                    acc["requestBody"] = merge_string_body(get(acc, "requestBody"), get(cur, "requestBody"))
                    acc["responseBody"] = merge_string_body(get(acc, "responseBody"), get(cur, "responseBody"))
                    acc["timestamp"] = acc["timestamp"] if acc["timestamp"] > cur["timestamp"] else cur["timestamp"]
                    ar, cr = get(acc, "replica"), get(cur, "replica")
                    if truthy(ar) and truthy(cr):
                        acc["replica"] = ar + cr
                bodies = parse_bodies(acc)
                rep = get(acc, "replica")
                combined.append(
                    {
                        **base,
                        "status": status,
                        "combined": len(sub),
                        "avgReplica": rep / len(sub) if truthy(rep) else UNDEF,
                        "latestTimestamp": acc["timestamp"],
                        "latency": {"mean": to_precise(mean), "cv": to_precise(cv)},
                        "requestContentType": get(acc, "requestContentType"),
                        "responseContentType": get(acc, "responseContentType"),
                        **bodies,
                    }
                )
        return CombinedRealtimeDataList(combined)


# --------------------------------------------------------------------------
# CombinedRealtimeDataList  (src/classes/CombinedRealtimeDataList.ts)
# --------------------------------------------------------------------------
def _scale_shift(mean1: float, mean2: float) -> int:
    """CombinedRealtimeDataList.ts:322-332."""

    def safe_log10(x):
        if x <= 0:
            return 0
        return math.floor(math.log10(x))

    return math.floor((safe_log10(mean1) + safe_log10(mean2)) / 2)


def combine_latency_cv_and_mean(n1, mean1, cv1, n2, mean2, cv2):
    """CombinedRealtimeDataList.ts:278-315."""
    shift = _scale_shift(mean1, mean2)
    scale = math.pow(10, shift)
    mean1s = mean1 / scale
    mean2s = mean2 / scale
    std1s = cv1 * mean1s
    std2s = cv2 * mean2s
    total = n1 + n2
    mean_total = (n1 * mean1s + n2 * mean2s) / total
    # JS `x ** 2` is Math.pow(x, 2), whose fdlibm core returns x * x for y == 2
    # (V8 base/ieee754 pow); C pow(x, 2.0) is only within 0.52 ulp of it
    var1 = std1s * std1s
    var2 = std2s * std2s
    d1 = mean1s - mean_total
    d2 = mean2s - mean_total
    pooled = (n1 * var1 + n2 * var2 + n1 * (d1 * d1) + n2 * (d2 * d2)) / total
    std_total = math.sqrt(pooled)
    cv_total = 0 if mean_total == 0 else std_total / mean_total
    return mean_total * scale, cv_total


class CombinedRealtimeDataList:
    def __init__(self, data: List[dict]):
        self._data = data

    def toJSON(self):
        return self._data

    def getContainingNamespaces(self):
        return list(dict.fromkeys(get(r, "namespace") for r in self._data))

    def adjustTimestamp(self, to):
        return CombinedRealtimeDataList([{**r, "latestTimestamp": to * 1000} for r in self._data])

    def toHistoricalData(self, serviceDependencies, replicas=None, labelMap=None):
        """CombinedRealtimeDataList.ts:26-150: rows bucketed by the minute of their
        latestTimestamp (Utils.BelongsToMinuteTimestamp, Utils.ts:135-141), then
        per minute the endpoint and service summaries and RiskAnalyzer.RealtimeRisk.
        Dates are given as the ISO strings their JSON form has."""
        replicas = replicas or []
        dates: Dict[int, List[dict]] = {}
        for r in self._data:
            dates.setdefault(belongs_to_minute(r["latestTimestamp"] / 1000), []).append(r)
        out = []
        for time, daily in dates.items():
            risks = RiskAnalyzer.RealtimeRisk(daily, serviceDependencies, replicas)
            emap: Dict[str, List[dict]] = {}
            smap: Dict[str, List[dict]] = {}
            for r in daily:
                emap.setdefault(r["uniqueEndpointName"], []).append(r)
                smap.setdefault(r["uniqueServiceName"], []).append(r)
            eps = []
            for uen, rows in emap.items():
                tok = uen.split("\t")
                req = rerr = serr = 0
                for c in rows:
                    req += c["combined"]
                    if str(c["status"]).startswith("4"):
                        rerr += c["combined"]
                    if str(c["status"]).startswith("5"):
                        serr += c["combined"]
                valid = [c for c in rows if get(c["latency"], "mean") is not UNDEF and c["latency"].get("mean") is not None]
                tot = 0.0
                for c in valid:
                    tot = tot + c["latency"]["mean"]
                mean = tot / len(valid) if valid else math.nan
                e = {
                    "latencyMean": mean if math.isfinite(mean) else 0,
                    "latencyCV": max((c["latency"].get("cv") or 0) for c in rows),
                    "method": tok[3] if len(tok) > 3 else UNDEF,
                    "requestErrors": rerr,
                    "requests": req,
                    "serverErrors": serr,
                    "uniqueEndpointName": uen,
                    "uniqueServiceName": "\t".join(tok[:3]) if len(tok) >= 3 else UNDEF,
                }
                if labelMap is not None and uen in labelMap:
                    e["labelName"] = labelMap[uen]
                eps.append(strip_undef(e))
            svcs = []
            for usn, rows in smap.items():
                tok = usn.split("\t")
                mine = [e for e in eps if e.get("uniqueServiceName") == usn]
                req = rerr = serr = 0
                for e in mine:
                    rerr += e["requestErrors"]
                    serr += e["serverErrors"]
                    req += e["requests"]
                valid = [c for c in rows if isinstance(c["latency"].get("mean"), (int, float))
                         and math.isfinite(c["latency"]["mean"])]
                tot = 0.0
                for c in valid:
                    tot = tot + c["latency"]["mean"]
                mean = tot / len(valid) if valid else math.nan
                risk = next(x for x in risks if x["uniqueServiceName"] == usn)
                svcs.append(strip_undef({
                    "date": iso_minute(time),
                    "endpoints": mine,
                    "service": tok[0],
                    "namespace": tok[1] if len(tok) > 1 else UNDEF,
                    "version": tok[2] if len(tok) > 2 else UNDEF,
                    "requests": req,
                    "requestErrors": rerr,
                    "serverErrors": serr,
                    "latencyMean": mean if math.isfinite(mean) else 0,
                    "latencyCV": max((c["latency"].get("cv") or 0) for c in rows),
                    "uniqueServiceName": usn,
                    "risk": risk.get("norm", UNDEF),
                }))
            out.append({"date": iso_minute(time), "services": svcs})
        return out

    def combineWith(self, other: "CombinedRealtimeDataList"):
        """CombinedRealtimeDataList.ts:183-263 (body/schema merge out of scope)."""
        groups: Dict[str, List[dict]] = {}
        for r in self._data + other._data:
            groups.setdefault(f"{r['uniqueEndpointName']}\t{js_str(get(r, 'status'))}", []).append(r)
        out = []
        for group in groups.values():
            sample = group[0]
            n = 0
            for c in group:
                n = n + c["combined"]
            prev = sample  # reduce without initial value mutates group[0]
            for cur in group[1:]:
                if truthy(get(prev, "avgReplica")) and truthy(get(cur, "avgReplica")):
                    prev["avgReplica"] = prev["avgReplica"] + cur["avgReplica"]
                prev["latestTimestamp"] = js_max([prev["latestTimestamp"], cur["latestTimestamp"]])
                prev["requestBody"] = js_merge(get(prev, "requestBody"), get(cur, "requestBody"))
                prev["responseBody"] = js_merge(get(prev, "responseBody"), get(cur, "responseBody"))
                if truthy(prev["requestBody"]):
                    prev["requestSchema"] = object_to_interface_string(prev["requestBody"])
                if truthy(prev["responseBody"]):
                    prev["responseSchema"] = object_to_interface_string(prev["responseBody"])
            acc = {"mean": 0.0, "cv": 0.0, "n": 0}
            for cur in group:
                m, c = combine_latency_cv_and_mean(
                    acc["n"], acc["mean"], acc["cv"], cur["combined"], cur["latency"]["mean"], cur["latency"]["cv"]
                )
                acc = {"mean": m, "cv": c, "n": acc["n"] + cur["combined"]}
            out.append(
                {
                    "uniqueEndpointName": sample["uniqueEndpointName"],
                    "uniqueServiceName": get(sample, "uniqueServiceName"),
                    "service": get(sample, "service"),
                    "namespace": get(sample, "namespace"),
                    "version": get(sample, "version"),
                    "method": get(sample, "method"),
                    "status": get(sample, "status"),
                    "combined": n,
                    "requestContentType": get(sample, "requestContentType"),
                    "responseContentType": get(sample, "responseContentType"),
                    "latestTimestamp": prev["latestTimestamp"],
                    "requestBody": get(prev, "requestBody"),
                    "requestSchema": get(prev, "requestSchema"),
                    "responseBody": get(prev, "responseBody"),
                    "responseSchema": get(prev, "responseSchema"),
                    "latency": {"mean": to_precise(acc["mean"]), "cv": to_precise(acc["cv"])},
                }
            )
        return CombinedRealtimeDataList(out)


# --------------------------------------------------------------------------
# EndpointDependencies  (src/classes/EndpointDependencies.ts)
# --------------------------------------------------------------------------
def parse_threshold_to_ms(s):
    r"""EndpointDependencies.parseThresholdToMilliseconds (EndpointDependencies.ts:20-31):
    /(?:(\d+)d)?(?:(\d+)h)?(?:(\d+)m)?/ with String.match (first match, which
    may be the empty one at index 0), parseInt base 10, JS number arithmetic."""
    if not s:
        return 0
    m = re.match(r"(?:([0-9]+)d)?(?:([0-9]+)h)?(?:([0-9]+)m)?", s)
    if m is None:
        return 0
    days = float(int(m.group(1))) if m.group(1) else 0.0
    hours = float(int(m.group(2))) if m.group(2) else 0.0
    minutes = float(int(m.group(3))) if m.group(3) else 0.0
    return ((days * 86400) + (hours * 3600) + (minutes * 60)) * 1000


# GlobalSettings.DeprecatedEndpointThreshold (GlobalSettings.ts:79), parsed
# into the class's static (EndpointDependencies.ts:33-36), and Date.now():
# unset / the wall clock unless a test pins them
DEPRECATED_THRESHOLD_MS = 0
DATE_NOW = None


def _date_now():
    return DATE_NOW() if DATE_NOW is not None else int(time.time() * 1000)


class EndpointDependencies:
    def __init__(self, deps: List[dict]):
        self._deps = self._filter_out_deprecated(deps)

    @staticmethod
    def _filter_out_deprecated(deps):
        """EndpointDependencies.ts:44-74 (mutates the kept rows' lists)."""
        now = _date_now()
        cut = 0 if DEPRECATED_THRESHOLD_MS == 0 else now - DEPRECATED_THRESHOLD_MS
        if cut == 0:
            return deps
        names = set()
        kept = []
        for dep in deps:
            if dep["lastUsageTimestamp"] < cut:
                names.add(dep["endpoint"]["uniqueEndpointName"])
            else:
                kept.append(dep)
        for dep in kept:
            dep["dependingBy"] = [x for x in dep["dependingBy"] if x["endpoint"]["uniqueEndpointName"] not in names]
            dep["dependingOn"] = [x for x in dep["dependingOn"] if x["endpoint"]["uniqueEndpointName"] not in names]
        return kept

    def toJSON(self):
        return self._deps

    def trim(self):
        """EndpointDependencies.ts:91-112."""
        out = []
        for d in self._deps:
            on: Dict[str, dict] = {}
            for x in d["dependingOn"]:
                on[f"{js_str(x['distance'])}\t{x['endpoint']['uniqueEndpointName']}"] = x
            by: Dict[str, dict] = {}
            for x in d["dependingBy"]:
                by[f"{js_str(x['distance'])}\t{x['endpoint']['uniqueEndpointName']}"] = x
            out.append({**d, "dependingBy": list(by.values()), "dependingOn": list(on.values())})
        return EndpointDependencies(out)

    def label(self, label_map: Optional[Dict[str, str]] = None):
        """EndpointDependencies.ts:114-153 with the DataCache lookup replaced by
        an explicit ``uniqueEndpointName -> label`` map (None -> undefined)."""

        def ep_name(u):
            return label_map.get(u, UNDEF) if label_map else UNDEF

        out = []
        for d in self._deps:
            out.append(
                {
                    "endpoint": {**d["endpoint"], "labelName": ep_name(d["endpoint"]["uniqueEndpointName"])},
                    "isDependedByExternal": d["isDependedByExternal"],
                    "lastUsageTimestamp": d["lastUsageTimestamp"],
                    "dependingOn": [
                        {**x, "endpoint": {**x["endpoint"], "labelName": ep_name(x["endpoint"]["uniqueEndpointName"])}}
                        for x in d["dependingOn"]
                    ],
                    "dependingBy": [
                        {**x, "endpoint": {**x["endpoint"], "labelName": ep_name(x["endpoint"]["uniqueEndpointName"])}}
                        for x in d["dependingBy"]
                    ],
                }
            )
        return out

    # ---- merge ------------------------------------------------------------
    @staticmethod
    def _map_obj(d):
        return {
            "endpoint": d,
            "by": {f"{x['endpoint']['uniqueEndpointName']}\t{js_str(x['distance'])}" for x in d["dependingBy"]},
            "on": {f"{x['endpoint']['uniqueEndpointName']}\t{js_str(x['distance'])}" for x in d["dependingOn"]},
        }

    def combineWith(self, other: "EndpointDependencies"):
        """EndpointDependencies.ts:499-542 (mutates rows exactly like the TS)."""
        m: Dict[str, dict] = {}
        for d in self._deps:
            m[d["endpoint"]["uniqueEndpointName"]] = self._map_obj(d)
        for d in other._deps:
            name = d["endpoint"]["uniqueEndpointName"]
            ex = m.get(name)
            if ex is not None:
                d["lastUsageTimestamp"] = js_max([d["lastUsageTimestamp"], ex["endpoint"]["lastUsageTimestamp"]])
                for dep in d["dependingBy"]:
                    k = f"{dep['endpoint']['uniqueEndpointName']}\t{js_str(dep['distance'])}"
                    if k not in ex["by"]:
                        ex["endpoint"]["dependingBy"].append(dep)
                        ex["by"].add(k)
                for dep in d["dependingOn"]:
                    k = f"{dep['endpoint']['uniqueEndpointName']}\t{js_str(dep['distance'])}"
                    if k not in ex["on"]:
                        ex["endpoint"]["dependingOn"].append(dep)
                        ex["on"].add(k)
            else:
                m[name] = self._map_obj(d)
        return EndpointDependencies([v["endpoint"] for v in m.values()])

    # ---- service level views -----------------------------------------------
    def toServiceDependencies(self):
        """EndpointDependencies.ts:369-410."""
        deps = self._deps
        templates = list(dict.fromkeys(d["endpoint"]["uniqueServiceName"] for d in deps))
        out = []
        for usn in templates:
            dependency = [d for d in deps if d["endpoint"]["uniqueServiceName"] == usn]
            link_map = self._service_links(dependency)
            service, namespace, version = (usn.split("\t") + [UNDEF] * 3)[:3]
            links = []
            for lusn, info in link_map.items():
                ls, ln, lv = (lusn.split("\t") + [UNDEF] * 3)[:3]
                links.append({"service": ls, "namespace": ln, "version": lv, **info, "uniqueServiceName": lusn})
            out.append(
                {
                    "service": service,
                    "namespace": namespace,
                    "version": version,
                    "dependency": dependency,
                    "links": links,
                    "uniqueServiceName": usn,
                }
            )
        return out

    @staticmethod
    def _service_links(dependency):
        """EndpointDependencies.ts:412-470."""
        link_set: Dict[str, None] = {}
        for dep in dependency:
            for x in list(dep["dependingOn"]) + list(dep["dependingBy"]):
                e = x["endpoint"]
                k = (
                    f"{e['uniqueServiceName']}\t{js_str(get(e, 'method'))}\t{js_str(get(e, 'labelName'))}"
                    f"\t{x['type']}\t{js_str(x['distance'])}"
                )
                link_set[k] = None
        detail: Dict[str, Dict[int, dict]] = {}
        for k in link_set:
            tok = k.split("\t")
            service, namespace, version, typ, dist_s = tok[0], tok[1], tok[2], tok[5], tok[6]
            usn = f"{service}\t{namespace}\t{version}"
            distance = int(dist_s)
            existing = detail.get(usn, {})
            ed = existing.get(distance, {"count": 0, "dependingBy": 0, "dependingOn": 0, "distance": distance})
            existing[distance] = {
                "count": ed["count"] + 1,
                "dependingBy": ed["dependingBy"] + (1 if typ == "CLIENT" else 0),
                "dependingOn": ed["dependingOn"] + (1 if typ == "SERVER" else 0),
                "distance": distance,
            }
            detail[usn] = existing
        link_map: Dict[str, dict] = {}
        for usn, dm in detail.items():
            details = list(dm.values())
            agg = {"count": 0, "dependingBy": 0, "dependingOn": 0}
            for c in details:
                agg["count"] += c["count"]
                agg["dependingBy"] += c["dependingBy"]
                agg["dependingOn"] += c["dependingOn"]
            link_map[usn] = {"details": details, **agg}
        return link_map

    def toChordData(self):
        """EndpointDependencies.ts:472-497."""

        def name_to_id(usn):
            s, n, v = (usn.split("\t") + ["undefined"] * 3)[:3]
            return f"{s}.{n} ({v})"

        links = []
        for s in self.toServiceDependencies():
            for l in s["links"]:
                links.append({"from": s["uniqueServiceName"], "to": l["uniqueServiceName"], "value": l["dependingOn"]})
        links = [l for l in links if l["value"] > 0]
        nodes: Dict[str, None] = {}
        for l in links:
            nodes[l["from"]] = None
            nodes[l["to"]] = None
        return {
            "nodes": [{"id": name_to_id(n), "name": n} for n in nodes],
            "links": [{**l, "from": name_to_id(l["from"]), "to": name_to_id(l["to"])} for l in links],
        }

    def toServiceEndpointCohesion(self):
        """EndpointDependencies.ts:565-612."""
        sm: Dict[str, List[dict]] = {}
        for d in self._deps:
            sm.setdefault(d["endpoint"]["uniqueServiceName"], []).append(d)
        out = []
        for usn, endpoints in sm.items():
            util: Dict[str, Dict[str, None]] = {}
            for e in endpoints:
                for dep in e["dependingBy"]:
                    if dep["distance"] != 1:
                        continue
                    util.setdefault(dep["endpoint"]["uniqueServiceName"], {})[e["endpoint"]["uniqueEndpointName"]] = None
            consumers = [{"uniqueServiceName": k, "consumes": len(v)} for k, v in util.items()]
            coh = 0
            if len(endpoints) > 0 and len(consumers) > 0:
                coh = 0
                for c in consumers:
                    coh = coh + c["consumes"] / len(endpoints)
                coh /= len(consumers)
            out.append(
                {
                    "uniqueServiceName": usn,
                    "totalEndpoints": len(endpoints),
                    "consumers": consumers,
                    "endpointUsageCohesion": coh,
                }
            )
        return out

    def toServiceInstability(self):
        """EndpointDependencies.ts:614-641."""
        out = []
        for s in self.toServiceDependencies():
            by = on = 0
            for l in s["links"]:
                if l["dependingBy"] > 0:
                    by += 1
                if l["dependingOn"] > 0:
                    on += 1
            inst = 0 if on + by == 0 else on / (on + by)
            out.append(
                {
                    "uniqueServiceName": s["uniqueServiceName"],
                    "name": f"{js_str(s['service'])}.{js_str(s['namespace'])} ({js_str(s['version'])})",
                    "dependingBy": by,
                    "dependingOn": on,
                    "instability": inst,
                }
            )
        return out

    def toServiceCoupling(self):
        """EndpointDependencies.ts:643-657."""
        out = []
        for c in RiskAnalyzer.AbsoluteCriticalityOfServices(self.toServiceDependencies()):
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
        """EndpointDependencies.ts:157-265 (base nodes and links; thresholds
        unset so every node is Active)."""
        sem: Dict[str, List[dict]] = {}
        for dep in self._deps:
            sem.setdefault(f"{js_str(dep['endpoint']['service'])}\t{js_str(dep['endpoint']['namespace'])}", []).append(dep)
        labels, link_set = set(), set()
        nodes = [{"id": "null", "group": "null", "name": "external requests", "usageStatus": "Active"}]
        links = []
        for service, eps in sem.items():
            nodes.append({"id": service, "group": service, "name": service.replace("\t", ".", 1), "usageStatus": "Active"})
            for e in eps:
                ep = e["endpoint"]
                nid = f"{ep['uniqueServiceName']}\t{js_str(get(ep, 'method'))}\t{js_str(get(ep, 'labelName'))}"
                if nid not in labels:
                    nodes.append({"id": nid, "group": service, "usageStatus": "Active"})
                    labels.add(nid)
                if f"{service}\t{nid}" not in link_set:
                    links.append({"source": service, "target": nid})
                    link_set.add(f"{service}\t{nid}")
                for dep in e["dependingOn"]:
                    if dep["distance"] != 1:
                        continue
                    de = dep["endpoint"]
                    did = f"{de['uniqueServiceName']}\t{js_str(get(de, 'method'))}\t{js_str(get(de, 'labelName'))}"
                    if f"{nid}\t{did}" not in link_set:
                        links.append({"source": nid, "target": did})
                        link_set.add(f"{nid}\t{did}")
                if e["isDependedByExternal"] and f"null\t{nid}" not in link_set:
                    links.append({"source": "null", "target": nid})
                    link_set.add(f"null\t{nid}")
        return {"nodes": nodes, "links": links}


# --------------------------------------------------------------------------
# Normalizer  (src/utils/Normalizer.ts)
# --------------------------------------------------------------------------
class Normalizer:
    @staticmethod
    def BetweenFixedNumber(inp):
        base, ratio = 0.1, 1 - 0.1
        mx, mn = js_max(inp), js_min(inp)
        if mx - mn == 0:
            return [0.1]  # Normalizer.ts:22 (a one-element list, reproduced)
        return [((v - mn) / (mx - mn)) * ratio + base for v in inp]

    @staticmethod
    def Sigmoid(inp):
        return [1 / (1 + math.exp(-v)) for v in inp]

    @staticmethod
    def SigmoidAdj(inp):
        z = 2 * math.log(3)
        return [to_precise(1 / (1 + math.exp(-z * (v - 1.5)))) for v in inp]

    @staticmethod
    def FixedRatio(inp):
        mx = js_max(inp)
        if mx == 0:
            return inp
        return [v / mx for v in inp]

    @staticmethod
    def Linear(inp, minimum=0.1):
        if minimum >= 1:
            return inp
        return [n * (1 - minimum) + minimum for n in Normalizer.FixedRatio(inp)]


def _locale_tables():
    """ICU root tables as the reference's Node reports them
    (tests/golden/locale_order.json, made by tests/golden/gen_locale_order.js):
    whitespace/punctuation primary order, ignorable controls, and the
    secondary order of the combining marks U+0300..U+036F."""
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "locale_order.json")
    d = json.load(open(path))
    ign = set(d["punct_ignorable"])
    punct = {c: i for i, c in enumerate(c for c in d["punct_sorted"] if c not in ign)}
    marks, r = {}, 0
    for i, m in enumerate(d["marks_sorted"]):
        if i and d["marks_signs"][i - 1] != 0:
            r += 1
        marks[m] = r
    return punct, ign, marks


_LOCALE = None


def _locale_key(s: str):
    """localeCompare (ICU root, en-US) as three levels: primary (whitespace <
    punctuation < digits < case-folded base letters; ignorable controls
    skipped), secondary (NFD combining marks per letter), tertiary (case)."""
    import unicodedata

    global _LOCALE
    if _LOCALE is None:
        _LOCALE = _locale_tables()
    punct, ign, marks = _LOCALE
    prim, sec, tert = [], [], []
    for ch in unicodedata.normalize("NFD", s):
        if ord(ch) in marks:
            if sec:
                sec[-1] = sec[-1] + (marks[ord(ch)],)
            continue
        if ch in ign:
            continue
        if ch in punct:
            prim.append((1, punct[ch]))
        elif ch.isdigit() and ch.isascii():
            prim.append((2, ch))
        elif ch.isalpha() and ch.isascii():
            prim.append((3, ch.lower()))
        else:
            prim.append((4, ord(ch)))
        sec.append(())
        tert.append(1 if ch.isupper() else 0)
    return (prim, sec, tert)


def _sort_locale(items, key):
    return sorted(items, key=lambda x: _locale_key(key(x)))


# --------------------------------------------------------------------------
# RiskAnalyzer  (src/utils/RiskAnalyzer.ts)
# --------------------------------------------------------------------------
class RiskAnalyzer:
    MINIMUM_PROB = 0.01

    @staticmethod
    def RealtimeRisk(data, dependencies, replicas):
        """RiskAnalyzer.ts:10-49."""
        impacts = RiskAnalyzer.Impact(dependencies, replicas)
        probs = RiskAnalyzer.Probability(data)
        risks = []
        for s in dict.fromkeys(d["uniqueServiceName"] for d in data):
            sn, ns, sv = (s.split("\t") + [UNDEF] * 3)[:3]
            imp = next((i["impact"] for i in impacts if i["uniqueServiceName"] == s), UNDEF)
            imp = imp if truthy(imp) else 0
            pr = next((p["probability"] for p in probs if p["uniqueServiceName"] == s), UNDEF)
            pr = pr if truthy(pr) else RiskAnalyzer.MINIMUM_PROB
            risks.append(
                {
                    "uniqueServiceName": s,
                    "service": sn,
                    "namespace": ns,
                    "version": sv,
                    "risk": imp * pr,
                    "impact": imp,
                    "probability": pr,
                }
            )
        norm = Normalizer.BetweenFixedNumber([r["risk"] for r in risks])
        return [{**r, "norm": norm[i] if i < len(norm) else UNDEF} for i, r in enumerate(risks)]

    @staticmethod
    def Impact(dependencies, replicas):
        """RiskAnalyzer.ts:51-85 (localeCompare sort vs code-unit sort kept)."""
        rf = RiskAnalyzer.RelyingFactor(dependencies)
        acs = RiskAnalyzer.AbsoluteCriticalityOfServices(dependencies)

        def norm(lst):
            return Normalizer.FixedRatio([x["factor"] for x in _sort_locale(lst, lambda x: x["uniqueServiceName"])])

        nrf, nacs = norm(rf), norm(acs)
        raw = []
        for i, usn in enumerate(sorted(d["uniqueServiceName"] for d in dependencies)):
            rep = next((r["replicas"] for r in replicas if r["uniqueServiceName"] == usn), UNDEF)
            raw.append({"uniqueServiceName": usn, "impact": (nrf[i] + nacs[i]) / (rep if truthy(rep) else 1)})
        ni = Normalizer.Linear([r["impact"] for r in raw])
        return [{**r, "impact": ni[i]} for i, r in enumerate(raw)]

    @staticmethod
    def Probability(data):
        """RiskAnalyzer.ts:87-122."""
        rel = RiskAnalyzer.ReliabilityMetric(data)
        raw = RiskAnalyzer.InvokeProbabilityAndErrorRate(data)
        mp = RiskAnalyzer.MINIMUM_PROB
        npro = [r["probability"] * (1 - mp) + mp for r in raw]
        nerr = [r["errorRate"] * (1 - mp) + mp for r in raw]
        base = Normalizer.Linear([p * nerr[i] for i, p in enumerate(npro)], mp)
        base_map = {raw[i]["uniqueServiceName"]: b for i, b in enumerate(base)}
        out = []
        for r in rel:
            prob = base_map[r["uniqueServiceName"]]
            p = r["norm"] * (mp if prob < mp else prob)
            out.append({"uniqueServiceName": r["uniqueServiceName"], "probability": p * (1 - mp) + mp})
        return out

    @staticmethod
    def RelyingFactor(dependencies):
        """RiskAnalyzer.ts:124-137."""
        fm: Dict[str, float] = {}
        for d in dependencies:
            f = 0
            for l in d["links"]:
                for c in l["details"]:
                    f = f + c["dependingBy"] / c["distance"]
            gw = any(len(x["dependingBy"]) == 0 for x in d["dependency"])
            fm[d["uniqueServiceName"]] = f + (1 if gw else 0)
        return [{"uniqueServiceName": k, "factor": v} for k, v in fm.items()]

    @staticmethod
    def AbsoluteCriticalityOfServices(dependencies):
        """RiskAnalyzer.ts:145-169."""
        out = []
        for d in dependencies:
            gw = any(len(x["dependingBy"]) == 0 for x in d["dependency"])
            ais, ads = (1 if gw else 0), 0
            for l in d["links"]:
                for c in l["details"]:
                    if c["distance"] != 1:
                        continue
                    if c["dependingBy"] > 0:
                        ais += 1
                    if c["dependingOn"] > 0:
                        ads += 1
            out.append({"uniqueServiceName": d["uniqueServiceName"], "factor": ais * ads, "ais": ais, "ads": ads})
        return out

    @staticmethod
    def InvokeProbabilityAndErrorRate(data, include_request_error=False):
        """RiskAnalyzer.ts:171-213."""
        counts: Dict[str, dict] = {}
        for d in data:
            st = d["status"]
            is_err = st.startswith("5") or (include_request_error and st.startswith("4"))
            p = counts.get(d["uniqueServiceName"], {"count": 0, "error": 0})
            counts[d["uniqueServiceName"]] = {
                "count": p["count"] + d["combined"],
                "error": p["error"] + (d["combined"] if is_err else 0),
            }
        total = 0
        for v in counts.values():
            total = total + v["count"]
        out = []
        for k, v in counts.items():
            out.append(
                {
                    "uniqueServiceName": k,
                    "probability": v["count"] / total if total else math.nan,
                    "errorRate": v["error"] / v["count"] if v["count"] else math.nan,
                }
            )
        return out

    @staticmethod
    def ReliabilityMetric(data):
        """RiskAnalyzer.ts:215-226."""
        rm = RiskAnalyzer.GetLatencyCVOfServices(data)
        norm = Normalizer.SigmoidAdj([m["metric"] for m in rm])
        return [{**m, "norm": norm[i]} for i, m in enumerate(rm)]

    @staticmethod
    def GetLatencyCVOfServices(data):
        """RiskAnalyzer.ts:228-248."""
        dm: Dict[str, List[dict]] = {}
        for s in data:
            dm.setdefault(s["uniqueServiceName"], []).append(s)
        out = []
        for usn, lst in dm.items():
            total = 0
            ssum = 0
            for d in lst:
                ssum += d["latency"]["cv"] * d["combined"]
                total += d["combined"]
            out.append({"uniqueServiceName": usn, "metric": ssum / total if total else math.nan})
        return out


# --------------------------------------------------------------------------
# bodies: Utils.Merge / MergeStringBody / ObjectToInterfaceString
# --------------------------------------------------------------------------
def js_parse(text):
    """JSON.parse (SyntaxError -> ValueError).  JS numbers are doubles."""
    if not isinstance(text, str):
        raise ValueError("JSON.parse of a non-string")

    def num(tok):
        v = int(tok)
        return v if -(2 ** 53) < v < 2 ** 53 else float(tok)

    def bad(tok):
        raise ValueError(tok)

    return json.loads(text, parse_int=num, parse_constant=bad)


def js_stringify(v):
    """JSON.stringify of a parsed JSON value.  Only ever re-parsed here, so
    Python's float spelling (1e+16 for 10000000000000000) is equivalent."""
    if v is UNDEF:
        return UNDEF
    return json.dumps(v, ensure_ascii=False, separators=(",", ":"), allow_nan=False)


def _spread(x) -> dict:
    if isinstance(x, dict):
        return dict(x)
    if isinstance(x, str):
        units = x.encode("utf-16-le", "surrogatepass")
        return {str(k // 2): units[k:k + 2].decode("utf-16-le", "surrogatepass") for k in range(0, len(units), 2)}
    return {}


def js_merge(a, b):
    """Utils.Merge (Utils.ts:279-291)."""
    if isinstance(a, list) and isinstance(b, list):
        return a[:10] + b[:10]
    if not isinstance(a, list) and not isinstance(b, list):
        out = _spread(a)
        out.update(_spread(b))
        return out
    return a if truthy(a) else b


def merge_string_body(a, b):
    """Utils.MergeStringBody (Utils.ts:293-309)."""
    if not (truthy(a) and truthy(b)):
        return a if truthy(a) else b
    pa = pb = UNDEF
    try:
        pa = js_parse(a)
    except ValueError:
        pass
    try:
        pb = js_parse(b)
    except ValueError:
        pass
    if truthy(pa) and truthy(pb):
        return js_stringify(js_merge(pa, pb))
    return js_stringify(pa if truthy(pa) else pb)


JSON_TO_TS = None  # a json-to-ts restatement (obj, rootName) -> [interface strings]; absent


def _primitive(v):
    return not isinstance(v, (dict, list))


def _js_typeof(v):
    if v is None:
        return "object"
    if v is UNDEF:
        return "undefined"
    if v is True or v is False:
        return "boolean"
    return {int: "number", float: "number", str: "string"}.get(type(v), "object")


def _sort_obj(o):
    if isinstance(o, list):
        return o if all(_primitive(x) for x in o) else [_sort_obj(x) for x in o if not _primitive(x)]
    out = {}
    for k in sorted(o, key=lambda t: [ord(c) for c in t.encode("utf-16-be", "surrogatepass").decode("latin-1")]):
        v = o[k]
        if isinstance(v, list):
            if v and all(isinstance(x, dict) for x in v):
                v = [_sort_obj(x) for x in v]
        elif isinstance(v, dict):
            v = _sort_obj(v)
        out[k] = v
    return out


def _members(o):
    out = ""
    for k in o:
        v = o[k]
        if not re.match(r"^[A-Za-z_][A-Za-z0-9_]*$", k) or isinstance(v, (dict, list)):
            return None
        out += "  %s?: any;\n" % k if v is None else "  %s: %s;\n" % (k, _js_typeof(v))
    return out


def _to_ts(o, root):
    """JsonToTS (json-to-ts 1.7) for single-interface shapes only (the format
    of tests/Utils.test.ts:17-30,58-69): a flat object, or a non-empty array
    of flat objects that all give the same members."""
    body = None
    if isinstance(o, dict):
        body = _members(o)
    elif isinstance(o, list) and o and all(isinstance(x, dict) for x in o):
        each = [_members(x) for x in o]
        body = each[0] if None not in each and len(set(each)) == 1 else None
    if body is not None:
        return ["interface %s {\n%s}" % (root, body)]
    if JSON_TO_TS is None:
        raise NotImplementedError("json-to-ts")
    return list(JSON_TO_TS(o, root))


def object_to_interface_string(o, name="Root"):
    """Utils.ObjectToInterfaceString (Utils.ts:14-36)."""
    if _primitive(o):
        return _js_typeof(o)
    so = _sort_obj(o)
    if isinstance(so, list):
        if len(o) == 0:
            return "interface %s extends Array<any>{}" % name
        if _primitive(o[0]):
            return "interface %s extends Array<%s>{}" % (name, _js_typeof(o[0]))
        return "interface %s extends Array<ArrayItem>{}\n" % name + "\n".join(_to_ts(so, "ArrayItem"))
    return "\n".join(_to_ts(so, name))


def parse_bodies(acc):
    """RealtimeDataList.parseRequestResponseBody (RealtimeDataList.ts:120-155)."""
    out = {}
    for side in ("request", "response"):
        if get(acc, side + "ContentType") != "application/json":
            continue
        try:
            body = js_parse(get(acc, side + "Body"))
        except ValueError:
            continue
        out[side + "Body"] = body
        out[side + "Schema"] = object_to_interface_string(body)
    return out


# --------------------------------------------------------------------------
# Envoy logs: KubernetesService.ParseEnvoyLogs + classes/EnvoyLog.ts
# --------------------------------------------------------------------------
class Date:
    """new Date(iso) -> getTime() in ms (NaN if unparsable), fraction truncated."""

    def __init__(self, text):
        self.text = text
        m = re.match(r"^(\d{4})-(\d\d)-(\d\d)T(\d\d):(\d\d):(\d\d)(?:\.(\d+))?(Z|[+-]\d\d:\d\d)?$", text or "")
        if not m:
            self.t = float("nan")
            return
        import datetime

        y, mo, d, h, mi, se, fr, tz = m.groups()
        try:
            dt = datetime.datetime(int(y), int(mo), int(d), int(h), int(mi), int(se), tzinfo=datetime.timezone.utc)
        except ValueError:
            self.t = float("nan")
            return
        ms = int(dt.timestamp()) * 1000 + int(((fr or "") + "000")[:3])
        if tz and tz != "Z":
            off = (int(tz[1:3]) * 60 + int(tz[4:6])) * 60000
            ms = ms - off if tz[0] == "+" else ms + off
        self.t = float(ms)

    def getTime(self):
        return self.t


def parse_envoy_logs(lines, namespace, pod):
    """KubernetesService.ParseEnvoyLogs (KubernetesService.ts:201-242)."""
    term = "\n\r\u2028\u2029"
    first_trace = {}
    logs = []
    for line in lines:
        cols = line.split("\t")
        if len(cols) < 2:
            raise TypeError("log is undefined")
        t, log = cols[0], cols[1]
        h = re.search(r"\[(Request|Response) ([A-Za-z0-9_\-]+)/([A-Za-z0-9_]+)/([A-Za-z0-9_]+)/([A-Za-z0-9_]+)\]", log)
        if not h or not h.group(2):
            continue
        typ, rid, tid, sid, pid = h.groups()
        st = re.search(r"\[Status\] ([0-9]+)", log)
        mp = re.search(r"(GET|POST|PUT|DELETE|PATCH|HEAD|OPTIONS) ([^\]]+)", log)
        ct = re.search(r"\[ContentType ([^\]]*)\]", log)
        bd = re.search("\\[Body\\] ([^" + term + "]*)", log)
        if rid not in first_trace and tid != "NO_ID":
            first_trace[rid] = tid
        e = {"timestamp": Date(t), "type": typ, "requestId": rid, "traceId": tid, "spanId": sid,
             "parentSpanId": pid, "namespace": namespace, "podName": pod}
        if mp:
            e["method"], e["path"] = mp.group(1), mp.group(2)
        if st:
            e["status"] = st.group(1)
        if bd:
            e["body"] = bd.group(1)
        if ct:
            e["contentType"] = ct.group(1)
        logs.append(e)
    for e in logs:
        e["traceId"] = first_trace.get(e["requestId"]) or "NO_ID"
    return EnvoyLogs(logs)


class EnvoyLogs:
    def __init__(self, logs):
        self.logs = logs

    def toJSON(self):
        return self.logs

    def toStructured(self):
        if not self.logs:
            return []
        by_id: Dict[str, Dict[str, dict]] = {}
        for e in self.logs:
            by_id.setdefault(js_str(get(e, "requestId")) + "/" + js_str(get(e, "traceId")), {})[get(e, "spanId")] = e
        if any("NO_ID" in m for m in by_id.values()):
            return self.toStructuredFallback()
        res = []
        for key, spans in by_id.items():
            parts = key.split("/")
            traces = []
            for sid, e in spans.items():
                par = spans.get(get(e, "parentSpanId"))
                if get(e, "type") == "Response" and par is not None and get(par, "type") == "Request":
                    traces.append({"traceId": parts[1], "spanId": sid, "parentSpanId": get(e, "parentSpanId"),
                                   "request": par, "response": e, "isFallback": False})
            res.append({"requestId": parts[0], "traces": traces})
        return res

    def toStructuredFallback(self):
        if not self.logs:
            return []
        groups: Dict[str, List[dict]] = {}
        for e in self.logs:
            if truthy(get(e, "requestId")):
                groups.setdefault(js_str(e["requestId"]) + "/" + js_str(get(e, "traceId")), []).append(e)
        res = []
        for key, logs in groups.items():
            parts = key.split("/")
            open_reqs = []
            by_span: Dict[Any, dict] = {}
            for e in logs:
                if get(e, "type") == "Request":
                    open_reqs.append(e)
                if get(e, "type") == "Response":
                    if not open_reqs:
                        continue
                    q = open_reqs.pop()
                    by_span[get(q, "spanId")] = {"traceId": parts[1], "request": q, "response": e,
                                                 "spanId": get(q, "spanId"), "parentSpanId": get(q, "parentSpanId"),
                                                 "isFallback": True}
            res.append({"requestId": parts[0], "traces": list(by_span.values())})
        return res

    @staticmethod
    def CombineToStructuredEnvoyLogs(all_logs):
        return EnvoyLogs.FillMissingId(EnvoyLogs.CombineStructuredEnvoyLogs([l.toStructured() for l in all_logs]))

    @staticmethod
    def CombineStructuredEnvoyLogs(structured):
        merged: Dict[str, list] = {}
        for per_service in structured:
            for l in per_service:
                merged[l["requestId"]] = merged.get(l["requestId"], []) + l["traces"]
        out = []
        for rid, traces in merged.items():
            times = [t["request"]["timestamp"].getTime() if isinstance(t["request"].get("timestamp"), Date)
                     else float("nan") for t in traces]
            if any(x < 0 for x in times):
                raise NotImplementedError("sort with pre-1970 request times")
            out.append({"requestId": rid, "traces": traces})  # (comparator >= 0 or NaN: order kept)
        return out

    @staticmethod
    def FillMissingId(logs):
        parents = {}
        for l in logs:
            for t in l["traces"]:
                p = get(t, "parentSpanId")
                if truthy(p) and p != "NO_ID":
                    parents[js_str(l["requestId"]) + "/" + js_str(get(t, "spanId"))] = p
        for l in logs:
            for t in l["traces"]:
                p = parents.get(js_str(l["requestId"]) + "/" + js_str(get(t, "spanId")))
                t["parentSpanId"] = p if truthy(p) else get(t, "parentSpanId")
        return logs
