"""Envoy access logs -> structured logs -> realtime-row bodies.

Host-side by design (string / JSON work, no per-span arithmetic): the
reference's own pipeline in front of Traces.combineLogsToRealtimeData
(RealtimeWorkerImpl.ts:44-62):

* :func:`envoy_log_lines` / :func:`ParseEnvoyLogs`  KubernetesService.ts:178-242
* :class:`EnvoyLogs` (toStructured, toStructuredFallback,
  CombineToStructuredEnvoyLogs, CombineStructuredEnvoyLogs, FillMissingId)
                                                  classes/EnvoyLog.ts:7-149
* :func:`merge_string_body`, :func:`merge`        utils/Utils.ts:279-309
* :func:`parse_request_response_body`             RealtimeDataList.ts:120-155
* :func:`object_to_interface_string`             utils/Utils.ts:14-75; of the
  ``json-to-ts`` npm package it calls (package.json "^1.7.0", not in this
  image) only the single-interface outputs the reference's own vectors fix
  are restated (flat objects, arrays of one flat shape); nested shapes call
  the hook set with :func:`set_json_to_ts` and raise NotImplementedError
  without one (parity unpinned).

JS semantics kept where they are observable: JSON.parse / JSON.stringify
(number formatting, the JS grammar), truthiness, Map first-position /
last-value order, and Array.prototype.sort with the reference's one-argument
comparator (V8's TimSort, see :func:`_sort_by_request_time`).
"""
from __future__ import annotations

import json
import math
import re
from typing import Callable, Dict, List, Optional, Sequence

from .ingest import UNDEFINED, js_truthy

# ------------------------------------------------------------------------------
# JS values
# ------------------------------------------------------------------------------
_SAFE = 2 ** 53


class JSDate:
    """``new Date(string)`` for the ISO-8601 forms Envoy / Kubernetes print
    (other strings: an Invalid Date, getTime() = NaN).  Fractions beyond
    milliseconds are truncated, as V8 does; a time without an offset is
    taken as UTC (the pod clock's zone in the reference's deployment)."""

    _ISO = re.compile(r"^(\d{4})-(\d{2})-(\d{2})(?:T(\d{2}):(\d{2})(?::(\d{2})(?:\.(\d+))?)?(Z|[+-]\d{2}:\d{2})?)?$")

    def __init__(self, text):
        self.text = text
        self.ms = float("nan")
        m = self._ISO.match(text) if isinstance(text, str) else None
        if m:
            import calendar

            y, mo, d, h, mi, s, frac, tz = m.groups()
            try:
                secs = calendar.timegm((int(y), int(mo), int(d), int(h or 0), int(mi or 0), int(s or 0), 0, 0, 0))
            except (ValueError, OverflowError):
                return
            if not (1 <= int(mo) <= 12 and 1 <= int(d) <= 31 and int(h or 0) <= 24 and int(mi or 0) < 60
                    and int(s or 0) < 60):
                return
            ms = secs * 1000 + (int((frac or "0")[:3].ljust(3, "0")))
            if tz and tz != "Z":
                sign = 1 if tz[0] == "+" else -1
                ms -= sign * (int(tz[1:3]) * 60 + int(tz[4:6])) * 60000
            self.ms = float(ms)

    def getTime(self) -> float:
        return self.ms

    def __eq__(self, other):
        return isinstance(other, JSDate) and self.text == other.text

    def __repr__(self):
        return f"JSDate({self.text!r})"


def js_number_str(x: float) -> str:
    """Number::toString (ECMA-262 7.1.12.1) from the shortest round-trip digits."""
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, int) and abs(x) < _SAFE:
        return str(x)
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if x == 0:
        return "0"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))
    mant, _, exp = r.partition("e")
    e = int(exp) if exp else 0
    ip, _, fp = mant.partition(".")
    digits = (ip + fp).lstrip("0")
    # value = 0.<digits> * 10^n  with n = position of the decimal point
    n = len(ip.lstrip("0")) + e if ip.strip("0") else e - (len(fp) - len(fp.lstrip("0")))
    digits = digits.rstrip("0") or "0"
    k = len(digits)
    if k <= n <= 21:
        return sign + digits + "0" * (n - k)
    if 0 < n <= 21:
        return sign + digits[:n] + "." + digits[n:]
    if -6 < n <= 0:
        return sign + "0." + "0" * (-n) + digits
    ee = n - 1
    es = ("+" if ee >= 0 else "-") + str(abs(ee))
    if k == 1:
        return sign + digits + "e" + es
    return sign + digits[0] + "." + digits[1:] + "e" + es


def _js_int(s: str):
    v = int(s)
    return v if abs(v) < _SAFE else float(s)


def _no_constant(s):
    raise ValueError(f"Unexpected token {s[0]} in JSON")


def js_json_parse(text):
    """JSON.parse: the JSON grammar only (no NaN / Infinity), numbers are
    doubles (integers beyond 2^53 round as JS does).  Raises ValueError for a
    SyntaxError (also for a non-string argument: JSON.parse(undefined))."""
    if not isinstance(text, str):
        raise ValueError("Unexpected token u in JSON")
    return json.loads(text, parse_int=_js_int, parse_constant=_no_constant)


_ESC = {'"': '\\"', "\\": "\\\\", "\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r", "\t": "\\t"}


def _js_quote(s: str) -> str:
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch in _ESC:
            out.append(_ESC[ch])
        elif c < 0x20 or 0xD800 <= c <= 0xDFFF:  # (lone surrogates: well-formed JSON.stringify)
            out.append("\\u%04x" % c)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _ordered_keys(d: dict):
    """Own property order of a JS object: array-index keys ascending, then the
    other strings in insertion order."""
    idx = [k for k in d if k.isdigit() and (k == "0" or not k.startswith("0")) and int(k) < 2 ** 32 - 1]
    rest = [k for k in d if k not in set(idx)]
    return sorted(idx, key=int) + rest


def js_json_stringify(v):
    """JSON.stringify of a JSON-parsed value (returns UNDEFINED for undefined)."""
    if v is UNDEFINED:
        return UNDEFINED
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (int, float)):
        return js_number_str(v) if math.isfinite(float(v)) else "null"
    if isinstance(v, str):
        return _js_quote(v)
    if isinstance(v, list):
        return "[" + ",".join("null" if x is UNDEFINED else js_json_stringify(x) for x in v) + "]"
    if isinstance(v, dict):
        parts = []
        for k in _ordered_keys(v):
            s = js_json_stringify(v[k])
            if s is not UNDEFINED:
                parts.append(_js_quote(k) + ":" + s)
        return "{" + ",".join(parts) + "}"
    raise TypeError(f"not a JSON value: {type(v).__name__}")


# ------------------------------------------------------------------------------
# Utils.Merge / MergeStringBody (Utils.ts:279-309)
# ------------------------------------------------------------------------------
def merge(a, b):
    """Utils.Merge: arrays -> first 10 of each; two non-arrays -> {...a, ...b}
    (spreading a primitive adds nothing, a string spreads its characters);
    otherwise a || b."""
    if isinstance(a, list) and isinstance(b, list):
        return a[:10] + b[:10]
    if not isinstance(a, list) and not isinstance(b, list):
        out = {}
        for x in (a, b):
            if isinstance(x, dict):
                out.update(x)
            elif isinstance(x, str):  # spread by UTF-16 code unit
                u = x.encode("utf-16-le", "surrogatepass")
                out.update({str(i): u[2 * i: 2 * i + 2].decode("utf-16-le", "surrogatepass")
                            for i in range(len(u) // 2)})
        return out
    return a if js_truthy(a) else b


def merge_string_body(a=UNDEFINED, b=UNDEFINED):
    """Utils.MergeStringBody (Utils.ts:293-309)."""
    if js_truthy(a) and js_truthy(b):
        pa = pb = UNDEFINED
        try:
            pa = js_json_parse(a)
        except ValueError:
            pass
        try:
            pb = js_json_parse(b)
        except ValueError:
            pass
        if js_truthy(pa) and js_truthy(pb):
            return js_json_stringify(merge(pa, pb))
        return js_json_stringify(pa if js_truthy(pa) else pb)
    return a if js_truthy(a) else b


# ------------------------------------------------------------------------------
# Utils.ObjectToInterfaceString (Utils.ts:14-75)
# ------------------------------------------------------------------------------
_json_to_ts: Optional[Callable] = None


def set_json_to_ts(fn: Optional[Callable]):
    """Install a restatement of json-to-ts's ``JsonToTS(object, {rootName})``
    (returning the list of interface strings); None removes it."""
    global _json_to_ts
    _json_to_ts = fn


def _is_primitive(v) -> bool:
    return not isinstance(v, (dict, list))


def _typeof(v) -> str:
    if v is UNDEFINED:
        return "undefined"
    if v is None:
        return "object"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    return "object"


def _sort_object(obj):
    if isinstance(obj, list):
        if all(_is_primitive(o) for o in obj):
            return obj
        return [_sort_object(o) for o in obj if not _is_primitive(o)]
    out = {}
    for k in sorted(obj.keys(), key=lambda s: s.encode("utf-16-be")):  # Array.prototype.sort: UTF-16 order
        o = obj[k]
        if isinstance(o, list) and len(o) > 0:
            if all(isinstance(i, dict) for i in o):
                o = [_sort_object(i) for i in o]
        elif isinstance(o, dict):
            o = _sort_object(o)
        out[k] = o
    return out


_IDENT = re.compile(r"^[a-zA-Z_][a-zA-Z\d_]*$")


def _flat_members(obj: dict):
    """`  key: type;` lines of an object whose values are all primitives, or
    None.  A null member is optional `any` (json-to-ts; tests/Utils.test.ts:
    58-69 shows `originId?: any;`)."""
    lines = []
    for k, v in obj.items():  # (already sorted by Utils.sortObject)
        if not _IDENT.match(k) or isinstance(v, (dict, list)):
            return None
        lines.append(f"  {k}?: any;\n" if v is None else f"  {k}: {_typeof(v)};\n")
    return lines


def _json_to_ts_call(obj, root: str) -> List[str]:
    """JsonToTS(obj, {rootName}) for the shapes whose output the reference's
    own vectors fix: one interface `interface <Name> {\n` + one `  key: type;\n`
    per member + `}` (tests/Utils.test.ts:17-30, 58-69), for
      * an object of primitive members (the empty object included: every
        cache merge meets it, Utils.Merge(undefined, undefined) is {},
        CombinedRealtimeDataList.ts:212-223);
      * an array of such objects with one member set and one type per member
        (the root's element interface is named by the rootName).
    Nested objects, arrays inside objects, and arrays whose elements differ
    (json-to-ts names nested interfaces and merges optional members) go to the
    hook of set_json_to_ts, or raise."""
    if isinstance(obj, dict):
        lines = _flat_members(obj)
        if lines is not None:
            return [f"interface {root} {{\n" + "".join(lines) + "}"]
    elif isinstance(obj, list) and obj and all(isinstance(o, dict) for o in obj):
        first = _flat_members(obj[0])
        if first is not None and all(_flat_members(o) == first for o in obj[1:]):
            return [f"interface {root} {{\n" + "".join(first) + "}"]
    if _json_to_ts is None:
        raise NotImplementedError(
            "Utils.ObjectToInterfaceString needs json-to-ts for nested objects (not in this image; "
            "install a restatement with kmamiz_amd.envoy.set_json_to_ts)")
    return list(_json_to_ts(obj, root))


def object_to_interface_string(obj, name: str = "Root") -> str:
    if _is_primitive(obj):
        return _typeof(obj)
    srt = _sort_object(obj)
    if isinstance(srt, list):
        array_type, appending = "Array<any>{}", ""
        if len(obj) > 0:
            if _is_primitive(obj[0]):
                array_type = f"Array<{_typeof(obj[0])}>{{}}"
            else:
                array_type = "Array<ArrayItem>{}\n"
                appending = "\n".join(_json_to_ts_call(srt, "ArrayItem"))
        return f"interface {name} extends {array_type}{appending}"
    return "\n".join(_json_to_ts_call(srt, name))


def parse_request_response_body(data: dict) -> dict:
    """RealtimeDataList.parseRequestResponseBody (RealtimeDataList.ts:120-155):
    for application/json content types, the parsed body and its schema; a body
    that does not parse (or a schema that throws) leaves both undefined."""
    out = {}
    for side in ("request", "response"):
        if data.get(f"{side}ContentType", UNDEFINED) == "application/json":
            try:
                body = js_json_parse(data.get(f"{side}Body", UNDEFINED))
            except ValueError:
                continue
            out[f"{side}Body"] = body
            out[f"{side}Schema"] = object_to_interface_string(body)
    return out


# ------------------------------------------------------------------------------
# KubernetesService.getEnvoyLogs / ParseEnvoyLogs (KubernetesService.ts:178-242)
# ------------------------------------------------------------------------------
_STRIP = re.compile("\\t[^\\n\\r\u2028\u2029]*envoy (lua|wasm)[^\\n\\r\u2028\u2029]*\\t(script|wasm) log[^:]*: ")
_HDR = re.compile(r"\[(Request|Response) ([\w\-_]+)/([\w_]+)/([\w_]+)/([\w_]+)\]", re.ASCII)
_STATUS = re.compile(r"\[Status\] ([0-9]+)")
_METHOD = re.compile(r"(GET|POST|PUT|DELETE|PATCH|HEAD|OPTIONS) ([^\]]+)")
_CTYPE = re.compile(r"\[ContentType ([^\]]*)]")
_BODY = re.compile("\\[Body\\] ([^\\n\\r\u2028\u2029]*)")


def envoy_log_lines(text: str) -> List[str]:
    """The istio-proxy log lines getEnvoyLogs keeps, with the Envoy prefix
    between the time and the script output collapsed to one tab (the second
    .replace there takes a literal string and never matches)."""
    out = []
    for line in text.split("\n"):
        if "script log: " in line or "wasm log " in line:
            out.append(_STRIP.sub("\t", line, count=1).replace("\tthread.*", ""))
    return out


def _group(m, i):
    return m.group(i) if m else UNDEFINED


def ParseEnvoyLogs(logs: Sequence[str], namespace: str, podName: str) -> "EnvoyLogs":
    id_map: Dict[str, str] = {}
    out = []
    for l in logs:
        parts = l.split("\t")
        time, log = parts[0], (parts[1] if len(parts) > 1 else UNDEFINED)
        if log is UNDEFINED:
            raise TypeError("Cannot read properties of undefined (reading 'match')")
        m = _HDR.search(log)
        typ, request_id, trace_id, span_id, parent = (_group(m, i) for i in range(1, 6))
        if not js_truthy(request_id):
            continue
        status = _group(_STATUS.search(log), 1)
        mm = _METHOD.search(log)
        method, path = _group(mm, 1), _group(mm, 2)
        ctype = _group(_CTYPE.search(log), 1)
        body = _group(_BODY.search(log), 1)
        if request_id not in id_map and trace_id != "NO_ID":
            id_map[request_id] = trace_id
        out.append({"timestamp": JSDate(time), "type": typ, "requestId": request_id, "traceId": trace_id,
                    "spanId": span_id, "parentSpanId": parent, "method": method, "path": path, "status": status,
                    "body": body, "contentType": ctype, "namespace": namespace, "podName": podName})
    for e in out:
        e["traceId"] = id_map.get(e["requestId"]) or "NO_ID"
    return EnvoyLogs([{k: v for k, v in e.items() if v is not UNDEFINED} for e in out])


# ------------------------------------------------------------------------------
# EnvoyLogs (classes/EnvoyLog.ts)
# ------------------------------------------------------------------------------
def _g(o: dict, k):
    return o.get(k, UNDEFINED)


def _sort_by_request_time(traces: List[dict]) -> List[dict]:
    """``traces.sort((t) => t.request.timestamp.getTime())`` (EnvoyLog.ts:121):
    the comparator reads only its FIRST argument, so V8's TimSort (Node 12)
    moves an element only when that element's request time is negative.  With
    every time >= 0 or NaN the array is one ascending run: unchanged.  Short
    arrays (< 64, a single run + binary insertion) are restated exactly;
    longer ones with pre-1970 times would need TimSort's merges and raise."""
    n = len(traces)
    if n < 2:
        return traces

    def neg(t):
        v = t["request"]["timestamp"].getTime() if isinstance(t["request"].get("timestamp"), JSDate) else float("nan")
        return v < 0  # (NaN compares false: treated as >= 0)

    if not any(neg(t) for t in traces):
        return traces
    if n >= 64:
        raise NotImplementedError("Array.prototype.sort merge phase with pre-1970 request times")
    a = list(traces)
    run = 2
    desc = neg(a[1])
    for i in range(2, n):
        if desc != neg(a[i]):
            break
        run += 1
    if desc:
        a[:run] = a[:run][::-1]
    for start in range(run, n):
        pivot = a[start]
        lo, hi = 0, start
        while lo < hi:
            mid = lo + ((hi - lo) >> 1)
            if neg(pivot):
                hi = mid
            else:
                lo = mid + 1
        a[lo + 1: start + 1] = a[lo:start]
        a[lo] = pivot
    traces[:] = a
    return traces


class EnvoyLogs:
    def __init__(self, envoyLogs: List[dict]):
        self._envoyLogs = envoyLogs

    def toJSON(self):
        return self._envoyLogs

    def toStructured(self) -> List[dict]:
        """EnvoyLog.ts:17-55."""
        if len(self._envoyLogs) == 0:
            return []
        log_map: Dict[str, Dict] = {}
        span_ids = set()
        for e in self._envoyLogs:
            key = f"{_s(_g(e, 'requestId'))}/{_s(_g(e, 'traceId'))}"
            log_map.setdefault(key, {})[_g(e, "spanId")] = e
            span_ids.add(_g(e, "spanId"))
        if "NO_ID" in span_ids:
            return self.toStructuredFallback()
        out = []
        for key, span_map in log_map.items():
            request_id, trace_id = (key.split("/") + [UNDEFINED])[:2]
            traces = []
            for span_id, log in span_map.items():
                p = _g(log, "parentSpanId")
                if _g(log, "type") == "Response" and p in span_map and _g(span_map[p], "type") == "Request":
                    traces.append({"traceId": trace_id, "spanId": span_id, "parentSpanId": p,
                                   "request": span_map[p], "response": log, "isFallback": False})
            out.append({"requestId": request_id, "traces": traces})
        return out

    def toStructuredFallback(self) -> List[dict]:
        """EnvoyLog.ts:57-99: pair each Response with the last open Request."""
        if len(self._envoyLogs) == 0:
            return []
        logs_map: Dict[str, List[dict]] = {}
        for log in self._envoyLogs:
            if js_truthy(_g(log, "requestId")):
                logs_map.setdefault(f"{_s(log['requestId'])}/{_s(_g(log, 'traceId'))}", []).append(log)
        out = []
        for key, logs in logs_map.items():
            request_id, trace_id = (key.split("/") + [UNDEFINED])[:2]
            stack: List[dict] = []
            trace_map: Dict = {}
            for log in logs:
                if _g(log, "type") == "Request":
                    stack.append(log)
                if _g(log, "type") == "Response":
                    if not stack:
                        stack = []
                        continue
                    req = stack.pop()
                    trace_map[_g(req, "spanId")] = {"traceId": trace_id, "request": req, "response": log,
                                                    "spanId": _g(req, "spanId"), "parentSpanId": _g(req, "parentSpanId"),
                                                    "isFallback": True}
            out.append({"requestId": request_id, "traces": list(trace_map.values())})
        return out

    @staticmethod
    def CombineToStructuredEnvoyLogs(logs: Sequence["EnvoyLogs"]) -> List[dict]:
        """EnvoyLog.ts:101-106 (what RealtimeWorkerImpl.ts:62 passes on)."""
        return EnvoyLogs.FillMissingId(EnvoyLogs.CombineStructuredEnvoyLogs([l.toStructured() for l in logs]))

    @staticmethod
    def CombineStructuredEnvoyLogs(logs: Sequence[List[dict]]) -> List[dict]:
        """EnvoyLog.ts:108-126."""
        log_map: Dict = {}
        for service_log in logs:
            for log in service_log:
                log_map.setdefault(log["requestId"], []).extend(log["traces"])
        return [{"requestId": rid, "traces": _sort_by_request_time(traces)} for rid, traces in log_map.items()]

    @staticmethod
    def FillMissingId(logs: List[dict]) -> List[dict]:
        """EnvoyLog.ts:128-148 (mutates the traces' parentSpanId)."""
        id_map: Dict[str, str] = {}
        for l in logs:
            for t in l["traces"]:
                p = _g(t, "parentSpanId")
                if js_truthy(p) and p != "NO_ID":
                    id_map[f"{_s(l['requestId'])}/{_s(_g(t, 'spanId'))}"] = p
        for l in logs:
            for t in l["traces"]:
                v = id_map.get(f"{_s(l['requestId'])}/{_s(_g(t, 'spanId'))}")
                t["parentSpanId"] = v if js_truthy(v) else _g(t, "parentSpanId")
        return logs


def _s(v) -> str:
    """Template-literal string of a log field."""
    from .ingest import tpl

    return tpl(v)
