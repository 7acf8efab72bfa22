"""Service-level risk (tail of the path).

Mirror of ``src/utils/RiskAnalyzer.ts`` and ``src/utils/Normalizer.ts`` over
the combined stats (engine K3 output) and service dependencies.  Host code:
at most a few thousand services, O(services + links).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

MINIMUM_PROB = 0.01


def _to_precise(x: float) -> float:
    t = (x + 2.220446049250313e-16) * 1e14
    if not math.isfinite(t):  # Math.round(NaN / +-Infinity) is itself
        return t / 1e14
    r = math.floor(t)
    if t - r >= 0.5:
        r += 1
    return float(r) / 1e14


# JS number semantics the reference's arithmetic relies on: Math.max/min
# propagate NaN (and give -/+Infinity on no arguments), `x || d` replaces 0 and
# NaN, and a division by zero gives NaN or +-Infinity instead of raising.
def _js_max(inp) -> float:
    if any(math.isnan(v) for v in inp):
        return math.nan
    return max(inp) if inp else -math.inf


def _js_min(inp) -> float:
    if any(math.isnan(v) for v in inp):
        return math.nan
    return min(inp) if inp else math.inf


def _js_or(v, default):
    return default if v is None or v == 0 or (isinstance(v, float) and math.isnan(v)) else v


def _js_div(a: float, b: float) -> float:
    if b != 0:
        return a / b
    if a == 0 or math.isnan(a):
        return math.nan
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


class Normalizer:
    """Normalizer.ts:17-70."""

    @staticmethod
    def Numbers(inp: Sequence[float], strategy, *args):
        return strategy(list(inp), *args)

    class Strategy:
        @staticmethod
        def BetweenFixedNumber(inp):
            hi, lo = _js_max(inp), _js_min(inp)
            if hi - lo == 0:
                return [0.1]  # Normalizer.ts:22, a single element, as in the TS
            return [((v - lo) / (hi - lo)) * 0.9 + 0.1 for v in inp]

        @staticmethod
        def Sigmoid(inp):
            return [1 / (1 + math.exp(-v)) for v in inp]

        @staticmethod
        def SigmoidAdj(inp):
            z = 2 * math.log(3)
            return [_to_precise(1 / (1 + math.exp(-z * (v - 1.5)))) for v in inp]

        @staticmethod
        def FixedRatio(inp):
            hi = _js_max(inp)
            return inp if hi == 0 else [_js_div(v, hi) for v in inp]

        @staticmethod
        def Linear(inp, minimum=0.1):
            if minimum >= 1:
                return inp
            return [v * (1 - minimum) + minimum for v in Normalizer.Strategy.FixedRatio(inp)]


def _gateway(dep) -> bool:
    if "gateway" in dep:  # the compact form of tail.ServiceTail.service_deps_compact()
        return dep["gateway"]
    return any(len(d["dependingBy"]) == 0 for d in dep["dependency"])


def absolute_criticality(service_deps: List[dict]) -> List[dict]:
    """RiskAnalyzer.ts:145-169: AIS = distance-1 dependents (+1 for a gateway),
    ADS = distance-1 dependencies, ACS = AIS * ADS."""
    out = []
    for s in service_deps:
        ais = 1 if _gateway(s) else 0
        ads = 0
        for l in s["links"]:
            for det in l["details"]:
                if det["distance"] == 1:
                    ais += det["dependingBy"] > 0
                    ads += det["dependingOn"] > 0
        out.append({"uniqueServiceName": s["uniqueServiceName"], "factor": ais * ads, "ais": ais, "ads": ads})
    return out


def relying_factor(service_deps: List[dict]) -> List[dict]:
    """RiskAnalyzer.ts:124-137."""
    fm: Dict[str, float] = {}
    for s in service_deps:
        f = 0
        for l in s["links"]:
            for det in l["details"]:
                f = f + det["dependingBy"] / det["distance"]
        fm[s["uniqueServiceName"]] = f + (1 if _gateway(s) else 0)
    return [{"uniqueServiceName": k, "factor": v} for k, v in fm.items()]


# String.prototype.localeCompare as the reference's Node runs it (ICU root
# order, en-US; pinned by tests/golden/locale_order.json, generated with that
# Node by tests/golden/gen_locale_order.js): three levels --
#   primary   whitespace < punctuation (in the order below) < digits < letters
#             (case-folded; accented letters by their base letter); C0 controls
#             other than whitespace are ignorable
#   secondary the combining marks of each letter (NFD), in ICU's mark order
#   tertiary  lowercase < uppercase
# Letters without a canonical decomposition outside ASCII (ae ligature,
# o-stroke, sharp s, ...) sort after all ASCII letters here: parity unpinned.
_PUNCT = "\t\n\x0b\x0c\r _-,;:!?.'\"()[]{}@*/\\&#%`^+<=>|~$"
_PUNCT_RANK = {c: i for i, c in enumerate(_PUNCT)}
_IGNORABLE = {chr(i) for i in list(range(0, 9)) + list(range(14, 32))}
# combining marks U+0300..U+036F in ICU's secondary order (equal ranks tie)
_MARK_ORDER = [
    (0x34f,), (0x332,), (0x313, 0x343), (0x314,), (0x301, 0x341), (0x300, 0x340), (0x306,), (0x302,), (0x30c,),
    (0x30a,), (0x342,), (0x308,), (0x344,), (0x30b,), (0x303,), (0x307,), (0x338,), (0x327,), (0x328,),
    (0x304,), (0x30d, 0x30e, 0x312, 0x315, 0x31a, 0x33d, 0x33e, 0x33f, 0x346, 0x34a, 0x34b, 0x34c, 0x350, 0x351,
     0x352, 0x357, 0x35b, 0x35d, 0x35e),
    (0x316, 0x317, 0x318, 0x319, 0x31c, 0x31d, 0x31e, 0x31f, 0x320, 0x329, 0x32a, 0x32b, 0x32c, 0x32f, 0x333,
     0x33a, 0x33b, 0x33c, 0x347, 0x348, 0x349, 0x34d, 0x34e, 0x353, 0x354, 0x355, 0x356, 0x359, 0x35a, 0x35c,
     0x35f, 0x362),
    (0x336, 0x337), (0x335,), (0x305,), (0x309,), (0x30f,), (0x310,), (0x311,), (0x31b,), (0x321,), (0x322,),
    (0x323,), (0x324,), (0x325,), (0x326,), (0x32d,), (0x32e,), (0x330,), (0x331,), (0x334,), (0x339,), (0x345,),
    (0x358,), (0x360,), (0x361,), (0x363,), (0x368,), (0x369,), (0x364,), (0x36a,), (0x365,), (0x36b,), (0x366,),
    (0x36c,), (0x36d,), (0x367,), (0x36e,), (0x36f,)]
_MARK_RANK = {m: r for r, ms in enumerate(_MARK_ORDER) for m in ms}


def _collation_key(s: str):
    import unicodedata

    prim, sec, ter = [], [], []
    for ch in unicodedata.normalize("NFD", s):
        o = ord(ch)
        if o in _MARK_RANK:
            if sec:
                sec[-1] = sec[-1] + (_MARK_RANK[o],)
            continue
        if ch in _IGNORABLE:
            continue
        if ch in _PUNCT_RANK:
            prim.append((1, _PUNCT_RANK[ch]))
            ter.append(0)
        elif "0" <= ch <= "9":
            prim.append((2, o))
            ter.append(0)
        elif ch.isascii() and ch.isalpha():
            prim.append((3, ord(ch.lower())))
            ter.append(1 if ch.isupper() else 0)
        else:
            prim.append((4, o))
            ter.append(0)
        sec.append(())
    return prim, sec, ter


def impact(service_deps: List[dict], replicas: List[dict]) -> List[dict]:
    """RiskAnalyzer.ts:51-85 (localeCompare-sorted factors zipped with a
    code-unit-sorted name list, as the TS does)."""

    def norm(lst):
        lst = sorted(lst, key=lambda x: _collation_key(x["uniqueServiceName"]))
        return Normalizer.Strategy.FixedRatio([x["factor"] for x in lst])

    nrf = norm(relying_factor(service_deps))
    nacs = norm(absolute_criticality(service_deps))
    rep = {}
    for r in replicas or []:
        rep.setdefault(r["uniqueServiceName"], r.get("replicas"))
    raw = []
    for i, usn in enumerate(sorted(s["uniqueServiceName"] for s in service_deps)):
        div = rep.get(usn) or 1
        raw.append({"uniqueServiceName": usn, "impact": (nrf[i] + nacs[i]) / div})
    ni = Normalizer.Strategy.Linear([r["impact"] for r in raw])
    return [{**r, "impact": ni[i]} for i, r in enumerate(raw)]


def probability(data: List[dict]) -> List[dict]:
    """RiskAnalyzer.ts:87-122, 171-248."""
    # latency CV per service weighted by request count (228-248)
    cv: Dict[str, List[float]] = {}
    for d in data:
        a = cv.setdefault(d["uniqueServiceName"], [0.0, 0])
        a[0] += d["latency"]["cv"] * d["combined"]
        a[1] += d["combined"]
    rel_names = list(cv)
    rel_norm = Normalizer.Strategy.SigmoidAdj([_js_div(cv[k][0], cv[k][1]) for k in rel_names])
    # invoke probability and 5xx error rate (171-213)
    cnt: Dict[str, List[int]] = {}
    for d in data:
        a = cnt.setdefault(d["uniqueServiceName"], [0, 0])
        a[0] += d["combined"]
        a[1] += d["combined"] if str(d["status"]).startswith("5") else 0
    total = 0
    for v in cnt.values():
        total += v[0]
    names = list(cnt)
    npro = [_js_div(cnt[k][0], total) * (1 - MINIMUM_PROB) + MINIMUM_PROB for k in names]
    nerr = [_js_div(cnt[k][1], cnt[k][0]) * (1 - MINIMUM_PROB) + MINIMUM_PROB for k in names]
    base = Normalizer.Strategy.Linear([p * nerr[i] for i, p in enumerate(npro)], MINIMUM_PROB)
    base_of = dict(zip(names, base))
    out = []
    for k, nm in zip(rel_names, rel_norm):
        b = base_of[k]
        p = nm * (MINIMUM_PROB if b < MINIMUM_PROB else b)
        out.append({"uniqueServiceName": k, "probability": p * (1 - MINIMUM_PROB) + MINIMUM_PROB})
    return out


def realtime_risk(data: List[dict], service_deps: List[dict], replicas: List[dict]) -> List[dict]:
    """RiskAnalyzer.RealtimeRisk (RiskAnalyzer.ts:10-49)."""
    imp = {}
    for i in impact(service_deps, replicas):
        imp.setdefault(i["uniqueServiceName"], i["impact"])
    prob = {}
    for p in probability(data):
        prob.setdefault(p["uniqueServiceName"], p["probability"])
    risks = []
    for usn in dict.fromkeys(d["uniqueServiceName"] for d in data):
        s, n, v = (usn.split("\t") + [None] * 3)[:3]
        i = _js_or(imp.get(usn), 0)
        p = _js_or(prob.get(usn), MINIMUM_PROB)
        risks.append(
            {"uniqueServiceName": usn, "service": s, "namespace": n, "version": v, "risk": i * p, "impact": i,
             "probability": p}
        )
    norm = Normalizer.Strategy.BetweenFixedNumber([r["risk"] for r in risks])
    return [{**r, **({"norm": norm[i]} if i < len(norm) else {})} for i, r in enumerate(risks)]
