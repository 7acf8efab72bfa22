"""The two pieces of hidden state the reference's EndpointDependencies
constructor reads (SURVEY.md 8b "Hidden state"): ``GlobalSettings.
DeprecatedEndpointThreshold`` (``DEPRECATED_ENDPOINT_THRESHOLD``,
src/GlobalSettings.ts:50,79) and ``Date.now()`` (EndpointDependencies.ts:49).

The TS parses the threshold once, when the class loads (a static field,
EndpointDependencies.ts:33-36); here it is parsed when this module is imported,
and :func:`set_deprecated_threshold` / :func:`set_clock` replace either for a
deployment that configures them in-process, or for tests that pin them.
"""
from __future__ import annotations

import os
import re
import time
from typing import Callable, Optional

# EndpointDependencies.ts:22 (`\d` of a JS RegExp is ASCII only)
_THRESHOLD_RE = re.compile(r"(?:([0-9]+)d)?(?:([0-9]+)h)?(?:([0-9]+)m)?")


def parse_threshold_ms(s: Optional[str]) -> float:
    """EndpointDependencies.parseThresholdToMilliseconds (EndpointDependencies.ts:20-31).

    ``String.prototype.match`` without the g flag returns the first match, and
    this pattern matches the empty string at position 0 whenever the text does
    not start with ``<digits>d|h|m``: "x1d", " 2h", "30s" and "12" are 0 ms.
    Arithmetic in doubles, as JS numbers."""
    if not s:
        return 0
    m = _THRESHOLD_RE.match(s)  # anchored at 0: the empty match there always succeeds
    days, hours, minutes = (float(int(g, 10)) if g else 0.0 for g in m.groups())
    v = ((days * 86400) + (hours * 3600) + (minutes * 60)) * 1000
    return int(v) if v == int(v) and abs(v) < 2 ** 53 else v


_deprecated_ms = parse_threshold_ms(os.environ.get("DEPRECATED_ENDPOINT_THRESHOLD") or "")
_clock: Callable[[], float] = lambda: int(time.time() * 1000)  # Date.now(): integer ms


def set_deprecated_threshold(s: Optional[str]) -> None:
    """Re-parse the threshold (as the TS would on a restart with the new env)."""
    global _deprecated_ms
    _deprecated_ms = parse_threshold_ms(s or "")


def set_clock(fn: Optional[Callable[[], float]]) -> None:
    """Replace ``Date.now()`` (None restores the wall clock)."""
    global _clock
    _clock = fn if fn is not None else (lambda: int(time.time() * 1000))


def deprecated_threshold_ms() -> float:
    return _deprecated_ms


def deprecated_cutoff() -> float:
    """EndpointDependencies.ts:49-54: ``now - threshold``, or 0 (no filter)
    when the threshold is 0 -- and also when ``now - threshold`` is exactly 0,
    since the TS tests the difference, not the threshold."""
    if _deprecated_ms == 0:
        return 0
    return _clock() - _deprecated_ms


def filter_out_deprecated(deps: list, cutoff: float) -> list:
    """EndpointDependencies.filterOutDeprecatedEndpoint (EndpointDependencies.ts:44-74)
    over TEndpointDependency dicts, for a cutoff from :func:`deprecated_cutoff`:
    rows used before the cutoff are dropped, and their names leave every
    remaining row's lists.  Like the TS it assigns the filtered lists into the
    row objects it keeps (callers holding those rows see the change)."""
    if cutoff == 0:
        return deps
    gone = set()
    kept = []
    for d in deps:
        if d["lastUsageTimestamp"] < cutoff:
            gone.add(d["endpoint"]["uniqueEndpointName"])
        else:
            kept.append(d)
    for d in kept:
        d["dependingBy"] = [x for x in d["dependingBy"] if x["endpoint"]["uniqueEndpointName"] not in gone]
        d["dependingOn"] = [x for x in d["dependingOn"] if x["endpoint"]["uniqueEndpointName"] not in gone]
    return kept
