"""Cross-window merges of the cache layer in columnar form.

Every 5 s the reference merges the window's results into two caches:

* ``CCombinedRealtimeData.setData`` (Cacheable/CCombinedRealtimeData.ts:47-53):
  drop rows whose ``service`` is falsy, then ``cached.combineWith(update)``
  (CombinedRealtimeDataList.ts:183-263: group by endpoint + status, sum the
  counts, max the timestamps, fold (n, mean, cv) pairwise with the decimal
  shift of 278-332, ToPrecise);
* ``CEndpointDependencies.setData`` (Cacheable/CEndpointDependencies.ts:46-48)
  of ``existing.combineWith(newDep)`` (RealtimeWorkerImpl.ts:67-70,
  Initializer.ts:92): one merged row per endpoint, new (name, distance)
  entries appended in the order combineWith meets them, then ``trim()``.

Here both caches are columns with stable ids (an endpoint registry that
outlives the windows), and a merge is a handful of vectorised set operations
over them -- never a per-span or per-object loop.  The window side comes
straight from the engine: the combined groups (K3) and the reduced graph with
its exact entry order (``kmz_run(KMZ_RUN_DEPS | KMZ_RUN_DEP_ORDER)``,
kmz_order.hip).  Objects are built only by ``toJSON()``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import settings
from .ingest import UNDEFINED, js_truthy, tpl

I64_MIN = np.iinfo(np.int64).min
_U = np.uint64


def _clean(d: dict) -> dict:
    return {k: v for k, v in d.items() if v is not UNDEFINED}


def _freeze(fields: dict):
    return tuple(sorted(((k, type(v).__name__, v if v is not UNDEFINED else None) for k, v in fields.items()),
                        key=lambda t: t[0]))


class _Registry:
    """uniqueEndpointName -> stable id, and interned ToEndpointInfo field sets
    (everything of an endpoint info but its timestamp).  Append-only, so every
    cache state and window built on one registry shares it: ids never change."""

    def __init__(self):
        self.names: List[str] = []
        self.index: Dict[str, int] = {}
        self.infos: List[dict] = []
        self.info_index: Dict[tuple, int] = {}
        self._by_obj: Dict[int, tuple] = {}  # id(fields dict) -> (dict, info id)

    def info_of_obj(self, fields: dict) -> int:
        """info_id of a long-lived fields dict (the ingest's per-shape Identity
        objects are cached across batches): interned once per object."""
        hit = self._by_obj.get(id(fields))
        if hit is not None and hit[0] is fields:
            return hit[1]
        i = self.info_id(fields)
        self._by_obj[id(fields)] = (fields, i)
        return i

    def name_id(self, name: str) -> int:
        i = self.index.get(name)
        if i is None:
            i = self.index[name] = len(self.names)
            self.names.append(name)
        return i

    def info_id(self, fields: dict) -> int:
        k = _freeze(fields)
        i = self.info_index.get(k)
        if i is None:
            i = self.info_index[k] = len(self.infos)
            self.infos.append(dict(fields))
        return i


# ------------------------------------------------------------------------------
# dependency cache
# ------------------------------------------------------------------------------
class ReducedDependencies:
    """EndpointDependencies in reduced form (one merged row per endpoint), as
    columns.  Rows: ``row_ep`` (registry id, in row order), ``row_info`` /
    ``row_ts`` (the row's ``endpoint``), ``row_last`` (lastUsageTimestamp),
    ``row_ext`` (isDependedByExternal).  Entries: ``e_row`` (the row's endpoint),
    ``e_side`` (0 dependingBy, 1 dependingOn), ``e_ep`` / ``e_dist`` (the entry's
    endpoint name and distance), ``e_info`` / ``e_ts`` (its endpoint info),
    ``e_ord`` (its place in the row's list: increasing)."""

    def __init__(self, reg: Optional[_Registry] = None):
        self.reg = reg or _Registry()
        z = np.zeros(0, np.int64)
        self.row_ep, self.row_info = z.copy(), z.copy()
        self.row_ts, self.row_last = np.zeros(0), np.zeros(0)
        self.row_last_int = np.zeros(0, bool)  # lastUsageTimestamp is the integer 0 (no usage)
        self.row_ext = np.zeros(0, bool)
        self.e_row, self.e_side, self.e_ep, self.e_dist, self.e_info, self.e_ord = (z.copy() for _ in range(6))
        self.e_ts = np.zeros(0)
        self.next_ord = 0

    # -- construction -----------------------------------------------------------
    @classmethod
    def from_window(cls, entries: np.ndarray, row_ts: np.ndarray, row_shape: np.ndarray, endpoints: np.ndarray,
                    names: Sequence[str], shape_fields, reg: Optional[_Registry] = None) -> "ReducedDependencies":
        """The engine's reduced graph of one window (EndpointDependencies([])
        .combineWith(traces.toEndpointDependencies()).trim()): kmz_get_dep_entries
        + kmz_get_endpoints.  ``names[e]`` is the uniqueEndpointName of window
        dependency endpoint e, ``shape_fields(s)`` the ToEndpointInfo fields of
        shape s (Traces.ts:213-241)."""
        lt = endpoints["last_ts"]
        none = lt == I64_MIN
        last_ms = np.where(none, 0.0, np.maximum(0.0, np.where(none, 0, lt) / 1000))
        return cls.from_columns(entries, row_ts, row_shape, endpoints["first_row"], endpoints["has_row"] != 0,
                                endpoints["external"] != 0, last_ms, none, names, shape_fields, reg)

    @classmethod
    def from_columns(cls, entries, row_ts, row_shape, first_row, has_row, external, last_ms, last_none, names,
                     shape_fields, reg: Optional[_Registry] = None) -> "ReducedDependencies":
        out = cls(reg)
        R = out.reg
        emap = np.array([R.name_id(n) if n is not None else -1 for n in names] or [-1], dtype=np.int64)
        has = np.nonzero(has_row)[0]
        has = has[np.argsort(first_row[has], kind="stable")]
        used = np.concatenate([entries["shape"], row_shape[has]])
        shapes = np.nonzero(np.bincount(used))[0] if len(used) else used  # distinct shapes, O(n)
        smap = np.full(int(shapes.max()) + 1 if len(shapes) else 1, -1, np.int64)
        for s in shapes.tolist():
            smap[s] = R.info_of_obj(shape_fields(s))
        out.row_ep = emap[has]
        out.row_info = smap[row_shape[has]]
        out.row_ts = row_ts[has] / 1000
        out.row_last_int = np.asarray(last_none)[has]
        out.row_last = np.asarray(last_ms, np.float64)[has]
        out.row_ext = np.asarray(external)[has]
        k = entries["key"]
        side = (k & _U(1)).astype(np.int64)
        a = (k >> _U(40)).astype(np.int64)
        d = ((k >> _U(16)) & _U(0xFFFFFF)).astype(np.int64)
        out.e_side = side
        out.e_dist = ((k >> _U(1)) & _U(0x7FFF)).astype(np.int64)
        out.e_row = emap[np.where(side == 1, a, d)]
        out.e_ep = emap[np.where(side == 1, d, a)]
        out.e_info = smap[entries["shape"]]
        out.e_ts = entries["ts"] / 1000
        # within a merged row: by the contributing row, then the row's own
        # order (side 1: the first descendant's index; side 0: the distance).
        # Both are flatten indices < 2^31, so (row, within) packs into one
        # order-preserving int64 and no sort is needed here.
        within = np.where(side == 1, entries["pos"], out.e_dist.astype(np.uint64))
        if len(k) and (int(entries["row"].max()) >= 1 << 31 or int(within.max()) >= 1 << 32):
            o = np.lexsort((within, entries["row"]))
            out.e_ord = np.empty(len(o), np.int64)
            out.e_ord[o] = np.arange(len(o), dtype=np.int64)
        else:
            out.e_ord = ((entries["row"] << _U(32)) | within).astype(np.int64)
        out.next_ord = int(out.e_ord.max()) + 1 if len(k) else 0
        return out.filtered()  # (every EndpointDependencies built on the way filters, EndpointDependencies.ts:41)

    @classmethod
    def from_json(cls, rows: Sequence[dict], merge_rows: bool = False,
                  reg: Optional[_Registry] = None) -> "ReducedDependencies":
        """Columns of TEndpointDependency objects (e.g. the cache's Mongo copy).
        ``merge_rows=False`` reads them as ``this`` of combineWith (a later row
        of the same endpoint replaces an earlier one, at the earlier one's
        position: Map.set, EndpointDependencies.ts:508-513); ``True`` as its
        argument (later rows append their unseen entries, 514-535).  Each row's
        lists are deduplicated as trim() does (first position, last value)."""
        out = cls(reg)
        R = out.reg
        order: List[int] = []
        by_ep: Dict[int, list] = {}
        rows = settings.filter_out_deprecated(list(rows), settings.deprecated_cutoff())  # new EndpointDependencies(rows)
        for r in rows:
            e = R.name_id(r["endpoint"]["uniqueEndpointName"])
            lists = []
            for side, lk in ((0, "dependingBy"), (1, "dependingOn")):
                seen: Dict[tuple, int] = {}
                lst: List[list] = []
                for x in r[lk]:
                    kk = (x["endpoint"]["uniqueEndpointName"], tpl(x["distance"]))
                    if kk in seen:
                        lst[seen[kk]][1] = x
                    else:
                        seen[kk] = len(lst)
                        lst.append([kk, x])
                lists.append(lst)
            if e not in by_ep:
                order.append(e)
                by_ep[e] = [r, lists, [{k for k, _ in lists[0]}, {k for k, _ in lists[1]}]]
            elif not merge_rows:
                by_ep[e] = [r, lists, [{k for k, _ in lists[0]}, {k for k, _ in lists[1]}]]
            else:
                slot = by_ep[e]
                for side in (0, 1):
                    for kk, x in lists[side]:
                        if kk not in slot[2][side]:
                            slot[2][side].add(kk)
                            slot[1][side].append([kk, x])
        rows_c = {"ep": [], "info": [], "ts": [], "last": [], "ext": []}
        ents = {"row": [], "side": [], "ep": [], "dist": [], "info": [], "ts": []}
        for e in order:
            r, lists, _ = by_ep[e]
            ep = r["endpoint"]
            rows_c["ep"].append(e)
            rows_c["info"].append(R.info_id({k: v for k, v in ep.items() if k != "timestamp"}))
            rows_c["ts"].append(ep["timestamp"])
            rows_c["last"].append(r["lastUsageTimestamp"])
            rows_c["ext"].append(bool(r["isDependedByExternal"]))
            for side in (0, 1):
                for (nm, _), x in lists[side]:
                    xe = x["endpoint"]
                    ents["row"].append(e)
                    ents["side"].append(side)
                    ents["ep"].append(R.name_id(nm))
                    ents["dist"].append(int(x["distance"]))
                    ents["info"].append(R.info_id({k: v for k, v in xe.items() if k != "timestamp"}))
                    ents["ts"].append(xe["timestamp"])
        out.row_ep = np.array(rows_c["ep"], np.int64)
        out.row_info = np.array(rows_c["info"], np.int64)
        out.row_ts = np.array(rows_c["ts"], np.float64)
        out.row_last_int = np.array([type(v) is int and v == 0 for v in rows_c["last"]], bool)
        out.row_last = np.array(rows_c["last"], np.float64)
        out.row_ext = np.array(rows_c["ext"], bool)
        out.e_row = np.array(ents["row"], np.int64)
        out.e_side = np.array(ents["side"], np.int64)
        out.e_ep = np.array(ents["ep"], np.int64)
        out.e_dist = np.array(ents["dist"], np.int64)
        out.e_info = np.array(ents["info"], np.int64)
        out.e_ts = np.array(ents["ts"], np.float64)
        out.e_ord = np.arange(len(out.e_row), dtype=np.int64)
        out.next_ord = len(out.e_row)
        return out.filtered() if merge_rows else out

    # -- the reference's methods --------------------------------------------------
    def filtered(self, cutoff: Optional[float] = None) -> "ReducedDependencies":
        """The constructor's deprecation filter (EndpointDependencies.ts:44-74)
        on the columns: rows with lastUsageTimestamp < cutoff go, and every
        entry naming one of their endpoints (or belonging to one) with them.
        ``cutoff`` defaults to settings.deprecated_cutoff() (now - threshold;
        0: no filter)."""
        if cutoff is None:
            cutoff = settings.deprecated_cutoff()
        if cutoff == 0 or not len(self.row_ep):
            return self
        last = np.where(self.row_last_int, 0.0, self.row_last)
        stale = last < cutoff
        if not stale.any():
            return self
        gone = self.row_ep[stale]
        out = ReducedDependencies(self.reg)
        keep = ~stale
        for f in ("row_ep", "row_info", "row_ts", "row_last", "row_last_int", "row_ext"):
            setattr(out, f, getattr(self, f)[keep])
        ek = ~(np.isin(self.e_row, gone) | np.isin(self.e_ep, gone))
        for f in ("e_row", "e_side", "e_ep", "e_dist", "e_info", "e_ts", "e_ord"):
            setattr(out, f, getattr(self, f)[ek])
        out.next_ord = self.next_ord
        return out

    def _ck(self, row, side, ep, dist):
        return (row.astype(_U) << _U(40)) | (ep.astype(_U) << _U(16)) | (dist.astype(_U) << _U(1)) | side.astype(_U)

    def combineWith(self, other) -> "ReducedDependencies":
        """EndpointDependencies.ts:499-542 on the columns: this's rows keep their
        place and values (the reference writes the max lastUsageTimestamp into
        the incoming row object, which it then drops, 516), new endpoints'
        rows follow in the argument's order, and each row's unseen (name,
        distance) entries are appended in the argument's order."""
        if not isinstance(other, ReducedDependencies):
            other = other.toReduced() if hasattr(other, "toReduced") else ReducedDependencies.from_json(
                other.toJSON(), merge_rows=True)
        out = ReducedDependencies(self.reg)
        R = out.reg
        if other.reg is R:  # one registry: ids already agree
            bmap = imap = None
        else:
            bmap = np.array([R.name_id(n) for n in other.reg.names] or [0], dtype=np.int64)
            imap = np.array([R.info_id(f) for f in other.reg.infos] or [0], dtype=np.int64)
        b_row = bmap[other.row_ep] if bmap is not None else other.row_ep
        new = ~np.isin(b_row, self.row_ep)
        out.row_ep = np.concatenate([self.row_ep, b_row[new]])
        out.row_info = np.concatenate([self.row_info, imap[other.row_info[new]] if imap is not None else
                                       other.row_info[new]])
        out.row_ts = np.concatenate([self.row_ts, other.row_ts[new]])
        out.row_last = np.concatenate([self.row_last, other.row_last[new]])
        out.row_last_int = np.concatenate([self.row_last_int, other.row_last_int[new]])
        out.row_ext = np.concatenate([self.row_ext, other.row_ext[new]])
        if len(other.e_row):
            br, be = (bmap[other.e_row], bmap[other.e_ep]) if bmap is not None else (other.e_row, other.e_ep)
            bck = self._ck(br, other.e_side, be, other.e_dist)
            fresh = ~np.isin(bck, self._ck(self.e_row, self.e_side, self.e_ep, self.e_dist))
        else:
            br = be = other.e_row
            fresh = np.zeros(0, bool)
        rank = np.empty(int(fresh.sum()), np.int64)
        rank[np.argsort(other.e_ord[fresh], kind="stable")] = np.arange(len(rank), dtype=np.int64)
        out.e_row = np.concatenate([self.e_row, br[fresh]])
        out.e_side = np.concatenate([self.e_side, other.e_side[fresh]])
        out.e_ep = np.concatenate([self.e_ep, be[fresh]])
        out.e_dist = np.concatenate([self.e_dist, other.e_dist[fresh]])
        out.e_info = np.concatenate([self.e_info, imap[other.e_info[fresh]] if imap is not None else
                                     other.e_info[fresh]])
        out.e_ts = np.concatenate([self.e_ts, other.e_ts[fresh]])
        out.e_ord = np.concatenate([self.e_ord, self.next_ord + rank])
        out.next_ord = self.next_ord + len(rank)
        return out.filtered()  # new EndpointDependencies(...) (EndpointDependencies.ts:539-541)

    def trim(self) -> "ReducedDependencies":
        """EndpointDependencies.ts:91-112: the lists need no dedup here (entries
        are unique per (row, side, name, distance) by construction); the new
        object's constructor filters deprecated endpoints."""
        return self.filtered()

    def getData(self, namespace: Optional[str] = None) -> "ReducedDependencies":
        """Cacheable/CEndpointDependencies.ts:51-59: the rows whose endpoint
        namespace matches."""
        if namespace is None:
            return self
        keep_info = np.array([f.get("namespace", UNDEFINED) == namespace for f in self.reg.infos] or [False])
        keep = keep_info[self.row_info]
        eps = self.row_ep[keep]
        out = ReducedDependencies(self.reg)
        for f in ("row_ep", "row_info", "row_ts", "row_last", "row_last_int", "row_ext"):
            setattr(out, f, getattr(self, f)[keep])
        ek = np.isin(self.e_row, eps)
        for f in ("e_row", "e_side", "e_ep", "e_dist", "e_info", "e_ts", "e_ord"):
            setattr(out, f, getattr(self, f)[ek])
        out.next_ord = self.next_ord
        return out

    def __len__(self):
        return len(self.row_ep)

    def n_entries(self) -> int:
        return len(self.e_row)

    def toJSON(self) -> List[dict]:
        infos = self.reg.infos

        def info(i, ts):
            return _clean({**infos[i], "timestamp": ts})

        pos = np.full(max(len(self.reg.names), 1), -1, np.int64)
        pos[self.row_ep] = np.arange(len(self.row_ep))
        o = np.lexsort((self.e_ord, self.e_side, pos[self.e_row]))
        rows_of = pos[self.e_row][o]
        bounds = np.searchsorted(rows_of, np.arange(len(self.row_ep) + 1))
        side, dist, einf, ets = (self.e_side[o].tolist(), self.e_dist[o].tolist(), self.e_info[o].tolist(),
                                 self.e_ts[o].tolist())
        out = []
        last = self.row_last.tolist()
        for k, (ri, rts, ext, lint) in enumerate(zip(self.row_info.tolist(), self.row_ts.tolist(),
                                                     self.row_ext.tolist(), self.row_last_int.tolist())):
            by, on = [], []
            for j in range(int(bounds[k]), int(bounds[k + 1])):
                x = {"endpoint": info(einf[j], ets[j]), "distance": dist[j], "type": "SERVER" if side[j] else "CLIENT"}
                (on if side[j] else by).append(x)
            out.append({
                "endpoint": info(ri, rts),
                "lastUsageTimestamp": 0 if lint else last[k],
                "isDependedByExternal": bool(ext),
                "dependingBy": by,
                "dependingOn": on,
            })
        return out


class CEndpointDependencies:
    """Cacheable/CEndpointDependencies.ts:1-61 over the columns (no Mongo)."""

    uniqueName = "EndpointDependencies"

    def __init__(self, initData: Optional[ReducedDependencies] = None):
        self._data = initData

    def setData(self, update) -> None:
        """``super.setData(update.trim())``.  A ReducedDependencies stays columnar;
        anything else (the worker's first tick stores newDep itself, one row
        per span id, RealtimeWorkerImpl.ts:68-70) is kept as its trimmed rows."""
        self._data = update.trim()

    def getData(self, namespace: Optional[str] = None):
        if self._data is None:
            return None
        if isinstance(self._data, ReducedDependencies):
            return self._data.getData(namespace)
        if namespace:
            from .classes import EndpointDependencies

            return EndpointDependencies([d for d in self._data.toJSON()
                                         if d["endpoint"].get("namespace", UNDEFINED) == namespace])
        return self._data


def merge_shard_entries(parts):
    """The reduced graph's entry records of traceId shards -> those of the whole
    batch.  parts: (entries, row_ts, row_shape, first_row) per shard, indices
    global (kmz_set_index_map).  A row and every descendant row of it belong to
    one trace, hence to one shard: per key the record with the smallest row is
    the whole batch's; per endpoint the first row is the smallest first row."""
    ents = np.concatenate([p[0] for p in parts])
    o = np.lexsort((ents["row"], ents["key"]))
    ents = ents[o]
    keep = np.ones(len(ents), bool)
    keep[1:] = ents["key"][1:] != ents["key"][:-1]
    fr = np.stack([p[3] for p in parts])
    best = np.argmin(fr, axis=0)
    cols = np.arange(fr.shape[1])
    row_ts = np.stack([p[1] for p in parts])[best, cols]
    row_shape = np.stack([p[2] for p in parts])[best, cols]
    return ents[keep], row_ts, row_shape


def worker_dependencies(existing: Optional[ReducedDependencies], new) -> object:
    """RealtimeWorkerImpl.ts:67-70: ``existingDep ? new EndpointDependencies(
    existingDep).combineWith(newDep) : newDep``."""
    return existing.combineWith(new) if existing is not None else new


# ------------------------------------------------------------------------------
# combined realtime data cache
# ------------------------------------------------------------------------------
_BASE = ("uniqueServiceName", "service", "namespace", "version", "method", "requestContentType",
         "responseContentType")


_BODY_FIELDS = ("requestBody", "requestSchema", "responseBody", "responseSchema")


def _undef_col(n: int) -> np.ndarray:
    c = np.empty(n, dtype=object)
    c[:] = [UNDEFINED] * n
    return c


def _merge_bodies(body: Dict[str, np.ndarray], g: np.ndarray, rank: np.ndarray, head: np.ndarray, G: int):
    """The body half of combineWith's reduce (CombinedRealtimeDataList.ts:
    204-226): a group of one row keeps its row's bodies and schemas; a longer
    group folds Utils.Merge over its rows from the first and re-derives the
    schema of each truthy result.  Rows without bodies (or with {}) merge to {}
    whose schema is one constant: that case is vectorised, the rest loops."""
    from .envoy import merge, object_to_interface_string

    out = {f: body[f][head].copy() for f in _BODY_FIELDS}
    size = np.bincount(g, minlength=G)
    multi = size > 1
    if not multi.any():
        return out
    for side in ("request", "response"):
        b = body[side + "Body"]
        plain = np.array([v is UNDEFINED or (isinstance(v, dict) and not v) for v in b.tolist()], bool)
        all_plain = np.ones(G, bool)
        np.logical_and.at(all_plain, g, plain)
        fast = np.nonzero(multi & all_plain)[0]
        schema = object_to_interface_string({}) if len(fast) else None
        for k in fast.tolist():
            out[side + "Body"][k] = {}
            out[side + "Schema"][k] = schema
        slow = np.nonzero(multi & ~all_plain)[0]
        if len(slow):
            members = np.lexsort((rank, g))
            starts = np.searchsorted(g[members], np.arange(G + 1))
            sch = body[side + "Schema"]
            for k in slow.tolist():
                idx = members[starts[k]:starts[k + 1]]
                acc, sc = b[idx[0]], sch[idx[0]]
                for r in idx[1:].tolist():
                    acc = merge(acc, b[r])
                    if js_truthy(acc):
                        sc = object_to_interface_string(acc)
                out[side + "Body"][k] = acc
                out[side + "Schema"][k] = sc
    return out


def _safe_log10_floor(x: np.ndarray) -> np.ndarray:
    """Math.floor(Math.log10(x)) for x > 0, else 0 (CombinedRealtimeDataList.ts:322-330)."""
    u, inv = np.unique(x, return_inverse=True)
    e = np.array([math.floor(math.log10(v)) if v > 0 else 0 for v in u.tolist()], np.int64)
    return e[inv].reshape(x.shape)


def pooled(n1, m1, c1, n2, m2, c2):
    """combineLatencyCVAndMean (CombinedRealtimeDataList.ts:278-315) on arrays,
    the operations in the reference's order (fp64, no contraction)."""
    shift = (_safe_log10_floor(m1) + _safe_log10_floor(m2)) // 2
    us, inv = np.unique(shift, return_inverse=True)
    scale = np.array([math.pow(10, int(s)) for s in us.tolist()])[inv].reshape(shift.shape)
    n1 = n1.astype(np.float64)
    n2 = n2.astype(np.float64)
    a, b = m1 / scale, m2 / scale
    sa, sb = c1 * a, c2 * b
    tot = n1 + n2
    mt = (n1 * a + n2 * b) / tot
    da, db = a - mt, b - mt
    pv = (n1 * (sa * sa) + n2 * (sb * sb) + n1 * (da * da) + n2 * (db * db)) / tot
    with np.errstate(divide="ignore", invalid="ignore"):
        cv = np.where(mt == 0, 0.0, np.sqrt(pv) / mt)
    return mt * scale, cv


def to_precise(x: np.ndarray) -> np.ndarray:
    """Utils.ToPrecise (Utils.ts:311-313) on arrays."""
    t = (x + 2.220446049250313e-16) * 1e14
    r = np.floor(t)
    r = np.where(t - r >= 0.5, r + 1.0, r)
    return r / 1e14


class _CombinedTables:
    """Interned group keys (``uniqueEndpointName\tstatus``) and sample metas of
    combined rows; append-only, shared by every cache state built on it."""

    def __init__(self):
        self.keys: Dict[str, int] = {}
        self.metas: List[dict] = []
        self.meta_index: Dict[tuple, int] = {}
        self.memo: Dict[tuple, tuple] = {}  # (id(endpoint fields), status text) -> (key id, meta id)
        self._hold: List[dict] = []  # keeps the memo's field dicts alive

    def key_id(self, k: str) -> int:
        i = self.keys.get(k)
        if i is None:
            i = self.keys[k] = len(self.keys)
        return i

    def meta_id(self, m: dict) -> int:
        f = _freeze(m)
        i = self.meta_index.get(f)
        if i is None:
            i = self.meta_index[f] = len(self.metas)
            self.metas.append(m)
        return i


class CombinedColumns:
    """CombinedRealtimeDataList as columns: one row per (endpoint, status),
    ``key`` the interned ``uniqueEndpointName\tstatus`` (CombinedRealtimeDataList
    .ts:188-190), ``meta`` the row's sample fields (uniqueEndpointName, status,
    and _BASE), ``combined`` / ``latest`` / ``mean`` / ``cv``."""

    def __init__(self, tab: Optional[_CombinedTables] = None):
        self.tab = tab or _CombinedTables()
        self.key = np.zeros(0, np.int64)
        self.meta = np.zeros(0, np.int64)
        self.combined = np.zeros(0, np.int64)
        self.latest = np.zeros(0, np.float64)
        self.latest_int = np.zeros(0, bool)
        self.mean = np.zeros(0)
        self.cv = np.zeros(0)
        # parsed bodies and their schemas (Envoy logs; Python objects, UNDEFINED = absent)
        self.body = {f: _undef_col(0) for f in _BODY_FIELDS}

    @classmethod
    def from_json(cls, rows: Sequence[dict], like: Optional["CombinedColumns"] = None) -> "CombinedColumns":
        out = cls(like.tab if like else None)
        T = out.tab
        key, meta, comb, lat, lint, mean, cv = [], [], [], [], [], [], []
        body = {f: _undef_col(len(rows)) for f in _BODY_FIELDS}
        for j, r in enumerate(rows):
            for f in _BODY_FIELDS:
                if f in r:
                    body[f][j] = r[f]
            key.append(T.key_id(f"{r['uniqueEndpointName']}\t{tpl(r.get('status', UNDEFINED))}"))
            meta.append(T.meta_id({f: r.get(f, UNDEFINED) for f in ("uniqueEndpointName", "status") + _BASE}))
            comb.append(int(r["combined"]))
            lat.append(r["latestTimestamp"])
            lint.append(type(r["latestTimestamp"]) is int)
            mean.append(r["latency"]["mean"])
            cv.append(r["latency"]["cv"])
        out.key = np.array(key, np.int64)
        out.meta = np.array(meta, np.int64)
        out.combined = np.array(comb, np.int64)
        out.latest = np.array(lat, np.float64)
        out.latest_int = np.array(lint, bool)
        out.mean = np.array(mean, np.float64)
        out.cv = np.array(cv, np.float64)
        out.body = body
        return out

    @classmethod
    def from_groups(cls, groups: np.ndarray, n_status: int, ep_fields, statuses: Sequence,
                    like: Optional["CombinedColumns"] = None, used: Optional[np.ndarray] = None) -> "CombinedColumns":
        """Columns of RealtimeDataList.toCombinedRealtimeData() straight from the
        engine's dense groups (kmz_get_groups, [n_ep * n_status]): used groups
        ordered by their endpoint's first row, then their own first row
        (RealtimeDataList.ts:22-45).  ep_fields(e): the row fields of endpoint e
        (Traces.ts:73-99; long-lived dicts, memoised by identity); statuses[s]:
        the interned status values.  No Envoy logs here (no content types).
        With ``used`` (kmz_fetch_used's ids), ``groups`` holds only the used
        groups, groups[k] the one of id used[k]."""
        out = cls(like.tab if like else None)
        T = out.tab
        if used is None:
            used = np.nonzero(groups["combined"] > 0)[0]
            groups = groups[used]
        used = np.asarray(used, dtype=np.int64)
        ep, st = used // n_status, used % n_status
        first = groups["first"]
        if len(used):
            epf = np.full(int(ep.max()) + 1, np.iinfo(np.uint64).max, np.uint64)
            np.minimum.at(epf, ep, first)
            o = np.lexsort((first, epf[ep]))
            used, ep, st, groups = used[o], ep[o], st[o], groups[o]
        st_txt = [tpl(v) for v in statuses]
        keys, metas = [], []
        for e, s in zip(ep.tolist(), st.tolist()):
            f = ep_fields(e)
            hit = T.memo.get((id(f), st_txt[s]))
            if hit is None:
                T._hold.append(f)
                sv = statuses[s]
                hit = T.memo[(id(f), st_txt[s])] = (
                    T.key_id(f"{f['uniqueEndpointName']}\t{st_txt[s]}"),
                    T.meta_id({"uniqueEndpointName": f["uniqueEndpointName"], "status": sv,
                               **{b: f.get(b, UNDEFINED) for b in _BASE}}))
            keys.append(hit[0])
            metas.append(hit[1])
        out.key = np.array(keys, np.int64)
        out.meta = np.array(metas, np.int64)
        out.combined = groups["combined"].astype(np.int64)
        out.latest = groups["latest_timestamp"].astype(np.float64)
        out.latest_int = np.ones(len(used), bool)
        out.mean = groups["mean"].astype(np.float64)
        out.cv = groups["cv"].astype(np.float64)
        out.body = {f: _undef_col(len(used)) for f in _BODY_FIELDS}
        return out

    def _adopt(self, other: "CombinedColumns"):
        """other's key / meta ids in this's tables (identity when shared)."""
        if other.tab is self.tab:
            return None, None
        kinv = [None] * len(other.tab.keys)
        for k, i in other.tab.keys.items():
            kinv[i] = k
        kmap = np.array([self.tab.key_id(k) for k in kinv] or [0], np.int64)
        mmap = np.array([self.tab.meta_id(m) for m in other.tab.metas] or [0], np.int64)
        return kmap, mmap

    def filter_service(self) -> "CombinedColumns":
        """``update.toJSON().filter((rl) => rl.service)`` (CCombinedRealtimeData.ts:48-50)."""
        ok = np.array([js_truthy(m.get("service", UNDEFINED)) for m in self.tab.metas] or [False])
        return self._take(ok[self.meta] if len(self.meta) else np.zeros(0, bool))

    def filter_namespace(self, namespace: str) -> "CombinedColumns":
        ok = np.array([m.get("namespace", UNDEFINED) == namespace for m in self.tab.metas] or [False])
        return self._take(ok[self.meta] if len(self.meta) else np.zeros(0, bool))

    def _take(self, sel) -> "CombinedColumns":
        out = CombinedColumns(self.tab)
        for f in ("key", "meta", "combined", "latest", "latest_int", "mean", "cv"):
            setattr(out, f, getattr(self, f)[sel])
        out.body = {f: v[sel] for f, v in self.body.items()}
        return out

    def combineWith(self, other: "CombinedColumns") -> "CombinedColumns":
        """CombinedRealtimeDataList.ts:183-263 over the columns.  Groups in
        first-appearance order of this + other; the sample (and its meta) is the
        group's first row; the latency fold starts from (0, 0, 0) and takes the
        rows in list order, one rank of rows per step."""
        out = CombinedColumns(self.tab)
        kmap, mmap = out._adopt(other)
        key = np.concatenate([self.key, kmap[other.key] if kmap is not None else other.key])
        meta = np.concatenate([self.meta, mmap[other.meta] if mmap is not None else other.meta])
        comb = np.concatenate([self.combined, other.combined])
        lat = np.concatenate([self.latest, other.latest])
        lint = np.concatenate([self.latest_int, other.latest_int])
        mean = np.concatenate([self.mean, other.mean])
        cv = np.concatenate([self.cv, other.cv])
        if len(key) == 0:
            return out
        uk, first, inv = np.unique(key, return_index=True, return_inverse=True)
        g_order = np.argsort(first, kind="stable")  # groups in first-appearance order
        gid = np.empty(len(uk), np.int64)
        gid[g_order] = np.arange(len(uk))
        g = gid[inv]  # group of each row (0.. in output order)
        G = len(uk)
        # rank of each row within its group (list order)
        o = np.lexsort((np.arange(len(g)), g))
        starts = np.searchsorted(g[o], np.arange(G))
        rank = np.empty(len(g), np.int64)
        rank[o] = np.arange(len(g)) - starts[g[o]]
        head = o[starts]  # each group's sample row
        n = np.zeros(G, np.int64)
        m = np.zeros(G)
        c = np.zeros(G)
        best = lat[head].copy()
        best_int = lint[head].copy()
        for r in range(int(rank.max()) + 1):
            rows = np.nonzero(rank == r)[0]
            gg = g[rows]
            m[gg], c[gg] = pooled(n[gg], m[gg], c[gg], comb[rows], mean[rows], cv[rows])
            n[gg] += comb[rows]
            if r:
                up = lat[rows] > best[gg]  # Math.max(prev, curr) (keeps prev on ties)
                best[gg[up]] = lat[rows][up]
                best_int[gg[up]] = lint[rows][up]
        out.body = _merge_bodies({f: np.concatenate([self.body[f], other.body[f]]) for f in _BODY_FIELDS}, g, rank,
                                 head, G)
        out.key = key[head]
        out.meta = meta[head]
        out.combined = n
        out.latest = best
        out.latest_int = best_int
        out.mean = to_precise(m)
        out.cv = to_precise(c)
        return out

    def __len__(self):
        return len(self.key)

    def toJSON(self) -> List[dict]:
        out = []
        bodies = [self.body[f].tolist() for f in _BODY_FIELDS]
        for j, (mi, n, lt, li, mu, cv) in enumerate(zip(self.meta.tolist(), self.combined.tolist(), self.latest.tolist(),
                                                        self.latest_int.tolist(), self.mean.tolist(), self.cv.tolist())):
            m = self.tab.metas[mi]
            out.append(_clean({
                "uniqueEndpointName": m["uniqueEndpointName"],
                "uniqueServiceName": m["uniqueServiceName"],
                "service": m["service"],
                "namespace": m["namespace"],
                "version": m["version"],
                "method": m["method"],
                "status": m["status"],
                "combined": n,
                "requestContentType": m["requestContentType"],
                "responseContentType": m["responseContentType"],
                "latestTimestamp": int(lt) if li else lt,
                **{f: bodies[k][j] for k, f in enumerate(_BODY_FIELDS)},
                "latency": {"mean": mu, "cv": cv},
            }))
        return out


class CCombinedRealtimeData:
    """Cacheable/CCombinedRealtimeData.ts:8-67 over the columns (no Mongo)."""

    uniqueName = "CombinedRealtimeData"

    def __init__(self, initData: Optional[CombinedColumns] = None):
        self._data = initData

    def setData(self, update) -> None:
        if not isinstance(update, CombinedColumns):
            update = CombinedColumns.from_json(update.toJSON(), like=self._data)
        update = update.filter_service()
        self._data = self._data.combineWith(update) if self._data is not None else update

    def reset(self):
        self._data = None

    def getData(self, namespace: Optional[str] = None) -> Optional[CombinedColumns]:
        if namespace and self._data is not None:
            return self._data.filter_namespace(namespace)
        return self._data
