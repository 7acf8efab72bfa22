"""Engine: one HIP context (one GPU, one stream) holding a device-resident
span batch and running the four hot-path kernels on it.

This is the Python face of ``include/kmz.h``; the TypeScript-facing mirror of
the reference classes lives in :mod:`kmamiz_amd.classes`.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib as L


@dataclass
class SpanBatch:
    """Columnar span batch in flatten order (layout of ``kmz_spans``)."""

    span_id: np.ndarray  # u64
    parent_id: np.ndarray  # u64, 0 = none
    kind: np.ndarray  # u8
    shape: np.ndarray  # u32
    status: np.ndarray  # u16
    duration: np.ndarray  # u32 (us)
    timestamp: np.ndarray  # i64 (us)
    index_base: int = 0

    def __post_init__(self):
        self.span_id = np.ascontiguousarray(self.span_id, dtype=np.uint64)
        self.parent_id = np.ascontiguousarray(self.parent_id, dtype=np.uint64)
        self.kind = np.ascontiguousarray(self.kind, dtype=np.uint8)
        self.shape = np.ascontiguousarray(self.shape, dtype=np.uint32)
        self.status = np.ascontiguousarray(self.status, dtype=np.uint16)
        self.duration = np.ascontiguousarray(self.duration, dtype=np.uint32)
        self.timestamp = np.ascontiguousarray(self.timestamp, dtype=np.int64)
        n = len(self.span_id)
        for f in ("parent_id", "kind", "shape", "status", "duration", "timestamp"):
            if len(getattr(self, f)) != n:
                raise ValueError(f"column {f} has {len(getattr(self, f))} rows, expected {n}")

    def __len__(self):
        return len(self.span_id)

    def c_struct(self) -> L.Spans:
        return L.Spans(
            len(self),
            L.ptr(self.span_id),
            L.ptr(self.parent_id),
            L.ptr(self.kind),
            L.ptr(self.shape),
            L.ptr(self.status),
            L.ptr(self.duration),
            L.ptr(self.timestamp),
            int(self.index_base),
        )


@dataclass
class ShapeTable:
    rt_ep: np.ndarray
    tag_ep: np.ndarray
    dep_ep: np.ndarray
    n_rt_ep: int
    n_tag_ep: int
    n_dep_ep: int
    n_status: int

    def __post_init__(self):
        self.rt_ep = np.ascontiguousarray(self.rt_ep, dtype=np.uint32)
        self.tag_ep = np.ascontiguousarray(self.tag_ep, dtype=np.uint32)
        self.dep_ep = np.ascontiguousarray(self.dep_ep, dtype=np.uint32)

    def c_struct(self) -> L.Shapes:
        return L.Shapes(
            len(self.rt_ep),
            L.ptr(self.rt_ep),
            L.ptr(self.tag_ep),
            L.ptr(self.dep_ep),
            self.n_rt_ep,
            self.n_tag_ep,
            self.n_dep_ep,
            max(1, self.n_status),
        )


class Engine:
    """One ``kmz_ctx``.  ``stream`` is an optional hipStream_t (int/pointer)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        self._lib = L.lib()
        self.ctx = self._lib.kmz_create(device, C.c_void_p(stream) if stream else None)
        # (the hipStream_t handle it launches on; None: its own -- a handle of 0,
        # torch's default stream, also means its own, unordered with torch's)
        self.stream = stream if stream else None
        if not self.ctx:
            raise RuntimeError(f"kmz_create({device}) failed: no HIP device visible (the engine has no CPU path)")
        self.n = 0
        self.index_base = 0
        self.n_dep_ep = 0
        self.n_status = 1
        self._pinned = {}  # name -> (ptr, bytes): reused page-locked result buffers
        self._shapes = None  # the loaded batch's ShapeTable (or a synthetic config number)

    def close(self):
        if getattr(self, "ctx", None):
            self._lib.kmz_destroy(self.ctx)
            self.ctx = None
        for ptr_, _ in getattr(self, "_pinned", {}).values():
            self._lib.kmz_host_free(ptr_)
        self._pinned = {}

    def _pinned_array(self, name: str, count: int, dtype) -> np.ndarray:
        """numpy view of a reused page-locked buffer (D2H at full PCIe rate)."""
        dtype = np.dtype(dtype)
        nbytes = max(8, count * dtype.itemsize)
        cur = self._pinned.get(name)
        if cur is None or cur[1] < nbytes:
            if cur is not None:
                self._lib.kmz_host_free(cur[0])
            p = self._lib.kmz_host_alloc(max(nbytes, 2 * (cur[1] if cur else 0)))
            if not p:
                raise MemoryError("kmz_host_alloc failed")
            cur = (p, max(nbytes, 2 * (cur[1] if cur else 0)))
            self._pinned[name] = cur
        buf = (C.c_char * cur[1]).from_address(cur[0])
        return np.frombuffer(buf, dtype=dtype, count=count)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- input ---------------------------------------------------------------
    def load(self, batch: SpanBatch, shapes: ShapeTable):
        self.gen += 1
        self._loaded_token = None
        s = batch.c_struct()
        sh = shapes.c_struct()
        L.check(self.ctx, self._lib.kmz_load(self.ctx, C.byref(s), C.byref(sh), L.MEM_HOST))
        self.n = len(batch)
        self.index_base = batch.index_base
        self.n_dep_ep = shapes.n_dep_ep
        self.n_status = max(1, shapes.n_status)
        self._shapes = shapes

    # ---- K1 on the device: Zipkin JSON -> columns (kmz_json_parse) -------------
    def json_parse(self, data=None, ptr: Optional[int] = None, length: int = 0, device: bool = False):
        """Parse Trace[][] JSON on the GPU: ``data`` (bytes-like, host) or a raw
        ``ptr`` + ``length`` (host memory, e.g. pinned, or device memory with
        device=True).  -> (n_spans, n_shapes, n_statuses), or None outside the
        fast path (nothing loaded: parse on the host)."""
        self.gen += 1  # kmz_json_parse overwrites the columns and drops the last run, even on E_UNSUPPORTED
        self._loaded_token = None  # (no drop-in Traces owns the loaded batch any more)
        n, ns, nt = C.c_uint64(), C.c_uint32(), C.c_uint32()
        if ptr is None:
            buf = data if isinstance(data, bytes) else bytes(data)
            src, length = C.c_char_p(buf), len(buf)
        else:
            src = C.c_void_p(ptr)
        rc = self._lib.kmz_json_parse(self.ctx, src, length, L.MEM_DEVICE if device else L.MEM_HOST, C.byref(n),
                                      C.byref(ns), C.byref(nt))
        if rc == L.E_UNSUPPORTED:
            return None
        L.check(self.ctx, rc)
        return int(n.value), int(ns.value), int(nt.value)

    def json_fields(self, n_shapes: int, n_statuses: int):
        """(shape_fields [n_shapes*7, 2], status_fields [n_statuses, 2]) of the last json_parse."""
        sf = np.zeros((max(1, n_shapes) * 7, 2), np.uint64)
        tf = np.zeros((max(1, n_statuses), 2), np.uint64)
        L.check(self.ctx, self._lib.kmz_json_fields(self.ctx, L.ptr(sf), L.ptr(tf)))
        return sf[: n_shapes * 7], tf[:n_statuses]

    def json_known(self, n_shapes: int, n_statuses: int):
        """Ids remembered from earlier json_load calls for this batch's raw shapes /
        statuses (kmz_json_known); NONE32 where new."""
        ks = np.zeros(max(1, n_shapes), np.uint32)
        kt = np.zeros(max(1, n_statuses), np.uint32)
        L.check(self.ctx, self._lib.kmz_json_known(self.ctx, L.ptr(ks), L.ptr(kt)))
        return ks[:n_shapes], kt[:n_statuses]

    def json_load(self, shape_of_raw: np.ndarray, status_of_raw: np.ndarray, shapes: ShapeTable, index_base: int = 0,
                  n: Optional[int] = None):
        self.gen += 1
        self._loaded_token = None
        sm = np.ascontiguousarray(shape_of_raw, dtype=np.uint32)
        tm = np.ascontiguousarray(status_of_raw, dtype=np.uint32)
        sh = shapes.c_struct()
        L.check(self.ctx, self._lib.kmz_json_load(self.ctx, L.ptr(sm), L.ptr(tm), C.byref(sh), index_base))
        self.n = n if n is not None else self.n
        self.index_base = index_base
        self.n_dep_ep = shapes.n_dep_ep
        self.n_status = max(1, shapes.n_status)
        self._shapes = shapes

    def spans(self) -> SpanBatch:
        """The loaded batch's columns, copied to the host (kmz_get_spans)."""
        n = self.n
        cols = dict(span_id=np.zeros(n, np.uint64), parent_id=np.zeros(n, np.uint64), kind=np.zeros(n, np.uint8),
                    shape=np.zeros(n, np.uint32), status=np.zeros(n, np.uint16), duration=np.zeros(n, np.uint32),
                    timestamp=np.zeros(n, np.int64))
        L.check(self.ctx, self._lib.kmz_get_spans(self.ctx, *(L.ptr(cols[k]) for k in (
            "span_id", "parent_id", "kind", "shape", "status", "duration", "timestamp")), n))
        return SpanBatch(index_base=self.index_base, **cols)

    def load_synthetic(self, config: int, seed: int, trace_begin: int, trace_end: int) -> int:
        self.gen += 1
        self._loaded_token = None
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_synth_load(self.ctx, config, seed, trace_begin, trace_end, C.byref(n)))
        d = L.SynthDesc()
        self._lib.kmz_synth_describe(config, C.byref(d))
        self.n = n.value
        self.n_dep_ep = d.n_endpoints
        self.n_status = d.n_status
        self._shapes = config
        return self.n

    def load_synthetic_shard(self, config: int, seed: int, trace_begin: int, trace_end: int, world: int,
                             rank: int) -> int:
        """The traces of [trace_begin, trace_end) with shard(traceId) == rank
        (kmz_synth_load_shard), with their global flatten indices."""
        self.gen += 1
        self._loaded_token = None
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_synth_load_shard(self.ctx, config, seed, trace_begin, trace_end, world, rank,
                                                         C.byref(n)))
        d = L.SynthDesc()
        self._lib.kmz_synth_describe(config, C.byref(d))
        self.n = n.value
        self.index_base = 0
        self.n_dep_ep = d.n_endpoints
        self.n_status = d.n_status
        self._shapes = config
        return self.n

    def shape_table(self):
        """The ShapeTable the loaded batch is indexed by."""
        if isinstance(self._shapes, int):
            from . import synth

            return synth.shape_table(self._shapes)
        return self._shapes

    def global_index(self) -> np.ndarray:
        """Global flatten index (Traces.ts:29) of every loaded span, as the
        run's results report them (kmz_get_global_index)."""
        out = np.zeros(max(1, self.n), np.uint64)
        L.check(self.ctx, self._lib.kmz_get_global_index(self.ctx, L.ptr(out), len(out), L.MEM_HOST))
        return out[: self.n]

    def set_triples(self, src_ptr: int, n: int, device: bool):
        """Replace the run's edge set with n keys (kmz_set_triples)."""
        self.gen += 1
        L.check(self.ctx, self._lib.kmz_set_triples(self.ctx, C.c_void_p(src_ptr) if n else None, n,
                                                    L.MEM_DEVICE if device else L.MEM_HOST))

    def set_index_map(self, local_start: np.ndarray, global_start: np.ndarray):
        """Local -> global flatten-index runs of a non-contiguous shard
        (kmz_set_index_map): results then report global indices."""
        self.gen += 1  # (clears the last run)
        ls = np.ascontiguousarray(local_start, dtype=np.uint64)
        gs = np.ascontiguousarray(global_start, dtype=np.uint64)
        if len(ls) != len(gs):
            raise ValueError("local_start and global_start differ in length")
        L.check(self.ctx, self._lib.kmz_set_index_map(self.ctx, L.ptr(ls), L.ptr(gs), len(ls)))
        self.index_base = 0

    # ---- compute -------------------------------------------------------------
    # every call that changes the device results bumps `gen`, so a result
    # object can tell whether the engine still holds its run
    gen = 0

    def run(self, flags: int):
        self.gen += 1
        L.check(self.ctx, self._lib.kmz_run(self.ctx, flags))

    def run_begin(self, flags: int):
        """``run`` in two halves (kmz_run_begin / _end): the run is enqueued
        here, the caller's host work between the two overlaps its kernels, and
        ``run_end`` waits for it.  No other engine call in between."""
        self.gen += 1
        L.check(self.ctx, self._lib.kmz_run_begin(self.ctx, flags))

    def run_end(self):
        L.check(self.ctx, self._lib.kmz_run_end(self.ctx))

    def sync(self):
        L.check(self.ctx, self._lib.kmz_sync(self.ctx))

    # ---- results -------------------------------------------------------------
    def info(self) -> dict:
        i = L.Info()
        L.check(self.ctx, self._lib.kmz_get_info(self.ctx, C.byref(i)))
        return {f: getattr(i, f) for f, _ in L.Info._fields_}

    def groups(self, copy: bool = True) -> np.ndarray:
        """Finalised groups; copy=False returns a view of a reused pinned buffer."""
        G = self.info()["n_groups"]
        out = self._pinned_array("groups", G, L.GROUP_DTYPE)
        L.check(self.ctx, self._lib.kmz_get_groups(self.ctx, L.ptr(out), G))
        return out.copy() if copy else out

    def endpoints(self) -> np.ndarray:
        out = np.zeros(self.n_dep_ep, dtype=L.ENDPOINT_DTYPE)
        L.check(self.ctx, self._lib.kmz_get_endpoints(self.ctx, L.ptr(out), self.n_dep_ep))
        return out

    def triples(self, sort: bool = True, copy: bool = True) -> np.ndarray:
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_get_triples(self.ctx, None, 0, C.byref(n)))  # no sync after a run
        out = self._pinned_array("triples", n.value, np.uint64)
        L.check(self.ctx, self._lib.kmz_get_triples(self.ctx, L.ptr(out), n.value, C.byref(n)))
        if copy or sort:
            out = out.copy()
        if sort:
            out.sort()
        return out

    def fetch(self, groups: bool = True, deps: bool = True, keys: bool = True):
        """All result sets of the last run with one stream synchronisation
        (kmz_fetch).  Returns (groups, triples, endpoints); groups and triples
        are views of reused pinned buffers (valid until the next fetch),
        triples unordered.  ``keys=False`` leaves the edge keys in HBM (a
        consumer on the device, e.g. kmz_tail_run, reads them there) and
        returns None for them."""
        info = self.info()  # the run's cached read-back: no device round trip
        keys = keys and deps
        g = self._pinned_array("groups", info["n_groups"], L.GROUP_DTYPE) if groups else None
        t = self._pinned_array("triples", info["n_triples"], np.uint64) if keys else None
        e = np.empty(self.n_dep_ep, dtype=L.ENDPOINT_DTYPE) if deps else None  # (kmz_fetch sets every entry)
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_fetch(self.ctx, L.ptr(g) if groups else None, len(g) if groups else 0,
                                              L.ptr(t) if keys else None, len(t) if keys else 0,
                                              C.byref(n) if deps else None, L.ptr(e) if deps else None,
                                              len(e) if deps else 0))
        return g, t, e

    def fetch_used(self, deps: bool = True, keys: bool = True):
        """``fetch`` with only the used groups (kmz_fetch_used): returns (ids,
        groups, triples, endpoints); ids[k] is groups[k]'s index in the dense
        array (ascending).  ids / groups / triples are views of reused pinned
        buffers, valid until the next fetch."""
        info = self.info()
        keys = keys and deps
        nu = C.c_uint64()
        G = info["n_groups"]  # (buffers for every group: one call, the count comes with the copies)
        ids = self._pinned_array("gids", G, np.uint32)
        g = self._pinned_array("gused", G, L.GROUP_DTYPE)
        t = self._pinned_array("triples", info["n_triples"], np.uint64) if keys else None
        e = np.empty(self.n_dep_ep, dtype=L.ENDPOINT_DTYPE) if deps else None
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_fetch_used(self.ctx, L.ptr(ids), L.ptr(g), len(g), C.byref(nu),
                                                   L.ptr(t) if keys else None, len(t) if keys else 0,
                                                   C.byref(n) if deps else None, L.ptr(e) if deps else None,
                                                   len(e) if deps else 0))
        return ids[: nu.value], g[: nu.value], t, e

    def fetch_begin(self, groups: bool = True, deps: bool = True, keys: bool = True):
        """First half of ``fetch`` for a loop over consecutive batches
        (kmz_fetch_begin): the results of the last run are copied on the
        device and queued to the host on a transfer stream, so the next run's
        kernels overlap the copies.  ``fetch_end()`` returns them.  The pinned
        buffers alternate between two sets: a result stays valid until the
        second fetch after it."""
        info = self.info()
        keys = keys and deps
        slot = self._fslot = getattr(self, "_fslot", 0) ^ 1
        g = self._pinned_array(f"groups{slot}", info["n_groups"], L.GROUP_DTYPE) if groups else None
        t = self._pinned_array(f"triples{slot}", info["n_triples"], np.uint64) if keys else None
        e = np.empty(self.n_dep_ep, dtype=L.ENDPOINT_DTYPE) if deps else None  # (set by kmz_fetch_end)
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_fetch_begin(self.ctx, L.ptr(g) if groups else None, len(g) if groups else 0,
                                                    L.ptr(t) if keys else None, len(t) if keys else 0,
                                                    C.byref(n) if deps else None, L.ptr(e) if deps else None,
                                                    len(e) if deps else 0))
        self._fopen = (g, t, e)
        return self._fopen

    def fetch_end(self):
        """-> (groups, triples, endpoints) of the open ``fetch_begin`` (None
        if none is open), after its copies have landed."""
        out = getattr(self, "_fopen", None)
        L.check(self.ctx, self._lib.kmz_fetch_end(self.ctx))
        self._fopen = None
        return out

    def span_links(self):
        cp = np.zeros(self.n, dtype=np.uint32)
        rp = np.zeros(self.n, dtype=np.uint64)
        L.check(self.ctx, self._lib.kmz_get_span_links(self.ctx, L.ptr(cp), L.ptr(rp), self.n))
        return cp, rp

    def dep_entries(self):
        """-> (entries DEP_ENTRY_DTYPE, row_ts int64[n_dep], row_shape uint32[n_dep]) of the last
        run with RUN_DEPS | RUN_DEP_ORDER (kmz_get_dep_entries)."""
        m = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_get_dep_entries(self.ctx, None, 0, C.byref(m), None, None, 0))
        out = np.zeros(m.value, dtype=L.DEP_ENTRY_DTYPE)
        rts = np.zeros(self.n_dep_ep, dtype=np.int64)
        rsh = np.zeros(self.n_dep_ep, dtype=np.uint32)
        L.check(self.ctx, self._lib.kmz_get_dep_entries(self.ctx, L.ptr(out), m.value, C.byref(m), L.ptr(rts),
                                                        L.ptr(rsh), self.n_dep_ep))
        return out, rts, rsh

    # ---- multi-GPU partials ----------------------------------------------------
    def group_partials_ptr(self):
        p, g = C.c_void_p(), C.c_uint64()
        L.check(self.ctx, self._lib.kmz_group_partials(self.ctx, C.byref(p), C.byref(g)))
        return p.value, g.value

    def endpoint_partials_ptr(self):
        p, e = C.c_void_p(), C.c_uint64()
        L.check(self.ctx, self._lib.kmz_endpoint_partials(self.ctx, C.byref(p), C.byref(e)))
        return p.value, e.value

    def partials_words(self, which: int) -> int:
        w = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_partials_size(self.ctx, which, C.byref(w)))
        return w.value

    def export_partials(self, which: int, dst_ptr: int, words: int, device: bool):
        L.check(self.ctx, self._lib.kmz_partials_copy(self.ctx, which, C.c_void_p(dst_ptr), words,
                                                      L.MEM_DEVICE if device else L.MEM_HOST, 0))

    def import_partials(self, which: int, src_ptr: int, words: int, device: bool):
        self.gen += 1
        L.check(self.ctx, self._lib.kmz_partials_copy(self.ctx, which, C.c_void_p(src_ptr), words,
                                                      L.MEM_DEVICE if device else L.MEM_HOST, 1))

    def finalize(self):
        self.gen += 1
        L.check(self.ctx, self._lib.kmz_finalize(self.ctx))

    def merge_triples(self, src_ptr: int, n: int, device: bool):
        """Union other shards' edge keys (u64, 0 = padding) into this run's set."""
        self.gen += 1
        L.check(self.ctx, self._lib.kmz_merge_triples(self.ctx, C.c_void_p(src_ptr), n,
                                                      L.MEM_DEVICE if device else L.MEM_HOST))

    # ---- multi-GPU sharding guard (kmz_guard.hip) -------------------------------
    def unresolved_parents(self, dst_ptr: int = 0, cap: int = 0, device: bool = False) -> int:
        """Count (and with dst_ptr, copy) the parent ids missing from this
        batch; raises KmzError(KMZ_E_UNSUPPORTED) on the span-table path."""
        n = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_unresolved_parents(self.ctx, C.c_void_p(dst_ptr) if dst_ptr else None, cap,
                                                           C.byref(n), L.MEM_DEVICE if device else L.MEM_HOST))
        return n.value

    def count_ids(self, src_ptr: int, n: int, device: bool) -> int:
        """How many of the given ids (0 = padding) are span ids of this batch."""
        f = C.c_uint64()
        L.check(self.ctx, self._lib.kmz_count_ids(self.ctx, C.c_void_p(src_ptr) if n else None, n,
                                                  L.MEM_DEVICE if device else L.MEM_HOST, C.byref(f)))
        return f.value

    def route_ids(self, world: int, dst_ptr: int, cap: int, device: bool) -> list:
        """This batch's span ids, hashed (the certificate's bijection) and
        grouped by owner rank (kmz_route_ids) into dst; -> counts per rank."""
        counts = np.zeros(max(1, world), np.uint64)
        L.check(self.ctx, self._lib.kmz_route_ids(self.ctx, world, C.c_void_p(dst_ptr) if dst_ptr else None, cap,
                                                  L.MEM_DEVICE if device else L.MEM_HOST, L.ptr(counts)))
        return [int(x) for x in counts[:world]]

    def route_ids_fixed(self, world: int, seg: int, dst_ptr: int, device: bool) -> None:
        """kmz_route_ids_fixed: ``world`` segments of ``seg`` words (count,
        then the values) at dst; with device memory only enqueued on the
        engine's stream (no host round trip)."""
        L.check(self.ctx, self._lib.kmz_route_ids_fixed(self.ctx, world, seg, C.c_void_p(dst_ptr),
                                                        L.MEM_DEVICE if device else L.MEM_HOST))

    def route_ids_join(self, world: int, seg: int, dst_ptr: int) -> None:
        """kmz_route_ids_join: the next run writes kmz_route_ids_fixed's
        segments (device memory at dst) from its join; nothing enqueued here."""
        L.check(self.ctx, self._lib.kmz_route_ids_join(self.ctx, world, seg, C.c_void_p(dst_ptr)))

    def route_wait(self, stream: int = 0) -> bool:
        """kmz_route_wait: ``stream`` (a hipStream_t handle; 0: the engine's)
        waits for the last run's routing.  -> whether the join wrote it."""
        j = C.c_int()
        L.check(self.ctx, self._lib.kmz_route_wait(self.ctx, C.c_void_p(stream) if stream else None, C.byref(j)))
        return bool(j.value)

    def id_repeats(self, src_ptr: int, n: int, device: bool) -> Optional[bool]:
        """Whether any of the n routed values occurs twice (kmz_id_repeats);
        None when the certificate cannot decide (the caller checks another way)."""
        r = C.c_uint32()
        rc = self._lib.kmz_id_repeats(self.ctx, C.c_void_p(src_ptr) if n else None, n,
                                      L.MEM_DEVICE if device else L.MEM_HOST, C.byref(r))
        if rc == L.E_UNSUPPORTED:
            return None
        L.check(self.ctx, rc)
        return bool(r.value)

    def id_repeats_seg_begin(self, segs_ptr: int, world: int, seg: int, stream: int = 0) -> None:
        """kmz_id_repeats_seg_begin: the certificate over ``world`` received
        fixed segments of ``seg`` words (device memory), enqueued on
        ``stream`` (a hipStream_t handle; 0: the engine's stream)."""
        L.check(self.ctx, self._lib.kmz_id_repeats_seg_begin(self.ctx, C.c_void_p(segs_ptr), world, seg,
                                                             C.c_void_p(stream) if stream else None))

    def id_repeats_seg_end(self):
        """-> (repeated: Optional[bool], max_count: int) (kmz_id_repeats_seg_end);
        repeated is None when the certificate cannot decide, and meaningless
        when max_count >= seg (a segment overflowed)."""
        r, m = C.c_uint32(), C.c_uint64()
        rc = self._lib.kmz_id_repeats_seg_end(self.ctx, C.byref(r), C.byref(m))
        if rc == L.E_UNSUPPORTED:
            return None, int(m.value)
        L.check(self.ctx, rc)
        return bool(r.value), int(m.value)

    def graph_stats(self):
        """(runs replayed from hipGraphs so far, graphs held) (kmz_get_graph_stats)."""
        n, k = C.c_uint64(), C.c_uint32()
        L.check(self.ctx, self._lib.kmz_get_graph_stats(self.ctx, C.byref(n), C.byref(k)))
        return int(n.value), int(k.value)

    # ---- RiskAnalyzer.RealtimeRisk's per-service sums (RiskAnalyzer.ts:18, 228-248)
    def set_service_map(self, sid_of_ep: np.ndarray, n_sid: int, is_5xx: np.ndarray):
        """Services of the stats endpoints (the groups' endpoint ids) and the
        5xx statuses, for ``service_sums`` (kmz_service_map_set; kept until
        replaced)."""
        sid = np.ascontiguousarray(sid_of_ep, dtype=np.uint32)
        m = np.ascontiguousarray(is_5xx, dtype=np.uint8)
        L.check(self.ctx, self._lib.kmz_service_map_set(self.ctx, L.ptr(sid), len(sid), int(n_sid), L.ptr(m), len(m)))
        self._n_sid = int(n_sid)

    def service_sums(self):
        """Per service over the finalised groups with combined > 0, on the
        device (kmz_service_sums): -> (order_ids, wsum, cnt, err) exactly as
        ``tail.service_sums`` returns them for the same rows: services in
        first-occurrence order, sum(cv * combined) added in ascending group
        order, sum(combined), sum(combined of 5xx)."""
        self.service_sums_begin()
        return self.service_sums_end()

    def service_sums_begin(self) -> None:
        """``service_sums`` enqueued only (kmz_service_sums_begin)."""
        L.check(self.ctx, self._lib.kmz_service_sums_begin(self.ctx))

    def service_sums_end(self):
        """Waits for ``service_sums_begin``'s sums: the same result as ``service_sums``."""
        out = np.empty(self._n_sid, dtype=L.SERVICE_SUM_DTYPE)
        L.check(self.ctx, self._lib.kmz_service_sums_end(self.ctx, L.ptr(out), len(out)))
        big = np.iinfo(np.uint64).max
        present = np.nonzero(out["first"] != big)[0]
        order = present[np.argsort(out["first"][present], kind="stable")]
        return order, out["wsum"][order], out["count"][order], out["err"][order]

    # ---- profiling -------------------------------------------------------------
    def set_profiling(self, on):
        """True / False: time every kernel id, or none.  A collection of
        names from ``_lib.KERNELS``: time only those (each timed id adds an
        event pair, i.e. launch gaps, to the run)."""
        if isinstance(on, bool) or on is None:
            L.check(self.ctx, self._lib.kmz_set_profiling(self.ctx, 1 if on else 0))
        else:
            mask = 0
            for k in on:
                mask |= 1 << L.KERNELS.index(k)
            L.check(self.ctx, self._lib.kmz_set_profiling_mask(self.ctx, mask))

    def kernel_times(self, reset: bool = False) -> dict:
        ms = np.zeros(len(L.KERNELS), dtype=np.float64)
        calls = np.zeros(len(L.KERNELS), dtype=np.uint64)
        L.check(self.ctx, self._lib.kmz_kernel_times(self.ctx, L.ptr(ms), L.ptr(calls), 1 if reset else 0))
        return {k: (float(ms[i]), int(calls[i])) for i, k in enumerate(L.KERNELS)}


def finalize_host(partials: np.ndarray, n_groups: int) -> np.ndarray:
    """Host finalisation of raw group partials (same arithmetic as the device)."""
    p = np.ascontiguousarray(partials, dtype=np.uint64)
    out = np.zeros(n_groups, dtype=L.GROUP_DTYPE)
    L.lib().kmz_finalize_host(L.ptr(p), n_groups, L.ptr(out))
    return out


def decode_triples(keys: np.ndarray):
    """key = anc_ep<<40 | desc_ep<<16 | distance<<1 | on  ->  column arrays."""
    k = np.asarray(keys, dtype=np.uint64)
    return (
        (k >> np.uint64(40)).astype(np.int64),
        ((k >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.int64),
        ((k >> np.uint64(1)) & np.uint64(0x7FFF)).astype(np.int64),
        (k & np.uint64(1)).astype(bool),
    )
