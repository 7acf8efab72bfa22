"""ctypes wrapper of oracle/_build/libkmz_oracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this.  See kmz_oracle.c for what it restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "_build", "libkmz_oracle.so")
SO_OMP = os.path.join(_HERE, "_build", "libkmz_cpu_omp.so")
_lib = None
_omp = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = C.CDLL(SO)
        P = C.c_void_p
        L.oracle_stats.restype = C.c_int
        L.oracle_stats.argtypes = [C.c_uint64, P, P, P, P, P, P, C.c_uint32, C.c_uint32, P, P, P, P, P]
        L.oracle_deps.restype = C.c_int
        L.oracle_deps.argtypes = [C.c_uint64, P, P, P, P, P, P, C.c_uint32, C.c_uint64, P, P, P, P, P, P]
        L.oracle_dep_entries.restype = C.c_int
        L.oracle_dep_entries.argtypes = [C.c_uint64, P, P, P, P, P, P, C.c_uint32, C.c_uint64, P, P, P, P]
        L.oracle_to_precise.restype = C.c_double
        L.oracle_to_precise.argtypes = [C.c_double]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def stats(batch, ep_of_shape: np.ndarray, n_ep: int, n_status: int):
    """-> dict of dense per-group arrays (sequential Welford, JS order)."""
    G = n_ep * n_status
    out = dict(
        combined=np.zeros(G, np.uint64),
        mean=np.zeros(G, np.float64),
        cv=np.zeros(G, np.float64),
        latest_timestamp=np.zeros(G, np.int64),
        first=np.zeros(G, np.uint64),
    )
    ep = np.ascontiguousarray(ep_of_shape, dtype=np.uint32)
    rc = lib().oracle_stats(
        len(batch), _p(batch.kind), _p(batch.shape), _p(batch.status), _p(batch.duration), _p(batch.timestamp),
        _p(ep), n_ep, n_status, _p(out["combined"]), _p(out["mean"]), _p(out["cv"]), _p(out["latest_timestamp"]),
        _p(out["first"]),
    )
    assert rc == 0
    used = out["first"] != np.uint64(0xFFFFFFFFFFFFFFFF)
    out["first"] = np.where(used, out["first"] + np.uint64(batch.index_base), out["first"])
    return out


def deps(batch, dep_ep: np.ndarray, n_ep: int):
    """-> (sorted unique edge keys, per-endpoint dict, counts dict)."""
    n = len(batch)
    cap = max(16, 2 * n + 16)
    keys = np.zeros(cap, np.uint64)
    nk = C.c_uint64()
    last = np.zeros(max(1, n_ep), np.float64)
    first = np.zeros(max(1, n_ep), np.uint64)
    ext = np.zeros(max(1, n_ep), np.uint8)
    counts = np.zeros(4, np.uint64)
    ep = np.ascontiguousarray(dep_ep, dtype=np.uint32)
    rc = lib().oracle_deps(
        n, _p(batch.span_id), _p(batch.parent_id), _p(batch.kind), _p(batch.shape), _p(batch.timestamp), _p(ep),
        n_ep, cap, _p(keys), C.byref(nk), _p(last), _p(first), _p(ext), _p(counts),
    )
    if rc == -4:  # more unique keys than 2n (deep chains): once more with the size it reported
        cap = nk.value
        keys = np.zeros(cap, np.uint64)
        last[:] = 0
        first[:] = 0
        ext[:] = 0
        counts[:] = 0
        rc = lib().oracle_deps(
            n, _p(batch.span_id), _p(batch.parent_id), _p(batch.kind), _p(batch.shape), _p(batch.timestamp), _p(ep),
            n_ep, cap, _p(keys), C.byref(nk), _p(last), _p(first), _p(ext), _p(counts),
        )
    if rc == -3:
        raise RuntimeError("cyclic parent chain")
    assert rc == 0, rc
    has = first != np.uint64(0xFFFFFFFFFFFFFFFF)
    first = np.where(has, first + np.uint64(batch.index_base), first)
    return (
        keys[: nk.value].copy(),
        dict(last=last[:n_ep], first=first[:n_ep], external=ext[:n_ep].astype(bool), has_row=has[:n_ep]),
        dict(rows=int(counts[0]), relations=int(counts[1]), max_depth=int(counts[2]), keys=int(counts[3])),
    )


ENTRY_DTYPE = np.dtype([("key", "<u8"), ("row", "<u8"), ("span", "<u8"), ("pos", "<u8"), ("ts", "<i8"),
                        ("shape", "<u4"), ("pad", "<u4")])


def dep_entries(batch, dep_ep: np.ndarray, n_ep: int):
    """oracle_dep_entries: the entry records of the reduced graph
    EndpointDependencies([]).combineWith(deps).trim(), sorted by key, plus the
    (timestamp, shape) of each endpoint's first row.  Indices are global."""
    n = len(batch)
    ep = np.ascontiguousarray(dep_ep, dtype=np.uint32)
    row_ts = np.zeros(max(1, n_ep), np.int64)
    row_shape = np.zeros(max(1, n_ep), np.uint32)
    cap = max(64, n // 4)
    while True:
        out = np.zeros(cap, ENTRY_DTYPE)
        m = C.c_uint64()
        rc = lib().oracle_dep_entries(
            n, _p(batch.span_id), _p(batch.parent_id), _p(batch.kind), _p(batch.shape), _p(batch.timestamp), _p(ep),
            n_ep, cap, _p(out), C.byref(m), _p(row_ts), _p(row_shape),
        )
        if rc == -4:
            cap = m.value
            continue
        if rc == -3:
            raise RuntimeError("cyclic parent chain")
        assert rc == 0, rc
        break
    out = out[: m.value]
    base = np.uint64(batch.index_base)
    for f in ("row", "span", "pos"):
        out[f] += base
    out = out[np.argsort(out["key"], kind="stable")]
    return out, row_ts[:n_ep], row_shape[:n_ep]


# ---- all-core OpenMP restatement (kmz_cpu_omp.c): the bench's cpu_baseline ----
def omp_lib():
    global _omp
    if _omp is None:
        if not os.path.exists(SO_OMP):
            build()
        L = C.CDLL(SO_OMP)
        P = C.c_void_p
        L.omp_stats.restype = C.c_int
        L.omp_stats.argtypes = [C.c_uint64, P, P, P, P, P, P, C.c_uint32, C.c_uint32, P, P, P, P, P]
        L.omp_deps.restype = C.c_int
        L.omp_deps.argtypes = [C.c_uint64, P, P, P, P, P, P, C.c_uint32, C.c_uint64, P, P, P, P, P, P]
        L.omp_threads.restype = C.c_int
        _omp = L
    return _omp


def omp_threads() -> int:
    return int(omp_lib().omp_threads())


def omp_stats(batch, ep_of_shape: np.ndarray, n_ep: int, n_status: int):
    """Same outputs as stats() (exact integer moments, 1e-9 of the Welford)."""
    G = n_ep * n_status
    out = dict(combined=np.zeros(G, np.uint64), mean=np.zeros(G, np.float64), cv=np.zeros(G, np.float64),
               latest_timestamp=np.zeros(G, np.int64), first=np.zeros(G, np.uint64))
    ep = np.ascontiguousarray(ep_of_shape, dtype=np.uint32)
    rc = omp_lib().omp_stats(
        len(batch), _p(batch.kind), _p(batch.shape), _p(batch.status), _p(batch.duration), _p(batch.timestamp),
        _p(ep), n_ep, n_status, _p(out["combined"]), _p(out["mean"]), _p(out["cv"]), _p(out["latest_timestamp"]),
        _p(out["first"]),
    )
    assert rc == 0
    used = out["first"] != np.uint64(0xFFFFFFFFFFFFFFFF)
    out["first"] = np.where(used, out["first"] + np.uint64(batch.index_base), out["first"])
    return out


def omp_deps(batch, dep_ep: np.ndarray, n_ep: int):
    """Same outputs as deps() for batches with unique span ids (-2: repeated id)."""
    n = len(batch)
    nk = C.c_uint64()
    last = np.zeros(max(1, n_ep), np.float64)
    first = np.zeros(max(1, n_ep), np.uint64)
    ext = np.zeros(max(1, n_ep), np.uint8)
    counts = np.zeros(4, np.uint64)
    ep = np.ascontiguousarray(dep_ep, dtype=np.uint32)
    args = (n, _p(batch.span_id), _p(batch.parent_id), _p(batch.kind), _p(batch.shape), _p(batch.timestamp), _p(ep),
            n_ep)
    rc = omp_lib().omp_deps(*args, 0, None, C.byref(nk), _p(last), _p(first), _p(ext), _p(counts))
    if rc == -2:
        raise ValueError("repeated span ids: use the sequential oracle")
    assert rc == 0, rc
    keys = np.zeros(max(1, nk.value), np.uint64)
    rc = omp_lib().omp_deps(*args, nk.value, _p(keys), C.byref(nk), _p(last), _p(first), _p(ext), _p(counts))
    assert rc == 0, rc
    has = first != np.uint64(0xFFFFFFFFFFFFFFFF)
    first = np.where(has, first + np.uint64(batch.index_base), first)
    return (
        keys[: nk.value].copy(),
        dict(last=last[:n_ep], first=first[:n_ep], external=ext[:n_ep].astype(bool), has_row=has[:n_ep]),
        dict(rows=int(counts[0]), relations=int(counts[1]), max_depth=int(counts[2]), keys=int(counts[3])),
    )
