"""ctypes binding of ``include/kmz.h`` (libkmz.so, built in-tree).

The product path is the HIP engine: importing this module fails loudly when
``kmamiz_amd/libkmz.so`` is missing, and :func:`create` raises when no GPU is
visible.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkmz.so")
if os.environ.get("KMZ_LIB_VARIANT"):  # diagnostic A/B builds (tools/variant.sh): libkmz_<variant>.so, in-tree
    LIB_PATH = os.path.join(_HERE, "libkmz_%s.so" % os.environ["KMZ_LIB_VARIANT"])

KIND_OTHER, KIND_SERVER, KIND_CLIENT = 0, 1, 2
NONE32 = 0xFFFFFFFF
NONE64 = 0xFFFFFFFFFFFFFFFF

RUN_STATS_RT, RUN_STATS_TAG, RUN_DEPS, RUN_SPAN_LINKS, RUN_DEP_ORDER = 1, 2, 4, 8, 16
RUN_NO_CERT = 32  # the multi-GPU guard checks the ids (kmz.h KMZ_RUN_NO_CERT)
MEM_HOST, MEM_DEVICE = 0, 1

ERRORS = {
    -1: "KMZ_E_ARG",
    -2: "KMZ_E_HIP",
    -3: "KMZ_E_CYCLE",
    -4: "KMZ_E_ZERO_ID",
    -5: "KMZ_E_RANGE",
    -6: "KMZ_E_OVERFLOW",
    -7: "KMZ_E_STATE",
    -8: "KMZ_E_RCCL",
}

KERNELS = ["memset", "build", "fixup", "resolve", "stats", "walk", "final", "join", "cert", "reduce", "pend", "check",
           "settle", "tail", "order", "json", "joinwalk"]
SYNTH_BOOKINFO, SYNTH_MESH, SYNTH_POWER = 2, 3, 5
PART_GROUPS, PART_ENDPOINTS, PART_TRIPLES = 0, 1, 2


class KmzError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class CycleError(KmzError):
    """The reference loops forever on a cyclic parentId chain (Traces.ts:131-142)."""


class Spans(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("span_id", C.c_void_p),
        ("parent_id", C.c_void_p),
        ("kind", C.c_void_p),
        ("shape", C.c_void_p),
        ("status", C.c_void_p),
        ("duration", C.c_void_p),
        ("timestamp", C.c_void_p),
        ("index_base", C.c_uint64),
    ]


class Shapes(C.Structure):
    _fields_ = [
        ("n_shapes", C.c_uint32),
        ("rt_ep", C.c_void_p),
        ("tag_ep", C.c_void_p),
        ("dep_ep", C.c_void_p),
        ("n_rt_ep", C.c_uint32),
        ("n_tag_ep", C.c_uint32),
        ("n_dep_ep", C.c_uint32),
        ("n_status", C.c_uint32),
    ]


class Info(C.Structure):
    _fields_ = [
        ("n_spans", C.c_uint64),
        ("n_server", C.c_uint64),
        ("n_rows", C.c_uint64),
        ("n_relations", C.c_uint64),
        ("n_triples", C.c_uint64),
        ("n_dups", C.c_uint64),
        ("max_depth", C.c_uint64),
        ("n_groups", C.c_uint64),
        ("flags", C.c_uint32),
        ("path", C.c_uint32),
        ("n_chains", C.c_uint64),
    ]


class SynthDesc(C.Structure):
    _fields_ = [("n_shapes", C.c_uint32), ("n_status", C.c_uint32), ("n_endpoints", C.c_uint32)]


GROUP_DTYPE = np.dtype(
    [("combined", "<u8"), ("first", "<u8"), ("latest_timestamp", "<i8"), ("mean", "<f8"), ("cv", "<f8")]
)
ENDPOINT_DTYPE = np.dtype([("last_ts", "<i8"), ("first_row", "<u8"), ("external", "<u4"), ("has_row", "<u4")])
# kmz_dep_entry: one entry of the reduced graph with its order (kmz.h)
DEP_ENTRY_DTYPE = np.dtype([("key", "<u8"), ("row", "<u8"), ("span", "<u8"), ("pos", "<u8"), ("ts", "<i8"),
                            ("shape", "<u4"), ("pad", "<u4")])
TAIL_DETAIL_DTYPE = np.dtype([("svc", "<u4"), ("lsvc", "<u4"), ("distance", "<u4"), ("count", "<u4"),
                              ("depending_by", "<u4"), ("depending_on", "<u4")])
TAIL_PAIR_DTYPE = np.dtype([("svc", "<u4"), ("consumer", "<u4"), ("consumes", "<u4")])
SERVICE_SUM_DTYPE = np.dtype([("wsum", "<f8"), ("count", "<f8"), ("err", "<f8"), ("first", "<u8")])  # kmz_service_sum


class TailMap(C.Structure):
    _fields_ = [
        ("svc", C.c_void_p),
        ("cls", C.c_void_p),
        ("lsvc", C.c_void_p),
        ("n_ep", C.c_uint32),
        ("n_svc", C.c_uint32),
        ("n_cls", C.c_uint32),
        ("n_lsvc", C.c_uint32),
    ]


class ZipkinBatch(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("span_id", C.POINTER(C.c_uint64)),
        ("parent_id", C.POINTER(C.c_uint64)),
        ("kind", C.POINTER(C.c_uint8)),
        ("shape", C.POINTER(C.c_uint32)),
        ("status", C.POINTER(C.c_uint32)),
        ("duration", C.POINTER(C.c_uint32)),
        ("timestamp", C.POINTER(C.c_int64)),
        ("n_shapes", C.c_uint32),
        ("n_statuses", C.c_uint32),
        ("shape_fields", C.POINTER(C.c_uint64)),
        ("status_fields", C.POINTER(C.c_uint64)),
    ]


E_UNSUPPORTED = -9
JSON_ABSENT = 0xFFFFFFFFFFFFFFFF


# (name, restype, argtypes) for every symbol declared in include/kmz.h
_P = C.c_void_p
SIGNATURES = [
    ("kmz_abi_version", C.c_int, []),
    ("kmz_create", _P, [C.c_int, _P]),
    ("kmz_destroy", None, [_P]),
    ("kmz_last_error", C.c_char_p, [_P]),
    ("kmz_sync", C.c_int, [_P]),
    ("kmz_load", C.c_int, [_P, C.POINTER(Spans), C.POINTER(Shapes), C.c_int]),
    ("kmz_run", C.c_int, [_P, C.c_uint32]),
    ("kmz_run_begin", C.c_int, [_P, C.c_uint32]),
    ("kmz_run_end", C.c_int, [_P]),
    ("kmz_get_info", C.c_int, [_P, C.POINTER(Info)]),
    ("kmz_get_groups", C.c_int, [_P, _P, C.c_uint64]),
    ("kmz_get_endpoints", C.c_int, [_P, _P, C.c_uint64]),
    ("kmz_get_triples", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("kmz_get_span_links", C.c_int, [_P, _P, _P, C.c_uint64]),
    ("kmz_get_dep_entries", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_uint64), _P, _P, C.c_uint64]),
    ("kmz_get_spans", C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, C.c_uint64]),
    ("kmz_json_parse", C.c_int, [_P, _P, C.c_uint64, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint32)]),
    ("kmz_json_fields", C.c_int, [_P, _P, _P]),
    ("kmz_json_load", C.c_int, [_P, _P, _P, C.POINTER(Shapes), C.c_uint64]),
    ("kmz_json_known", C.c_int, [_P, _P, _P]),
    ("kmz_json_forget", C.c_int, [_P]),
    ("kmz_fetch", C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, C.POINTER(C.c_uint64), _P, C.c_uint64]),
    ("kmz_fetch_begin", C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, C.POINTER(C.c_uint64), _P, C.c_uint64]),
    ("kmz_fetch_used", C.c_int, [_P, _P, _P, C.c_uint64, C.POINTER(C.c_uint64), _P, C.c_uint64,
                                 C.POINTER(C.c_uint64), _P, C.c_uint64]),
    ("kmz_fetch_end", C.c_int, [_P]),
    ("kmz_group_partials", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    ("kmz_endpoint_partials", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    ("kmz_partials_size", C.c_int, [_P, C.c_int, C.POINTER(C.c_uint64)]),
    ("kmz_partials_copy", C.c_int, [_P, C.c_int, _P, C.c_uint64, C.c_int, C.c_int]),
    ("kmz_merge_triples", C.c_int, [_P, _P, C.c_uint64, C.c_int]),
    ("kmz_set_triples", C.c_int, [_P, _P, C.c_uint64, C.c_int]),
    ("kmz_parse_zipkin", C.c_int, [C.c_char_p, C.c_uint64, C.c_int, C.POINTER(C.POINTER(ZipkinBatch))]),
    ("kmz_zipkin_free", None, [C.POINTER(ZipkinBatch)]),
    ("kmz_unresolved_parents", C.c_int, [_P, _P, C.c_uint64, C.POINTER(C.c_uint64), C.c_int]),
    ("kmz_count_ids", C.c_int, [_P, _P, C.c_uint64, C.c_int, C.POINTER(C.c_uint64)]),
    ("kmz_route_ids", C.c_int, [_P, C.c_uint32, _P, C.c_uint64, C.c_int, _P]),
    ("kmz_route_ids_fixed", C.c_int, [_P, C.c_uint32, C.c_uint64, _P, C.c_int]),
    ("kmz_route_ids_join", C.c_int, [_P, C.c_uint32, C.c_uint64, _P]),
    ("kmz_route_wait", C.c_int, [_P, _P, C.POINTER(C.c_int)]),
    ("kmz_get_graph_stats", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    ("kmz_id_repeats", C.c_int, [_P, _P, C.c_uint64, C.c_int, C.POINTER(C.c_uint32)]),
    ("kmz_id_repeats_seg_begin", C.c_int, [_P, _P, C.c_uint32, C.c_uint64, _P]),
    ("kmz_id_repeats_seg_end", C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    ("kmz_trace_shard", C.c_uint32, [C.c_char_p, C.c_uint64, C.c_uint32]),
    ("kmz_set_index_map", C.c_int, [_P, _P, _P, C.c_uint64]),
    ("kmz_get_global_index", C.c_int, [_P, _P, C.c_uint64, C.c_int]),
    ("kmz_tail_map_set", C.c_int, [_P, C.POINTER(TailMap)]),
    ("kmz_tail_run", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("kmz_tail_begin", C.c_int, [_P]),
    ("kmz_tail_end", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("kmz_tail_get", C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, _P, C.c_uint64]),
    ("kmz_tail_service_stats", C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, C.POINTER(C.c_uint32)]),
    ("kmz_tail_service_first", C.c_int, [_P, _P, C.c_uint64]),
    ("kmz_service_map_set", C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, C.c_uint32]),
    ("kmz_service_sums", C.c_int, [_P, _P, C.c_uint64]),
    ("kmz_service_sums_begin", C.c_int, [_P]),
    ("kmz_service_sums_end", C.c_int, [_P, _P, C.c_uint64]),
    ("kmz_finalize", C.c_int, [_P]),
    ("kmz_finalize_host", None, [_P, C.c_uint64, _P]),
    ("kmz_host_exp", None, [_P, _P, C.c_uint64]),
    ("kmz_host_alloc", _P, [C.c_uint64]),
    ("kmz_host_free", None, [_P]),
    ("kmz_set_profiling", C.c_int, [_P, C.c_int]),
    ("kmz_set_profiling_mask", C.c_int, [_P, C.c_uint32]),
    ("kmz_kernel_times", C.c_int, [_P, _P, _P, C.c_int]),
    ("kmz_synth_describe", C.c_int, [C.c_int, C.POINTER(SynthDesc)]),
    ("kmz_synth_load", C.c_int, [_P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("kmz_synth_load_shard", C.c_int,
     [_P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]),
    (
        "kmz_synth_host",
        C.c_int,
        [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P, _P, _P, _P, _P, _P, _P, _P, C.POINTER(C.c_uint64)],
    ),
    ("kmz_synth_shape_ids", C.c_int, [C.c_int, _P, _P, _P, C.c_uint32]),
]

_lib = None


def lib():
    """Load libkmz.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build()) first")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def check(ctx, rc):
    if rc != 0:
        msg = lib().kmz_last_error(ctx).decode(errors="replace") if ctx else ""
        if rc == -3:
            raise CycleError(rc, msg)
        raise KmzError(rc, msg)
    return rc
