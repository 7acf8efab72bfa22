"""kmamiz_amd -- MI355X-native engine for KMamiz's trace-processing hot path.

Zipkin spans -> realtime data -> (endpoint x status) combined stats + endpoint
dependency graph, as HIP kernels for gfx950 behind the C ABI in
``include/kmz.h`` (``libkmz.so``).  The classes mirror the reference's
TypeScript API (src/classes/*.ts) so callers switch by import.
"""
from ._lib import KmzError, CycleError  # noqa: F401
from .engine import Engine, SpanBatch, ShapeTable, finalize_host, decode_triples  # noqa: F401
from .classes import (  # noqa: F401
    Traces,
    RealtimeDataList,
    CombinedRealtimeDataList,
    EndpointDependencies,
    default_engine,
)

__all__ = [
    "Engine",
    "SpanBatch",
    "ShapeTable",
    "Traces",
    "RealtimeDataList",
    "CombinedRealtimeDataList",
    "EndpointDependencies",
    "KmzError",
    "CycleError",
    "finalize_host",
    "decode_triples",
    "default_engine",
]
