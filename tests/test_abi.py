"""The C ABI library loads and exports every symbol include/kmz.h declares
(no compute without a GPU), plus the host-only entry points."""
import ctypes as C
import os
import re

import numpy as np

from conftest import ROOT


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "kmz.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kmz_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported_and_bound():
    from kmamiz_amd import _lib

    L = _lib.lib()
    decl = declared_symbols()
    assert len(decl) >= 20
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for name in decl:
        assert hasattr(L, name), name  # exported by libkmz.so
        assert name in bound, name  # and bound with a signature
    assert L.kmz_abi_version() == 1


def test_library_is_the_in_tree_hip_build():
    from kmamiz_amd import _lib

    assert os.path.dirname(_lib.LIB_PATH) == os.path.join(ROOT, "kmamiz_amd")
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob  # a gfx950 code object is embedded


def test_structs_match_header():
    from kmamiz_amd import _lib

    assert C.sizeof(_lib.Spans) == 8 * 9
    assert C.sizeof(_lib.Shapes) == 4 + 4 + 8 * 3 + 4 * 4 + 0  # padded as the C struct
    assert _lib.GROUP_DTYPE.itemsize == 40
    assert _lib.ENDPOINT_DTYPE.itemsize == 24


def test_finalize_host_matches_welford():
    """Exact integer moments -> (mean, cv) within 1e-9 of the sequential Welford."""
    from kmamiz_amd import finalize_host
    from oracle import kmz_oracle as O

    rng = np.random.default_rng(1)
    for trial in range(200):
        n = int(rng.integers(1, 300))
        d = rng.integers(0, 10**7 if trial % 3 else 100, size=n).astype(np.uint64)
        if trial % 17 == 0:
            d[:] = d[0]  # zero variance
        dd = d * d
        part = np.array(
            [n, int(d.sum()), int((dd & np.uint64(0xFFFFFFFF)).sum()), int((dd >> np.uint64(32)).sum()),
             (1 << 63) + 5, 0],
            dtype=np.uint64,
        )
        g = finalize_host(part, 1)[0]
        mean, cv = O.welford_mean_cv([float(x) / 1000 for x in d])
        assert g["combined"] == n and g["latest_timestamp"] == 5
        assert g["mean"] == (O.to_precise(mean) if mean == 0 else g["mean"])
        assert abs(g["mean"] - O.to_precise(mean)) <= 1e-9 * abs(mean) + 1e-14
        assert abs(g["cv"] - O.to_precise(cv)) <= 1e-9 * abs(cv) + 1e-13


def test_create_without_gpu_returns_null_or_ctx():
    from conftest import have_gpu
    from kmamiz_amd import _lib

    ctx = _lib.lib().kmz_create(0, None)
    assert bool(ctx) == have_gpu()
    if ctx:
        _lib.lib().kmz_destroy(ctx)


def test_synthetic_host_generator_deterministic():
    from kmamiz_amd import synth

    a, off_a = synth.host_batch(synth.MESH, 10, 60)
    b, off_b = synth.host_batch(synth.MESH, 10, 60)
    assert a.span_id.tobytes() == b.span_id.tobytes() and a.index_base == b.index_base
    full, off = synth.host_batch(synth.MESH, 0, 60)
    k = int(off[10])
    assert np.array_equal(full.span_id[k:], a.span_id) and a.index_base == k
    assert len(np.unique(full.span_id)) == len(full)  # unique ids
    # every SERVER has a CLIENT parent in its trace, roots are CLIENT
    kinds = dict(zip(full.span_id.tolist(), full.kind.tolist()))
    srv = full.kind == 1
    assert all(kinds[p] == 2 for p in full.parent_id[srv].tolist())
    assert np.all(full.kind[full.parent_id == 0] == 2)


def test_host_exp_is_math_exp():
    """kmz_host_exp (the risk finish's SigmoidAdj exponentials in one call)
    returns Python's math.exp bit for bit: both are the C library's exp."""
    import math

    from kmamiz_amd import _lib

    rng = np.random.default_rng(7)
    x = np.concatenate([rng.normal(0, 3, 4000), rng.uniform(-700, 700, 4000),
                        [0.0, -0.0, 1e-300, -745.2, 709.7, math.inf, -math.inf, math.nan]])
    out = np.empty_like(x)
    _lib.lib().kmz_host_exp(_lib.ptr(x), _lib.ptr(out), len(x))
    ref = np.array([math.inf if v > 709.78 else math.exp(v) for v in x.tolist()])  # (math.exp raises on overflow)
    fin = ~np.isnan(ref)
    assert np.array_equal(np.isnan(out), ~fin)
    assert np.array_equal(out[fin].view(np.uint64), ref[fin].view(np.uint64))
