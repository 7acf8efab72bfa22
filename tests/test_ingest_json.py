"""Native Zipkin JSON ingest (kmz_parse_zipkin) against the
general path (json.loads + ingest.ingest_traces): same columns, same shapes
and statuses (compared by content), same fallbacks.  Host only."""
import json
import os

import numpy as np
import pytest

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _fixture(name):
    t = json.load(open(os.path.join(FIX, f"{name}.json")))
    return t if name == "MockTrace" else [t]


def _same(traces, threads=0):
    from kmamiz_amd.ingest import ingest_json, ingest_traces

    data = json.dumps(traces).encode()
    r = ingest_json(data, threads=threads)
    assert r is not None
    b1, d1 = r
    b2, d2, _ = ingest_traces(traces)
    for f in ("span_id", "parent_id", "kind", "duration", "timestamp"):
        assert np.array_equal(getattr(b1, f), getattr(b2, f)), f
    assert [d1.shapes[i] for i in b1.shape] == [d2.shapes[i] for i in b2.shape]
    assert [d1.statuses[i] for i in b1.status] == [d2.statuses[i] for i in b2.status]
    return b1, d1


@pytest.mark.parametrize("fx", ["MockTracePDAS", "MockTrace", "MockData2_traces"])
def test_fixture_json_matches_general_ingest(fx):
    _same(_fixture(fx))


@pytest.mark.parametrize("config", [2, 3, 5])
def test_synthetic_json_matches_general_ingest(config):
    from kmamiz_amd import synth

    batch, off = synth.host_batch(config, 0, 300)
    _same(synth.to_traces(config, batch, off))


def test_threads_give_the_same_batch():
    """Per-thread interning tables merge in first-occurrence order."""
    from kmamiz_amd import synth
    from kmamiz_amd.ingest import ingest_json

    batch, off = synth.host_batch(3, 0, 3000)
    data = json.dumps(synth.to_traces(3, batch, off)).encode()
    b1, d1 = ingest_json(data, threads=1)
    b8, d8 = ingest_json(data, threads=8)
    for f in ("span_id", "parent_id", "kind", "shape", "status", "duration", "timestamp"):
        assert np.array_equal(getattr(b1, f), getattr(b8, f)), f
    assert d1.shapes == d8.shapes and d1.statuses == d8.statuses
    assert np.array_equal(b1.span_id, batch.span_id) and np.array_equal(b1.timestamp, batch.timestamp)


@pytest.mark.parametrize("mutate", ["upper_id", "float_duration", "escaped_key", "string_tags", "zero_parent",
                                    "missing_id", "not_nested"])
def test_outside_the_fast_path_falls_back(mutate):
    from kmamiz_amd.ingest import ingest_json

    t = _fixture("MockTracePDAS")
    s = t[0][1]
    if mutate == "upper_id":
        s["id"] = s["id"].upper() if any(c.isalpha() for c in s["id"]) else "ABCDEF0123456789"
    elif mutate == "float_duration":
        s["duration"] = 1.5
    elif mutate == "escaped_key":
        data = json.dumps(t).replace('"kind"', '"\\u006bind"', 1).encode()
        assert ingest_json(data) is None
        return
    elif mutate == "string_tags":
        s["tags"] = "x"
    elif mutate == "zero_parent":
        s["parentId"] = "0" * 16
    elif mutate == "missing_id":
        del s["id"]
    elif mutate == "not_nested":
        t = t[0]
    assert ingest_json(json.dumps(t).encode()) is None


def test_falsy_parents_and_null_tags():
    t = _fixture("MockTracePDAS")
    t[0][0]["parentId"] = ""
    t[0][1]["tags"] = None
    t[0][2].pop("parentId", None)
    _same(t)


def test_escaped_values_and_pretty_printing():
    """Values are interned by raw text and decoded per shape: an escaped and a
    plain spelling of the same name are one shape after decoding."""
    from kmamiz_amd.ingest import ingest_json, ingest_traces

    t = _fixture("MockTracePDAS")
    data = json.dumps(t, indent=2).replace('/', '\\/').encode()  # "\/" decodes to "/"
    b1, d1 = ingest_json(data)
    b2, d2, _ = ingest_traces(t)
    assert [d1.shapes[i] for i in b1.shape] == [d2.shapes[i] for i in b2.shape]
    assert np.array_equal(b1.span_id, b2.span_id)
    t[0][0]["name"] = 'say "hi"\\n'
    _same(t)


@pytest.mark.parametrize("text", [b"[]", b" [ ] \n", b"[[]]", b"[[], []]"])
def test_empty_batches(text):
    from kmamiz_amd.ingest import ingest_json

    b, d = ingest_json(text, threads=4)
    assert len(b.span_id) == 0


def test_split_inside_a_string_reparses():
    """Byte splits land in a tag value full of the trace-boundary pattern; the
    range before a split never lands on it, so the batch is parsed on one
    thread and equals the general path."""
    from kmamiz_amd import synth

    batch, off = synth.host_batch(2, 0, 200)
    traces = synth.to_traces(2, batch, off)
    traces[len(traces) // 2][0]["tags"]["x"] = "]], [[" * 600_000  # ~3.6 MB
    _same(traces, threads=8)
