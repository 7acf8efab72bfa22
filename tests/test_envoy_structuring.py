"""the Envoy-log pipeline in front of
Traces.combineLogsToRealtimeData, and the JSON bodies it carries.

* KubernetesService.ParseEnvoyLogs (KubernetesService.ts:201-242) on the
  reference's own raw lines (MockLogsPDAS, tests/EnvoyLog.test.ts:4-15);
* EnvoyLogs.toStructured / toStructuredFallback / CombineToStructuredEnvoyLogs
  / FillMissingId (EnvoyLog.ts:17-149) vs the oracle on randomized logs;
* Utils.MergeStringBody / Merge / ObjectToInterfaceString (Utils.ts:14-75,
  279-309), JSON.parse / JSON.stringify semantics;
* combined rows with application/json bodies (RealtimeDataList.ts:53-89,
  120-155) on the GPU vs the oracle, and the cache merge of bodies
  (CombinedRealtimeDataList.ts:204-226) vs the reference's golden
  (CombinedRealtimeDataList.test.ts:25-31).

json-to-ts (package.json "^1.7.0") is absent: its single-interface outputs
fixed by tests/Utils.test.ts are restated; nested shapes go through a hook,
here a stand-in shared by the product and the oracle (parity unpinned).
"""
import copy
import json
import random

import pytest

from conftest import fixture
from oracle import kmz_oracle as O


def _stand_in(obj, root):
    return ["__ts__%s:%s" % (root, json.dumps(obj, sort_keys=True, ensure_ascii=False))]


@pytest.fixture
def ts_hook():
    from kmamiz_amd import envoy

    envoy.set_json_to_ts(_stand_in)
    O.JSON_TO_TS = _stand_in
    yield
    envoy.set_json_to_ts(None)
    O.JSON_TO_TS = None


def _plain(logs):
    """EnvoyLogs JSON with Dates as getTime() (both sides' Date stand-ins)."""
    def conv(v):
        if hasattr(v, "getTime"):
            t = v.getTime()
            return ("date", None if t != t else t)
        if isinstance(v, dict):
            return {k: conv(x) for k, x in v.items()}
        if isinstance(v, list):
            return [conv(x) for x in v]
        return v

    return conv(O.strip_undef(logs))


def test_parse_envoy_logs_reference_lines():
    from kmamiz_amd.envoy import ParseEnvoyLogs

    lines = fixture("MockLogsPDAS")
    logs = ParseEnvoyLogs(lines, "pdas", "user-service")
    assert len(logs.toJSON()) == len(lines)  # EnvoyLog.test.ts:11-13
    assert logs.toStructured()
    exp = O.parse_envoy_logs(lines, "pdas", "user-service")
    assert _plain(logs.toJSON()) == _plain(exp.toJSON())
    assert _plain(logs.toStructured()) == _plain(exp.toStructured())
    first = logs.toJSON()[0]
    assert first["timestamp"].getTime() == 1646208338224  # "...38.224642Z" truncated to ms, as V8
    assert first["method"] == "GET" and first["path"].startswith("user-service.pdas")
    assert logs.toJSON()[1]["contentType"] == "application/json" and logs.toJSON()[1]["body"].startswith('{"id"')


def test_envoy_log_lines():
    from kmamiz_amd.envoy import envoy_log_lines

    raw = ("2022-03-02T08:05:38.224642Z\twarning\tenvoy lua\tscript log: [Request a-b/t1/s1/p1] [GET x/y]\n"
           "2022-03-02T08:05:38.3Z\tinfo\tenvoy wasm\twasm log kmamiz: [Response a-b/t1/s2/s1] [Status] 200\n"
           "2022-03-02T08:05:39Z\tinfo\tsomething else\n")
    assert envoy_log_lines(raw) == ["2022-03-02T08:05:38.224642Z\t[Request a-b/t1/s1/p1] [GET x/y]",
                                    "2022-03-02T08:05:38.3Z\t[Response a-b/t1/s2/s1] [Status] 200"]


def _random_lines(rng, n_req=6, fallback=False):
    out = []
    for r in range(n_req):
        rid = f"req-{r}"
        tid = "NO_ID" if fallback and rng.random() < 0.5 else f"{rng.getrandbits(64):016x}"
        stack = []
        for k in range(rng.randint(1, 6)):
            sid = "NO_ID" if fallback and rng.random() < 0.3 else f"{rng.getrandbits(64):016x}"
            par = stack[-1] if stack and rng.random() < 0.7 else f"{rng.getrandbits(64):016x}"
            t = f"2022-03-02T08:05:{10 + k:02d}.{rng.randint(0, 999999):06d}Z"
            if rng.random() < 0.6:
                body = rng.choice(['{"a":1}', '{"b":"x","a":2}', "[1,2]", "plain"])
                out.append(f"{t}\t[Request {rid}/{tid}/{sid}/{par}] [POST svc.ns/api] [ContentType application/json]"
                           f" [Body] {body}")
                stack.append(sid)
            else:
                resp_of = stack.pop() if stack and rng.random() < 0.8 else sid
                out.append(f"{t}\t[Response {rid}/{tid}/{sid}/{resp_of}] [Status] {rng.choice([200, 404])}"
                           f" [ContentType text/plain] [Body] ok{k}")
    rng.shuffle(out)
    return out


@pytest.mark.parametrize("seed", range(12))
def test_structured_logs_vs_oracle(seed):
    from kmamiz_amd.envoy import EnvoyLogs, ParseEnvoyLogs

    rng = random.Random(seed)
    pods = [_random_lines(rng, fallback=seed % 3 == 0) for _ in range(3)]
    ours = EnvoyLogs.CombineToStructuredEnvoyLogs([ParseEnvoyLogs(p, "ns", f"pod{i}") for i, p in enumerate(pods)])
    ref = O.EnvoyLogs.CombineToStructuredEnvoyLogs([O.parse_envoy_logs(p, "ns", f"pod{i}")
                                                    for i, p in enumerate(pods)])
    assert _plain(ours) == _plain(ref)


def test_sort_with_one_argument_comparator():
    """traces.sort((t) => t.request.timestamp.getTime()) under V8's TimSort:
    only elements with a negative request time move."""
    from kmamiz_amd.envoy import JSDate, _sort_by_request_time

    def tr(ts, i):
        return {"i": i, "request": {"timestamp": JSDate(ts)}}

    a = [tr("2022-01-01T00:00:00Z", 0), tr("bad", 1), tr("2021-01-01T00:00:00Z", 2)]
    assert [x["i"] for x in _sort_by_request_time(list(a))] == [0, 1, 2]
    b = [tr("1960-01-01T00:00:00Z", 0), tr("1950-01-01T00:00:00Z", 1), tr("2022-01-01T00:00:00Z", 2),
         tr("1940-01-01T00:00:00Z", 3)]
    # descending run [0, 1] reversed, then 2 stays, 3 is inserted at the front
    assert [x["i"] for x in _sort_by_request_time(list(b))] == [3, 1, 0, 2]


def test_merge_string_body_and_json_semantics():
    from kmamiz_amd.envoy import js_json_parse, js_json_stringify, js_number_str, merge, merge_string_body
    from kmamiz_amd.ingest import UNDEFINED

    assert merge_string_body('{"a":1}', '{"b":2}') == '{"a":1,"b":2}'
    assert merge_string_body('{"a":1}', "nope") == '{"a":1}'
    assert merge_string_body("nope", "nah") is UNDEFINED  # JSON.stringify(undefined)
    assert merge_string_body("0", '{"x":1}') == '{"x":1}'  # parsed 0 is falsy
    assert merge_string_body("[1,2]", "[3]") == "[1,2,3]"
    assert merge_string_body(UNDEFINED, "abc") == "abc"
    assert merge_string_body("", "abc") == "abc"
    assert merge_string_body('"ab"', '{"z":1}') == '{"0":"a","1":"b","z":1}'  # string spread
    assert merge([1] * 12, [2] * 12) == [1] * 10 + [2] * 10
    assert merge(UNDEFINED, UNDEFINED) == {}
    assert js_json_stringify({"b": 1, "2": 0, "1": 0, "a": [1.5, None, "é\n"]}) == '{"1":0,"2":0,"b":1,"a":[1.5,null,"é\\n"]}'
    assert js_number_str(1e21) == "1e+21" and js_number_str(1e20) == "100000000000000000000"
    assert js_number_str(1e-7) == "1e-7" and js_number_str(0.000001) == "0.000001"
    assert js_json_parse("12345678901234567891") == 12345678901234567000.0
    with pytest.raises(ValueError):
        js_json_parse("NaN")
    for a, b in [('{"a":1}', '{"a":2,"c":[1]}'), ("[1]", "[2,3]"), ('"s"', "1"), ("null", '{"a":1}')]:
        assert merge_string_body(a, b) == O.merge_string_body(a, b) or json.loads(merge_string_body(a, b)) == \
            json.loads(O.merge_string_body(a, b))


def test_object_to_interface_string_golden():
    """tests/Utils.test.ts:32-69 (the array vector; the nested one needs
    json-to-ts's naming of nested interfaces, which is not restated)."""
    from kmamiz_amd.envoy import object_to_interface_string

    array = [
        {"id": "61d58fabd7cb2766e01db3c6", "originId": None, "ordinaryUserName": None,
         "dataRequesterName": "新創公司A", "dataHolderName": "台灣電力公司", "firstSignDate": 0,
         "secondSignDate": 0, "signState": 0},
        {"id": "61d58facd7cb2766e01db7b0", "originId": None, "ordinaryUserName": None,
         "dataRequesterName": "新創公司A", "dataHolderName": "台灣電力公司", "firstSignDate": 0,
         "secondSignDate": 0, "signState": -3},
    ]
    exp = ("interface ObjArray extends Array<ArrayItem>{}\n" "interface ArrayItem {\n"
           "  dataHolderName: string;\n" "  dataRequesterName: string;\n" "  firstSignDate: number;\n"
           "  id: string;\n" "  ordinaryUserName?: any;\n" "  originId?: any;\n" "  secondSignDate: number;\n"
           "  signState: number;\n" "}")
    assert object_to_interface_string(array, "ObjArray") == exp
    assert O.object_to_interface_string(array, "ObjArray") == exp
    assert object_to_interface_string(5) == "number" and object_to_interface_string(None) == "object"
    assert object_to_interface_string([1, "a"]) == "interface Root extends Array<number>{}"
    assert object_to_interface_string([]) == "interface Root extends Array<any>{}"
    with pytest.raises(NotImplementedError):
        object_to_interface_string({"nested": {"a": 1}})


def _resolve_markers(v):
    """The fixtures' schema strings were extracted with ObjectToInterfaceString
    stubbed as "__schema__" + JSON (tests/golden/extract_mockdata.py)."""
    from kmamiz_amd.envoy import object_to_interface_string

    if isinstance(v, dict):
        return {k: _resolve_markers(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_resolve_markers(x) for x in v]
    if isinstance(v, str) and v.startswith("__schema__"):
        return object_to_interface_string(json.loads(v[len("__schema__"):]))
    return v


def test_combined_merge_golden_with_bodies():
    """CombinedRealtimeDataList.test.ts:25-31: the whole row, bodies and
    schemas included (MockData.ts:4480-4560)."""
    from kmamiz_amd import CombinedRealtimeDataList
    from kmamiz_amd.cache import CombinedColumns

    a = _resolve_markers(fixture("MockBaseCrlData1"))
    b = _resolve_markers(fixture("MockBaseCrlData2"))
    exp = _resolve_markers(fixture("MockCombinedBaseData"))
    got = CombinedRealtimeDataList(copy.deepcopy(a)).combineWith(CombinedRealtimeDataList(copy.deepcopy(b))).toJSON()
    assert got == exp
    orc = O.CombinedRealtimeDataList(copy.deepcopy(a)).combineWith(O.CombinedRealtimeDataList(copy.deepcopy(b)))
    assert O.strip_undef(orc.toJSON()) == exp
    cols = CombinedColumns.from_json(copy.deepcopy(a)).combineWith(CombinedColumns.from_json(copy.deepcopy(b)))
    assert cols.toJSON() == exp


JSON_BODIES = ['{"a":1,"b":"x"}', '{"a":2}', '[{"k":1},{"k":2}]', "[1,2,3]", "0", "null", '"str"', "not json",
               '{"n":{"deep":1}}', "", '{"a":null}']


def json_logs(traces, rng, bodies=JSON_BODIES):
    logs = []
    for tr in traces:
        entries = []
        for s in tr:
            if rng.random() < 0.7:
                e = {"traceId": s["traceId"], "spanId": s["id"], "isFallback": rng.random() < 0.2,
                     "request": {"body": rng.choice(bodies)}, "response": {"body": rng.choice(bodies)}}
                for side in ("request", "response"):
                    ct = rng.choice(["application/json", "application/json", "text/plain", None])
                    if ct is not None:
                        e[side]["contentType"] = ct
                    if rng.random() < 0.1:
                        del e[side]["body"]
                entries.append(e)
        logs.append({"traces": entries})
    return logs


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_combined_with_json_bodies_equal_oracle(engine, seed, ts_hook):
    from kmamiz_amd import Traces, synth
    from test_gpu_parity import _stats_equal

    cfg = 2 if seed % 2 else 3
    batch, off = synth.host_batch(cfg, 0, 120)
    traces = synth.to_traces(cfg, batch, off)
    logs = json_logs(traces, random.Random(seed))
    ours = Traces(traces, engine=engine).combineLogsToRealtimeData(copy.deepcopy(logs))
    ref = O.Traces(traces).combineLogsToRealtimeData(copy.deepcopy(logs))
    assert ours.toJSON() == O.strip_undef(ref.toJSON())
    got = ours.toCombinedRealtimeData().toJSON()
    exp = O.strip_undef(ref.toCombinedRealtimeData().toJSON())
    _stats_equal(got, exp)
    fields = ("requestContentType", "responseContentType", "requestBody", "requestSchema", "responseBody",
              "responseSchema")
    for a, b in zip(got, exp):
        for k in fields:
            assert a.get(k) == b.get(k), k
    assert any("requestBody" in a for a in got)
    # the cache merge of two such windows (CCombinedRealtimeData.setData)
    from kmamiz_amd import CombinedRealtimeDataList
    from kmamiz_amd.cache import CombinedColumns

    merged = CombinedColumns.from_json(copy.deepcopy(got)).combineWith(CombinedColumns.from_json(copy.deepcopy(got)))
    mirror = CombinedRealtimeDataList(copy.deepcopy(got)).combineWith(CombinedRealtimeDataList(copy.deepcopy(got)))
    orc = O.CombinedRealtimeDataList(copy.deepcopy(exp)).combineWith(O.CombinedRealtimeDataList(copy.deepcopy(exp)))
    for a, b, c in zip(merged.toJSON(), mirror.toJSON(), O.strip_undef(orc.toJSON())):
        for k in fields:
            assert a.get(k) == b.get(k) == c.get(k), k


@pytest.mark.gpu
def test_pdas_with_its_own_envoy_logs(engine):
    """The PDAS trace fixture with the reference's PDAS log lines, through the
    worker's chain (RealtimeWorkerImpl.ts:60-64)."""
    from kmamiz_amd import Traces
    from kmamiz_amd.envoy import EnvoyLogs, ParseEnvoyLogs

    traces = [fixture("MockTracePDAS")]
    lines = fixture("MockLogsPDAS")
    ours_logs = EnvoyLogs.CombineToStructuredEnvoyLogs([ParseEnvoyLogs(lines, "pdas", "user-service")])
    ref_logs = O.EnvoyLogs.CombineToStructuredEnvoyLogs([O.parse_envoy_logs(lines, "pdas", "user-service")])
    ours = Traces(traces, engine=engine).combineLogsToRealtimeData(ours_logs)
    ref = O.Traces(traces).combineLogsToRealtimeData(ref_logs)
    assert ours.toJSON() == O.strip_undef(ref.toJSON())
    assert ours.toCombinedRealtimeData().toJSON() == O.strip_undef(ref.toCombinedRealtimeData().toJSON())


@pytest.mark.gpu
def test_nested_json_bodies_need_the_hook(engine):
    from kmamiz_amd import Traces

    traces = [fixture("MockTracePDAS")]
    logs = [{"traces": [{"traceId": s["traceId"], "spanId": s["id"], "isFallback": False,
                         "request": {"body": '{"n":{"deep":1}}', "contentType": "application/json"},
                         "response": {"body": "x"}} for s in traces[0]]}]
    with pytest.raises(NotImplementedError):
        Traces(traces, engine=engine).combineLogsToRealtimeData(logs).toCombinedRealtimeData()
