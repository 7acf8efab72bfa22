"""Pin the oracle: every known answer the reference's jest suite holds for the
hot path, from the fixtures extracted out of tests/MockData.ts."""
import math

import pytest

from conftest import fixture
from oracle import kmz_oracle as O


def test_traces_to_realtime_data():  # Traces.test.ts:12-15
    rl = O.Traces([fixture("MockTracePDAS")]).toRealTimeData()
    assert O.strip_undef(rl.toJSON()) == fixture("MockRlDataPDAS")


def test_traces_to_endpoint_dependencies():  # Traces.test.ts:17-21
    deps = O.Traces([fixture("MockTracePDAS")]).toEndpointDependencies()
    got = O.strip_undef(deps.toJSON())
    assert got == fixture("MockEndpointDependenciesPDAS")
    # first position / last value of the nested entry (MockData.ts:4286)
    assert got[3]["dependingOn"][0]["endpoint"]["timestamp"] == 1646208338227.724


def test_to_endpoint_info():  # Traces.test.ts:23-26
    assert O.strip_undef(O.Traces.ToEndpointInfo(fixture("MockTracePDAS")[0])) == fixture("MockEndpointInfoPDAS1")


def test_realtime_combined_welford():  # RealtimeDataList.test.ts:10-13
    c = O.RealtimeDataList(fixture("MockBaseRlData1")).toCombinedRealtimeData().toJSON()
    exp = fixture("MockBaseCrlData1")[0]
    assert c[0]["combined"] == 10 and c[0]["latency"] == {"mean": 100, "cv": 0.17888543819998}
    assert c[0]["latestTimestamp"] == exp["latestTimestamp"] and c[0]["avgReplica"] == 1


def test_combined_merge():  # CombinedRealtimeDataList.test.ts:25-31
    a = O.CombinedRealtimeDataList(fixture("MockBaseCrlData1"))
    b = O.CombinedRealtimeDataList(fixture("MockBaseCrlData2"))
    c = a.combineWith(b).toJSON()[0]
    exp = fixture("MockCombinedBaseData")[0]
    assert c["combined"] == 20 and c["latency"] == {"mean": 125, "cv": 0.25861167800391}
    assert c["latestTimestamp"] == exp["latestTimestamp"]


def test_explode_url():  # Utils.test.ts:72-85
    assert "\t".join(O.explode_url("http://example.com:8080/test/test")) == "example.com\t:8080\t/test/test"
    assert "\t".join(O.explode_url("https://192.168.1.1/test#123")) == "192.168.1.1\t\t/test#123"
    assert (
        "\t".join(O.explode_url("service.test.svc.cluster.local:80/test/endpoint"))
        == "service.test.svc.cluster.local\t:80\t/test/endpoint"
    )


def test_normalizer():  # Utils.test.ts:95-112
    assert O.Normalizer.BetweenFixedNumber([1, 2, 3]) == [0.1, 0.55, 1]
    assert O.Normalizer.Linear([1, 2, 3]) == [0.4, 0.7, 1]
    assert O.Normalizer.Sigmoid([1, 2, 3]) == [1 / (1 + math.exp(-v)) for v in (1, 2, 3)]
    assert O.Normalizer.FixedRatio([1, 2, 4]) == [0.25, 0.5, 1]


@pytest.fixture
def pdas_deps():
    return O.EndpointDependencies(fixture("MockEndpointDependenciesPDAS"))


def test_graph_data(pdas_deps):  # EndpointDependencies.test.ts:11-15
    g = pdas_deps.toGraphData()
    assert len(g["nodes"]) == 7 and len(g["links"]) == 6


def test_chord_data(pdas_deps):  # EndpointDependencies.test.ts:16-45
    assert pdas_deps.toChordData() == {
        "nodes": [
            {"id": "external-service.pdas (latest)", "name": "external-service\tpdas\tlatest"},
            {"id": "user-service.pdas (latest)", "name": "user-service\tpdas\tlatest"},
            {"id": "contract-service.pdas (latest)", "name": "contract-service\tpdas\tlatest"},
        ],
        "links": [
            {"from": "external-service.pdas (latest)", "to": "user-service.pdas (latest)", "value": 1},
            {"from": "external-service.pdas (latest)", "to": "contract-service.pdas (latest)", "value": 1},
        ],
    }


def test_service_dependencies(pdas_deps):  # EndpointDependencies.test.ts:46-48
    assert len(pdas_deps.toServiceDependencies()) == 3


def test_cohesion(pdas_deps):  # EndpointDependencies.test.ts:49-79
    assert pdas_deps.toServiceEndpointCohesion() == [
        {
            "uniqueServiceName": "user-service\tpdas\tlatest",
            "totalEndpoints": 2,
            "consumers": [{"uniqueServiceName": "external-service\tpdas\tlatest", "consumes": 1}],
            "endpointUsageCohesion": 0.5,
        },
        {
            "uniqueServiceName": "contract-service\tpdas\tlatest",
            "totalEndpoints": 1,
            "consumers": [{"uniqueServiceName": "external-service\tpdas\tlatest", "consumes": 1}],
            "endpointUsageCohesion": 1,
        },
        {"uniqueServiceName": "external-service\tpdas\tlatest", "totalEndpoints": 1, "consumers": [],
         "endpointUsageCohesion": 0},
    ]


def test_coupling(pdas_deps):  # EndpointDependencies.test.ts:80-104
    assert [(c["ais"], c["ads"], c["acs"]) for c in pdas_deps.toServiceCoupling()] == [(1, 0, 0), (1, 0, 0), (1, 2, 2)]


def test_instability(pdas_deps):  # EndpointDependencies.test.ts:105-128
    assert [(c["dependingBy"], c["dependingOn"], c["instability"]) for c in pdas_deps.toServiceInstability()] == [
        (1, 0, 0),
        (1, 0, 0),
        (0, 2, 1),
    ]


def test_js_round_semantics():
    assert O.js_round(0.49999999999999994) == 0
    assert O.js_round(-2.5) == -2
    assert O.js_round(2.5) == 3
    assert O.to_precise(0.1 + 0.2) == 0.3
