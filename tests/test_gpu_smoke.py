"""First GPU parity checks: reference fixtures through the engine."""
import numpy as np
import pytest

from conftest import fixture
from oracle import kmz_oracle as O

pytestmark = pytest.mark.gpu


def test_pdas_realtime_and_deps(engine):
    from kmamiz_amd import Traces, default_engine

    t = Traces([fixture("MockTracePDAS")], engine=engine)
    deps = t.toEndpointDependencies().toJSON()
    assert deps == fixture("MockEndpointDependenciesPDAS")
    crl = t.toRealTimeData().toCombinedRealtimeData().toJSON()
    exp = O.strip_undef(O.Traces([fixture("MockTracePDAS")]).toRealTimeData().toCombinedRealtimeData().toJSON())
    assert [ (c["uniqueEndpointName"], c["status"], c["combined"], c["latestTimestamp"]) for c in crl] == \
           [ (c["uniqueEndpointName"], c["status"], c["combined"], c["latestTimestamp"]) for c in exp]
    for a, b in zip(crl, exp):
        assert a["latency"]["mean"] == pytest.approx(b["latency"]["mean"], rel=1e-9)
        assert a["latency"]["cv"] == pytest.approx(b["latency"]["cv"], rel=1e-9, abs=1e-12)
