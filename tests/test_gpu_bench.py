"""bench.py's output contract on small batches (the driver parses this line):
one JSON line with the metric, the roofline of the dominant kernel (live
events in the timed region), the per-kernel table of the profiled pass and,
with the service tail on, the pipelined host finish.  Runs bench.py as a
child process on the GPU."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(*args):
    env = dict(os.environ)
    env.pop("KMZ_BENCH_TRACE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--cpu-seconds", "0", "--no-h2d", *args], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("extra", [("--spans", "2e6"), ("--config", "power", "--spans", "2e6"),
                                   ("--spans", "2e6", "--kernel-times", "live", "--fetch", "sync")])
def test_bench_line_contract(extra):
    d = _bench(*extra)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - d["config"]["spans_total"] / (d["ms_per_step"] * 1e-3)) <= 1e-3 * d["value"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernels", "kernels_source"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["kernels"] and all(v["calls_per_step"] > 0 for v in r["kernels"].values())
    if "power" in extra:
        assert d["config"]["service_tail"] is True
