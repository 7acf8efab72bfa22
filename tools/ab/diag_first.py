"""Diagnostic: why is the first step after a pause slower?  Times single steps
(run + fetch) after different pauses / profiling toggles."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

e = Engine(0)
e.load_synthetic(synth.MESH, synth.SEED, 0, 3650000)
F = L.RUN_STATS_TAG | L.RUN_DEPS


def step():
    e.run(F)
    e.fetch()


def timed(n=4):
    out = []
    for _ in range(n):
        t = time.perf_counter()
        step()
        out.append(round((time.perf_counter() - t) * 1e3, 2))
    return out


for _ in range(3):
    step()
print("steady", timed(), flush=True)
time.sleep(0.005)
print("after 5ms sleep", timed(), flush=True)
time.sleep(0.05)
print("after 50ms sleep", timed(), flush=True)
torch.cuda.synchronize()
print("after torch sync", timed(), flush=True)
e.set_profiling(True)
print("after set_profiling", timed(), flush=True)
e.set_profiling(False)
print("profiling off", timed(), flush=True)
e.set_profiling(True)
print("profiling on again", timed(), flush=True)
