"""Host time of one mesh step's calls (10^8 spans, as bench.py's default):
kmz_run_begin (the enqueue of the whole run), kmz_run_end (the wait), and the
fetch's two halves, median over steps.  A run_begin much longer than the
run's first kernels leaves the GPU idle at the head of the step.  With
KMZ_RUNBEGIN_PROFILE=1 the engine prints per-stage host times of run_begin
(kmz_api.hip)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    e = Engine(0, stream=stream.cuda_stream)
    n = e.load_synthetic(synth.MESH, synth.SEED, 0, 3650000)
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    t = {"run_begin": [], "run_end": [], "fetch_end": [], "fetch_begin": []}
    for i in range(12):
        a = time.perf_counter()
        e.run_begin(flags)
        b = time.perf_counter()
        e.run_end()
        c = time.perf_counter()
        e.fetch_end()
        d = time.perf_counter()
        e.fetch_begin()
        f = time.perf_counter()
        if i >= 2:
            for k, v in zip(t, (b - a, c - b, d - c, f - d)):
                t[k].append(v)
    e.fetch_end()
    print(json.dumps({"spans": n, **{k + "_us": round(float(np.median(v)) * 1e6, 1) for k, v in t.items()}}))


if __name__ == "__main__":
    main()
