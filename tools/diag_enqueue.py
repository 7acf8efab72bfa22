"""Diagnostic: host time of kmz_run_begin (the run's enqueue) against the
whole run, mesh 10^8 spans, engine on a torch stream as bench.py."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    e = Engine(0, stream=st.cuda_stream)
    ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 3657845
    e.load_synthetic(synth.MESH, synth.SEED, 0, ntr)
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    for _ in range(3):
        e.run(flags)
    beg, tot = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        e.run_begin(flags)
        t1 = time.perf_counter()
        e.run_end()
        t2 = time.perf_counter()
        beg.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    beg.sort()
    tot.sort()
    print(f"run_begin ms median {beg[10]:.3f} min {beg[0]:.3f} max {beg[-1]:.3f}; run ms median {tot[10]:.3f}")
    e.close()


if __name__ == "__main__":
    main()
