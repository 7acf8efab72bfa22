"""Kernel trace of the realtime tick (run it under rocprofv3 --kernel-trace):
TICKS calls of load + run + fetch on one synthetic 2 500-trace batch, as
tools/bench_tick.py times them, for one config and launch mode.  The trace's
per-tick launches and the gaps between them are summarised by
tools/tick_gaps.py.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o tick -- \
        python3 tools/tick_trace.py bookinfo direct 50
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bookinfo"
    mode = sys.argv[2] if len(sys.argv) > 2 else "direct"
    ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    if mode == "graph":
        os.environ["KMZ_HIPGRAPH"] = "1"
    elif mode == "direct":
        os.environ["KMZ_HIPGRAPH"] = "0"
    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    cfg = {"bookinfo": synth.BOOKINFO, "mesh": synth.MESH, "power": synth.POWER}[name]
    batch, _ = synth.host_batch(cfg, 0, 2500)
    table = synth.shape_table(cfg)
    e = Engine(0)
    for _ in range(ticks):
        e.load(batch, table)
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        e.fetch()
    print(name, mode, len(batch), "spans", "graph replays", e.graph_stats()[0], flush=True)
    e.close()


if __name__ == "__main__":
    main()
