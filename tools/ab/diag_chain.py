"""Diagnostic: K4 insert-path counters (KMZ_ABLATE bit 21) per run on the mesh."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["KMZ_ABLATE"] = str(1 << 21)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 3650000
e = Engine(0)
e.load_synthetic(synth.MESH, synth.SEED, 0, ntr)
buf = (C.c_ulonglong * 8)()
for k in range(3):
    L.lib().kmz__debug_chain(buf, 1)
    e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    L.lib().kmz__debug_chain(buf, 1)
    put, r0, r1, r2, rounds, tiles = list(buf)[:6]
    print(f"run {k}: spans to insert {put}, wait {r0}, inserted {r1}, joined {r2}, rounds/tile {rounds / max(1, tiles):.2f}, tiles {tiles}", flush=True)
