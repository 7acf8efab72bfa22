"""Diagnostic: engine info (rows, relations, chains, edge keys) for a synthetic config."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else synth.MESH
ntr = int(sys.argv[2]) if len(sys.argv) > 2 else 3650000
e = Engine(0)
e.load_synthetic(cfg, synth.SEED, 0, ntr)
e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
print(e.info(), flush=True)
