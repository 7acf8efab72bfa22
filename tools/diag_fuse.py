"""Diagnostic: k_join_chain phase clocks (KMZ_ABLATE bit 22), summed over
workgroups (s_memtime deltas of thread 0)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["KMZ_ABLATE"] = str(1 << 22)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 3650000
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else synth.MESH
e = Engine(0)
e.load_synthetic(cfg, synth.SEED, 0, ntr)
e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
names = ["load", "insert", "lookup", "contract+out", "cert1", "records+compact", "walk+probe", "check+elect",
         "leaders", "stats"]
f = L.lib().kmz__debug_fuse
buf = (C.c_ulonglong * 16)()
for k in range(2):
    f(buf, 1)
    e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    f(buf, 1)
    v = list(buf)[:10]
    tot = max(1, sum(v))
    print("run", k, " ".join(f"{nm}={x / tot * 100:.1f}%" for nm, x in zip(names, v)), "total", tot, flush=True)
