"""Diagnostic: k_join_window phase clocks (KMZ_ABLATE bit 23), summed over
workgroups, and k4_chain's (bit 22)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["KMZ_ABLATE"] = str((1 << 22) | (1 << 23))
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 3650000
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else synth.MESH
e = Engine(0)
e.load_synthetic(cfg, synth.SEED, 0, ntr)
e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
for fn, names, k in (("kmz__debug_join", ["load+fill", "insert", "lookup", "contract+write", "cert1"], 5),
                     ("kmz__debug_chain", ["loop/next", "fill", "hash+probe-issue", "check+elect", "leaders", "stats"], 6)):
    f = getattr(L.lib(), fn)
    buf = (C.c_ulonglong * 16)()
    f(buf, 1)
    e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    f(buf, 1)
    v = list(buf)[:k]
    tot = max(1, sum(v))
    print(fn, " ".join(f"{nm}={x / tot * 100:.1f}%" for nm, x in zip(names, v)), "total", tot, flush=True)
