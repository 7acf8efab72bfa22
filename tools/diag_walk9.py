"""Diagnostic: k4_tile9's phase clocks (a libkmz_<variant>.so built with
-DKMZ_T9_CLOCKS=1, selected by KMZ_LIB_VARIANT), config 3 at 10^8 spans:
s_memtime deltas seen by each workgroup's thread 0, summed over workgroups,
per run, as fractions and cycles per workgroup."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 3650000
e = Engine(0)
n = e.load_synthetic(synth.MESH, synth.SEED, 0, ntr)
buf = (C.c_ulonglong * 12)()
fn = L.lib().kmz__debug_walk9
names = ["window", "compact", "walk", "sigs", "probe", "claim", "lists", "rows", "end-of-round", "tile stats"]
for k in range(3):
    fn(buf, 1)
    e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    fn(buf, 0)
    v = list(buf)[:10]
    tot = max(1, sum(v))
    wgs = (n + 959) // 960
    print("run", k, "path", e.info()["path"], " ".join(f"{nm}={x / tot * 100:.1f}%" for nm, x in zip(names, v)),
          "cycles/wg", round(tot / wgs), flush=True)
