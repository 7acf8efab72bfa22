"""Diagnostic: the chain walk's list use per run (kmz__debug_chain_lists),
config 3 at 10^8 spans, for the build KMZ_LIB_VARIANT selects."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 3650000
e = Engine(0)
e.load_synthetic(synth.MESH, synth.SEED, 0, ntr)
buf = (C.c_ulonglong * 4)()
fn = L.lib().kmz__debug_chain_lists
fn.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
names = ["staged_keys", "deferred", "claims", "pending"]
for k in range(3):
    e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    fn(e.ctx, buf)
    i = e.info()
    print(os.environ.get("KMZ_LIB_VARIANT", "base"), "run", k, "chains", i["n_chains"], "path", i["path"],
          " ".join(f"{nm}={v}" for nm, v in zip(names, list(buf))), flush=True)
