"""Diagnostic: per-kernel times of the mesh pipeline under KMZ_ABLATE knobs
(bit 1 = skip edge-key dedup, 2 = skip the global edge set, 4 = skip global
endpoint atomics, 64 = skip certificate pass 1 in the join, 128 = skip its
global bin atomics).  Prints one JSON line per setting."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    from kmamiz_amd import Engine, synth
    from kmamiz_amd import _lib as L

    ntr = int(sys.argv[2])
    e = Engine(0)
    n = e.load_synthetic(synth.MESH, synth.SEED, 0, ntr)
    for _ in range(2):
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    e.kernel_times(reset=True)
    e.set_profiling(True)
    for _ in range(5):
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
    t = e.kernel_times(reset=True)
    print(json.dumps({"ablate": os.environ.get("KMZ_ABLATE", "0"), "n": n,
                      **{k: round(v[0] / max(1, v[1]), 3) for k, v in t.items()}}))
else:
    ntr = sys.argv[1] if len(sys.argv) > 1 else "3650000"
    for a in sys.argv[2:] or ["0", "1", "2", "4", "7"]:
        env = dict(os.environ, KMZ_ABLATE=a)
        subprocess.run([sys.executable, __file__, "child", ntr], env=env, check=True)
