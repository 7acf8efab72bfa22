"""Diagnostic: per-kernel times of the mesh pipeline under KMZ_ABLATE knobs
(K4 chain kernel: 256 = no table probe, 512 = no insert rounds, 1024 = no key
emission, 2048 = no hashing/probing/inserting).  Results are NOT correct under
a knob; only the times matter.  Prints one JSON line per setting."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    from kmamiz_amd import Engine, synth
    from kmamiz_amd import _lib as L

    ntr = int(sys.argv[2])
    e = Engine(0)
    n = e.load_synthetic(synth.MESH, synth.SEED, 0, ntr)
    for _ in range(2):
        try:
            e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        except Exception as ex:  # knobs may break invariants; timing still useful
            print("run error", ex, file=sys.stderr)
    e.kernel_times(reset=True)
    e.set_profiling(True)
    for _ in range(3):
        try:
            e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        except Exception as ex:
            print("run error", ex, file=sys.stderr)
    t = e.kernel_times(reset=True)
    print(json.dumps({"ablate": os.environ.get("KMZ_ABLATE", "0"), "n": n,
                      **{k: round(v[0] / max(1, v[1]), 3) for k, v in t.items() if v[1]}}), flush=True)
else:
    ntr = sys.argv[1] if len(sys.argv) > 1 else "3650000"
    for a in sys.argv[2:] or ["0", "256", "512", "1024", "2048"]:
        env = dict(os.environ, KMZ_ABLATE=a)
        subprocess.run([sys.executable, __file__, "child", ntr], env=env, check=True, timeout=120)
