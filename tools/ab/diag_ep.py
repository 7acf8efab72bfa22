"""Diagnostic (not product): endpoint records on the mesh, window vs table path
vs a host restatement; prints the first mismatches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

NTR = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
b, _ = synth.host_batch(3, 0, NTR)
n = len(b)
srv = b.kind == 1
E = 20000
exp_ts = np.full(E, np.iinfo(np.int64).min, np.int64)
np.maximum.at(exp_ts, b.shape[srv].astype(np.int64), b.timestamp[srv])
first = np.full(E, np.iinfo(np.int64).max, np.int64)
np.minimum.at(first, b.shape[srv].astype(np.int64), np.flatnonzero(srv))


def run(ablate=None, flags=L.RUN_STATS_TAG | L.RUN_DEPS | L.RUN_SPAN_LINKS):
    if ablate:
        os.environ["KMZ_ABLATE"] = ablate
    e = Engine(0)
    os.environ.pop("KMZ_ABLATE", None)
    e.load_synthetic(3, synth.SEED, 0, NTR)
    out = []
    for _ in range(2):
        e.run(flags)
        out.append((e.endpoints(), e.info(), e.groups()))
    e.close()
    return out


for tag, ab in (("window", None), ("table", "32")):
    for k, (ep, info, g) in enumerate(run(ab)):
        bad = np.flatnonzero(ep["last_ts"] != exp_ts)
        badf = np.flatnonzero((ep["first_row"].astype(np.int64) != first) & (first != np.iinfo(np.int64).max))
        gts = g["latest_timestamp"].reshape(E, 3)
        gbad = np.flatnonzero(np.where(g["combined"].reshape(E, 3) > 0, gts, np.iinfo(np.int64).min).max(1) != exp_ts)
        print(tag, k, "path", info["path"], "flags", info["flags"], "ts mismatches", len(bad), "first mismatches",
              len(badf), "group-ts mismatches", len(gbad))
        for x in bad[:5]:
            print("   ep", x, "got", ep["last_ts"][x], "exp", exp_ts[x], "grp", gts[x])
