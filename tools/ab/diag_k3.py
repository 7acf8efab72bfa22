"""Diagnostic (not product): K3 groups on the mesh vs a numpy restatement."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmamiz_amd import Engine, synth  # noqa: E402
from kmamiz_amd import _lib as L  # noqa: E402

for NTR in [int(x) for x in sys.argv[1:]] or [3000, 20000]:
    b, _ = synth.host_batch(3, 0, NTR)
    srv = b.kind == 1
    G = 20000 * 3
    g = b.shape[srv].astype(np.int64) * 3 + b.status[srv]
    cnt = np.bincount(g, minlength=G)
    ts = np.full(G, np.iinfo(np.int64).min, np.int64)
    np.maximum.at(ts, g, b.timestamp[srv])
    s1 = np.bincount(g, weights=b.duration[srv].astype(np.float64), minlength=G)
    for ab in (None, "8"):
        if ab:
            os.environ["KMZ_ABLATE"] = ab
        e = Engine(0)
        os.environ.pop("KMZ_ABLATE", None)
        e.load_synthetic(3, synth.SEED, 0, NTR)
        for k in range(3):
            e.run(L.RUN_STATS_TAG)
            r = e.groups()
            used = cnt > 0
            print(NTR, "ablate", ab, "run", k, "count mism", int((r["combined"] != cnt).sum()),
                  "ts mism", int((r["latest_timestamp"][used] != ts[used]).sum()),
                  "n_server", e.info()["n_server"], int(srv.sum()))
        e.close()
