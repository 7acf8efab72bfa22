"""Diagnostic: far-parent batch through each resolve/walk path (KMZ_ABLATE)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmamiz_amd import Engine, synth, _lib as L  # noqa: E402
from kmamiz_amd.engine import SpanBatch  # noqa: E402
from oracle import c_oracle  # noqa: E402

batch, _ = synth.host_batch(3, 0, 3000)
n = len(batch)
rng = np.random.default_rng(7)
perm = np.arange(n)
sel = np.flatnonzero(rng.random(n) < 0.02)
perm[sel] = perm[rng.permutation(sel)]
b = SpanBatch(batch.span_id[perm], batch.parent_id[perm], batch.kind[perm], batch.shape[perm],
              batch.status[perm], batch.duration[perm], batch.timestamp[perm], 0)
table = synth.shape_table(3)
okeys, oep, ocnt = c_oracle.deps(b, table.dep_ep, table.n_dep_ep)
print("oracle", ocnt, len(okeys))
# host reference of cparent
pos = {int(s): i for i, s in enumerate(b.span_id)}
par = np.array([pos.get(int(p), -1) if p else -1 for p in b.parent_id])
cp = np.full(n, 0xFFFFFFFF, dtype=np.uint64)
for i in range(n):
    if b.kind[i] == 2:
        continue
    j = par[i]
    while j >= 0 and b.kind[j] == 2:
        j = par[j]
    cp[i] = j if j >= 0 else 0xFFFFFFFF
for abl in ("0", "32", "16", "48"):
    os.environ["KMZ_ABLATE"] = abl
    e = Engine(0)
    e.load(b, table)
    try:
        e.run(L.RUN_DEPS | L.RUN_SPAN_LINKS)
        gcp, _ = e.span_links()
        bad = np.flatnonzero(gcp.astype(np.uint64) != cp)
        print(abl, "ok", e.info(), "cparent mismatches", len(bad), bad[:5], gcp[bad[:5]], cp[bad[:5]])
        print("   keys equal", np.array_equal(e.triples(), okeys))
    except Exception as ex:  # noqa: BLE001
        print(abl, "error", ex, e.info())
    e.close()
import ctypes
dbg = (ctypes.c_ulonglong * 64)()
L.lib().kmz__debug_k4(dbg)
print("dbg count", dbg[0])
for k in range(min(15, dbg[0])):
    i, f, c, w = dbg[1 + 4 * k: 5 + 4 * k]
    print("row", i, "first", f, "cur", c, "lcp", hex(w >> 32), "cparent[i]", w & 0xFFFFFFFF, "host cp[i]", int(cp[i]),
          "chain", [int(x) for x in [cp[i], cp[int(cp[i])] if cp[i] < n else -1]])
