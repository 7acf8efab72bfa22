import sys, os, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from kmamiz_amd import Engine, synth
from kmamiz_amd import _lib as L
config, t0, t1, world = 5, 7, 1500, 2
flags = L.RUN_STATS_TAG | L.RUN_DEPS
def partials(e):
    gw, ew = e.partials_words(L.PART_GROUPS), e.partials_words(L.PART_ENDPOINTS)
    g, ee = np.zeros(gw, np.uint64), np.zeros(ew, np.uint64)
    e.export_partials(L.PART_GROUPS, g.ctypes.data, gw, False)
    e.export_partials(L.PART_ENDPOINTS, ee.ctypes.data, ew, False)
    return g, ee
e = Engine(0)
parts = []
for r in range(world):
    e.load_synthetic_shard(config, synth.SEED, t0, t1, world, r); e.run(flags); parts.append(partials(e))
G = len(parts[0][0]) // 6
g = parts[0][0].copy()
for pg, _ in parts[1:]:
    g[:4*G] += pg[:4*G]; g[4*G:5*G] = np.maximum(g[4*G:5*G], pg[4*G:5*G]); g[5*G:] = np.minimum(g[5*G:], pg[5*G:])
e.load_synthetic(config, synth.SEED, t0, t1); e.run(flags); wg, _ = partials(e)
e2 = Engine(0); e2.load_synthetic(config, synth.SEED, t0, t1); e2.run(flags); wg2, _ = partials(e2)
print("fresh engine whole == reused engine whole:", np.array_equal(wg, wg2))
for name, w in (("reused", wg), ("fresh", wg2)):
    bad = np.nonzero(w != g)[0]
    print(name, "mismatches", len(bad), "fields", np.unique(bad // G)[:6], "groups", (bad % G)[:8])
    if len(bad):
        i = bad[0]; f = i // G; k = i % G
        print("  field", f, "group", k, "whole", [int(w[x*G+k]) for x in range(6)], "merged", [int(g[x*G+k]) for x in range(6)],
              [ [int(p[0][x*G+k]) for x in range(6)] for p in parts])
