"""How often does a chain-walk workgroup see a chain again?  (Diagnostic for
the K4 chain table's probe traffic)

Builds the mesh's (config 3) host batch, resolves every span's first
non-CLIENT ancestor, folds each non-CLIENT span's ancestry into a chain id
(the same recursive definition k4 interns: parent chain + (endpoint, kind))
and reports
  * distinct chains per 960-span tile against its walkers (repeats a per-tile
    LDS cache could serve),
  * the hit rate of a direct-mapped per-workgroup cache of K chain ids over a
    persistent workgroup's tiles (G workgroups taking tiles g, g+G, ...),
  * the share of walkers the K most frequent chains cover (the best any
    K-entry cache can do once warm).

usage: PYTHONPATH=. python tools/chain_reuse_sim.py [traces]
"""
import sys

import numpy as np

from kmamiz_amd import synth

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def chains(ntraces):
    b, _ = synth.host_batch(synth.MESH, 0, ntraces)
    tab = synth.shape_table(synth.MESH)
    n = len(b)
    order = np.argsort(b.span_id)
    ss = b.span_id[order]
    pos = np.minimum(np.searchsorted(ss, b.parent_id), n - 1)
    par = np.where((b.parent_id != 0) & (ss[pos] == b.parent_id), order[pos], -1)
    cp = par.copy()
    for _ in range(64):  # contract CLIENT ancestors
        nxt = np.where(cp >= 0, cp, 0)
        isc = (cp >= 0) & (b.kind[nxt] == 2)
        if not isc.any():
            break
        cp = np.where(isc, par[nxt], cp)
    dep = np.asarray(tab.dep_ep)[b.shape].astype(np.uint64)
    with np.errstate(over="ignore"):
        elem = (dep * np.uint64(0x9E3779B97F4A7C15) + b.kind.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)) & M64
        sig = np.zeros(n, np.uint64)
        done = cp < 0
        sig[done] = elem[done]
        for _ in range(64):
            todo = ~done & (cp >= 0) & done[np.maximum(cp, 0)]
            if not todo.any():
                break
            p = cp[todo]
            sig[todo] = ((sig[p] << np.uint64(7)) | (sig[p] >> np.uint64(57))) ^ elem[todo]
            done[todo] = True
    return n, np.nonzero(b.kind != 2)[0], sig


def main():
    ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    n, walkers, sig = chains(ntr)
    print("spans", n, "walkers", len(walkers), "distinct chains", len(np.unique(sig[walkers])))
    T = 960
    tiles = (n + T - 1) // T
    tile_of = walkers // T
    per = [sig[walkers[tile_of == t]] for t in range(tiles)]
    w = sum(len(x) for x in per)
    d = sum(len(np.unique(x)) for x in per)
    print("per tile: walkers %.1f distinct %.1f -> in-tile repeats %.3f" % (w / tiles, d / tiles, 1 - d / w))
    for G in (1024, 256):
        for K in (1024, 4096):
            hits = tot = 0
            sh = np.uint64(64 - int(np.log2(K)))
            for g in range(min(G, tiles)):
                cache = np.zeros(K, np.uint64)
                for t in range(g, tiles, G):
                    s = per[t]
                    with np.errstate(over="ignore"):
                        slot = ((s * np.uint64(0x9E3779B97F4A7C15)) >> sh).astype(np.int64)
                    hits += int((cache[slot] == s).sum())
                    tot += len(s)
                    cache[slot] = s
            print("G %d K %d: hit rate %.3f (%.1f tiles per workgroup)" % (G, K, hits / tot, tiles / G))
    _, c = np.unique(sig[walkers], return_counts=True)
    cs = np.cumsum(np.sort(c)[::-1]) / c.sum()
    for K in (256, 1024, 4096, 16384, 65536):
        print("top %d chains cover %.3f of walkers" % (K, cs[min(K, len(cs)) - 1]))


if __name__ == "__main__":
    main()
