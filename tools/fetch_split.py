"""Where a 2 500-trace tick's fetch goes (run once per config, then each
fetch variant timed over repeats of the same run's results): used groups
only, + edge keys, + endpoints (kmz_fetch_used), the dense kmz_fetch, and
the result sizes.  Prints one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    out = {}
    for name, cfg in (("bookinfo", synth.BOOKINFO), ("mesh", synth.MESH), ("power", synth.POWER)):
        e = Engine(0)
        batch, _ = synth.host_batch(cfg, 0, 2500)
        e.load(batch, synth.shape_table(cfg))
        e.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        res = {"n_triples": e.info()["n_triples"], "n_dep_ep": e.n_dep_ep, "groups_used": len(e.fetch_used()[0])}
        for label, fn in (("used_groups", lambda: e.fetch_used(deps=False)),
                          ("used_groups_keys", lambda: e.fetch_used(deps=True, keys=True)[:3]),
                          ("used_all", lambda: e.fetch_used()),
                          ("dense_all", lambda: e.fetch())):
            fn()
            ts = []
            for _ in range(50):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            res[label + "_us"] = round(float(np.median(ts)) * 1e6, 1)
        out[name] = res
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
