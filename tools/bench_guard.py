"""Cost of the cross-shard repeated-id guard on one GPU:
rank 0's shard of config 4 at world 2/4/8 (kmz_synth_load_shard), the routing
of its span-id hashes (kmz_route_ids, into device memory) and the certificate
over as many values as an owner receives (kmz_id_repeats, device memory),
timed over repeats, beside the shard's own step (kmz_run).  The all-to-all
itself is not timed here (one GPU).  Prints one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    ntr = 36578450  # 1e9 mesh spans (config 4)
    out = {"metric": "sharding guard cost per step, rank 0 of config 4", "unit": "ms", "worlds": {}}
    eng = Engine(0)
    for world in (2, 4, 8):
        n = eng.load_synthetic_shard(synth.MESH, synth.SEED, 0, ntr, world, 0)
        buf = torch.empty(n, dtype=torch.int64, device="cuda")
        eng.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        t = time.perf_counter()
        for _ in range(3):
            eng.run(L.RUN_STATS_TAG | L.RUN_DEPS)
        step = (time.perf_counter() - t) / 3
        eng.route_ids(world, buf.data_ptr(), n, True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            eng.route_ids(world, buf.data_ptr(), n, True)
        route = (time.perf_counter() - t) / 3
        assert eng.id_repeats(buf.data_ptr(), n, True) is False
        t = time.perf_counter()
        for _ in range(3):
            eng.id_repeats(buf.data_ptr(), n, True)
        check = (time.perf_counter() - t) / 3
        out["worlds"][world] = {"spans_rank0": n, "step_ms": round(step * 1e3, 3), "route_ms": round(route * 1e3, 3),
                                "certificate_ms": round(check * 1e3, 3),
                                "all_to_all_bytes_per_rank": 8 * n}
        del buf
        torch.cuda.empty_cache()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
