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
        # fixed segments (IdGuard's steady state: no counts exchange, no sync)
        seg = int(n / world * 1.125) + 1025
        fbuf = torch.empty(world * seg, dtype=torch.int64, device="cuda")
        eng.route_ids_fixed(world, seg, fbuf.data_ptr(), True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            eng.route_ids_fixed(world, seg, fbuf.data_ptr(), True)
        torch.cuda.synchronize()
        route_fixed = (time.perf_counter() - t) / 3
        del fbuf
        # what an owner receives: ~n values (hash-uniform owners, equal shards)
        assert eng.id_repeats(buf.data_ptr(), n, True) is False
        t = time.perf_counter()
        for _ in range(3):
            eng.id_repeats(buf.data_ptr(), n, True)
        check = (time.perf_counter() - t) / 3
        # the exchange over xGMI (not timed on one GPU): each rank sends
        # (world-1)/world of its 8-B hashes, one direct link per peer at
        # ~153 GB/s (MI355X_MICROARCH.md), all links at once
        peer_bytes = 8 * n / world
        out["worlds"][world] = {"spans_rank0": n, "step_ms": round(step * 1e3, 3), "route_ms": round(route * 1e3, 3),
                                "route_fixed_ms": round(route_fixed * 1e3, 3),
                                "certificate_ms": round(check * 1e3, 3),
                                "all_to_all_bytes_per_rank": int(8 * n * (world - 1) / world),
                                "all_to_all_ms_projected": round(peer_bytes / 153e9 * 1e3, 3),
                                "guard_ms_projected": round((route_fixed + check) * 1e3 + peer_bytes / 153e9 * 1e3, 3)}
        del buf
        torch.cuda.empty_cache()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
