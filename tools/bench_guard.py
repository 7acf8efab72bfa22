"""Cost of the cross-shard repeated-id guard on one GPU:
rank 0's shard of config 4 at world 2/4/8 (kmz_synth_load_shard).  Timed over
repeats, on the engine's stream = torch's (as bench.py):
  step_ms           the shard's own step with its certificate (kmz_run)
  step_nocert_ms    ... with KMZ_RUN_NO_CERT (the multi-GPU setting: the
                    guard checks every shard's ids, the run checks none)
  route_fixed_ms    kmz_route_ids_fixed, one pass (and route_fixed_hist_ms,
                    the histogram / scan / scatter form, KMZ_ABLATE2 bit 12)
  seg_certificate_ms  kmz_id_repeats_seg_begin/_end over world segments as
                    an owner receives them, alone
  guarded_step_ms   the whole guarded step as bench.py runs it at N > 1, with
                    the all-to-all stood in for by a device copy of the
                    segments on a stream of its own: routing, then the run
                    (no certificate) beside the copy + the segment
                    certificate on the guard's stream, then its verdict
  guarded_fold_ms   the same with the routing folded into the run's join
                    (kmz_route_ids_join; the copy waits for kmz_route_wait,
                    i.e. the join's end, then runs beside the rest of the
                    run), as bench.py runs it since round 6; step_route_ms:
                    the run with the routing armed and nothing else
The exchange over xGMI itself is not timed here (one GPU): its projection
is the bytes each rank sends over its peer links at ~153 GB/s each.  Prints
one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _timed(fn, reps=3):
    import torch

    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    import torch

    from kmamiz_amd import Engine
    from kmamiz_amd import _lib as L
    from kmamiz_amd import synth

    ntr = 36578450  # 1e9 mesh spans (config 4)
    out = {"metric": "sharding guard cost per step, rank 0 of config 4", "unit": "ms", "worlds": {}}
    stream = torch.cuda.Stream()  # (as bench.py: torch's current stream and the engine's, not handle 0)
    torch.cuda.set_stream(stream)
    eng = Engine(0, stream=stream.cuda_stream)
    os.environ["KMZ_ABLATE2"] = str(4096)
    eng_hist = Engine(0, stream=stream.cuda_stream)  # (the histogram routing form, for comparison)
    del os.environ["KMZ_ABLATE2"]
    gs = torch.cuda.Stream()
    cs = torch.cuda.Stream()
    flags = L.RUN_STATS_TAG | L.RUN_DEPS
    worlds = [int(w) for w in os.environ.get("KMZ_GUARD_WORLDS", "2,4,8").split(",")]
    for world in worlds:
        n = eng.load_synthetic_shard(synth.MESH, synth.SEED, 0, ntr, world, 0)
        step = _timed(lambda: eng.run(flags))
        step_nc = _timed(lambda: eng.run(flags | L.RUN_NO_CERT))
        seg = int(n / world * 1.125) + 1025
        send = torch.empty(world * seg, dtype=torch.int64, device="cuda")
        recv = torch.empty_like(send)
        route = _timed(lambda: eng.route_ids_fixed(world, seg, send.data_ptr(), True))
        eng_hist.load_synthetic_shard(synth.MESH, synth.SEED, 0, ntr, world, 0)
        route_hist = _timed(lambda: eng_hist.route_ids_fixed(world, seg, send.data_ptr(), True))
        eng_hist.load(synth.host_batch(synth.MESH, 0, 10)[0], synth.shape_table(synth.MESH))  # (free its columns)
        eng.route_ids_fixed(world, seg, send.data_ptr(), True)
        recv.copy_(send)
        torch.cuda.synchronize()

        def seg_cert():
            eng.id_repeats_seg_begin(recv.data_ptr(), world, seg, 0)
            rep, _ = eng.id_repeats_seg_end()
            assert rep is False

        cert = _timed(seg_cert)

        def guarded():
            eng.route_ids_fixed(world, seg, send.data_ptr(), True)
            cs.wait_stream(stream)
            with torch.cuda.stream(cs):
                recv.copy_(send)  # (stands in for the all-to-all)
            gs.wait_stream(cs)
            eng.id_repeats_seg_begin(recv.data_ptr(), world, seg, gs.cuda_stream)
            eng.run_begin(flags | L.RUN_NO_CERT)
            eng.run_end()
            rep, _ = eng.id_repeats_seg_end()
            assert rep is False

        guarded_ms = _timed(guarded)

        def routed_run():
            eng.route_ids_join(world, seg, send.data_ptr())
            eng.run(flags | L.RUN_NO_CERT)

        step_route = _timed(routed_run)
        in_join = eng.route_wait(0)

        def guarded_fold():
            eng.route_ids_join(world, seg, send.data_ptr())
            eng.run_begin(flags | L.RUN_NO_CERT)
            eng.route_wait(cs.cuda_stream)
            with torch.cuda.stream(cs):
                recv.copy_(send)  # (stands in for the all-to-all)
            gs.wait_stream(cs)
            eng.id_repeats_seg_begin(recv.data_ptr(), world, seg, gs.cuda_stream)
            eng.run_end()
            rep, _ = eng.id_repeats_seg_end()
            assert rep is False

        fold_ms = _timed(guarded_fold)
        peer_bytes = 8 * n / world
        a2a = peer_bytes / 153e9 * 1e3
        out["worlds"][world] = {"spans_rank0": n, "step_ms": round(step, 3), "step_nocert_ms": round(step_nc, 3),
                                "route_fixed_ms": round(route, 3), "route_fixed_hist_ms": round(route_hist, 3),
                                "seg_certificate_ms": round(cert, 3), "guarded_step_ms": round(guarded_ms, 3),
                                "step_route_ms": round(step_route, 3), "route_in_join": in_join,
                                "guarded_fold_ms": round(fold_ms, 3),
                                "guard_fold_ms_measured": round(fold_ms - step, 3),
                                "all_to_all_bytes_per_rank": int(8 * n * (world - 1) / world),
                                "all_to_all_ms_projected": round(a2a, 3),
                                # the guard's cost on the step: what the guarded step adds to the
                                # shard's certified step (the exchange overlaps the run)
                                "guard_ms_measured": round(guarded_ms - step, 3)}
        del send, recv
        torch.cuda.empty_cache()
    eng.close()
    eng_hist.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
