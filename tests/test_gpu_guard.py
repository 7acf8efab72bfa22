"""The cross-shard repeated-span-id guard on the GPU (kmz_guard.hip
kmz_route_ids, the certificate's kmz_id_repeats) against its host mirror
(kmamiz_amd.dist.route_ids_np) and a sort.  The reference's span map is global
(Traces.ts:117-123): an id in two shards must make the sharded run refuse."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("device", [False, True])
def test_route_ids_equals_host_mirror(engine, world, device):
    from kmamiz_amd import dist as kdist
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 3000)
    engine.load(batch, synth.shape_table(synth.MESH))
    n = len(batch)
    out = torch.zeros(n, dtype=torch.int64, device="cuda" if device else "cpu")
    counts = engine.route_ids(world, out.data_ptr(), n, device)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    h, c = kdist.route_ids_np(batch.span_id, world)
    assert counts == c.tolist()
    o = 0
    for r in range(world):  # each owner's segment holds exactly its hashes (order inside is free)
        assert np.array_equal(np.sort(got[o : o + counts[r]]), np.sort(h[o : o + counts[r]]))
        o += counts[r]


@pytest.mark.parametrize("m", [2, 1000, 1 << 20, 3_000_000])
def test_id_repeats_finds_one_repeat(engine, m):
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 20)
    engine.load(batch, synth.shape_table(synth.MESH))  # (any loaded batch: the check reads only its input)
    rng = np.random.default_rng(m)
    v = np.unique(rng.integers(1, 2**64 - 1, size=m + m // 8 + 8, dtype=np.uint64))[:m]
    rng.shuffle(v)
    assert len(v) == m
    assert engine.id_repeats(v.ctypes.data, m, False) is False
    w = v.copy()
    w[m - 1] = w[m // 3]
    assert engine.id_repeats(w.ctypes.data, m, False) is True
    d = torch.from_numpy(w.view(np.int64)).cuda()
    torch.cuda.synchronize()
    assert engine.id_repeats(d.data_ptr(), m, True) is True


def test_id_repeats_past_1e8_values(engine):
    """1.5e8 values: the certificate's split runs in rounds (2^10 sub-bins,
    k_cert_split_r); distinct values pass, one repeat is found."""
    from kmamiz_amd import synth

    batch, _ = synth.host_batch(synth.MESH, 0, 20)
    engine.load(batch, synth.shape_table(synth.MESH))
    m = 150_000_000
    v = torch.arange(1, m + 1, dtype=torch.int64, device="cuda") * 0x2545F4914F6CDD1D  # odd: distinct mod 2^64
    torch.cuda.synchronize()
    assert engine.id_repeats(v.data_ptr(), m, True) is False
    v[m - 7] = v[12345]
    torch.cuda.synchronize()
    assert engine.id_repeats(v.data_ptr(), m, True) is True
    del v
    torch.cuda.empty_cache()
