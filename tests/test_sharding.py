"""Multi-rank path on CPU: world_size-2 gloo.  Each rank
evaluates its slice of one ray batch and rank 0 gathers; the gathered buffer
must equal the single-process result bit for bit.  The per-rank compute here
is the oracle (no GPU in this container) -- what is under test is the
partitioning and the gather, which the GPU path (bench.py --gather) shares."""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sunsky_amd.sharding import gather_radiance, shard_range, shard_sizes

from helpers import angles_dict, hemisphere_wo

SCENE = angles_dict(6.0, 0.3, np.deg2rad(40), 0.1, 1.0, 1.0)


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 17, 1000, 1 << 16, (1 << 16) + 3])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0
    for a, b in spans:
        assert (a % 4 == 0 or a == b == n) and b >= a   # 16-byte aligned starts (empty tail shards excepted)
    sizes = shard_sizes(n, world)
    assert sum(sizes) == n and max(sizes) - min(sizes) <= 7   # one 4-ray block + a partial tail


def test_shard_range_errors():
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)
    with pytest.raises(ValueError):
        shard_range(10, 0, 0)


def _init(rank, world, store):
    # a file store in the test's own temporary directory: no port picked in advance that a
    # parallel test could take in between (pytest -n)
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)


def _worker(rank, world, store, n, out_path):
    _init(rank, world, store)
    try:
        import oracle as O
        wi = -hemisphere_wo(n, seed=5)          # every rank can regenerate the batch
        a, b = shard_range(n, rank, world)
        local = O.Oracle(SCENE, "rgb", "jit", "f32").eval(wi[a:b])
        full = gather_radiance(torch.from_numpy(np.ascontiguousarray(local.T)), n)
        if rank == 0:
            np.save(out_path, full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [4096 + 3, 10000])
def test_gloo_world2_gather_matches_single_process(tmp_path, n):
    store = str(tmp_path / "rdv")
    out = str(tmp_path / "full.npy")
    mp.start_processes(_worker, args=(2, store, n, out), nprocs=2, join=True, start_method="spawn")
    import oracle as O
    ref = O.Oracle(SCENE, "rgb", "jit", "f32").eval(-hemisphere_wo(n, seed=5)).T
    got = np.load(out)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def _key_worker(rank, world, store, out_path):
    from sunsky_amd.sharding import _group_key
    dev = torch.device("cuda", 0)               # a device object only: no GPU is touched
    keys = [_group_key(None, dev)]
    _init(rank, world, store)
    keys.append(_group_key(None, dev))
    dist.destroy_process_group()
    keys.append(_group_key(None, dev))
    if rank == 1:
        np.save(out_path, np.array(keys, dtype=object), allow_pickle=True)


def test_comm_cache_key_tracks_the_world(tmp_path):
    """the cached RCCL communicator is keyed by the group's rank and size, so a
    world of another size never reuses one, and a process without torch.distributed gets its
    own world-1 key (a same-size re-initialisation: the test below)."""
    store = str(tmp_path / "rdv")
    out = str(tmp_path / "keys.npy")
    mp.start_processes(_key_worker, args=(2, store, out), nprocs=2, join=True, start_method="spawn")
    keys = [tuple(k) for k in np.load(out, allow_pickle=True)]
    assert keys[0] == (None, 0, 0, 1) and keys[2] == keys[0]
    assert keys[1] == (None, 0, 1, 2)


class _FakeComm:
    """Stands in for RadianceComm (no GPU here): counts constructions and closes."""
    made = []

    def __init__(self, group, dev):
        self._h = len(_FakeComm.made) + 1
        _FakeComm.made.append(self)

    def close(self):
        self._h = None


def _reinit_worker(rank, world, store, out_path):
    from sunsky_amd.sharding import clear_radiance_comms, radiance_comm
    dev = torch.device("cuda", 0)               # a device object only: no GPU is touched
    _init(rank, world, store)
    a = radiance_comm(device=dev, _factory=_FakeComm)
    a2 = radiance_comm(device=dev, _factory=_FakeComm)
    dist.destroy_process_group()
    _init(rank, world, store + ".2")   # same rank, same size
    b = radiance_comm(device=dev, _factory=_FakeComm)
    res = [a is a2, b is not a, a._h is None, b._h is not None, len(_FakeComm.made)]
    clear_radiance_comms()
    res.append(b._h is None)
    dist.destroy_process_group()
    if rank == 1:
        np.save(out_path, np.array(res, dtype=object), allow_pickle=True)


def test_comm_cache_same_size_reinit_gets_a_new_communicator(tmp_path):
    """a world destroyed and re-initialised with the same rank and size has a new
    process group object; the cached communicator built over the old one is closed and a new
    one created, never reused."""
    store = str(tmp_path / "rdv")
    out = str(tmp_path / "reinit.npy")
    mp.start_processes(_reinit_worker, args=(2, store, out), nprocs=2, join=True, start_method="spawn")
    res = list(np.load(out, allow_pickle=True))
    assert res == [True, True, True, True, 2, True], res
