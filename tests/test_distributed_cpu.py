"""CPU (gloo, world_size 2): the data-parallel gradient averaging and the sweep sharder."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from vit_amd import parallel
    r, w, _ = parallel.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    g = torch.Generator().manual_seed(rank)
    flat = torch.randn(1_000_003, generator=g)
    expect = sum(torch.randn(1_000_003, generator=torch.Generator().manual_seed(k)) for k in range(world)) / world
    parallel.allreduce_flat(flat, bucket_mb=1.0)
    q.put((rank, float((flat - expect).abs().max())))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_flat_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err in res:
        assert err < 1e-5, (rank, err)


class _FlatModel:
    def __init__(self, flat):
        self.flat_grad = flat
        self.hook = None

    def set_grad_ready_hook(self, fn):
        self.hook = fn


def _worker_overlap(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from vit_amd import parallel
    parallel.init_from_env(backend="gloo")
    n = 100_003
    flat = torch.randn(n, generator=torch.Generator().manual_seed(rank))
    expect = sum(torch.randn(n, generator=torch.Generator().manual_seed(k)) for k in range(world)) / world
    m = _FlatModel(flat)
    red = parallel.OverlappedGradReduce(m)
    # block spans reported during "backward" (out of order, leaving gaps at both ends and between)
    m.hook(50_000, 70_000)
    m.hook(10_000, 30_000)
    m.hook(30_000, 50_000)
    red.finish()
    err = float((flat - expect).abs().max())
    # second step reuses the reducer: everything reduced again in finish() alone
    flat.copy_(torch.full((n,), float(rank)))
    red.finish()
    err2 = float((flat - (world - 1) / 2).abs().max())
    q.put((rank, err, err2))
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_grad_reduce_world2():
    """OverlappedGradReduce: block spans reduced as they are reported, the rest in finish()."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, err2 in res:
        assert err < 1e-5 and err2 < 1e-6, (rank, err, err2)


def test_shard_conditions_partition_and_chains():
    from vit_amd import parallel
    conds = parallel.length_sweep_conditions()
    assert len(conds) == 136  # the reference's grid (sweep.reference_length_grid)
    world = 8
    shards = [parallel.shard_conditions(conds, world, r) for r in range(world)]
    allc = sorted(c for s in shards for c in s)
    assert allc == sorted(conds)                       # exact partition
    for s in shards:                                   # start-epoch chains stay together
        starts = {c[0] for c in s}
        for st in starts:
            assert sorted(c for c in conds if c[0] == st) == sorted(c for c in s if c[0] == st)
    loads = [sum(c[1] for c in s) for s in shards]
    chain = {}
    for c in conds:
        chain[c[0]] = chain.get(c[0], 0) + c[1]
    assert max(loads) - min(loads) <= max(chain.values())  # LPT over whole chains
    assert shards == [parallel.shard_conditions(conds, world, r) for r in range(world)]  # deterministic


def test_bucket_bounds():
    from vit_amd import parallel
    assert parallel.bucket_bounds(10, 4) == [(0, 4), (4, 8), (8, 10)]
    assert parallel.bucket_bounds(86_567_656, 16 * 1024 * 1024)[-1][1] == 86_567_656


class _FeatModel(torch.nn.Module):
    """Stand-in with timm's forward_features surface: [B, 3, 4, 4] -> [B, 2, 16] (row 0 = CLS)."""
    global_pool = "token"

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.randn(48, 32, generator=torch.Generator().manual_seed(3)))

    def forward_features(self, x):
        return torch.tanh(x.flatten(1) @ self.w).reshape(x.shape[0], 2, 16)


def _rsa_inputs():
    import numpy as np
    g = torch.Generator().manual_seed(7)
    images = torch.randn(48, 3, 4, 4, generator=g)
    a = np.random.default_rng(8).random((48, 48))
    ref = (a + a.T) / 2
    np.fill_diagonal(ref, 0.0)
    return images, ref


def _worker_rsa(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from vit_amd import parallel, rsa
    parallel.init_from_env(backend="gloo")
    images, ref = _rsa_inputs()
    m = _FeatModel()
    out = {o: rsa.compute_rsa_score(m, images, ref, world=world, rank=rank, order=o) for o in ("image", "reference")}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 5])
def test_compute_rsa_score_world(world):
    """compute_rsa_score (MEAS:298-355) across gloo ranks: 'image' order equals the world-1 score;
    'reference' order reproduces the reference's rank-concatenated rows, including
    DistributedSampler's padding when 48 is not a multiple of the world size."""
    import numpy as np
    from vit_amd import rsa
    images, ref = _rsa_inputs()
    m = _FeatModel()
    single = rsa.compute_rsa_score(m, images, ref)
    emb = rsa.cls_embeddings(m, images)
    quirk = [i for r in range(world) for i in rsa.sampler_indices(48, world, r)][:48]
    want_ref = rsa.rsa(emb[quirk], ref)[:2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_rsa, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r]["image"] == (None, None) for r in range(1, world))
    assert np.allclose(res[0]["image"], single, rtol=0, atol=1e-12)
    assert np.allclose(res[0]["reference"], want_ref, rtol=0, atol=1e-12)
    assert abs(res[0]["reference"][0] - single[0]) > 1e-6  # the quirk changes the score


def test_sampler_indices_match_distributed_sampler():
    from torch.utils.data import DistributedSampler
    from vit_amd import rsa
    for n, world in ((48, 2), (48, 5), (7, 3), (3, 8)):
        for r in range(world):
            s = DistributedSampler(range(n), num_replicas=world, rank=r, shuffle=False)
            assert rsa.sampler_indices(n, world, r) == list(iter(s)), (n, world, r)
