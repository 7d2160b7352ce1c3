"""Multi-GPU layout (jleveldb_amd/shard.py) on the CPU: a
world_size-2 gloo job in which each rank generates its shard of the C4 block set
exactly as bench.py does on a GPU (splitmix64 from the shard's first word),
checksums it with the oracle, and the ranks then all-gather the results and
max-reduce their times.  Rank 0 checks the gathered results against the oracle
over the whole set: no data-path collective is needed for a bit-exact answer."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from jleveldb_amd import shard as shd

SEED = 0x4A4C4442


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n, q):
    import torch
    import torch.distributed as dist

    from oracle import oracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sh = shd.weak_shard(rank, world, n)
        data = oracle.fill_splitmix(n * 4096, SEED, sh.first_word)
        local = torch.from_numpy(oracle.fixed(data, 4096, n).view(np.int32))
        wall = shd.job_wall_time(0.01 * (rank + 1))
        gathered = shd.gather_results(local, world)
        if rank == 0:
            q.put((wall, gathered.numpy().view(np.uint32).copy()))
    finally:
        dist.destroy_process_group()


def test_weak_shards_gloo_world2():
    from oracle import oracle

    oracle.build()
    world, n = 2, 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    wall, got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert wall == pytest.approx(0.02)  # max over ranks
    whole = oracle.fill_splitmix(world * n * 4096, SEED, 0)
    assert np.array_equal(got, oracle.fixed(whole, 4096, world * n))
    assert shd.aggregate_rate(n * 4096, world, 1.0, 1) == pytest.approx(world * n * 4096 / 2**30)


@pytest.mark.parametrize("total,world", [(8 << 20, 8), (1000, 3), (7, 4), (0, 2)])
def test_strong_shards_cover_the_set(total, world):
    shards = [shd.strong_shard(r, world, total) for r in range(world)]
    assert shards[0].first_block == 0
    for a, b in zip(shards, shards[1:]):
        assert b.first_block == a.first_block + a.n_blocks
    assert sum(s.n_blocks for s in shards) == total
    assert max(s.n_blocks for s in shards) - min(s.n_blocks for s in shards) <= 1


def test_shard_first_word_matches_device_generator():
    # jl_fill_random_dev(first_word=r*n*512) on rank r == bytes of the global set
    from oracle import oracle

    oracle.build()
    n = 3
    whole = oracle.fill_splitmix(4 * n * 4096, SEED, 0)
    for r in range(4):
        sh = shd.weak_shard(r, 4, n)
        part = oracle.fill_splitmix(n * 4096, SEED, sh.first_word)
        assert np.array_equal(part, whole[sh.first_block * 4096:(sh.first_block + n) * 4096])
