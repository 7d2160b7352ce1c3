"""Multi-GPU layout (jleveldb_amd/shard.py) in multi-process
jobs over gloo.

* CPU (world_size 2 and 3): each rank takes its shard of a set exactly as
  bench.py does — C2/C4 fixed blocks generated from the shard's first splitmix64
  word, C3 variable blocks cut at the byte prefix sum, C5 logs cut on 32 KiB
  log-block boundaries — checksums / verifies it with the oracle, the ranks
  all-gather the (unequal) per-rank results, SUM-reduce the mismatch counts and
  MAX-reduce their times; rank 0 checks the gathered results against the
  oracle over the whole set.  This proves the layout: no data-path collective
  is needed for a bit-exact answer.
* GPU (`-m gpu`, world_size 2 on the box's one GPU, gloo for the collectives):
  the same C3 and C5 jobs with every rank running the PRODUCT (libjlcrc's
  jl_crc32c_batch_dev / jl_log_verify_dev on cuda:0) on its shard; the gathered
  results must equal the oracle over the whole set.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from jleveldb_amd import shard as shd
from jleveldb_amd import workloads as wl

SEED = 0x4A4C4442
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(rank, world, port, job, args, q):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        res = globals()[job](rank, world, *args)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


def _run_world(job, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, world, port, job, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


# ------------------------------------------------------------------ datasets
def _c3_set(n):
    from oracle import oracle

    lens = wl.c3_lengths(n, SEED)
    offs = wl.packed_offsets(lens)
    arena = oracle.fill_splitmix(int(lens.sum(dtype=np.uint64)) + 8, SEED + 3)
    return arena, offs, lens


def _c5_log(n_payloads, flips=()):
    from oracle import oracle

    rng = np.random.default_rng(SEED + 11)
    sizes = np.concatenate([rng.integers(0, 200, n_payloads // 2), rng.integers(1000, 70000, n_payloads // 10),
                            np.full(n_payloads - n_payloads // 2 - n_payloads // 10, 1056)])
    rng.shuffle(sizes)
    log = bytearray(oracle.log_write([rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in sizes]))
    for f in flips:
        log[f % len(log)] ^= 0x20
    return bytes(log)


def _live_u64(ev):
    ev = ev[ev["kind"] != 0]
    return np.stack([ev["offset"], ev["length"].astype(np.uint64), ev["type"].astype(np.uint64),
                     ev["kind"].astype(np.uint64)]).T.copy()


# ------------------------------------------------------------------ rank jobs
def _job_weak_fixed(rank, world, n):
    import torch

    from oracle import oracle

    sh = shd.weak_shard(rank, world, n)
    data = oracle.fill_splitmix(n * 4096, SEED, sh.first_word)
    local = torch.from_numpy(oracle.fixed(data, 4096, n).view(np.int32))
    wall = shd.job_wall_time(0.01 * (rank + 1))
    return wall, shd.gather_results(local).numpy().view(np.uint32).copy()


def _job_strong_unequal(rank, world, total):
    import torch

    sh = shd.strong_shard(rank, world, total)
    local = torch.arange(sh.first_block, sh.first_block + sh.n_blocks, dtype=torch.int64)
    return shd.gather_results(local).numpy().copy()


def _c3_rank(rank, world, n, product):
    import torch

    arena, offs, lens = _c3_set(n)
    sh = shd.byte_shard(rank, world, offs, lens)
    sl = slice(sh.first_block, sh.first_block + sh.n_blocks)
    part = np.ascontiguousarray(arena[sh.byte_lo:sh.byte_hi])
    loff = offs[sl] - np.uint64(sh.byte_lo)
    if product:
        import jleveldb_amd as jl

        torch.cuda.set_device(0)
        jl.init(0)
        dev = torch.device("cuda:0")
        got = jl.crc32c_batch_dev(torch.from_numpy(np.concatenate([part, np.zeros(16, np.uint8)])).to(dev),
                                  torch.from_numpy(loff.view(np.int64)).to(dev),
                                  torch.from_numpy(lens[sl].view(np.int32)).to(dev)).cpu()
        torch.cuda.synchronize()
    else:
        from oracle import oracle

        got = torch.from_numpy(oracle.batch(part, loff, lens[sl]).view(np.int32))
    nbytes = shd.gather_results(torch.tensor([sh.byte_hi - sh.byte_lo], dtype=torch.int64)).numpy()
    return nbytes, shd.gather_results(got).numpy().view(np.uint32).copy()


def _job_c3_oracle(rank, world, n):
    return _c3_rank(rank, world, n, False)


def _job_c3_product(rank, world, n):
    return _c3_rank(rank, world, n, True)


def _c5_rank(rank, world, n_payloads, flips, product):
    import torch

    import jleveldb_amd as jl

    log = np.frombuffer(_c5_log(n_payloads, flips), dtype=np.uint8)
    sh = shd.log_shard(rank, world, log.size)
    part = np.ascontiguousarray(log[sh.byte_lo:sh.byte_hi])
    if product:
        torch.cuda.set_device(0)
        jl.init(0)
        ev, n = jl.log_verify_dev(torch.from_numpy(part).to(torch.device("cuda:0")))
        ev = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
    else:
        from oracle import oracle

        ev = oracle.log_events(part)
    live = _live_u64(ev)
    live[:, 0] += np.uint64(sh.byte_lo)  # shard-relative header offsets -> file offsets
    bad = int((live[:, 3] == jl.LOG_BAD_CRC).sum())
    total_bad = shd.total_mismatches(bad)
    got = shd.gather_results(torch.from_numpy(live.reshape(-1).view(np.int64))).numpy().view(np.uint64)
    return total_bad, got.reshape(-1, 4).copy()


def _job_c5_oracle(rank, world, n_payloads, flips):
    return _c5_rank(rank, world, n_payloads, flips, False)


def _job_c5_product(rank, world, n_payloads, flips):
    return _c5_rank(rank, world, n_payloads, flips, True)


# ------------------------------------------------------------------ CPU tests
def test_weak_shards_gloo_world2():
    from oracle import oracle

    oracle.build()
    world, n = 2, 96
    wall, got = _run_world("_job_weak_fixed", world, n)
    assert wall == pytest.approx(0.02)  # max over ranks
    whole = oracle.fill_splitmix(world * n * 4096, SEED, 0)
    assert np.array_equal(got, oracle.fixed(whole, 4096, world * n))
    assert shd.aggregate_rate(n * 4096, world, 1.0, 1) == pytest.approx(world * n * 4096 / 2**30)


def test_gather_unequal_strong_shards_gloo_world3():
    got = _run_world("_job_strong_unequal", 3, 1000)  # 334 + 333 + 333 blocks
    assert np.array_equal(got, np.arange(1000))


@pytest.mark.parametrize("world", [2, 3])
def test_c3_byte_shards_gloo(world):
    from oracle import oracle

    oracle.build()
    n = 600
    nbytes, got = _run_world("_job_c3_oracle", world, n)
    arena, offs, lens = _c3_set(n)
    assert np.array_equal(got, oracle.batch(arena, offs, lens))
    total = int(lens.sum(dtype=np.uint64))
    assert int(nbytes.sum()) == total
    assert int(nbytes.max()) - total // world <= int(lens.max())  # byte-balanced to within one block


def test_c5_log_shards_gloo_world2():
    from oracle import oracle

    oracle.build()
    flips = (19, 32768 + 1000, 5 * 32768 + 77, 9 * 32768 + 4)
    total_bad, got = _run_world("_job_c5_oracle", 2, 400, flips)
    want = _live_u64(oracle.log_events(_c5_log(400, flips)))
    assert np.array_equal(got, want)
    assert total_bad == int((want[:, 3] == 2).sum()) >= 2


@pytest.mark.parametrize("total,world", [(8 << 20, 8), (1000, 3), (7, 4), (0, 2)])
def test_strong_shards_cover_the_set(total, world):
    shards = [shd.strong_shard(r, world, total) for r in range(world)]
    assert shards[0].first_block == 0
    for a, b in zip(shards, shards[1:]):
        assert b.first_block == a.first_block + a.n_blocks
    assert sum(s.n_blocks for s in shards) == total
    assert max(s.n_blocks for s in shards) - min(s.n_blocks for s in shards) <= 1


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_byte_and_log_shards_cover_the_set(world):
    lens = wl.c3_lengths(5000, SEED)
    offs = wl.packed_offsets(lens)
    bs = [shd.byte_shard(r, world, offs, lens) for r in range(world)]
    assert bs[0].first_block == 0 and sum(s.n_blocks for s in bs) == lens.size
    for a, b in zip(bs, bs[1:]):
        assert b.first_block == a.first_block + a.n_blocks
    for log_bytes in (0, 1, 32768, 32769, 10 * 32768 + 5):
        ls = [shd.log_shard(r, world, log_bytes) for r in range(world)]
        assert ls[0].byte_lo == 0 and ls[-1].byte_hi == log_bytes
        for a, b in zip(ls, ls[1:]):
            assert b.byte_lo == a.byte_hi and (a.byte_lo % 32768 == 0 or a.byte_lo == log_bytes)


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


def test_bench_refuses_more_gpus_than_visible():
    # bench.py --gpus N launches N ranks itself; without N GPUs it must fail loudly
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2 and "--gpus 64" in r.stderr


# ------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
def test_c3_byte_shards_product_world2(gpu, oracle):
    nbytes, got = _run_world("_job_c3_product", 2, 3000)
    arena, offs, lens = _c3_set(3000)
    assert np.array_equal(got, oracle.batch(arena, offs, lens))


@pytest.mark.gpu
def test_c5_log_shards_product_world2(gpu, oracle):
    flips = (19, 32768 + 1000, 5 * 32768 + 77, 9 * 32768 + 4, 40 * 32768 + 999)
    total_bad, got = _run_world("_job_c5_product", 2, 2000, flips)
    want = _live_u64(oracle.log_events(_c5_log(2000, flips)))
    assert np.array_equal(got, want)
    assert total_bad == int((want[:, 3] == 2).sum()) >= 2
