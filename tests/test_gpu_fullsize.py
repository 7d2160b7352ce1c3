"""Full-size parity at the BASELINE.json configs the bench reports beside C2.

* C3: 1M blocks, k ~ Zipf(1.1) on 1..64, len = 1024(k-1) + 1 + U[0,1023]
  (1 B - 64 KiB), packed back-to-back in one ~12 GB arena (unaligned starts):
  every block vs the multithreaded oracle (`oracle.batch`, restating
  J/util/Crc32C.java:85-93,119-162 and the mask :61-75), plus a one-byte flip
  that must change exactly that block's CRC.
* C4: the 8M x 4 KiB (32 GiB) set on one GPU as its 8 strong shards, each
  generated in place from its first splitmix64 word as a rank of bench.py
  --gpus 8 generates it: the shards' results concatenate to the results of one
  32 GiB launch and equal the oracle block for block; a one-byte flip changes
  exactly one CRC.
* C5: 2^17 x 32 KiB log blocks (4 GiB) written by the product's batched
  LogWriter (jl_log_layout + jl_log_emit_dev, J/db/LogWriter.java:88-161) from
  the three payload sets bench.py reports (1 056-B C1-shaped records; mixed
  1 B - 100 KiB records that fragment FIRST/MIDDLE/LAST; DBBench-default 131-B
  records, every block dense), verified device-resident (jl_log_verify_dev and
  the asynchronous form) and compared event-for-event with the oracle's
  readPhysicalRecord walk (J/db/LogReader.java:297-383), clean and with byte
  flips in three blocks; plus a 256 MiB log of 0-40 B records of random lengths
  (~1 200 events per block: dense blocks whose walk cannot speculate).
"""
import numpy as np
import pytest

from jleveldb_amd import shard as shd
from jleveldb_amd import workloads as wl

pytestmark = pytest.mark.gpu

THREADS = 16
SEED = 0x4A4C4442


def _live(ev):
    ev = ev[ev["kind"] != 0]
    return np.stack([ev["offset"], ev["length"].astype(np.uint64), ev["type"].astype(np.uint64),
                     ev["kind"].astype(np.uint64)])


def test_full_size_c3_block_for_block(gpu, jl, oracle):
    import torch

    lens = wl.c3_lengths(1 << 20, SEED)  # the set bench.py reports
    n = lens.size
    offs = wl.packed_offsets(lens)
    total = int(lens.sum(dtype=np.uint64))
    arena = torch.empty(total, dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(arena, SEED + 3)
    d_off = torch.from_numpy(offs.view(np.int64)).to(gpu)
    d_len = torch.from_numpy(lens.view(np.int32)).to(gpu)
    got = jl.crc32c_batch_dev(arena, d_off, d_len).cpu().numpy().view(np.uint32)
    host = arena.cpu().numpy()
    want = oracle.batch(host, offs, lens, threads=THREADS)
    assert np.array_equal(got, want)
    del host
    victim = 777_777
    arena[int(offs[victim]) + int(lens[victim]) - 1] ^= 0x40
    got2 = jl.crc32c_batch_dev(arena, d_off, d_len).cpu().numpy().view(np.uint32)
    assert list(np.nonzero(got2 != got)[0]) == [victim]


@pytest.mark.parametrize("payloads", list(wl.C5_SETS) + ["short_0_40"])
def test_full_size_c5_log_verify(gpu, jl, oracle, payloads):
    import torch

    if payloads == "short_0_40":
        # 0-40 B records, 256 MiB of log: ~1 200 events per 32 KiB block, every
        # block dense (lc_dense), flips included
        rng = np.random.default_rng(SEED + 11)
        lens = rng.integers(0, 41, (256 << 20) // 27).astype(np.uint32)
        lens = lens[: int(np.searchsorted(np.cumsum(lens.astype(np.uint64) + 7), 256 << 20))]
    else:
        lens = wl.c5_lengths(payloads, seed=SEED)  # the sets bench.py reports
    offs = wl.packed_offsets(lens)
    plan = jl.log_layout(offs, lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(src, SEED + 5)
    log = jl.log_emit_dev(src, plan)
    del src
    nb = int(plan["log_bytes"])
    assert log.numel() == nb

    def check():
        ev, n = jl.log_verify_dev(log)
        got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
        want = oracle.log_events(log.cpu().numpy())
        g, w = _live(got), _live(want)
        assert g.shape == w.shape and np.array_equal(g, w)
        # the asynchronous form: complete events for any density, no second call
        ev2 = torch.zeros(n * 16, dtype=torch.uint8, device=gpu)
        _, res = jl.log_verify_dev_async(log, events=ev2)
        r = res.cpu().numpy()
        assert int(r[0]) == n and int(r[2]) == 0
        assert torch.equal(ev2, ev[: n * 16])
        return want

    w = check()
    assert w.size == plan["len"].size and bool((w["kind"] == jl.LOG_OK).all())
    # flips in three log blocks: a flipped payload byte is BAD_CRC and drops the
    # rest of its 32 KiB block (J/db/LogReader.java:359-367); a flipped header
    # length is a bad-length report.  Either way the walk must match the oracle.
    for blk in (5, min(70_000, (nb >> 15) - 4), (nb >> 15) - 2):
        log[blk * 32768 + 20_000] ^= 0x01
    w = check()
    assert int(((w["kind"] != 0) & (w["kind"] != jl.LOG_OK)).sum()) >= 3


def test_full_size_c4_strong_shards(gpu, jl, oracle):
    import torch

    total, world = 8 << 20, 8
    data = torch.empty(total * 4096, dtype=torch.uint8, device=gpu)  # 32 GiB
    jl.fill_random_dev(data, SEED)
    whole = jl.crc32c_fixed_dev(data, 4096, total)
    for r in range(world):
        sh = shd.strong_shard(r, world, total)
        part = torch.empty(sh.n_blocks * 4096, dtype=torch.uint8, device=gpu)
        jl.fill_random_dev(part, SEED, first_word=sh.first_word)
        assert torch.equal(part[:1 << 20], data[sh.first_block * 4096:sh.first_block * 4096 + (1 << 20)])
        got = jl.crc32c_fixed_dev(part, 4096, sh.n_blocks)
        assert torch.equal(got, whole[sh.first_block:sh.first_block + sh.n_blocks]), f"shard {r}"
        del part, got
    torch.cuda.empty_cache()
    want = oracle.fixed(data.cpu().numpy(), 4096, total, threads=THREADS)
    ref = whole.cpu().numpy().view(np.uint32)
    assert np.array_equal(ref, want)
    victim = 6_543_210
    data[victim * 4096 + 1234] ^= 0x08
    got2 = jl.crc32c_fixed_dev(data, 4096, total).cpu().numpy().view(np.uint32)
    assert list(np.nonzero(got2 != ref)[0]) == [victim]
