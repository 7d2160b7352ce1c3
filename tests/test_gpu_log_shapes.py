"""Log verification (jl_log_verify_dev: lc_walk, lc_dense, the chunk rounds
through crc_gv4_kernel<MODE_LOG_CHUNK>, lc_combine, lc_apply) against the oracle's
readPhysicalRecord walk (J/db/LogReader.java:297-383), event for event, on log
shapes at the edges of its block classification:

* uniform runs of every length 0..300 (every start alignment; 1-byte crc ranges;
  blocks just below, at and above lc_walk's dense thresholds);
* dense blocks (DBBench-like 131-B records) holding one long record of 2.5-32 KB
  (lc_dense: one thread per record, any length);
* a uniform start followed by lengths that keep changing;
* blocks of 0-byte records (4 681 events per block);
* flipped bytes in the first, a middle and the last record of a block, and in a
  header length, for 131-B (dense) and 1 056-B (chunk rounds) records.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x4A4C4442


def _live(ev):
    ev = ev[ev["kind"] != 0]
    return np.stack([ev["offset"], ev["length"].astype(np.uint64), ev["type"].astype(np.uint64),
                     ev["kind"].astype(np.uint64)])


def _log(jl, gpu, lens, seed=SEED):
    import torch

    lens = np.asarray(lens, dtype=np.uint32)
    offs = np.zeros(lens.size, np.uint64)
    if lens.size > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    plan = jl.log_layout(offs, lens)
    src = torch.empty(max(1, int(lens.sum(dtype=np.uint64))), dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(src, seed)
    return jl.log_emit_dev(src, plan)


def _check(jl, oracle, log):
    ev, n = jl.log_verify_dev(log)
    got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
    want = oracle.log_events(log.cpu().numpy())
    g, w = _live(got), _live(want)
    assert g.shape == w.shape and np.array_equal(g, w)
    return want


def _runs(spec, reps=1):
    out = []
    for length, count in spec:
        out += [length] * count
    return out * reps


def test_uniform_runs_every_length(gpu, jl, oracle):
    lens = []
    for n in range(0, 301):
        lens += [n] * max(8, 4096 // (n + 7))  # a few blocks' worth per length, every alignment
    w = _check(jl, oracle, _log(jl, gpu, lens))
    assert bool((w["kind"] == jl.LOG_OK).all())


@pytest.mark.parametrize("long_len", [2500, 4090, 4200, 9000, 20000, 32000])
def test_dense_blocks_with_a_long_record(gpu, jl, oracle, long_len):
    # 6 x 131 B, one long record, 40 x 131 B, repeated: dense blocks holding a long record
    lens = _runs([(131, 6), (long_len, 1), (131, 40)], reps=60)
    log = _log(jl, gpu, lens)
    w = _check(jl, oracle, log)
    assert bool((w["kind"] == jl.LOG_OK).all())
    # a flip inside a long record: BAD_CRC there, the rest of its block dropped
    ok = w[(w["kind"] == jl.LOG_OK) & (w["length"] == long_len)]
    victim = int(ok["offset"][len(ok) // 2]) + 7 + long_len // 2
    log[victim] ^= 0x10
    w = _check(jl, oracle, log)
    assert int((w["kind"] == jl.LOG_BAD_CRC).sum()) >= 1


def test_uniform_start_then_changing_lengths(gpu, jl, oracle):
    rng = np.random.default_rng(SEED + 1)
    lens = []
    for _ in range(300):
        lens += [200] * 6 + list(rng.integers(1, 400, 60))
    _check(jl, oracle, _log(jl, gpu, lens))


def test_uniform_zero_length_records(gpu, jl, oracle):
    # 7-B records: ~4 681 events per block
    lens = [0] * (32768 // 7 * 40)
    _check(jl, oracle, _log(jl, gpu, lens))


@pytest.mark.parametrize("rec", [131, 1056])
def test_block_flips(gpu, jl, oracle, rec):
    lens = [rec] * ((64 << 20) // (rec + 7))
    log = _log(jl, gpu, lens)
    w = _check(jl, oracle, log)
    assert bool((w["kind"] == jl.LOG_OK).all())
    nb = log.numel() >> 15
    # first record's payload, a middle one, the block's last bytes, a header length byte
    for blk, off in ((3, 12), (nb // 2, 16_000), (nb // 3, 32_760), (nb - 3, 7 + rec + 7 + 4)):
        log[blk * 32768 + off] ^= 0x01
    w = _check(jl, oracle, log)
    assert int(((w["kind"] != 0) & (w["kind"] != jl.LOG_OK)).sum()) >= 3


def test_dense_list_in_chunks_random_lengths(gpu, jl, oracle):
    """~1.1 GiB of short records of random lengths (0-200 B) with runs of equal
    ones (mostly 1-3 long, some of 200-600): more than 32 768 dense blocks, so
    lc_dense takes its list in chunks of 2 (ld_chunk sizes them by the list), and
    every block walks 300+ runs in passes of 256 with runs that join the record
    before them (the look-back walk), trips past 257 records included.  Flips in
    payloads and in a header; every event against the oracle."""
    rng = np.random.default_rng(SEED + 7)
    m = (int(1.1 * (1 << 30)) // 107) // 3
    runs = np.where(rng.random(m) < 0.01, rng.integers(200, 600, m), rng.integers(1, 4, m))
    lens = np.repeat(rng.integers(0, 201, m), runs).astype(np.uint32)
    log = _log(jl, gpu, lens)
    assert log.numel() // 32768 > 32768
    for at in rng.integers(0, log.numel(), 6):
        log[int(at)] ^= 0x10
    w = _check(jl, oracle, log)
    assert int((w["kind"] == jl.LOG_BAD_CRC).sum()) >= 1


@pytest.mark.parametrize("seed", [101, 202])
def test_mixed_shapes_many_flips(gpu, jl, oracle, seed):
    """~2 GB logs mixing short random-length records (runs of 1-3 and of
    200-600 equal ones), DBBench-like 131-B stretches and long records
    (500 B - 40 KB: dense blocks' deferred records and chunk rounds), 300 bit
    flips; every live event against the oracle, checksum on and off (the
    stress that found lc_dense's first_bad race, at this size)."""
    rng = np.random.default_rng(seed)
    m = (int(1.0 * (1 << 30)) // 120) // 3
    kind = rng.random(m)
    runs = np.where(kind < 0.01, rng.integers(200, 600, m), rng.integers(1, 4, m))
    vals = np.where(kind > 0.999, rng.integers(500, 40000, m), rng.integers(0, 201, m))
    vals = np.where((kind > 0.5) & (kind < 0.52), 131, vals)
    log = _log(jl, gpu, np.repeat(vals, runs), seed=seed)
    for at in rng.integers(0, log.numel(), 300):
        log[int(at)] ^= 1 << int(rng.integers(0, 8))
    host = log.cpu().numpy()
    for checksum in (True, False):
        ev, n = jl.log_verify_dev(log, checksum)
        got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
        g, w = _live(got), _live(oracle.log_events(host, checksum=checksum))
        assert g.shape == w.shape and np.array_equal(g, w), checksum
