"""The one-launch small-log path (lc_small_kernel, log_chunks.hip; JL_OPT_LOG_SMALL_MAX)
against the oracle's readPhysicalRecord walk (J/db/LogReader.java:297-383), event
for event, and against the chunked path on the same logs.

Cases: the four C5 record shapes at the reference's call sizes (one WAL of the
4 MiB write buffer, J/Options.java:203, recovered at J/db/DBImpl.java:903) and
around them, with flips; blocks of more runs than one pass keeps (several passes
per block); runs of long records (the wave crc inside a trip); records of the
maximum fragment size; an unaligned device log; the EOF cases of a short last
block; a short event array; the asynchronous form; logs of alternating sizes
through one workspace (the look-back statuses of earlier calls must never
match); more blocks than the 64 statuses one look-back step reads.
"""
import ctypes

import numpy as np
import pytest

from jleveldb_amd import workloads as wl

pytestmark = pytest.mark.gpu

SEED = 0x4A4C4442
SMALL, CHUNKED = 64 << 20, 0


def _live(ev):
    ev = ev[ev["kind"] != 0]
    return np.stack([ev["offset"], ev["length"].astype(np.uint64), ev["type"].astype(np.uint64),
                     ev["kind"].astype(np.uint64)])


def _log(jl, gpu, lens, seed=SEED):
    import torch

    lens = np.asarray(lens, dtype=np.uint32)
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(max(1, int(lens.sum(dtype=np.uint64))), dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(src, seed)
    return jl.log_emit_dev(src, plan)


def _dev(jl, log, checksum=True):
    ev, n = jl.log_verify_dev(log, checksum)
    return ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE).copy()


def _both(jl, engine_options, oracle, log, checksum=True):
    """Small path == chunked path (all events, kind-0 drops included) == oracle (live events)."""
    engine_options(jl.OPT_LOG_SMALL_MAX, SMALL)
    small = _dev(jl, log, checksum)
    engine_options(jl.OPT_LOG_SMALL_MAX, CHUNKED)
    chunked = _dev(jl, log, checksum)
    engine_options(jl.OPT_LOG_SMALL_MAX, SMALL)
    assert small.size == chunked.size and np.array_equal(small, chunked)
    want = oracle.log_events(log.cpu().numpy(), checksum=checksum)
    g, w = _live(small), _live(want)
    assert g.shape == w.shape and np.array_equal(g, w)
    return small


@pytest.mark.parametrize("which", ["c1_1056", "mixed_1b_100k", "dbbench_131", "random_0_200"])
@pytest.mark.parametrize("mib", [0.25, 1, 4, 16])
def test_shapes_and_sizes(gpu, jl, oracle, engine_options, which, mib):
    lens = wl.c5_lengths(which, target=int(mib * (1 << 20)), seed=SEED + int(mib * 4))
    log = _log(jl, gpu, lens)
    nb = (log.numel() + 32767) >> 15
    rng = np.random.default_rng(SEED + nb)
    for _ in range(max(1, nb // 8)):  # flips in payloads and headers
        log[int(rng.integers(0, log.numel()))] ^= 1 << int(rng.integers(0, 8))
    for checksum in (True, False):
        _both(jl, engine_options, oracle, log, checksum)


@pytest.mark.parametrize("maxlen", [12, 40])
def test_more_runs_than_a_pass(gpu, jl, oracle, engine_options, maxlen):
    """0..maxlen-B records of random lengths: 700-2000 runs per block, kSRuns = 512
    kept per pass (2-4 passes), flips in later passes' records."""
    rng = np.random.default_rng(SEED + maxlen)
    lens = rng.integers(0, maxlen + 1, (3 << 20) // (maxlen // 2 + 7)).astype(np.uint32)
    log = _log(jl, gpu, lens)
    w = _both(jl, engine_options, oracle, log)
    ok = w[(w["kind"] == 1) & (w["length"] > 0)]
    for b in range(1, (log.numel() >> 15) - 1, 9):  # the last OK record of some blocks
        sel = ok[(ok["offset"] >> 15) == b]
        if sel.size:
            log[int(sel["offset"][-1]) + 7] ^= 0x40
    _both(jl, engine_options, oracle, log)


@pytest.mark.parametrize("big", [520, 2000, 9000, 32761])
def test_runs_of_long_records(gpu, jl, oracle, engine_options, big):
    """Equal long records (a trip extends their run; each checked by a wave), the
    maximum fragment payload 32761 B, and short ones around them; flips."""
    lens = ([big] * 5 + [100] * 3 + [big + 1] * 2) * 12
    log = _log(jl, gpu, lens)
    w = _both(jl, engine_options, oracle, log)
    longs = w[(w["kind"] == 1) & (w["length"] >= min(big, 520))]
    for i in range(0, longs.size, 7):
        h, n = int(longs["offset"][i]), int(longs["length"][i])
        log[h + 7 + (i * 131) % n] ^= 0x08
    _both(jl, engine_options, oracle, log)


@pytest.mark.parametrize("shift", [1, 5, 15])
def test_unaligned_device_log(gpu, jl, oracle, engine_options, shift):
    import torch

    log = _log(jl, gpu, wl.c5_lengths("random_0_200", target=2 << 20, seed=SEED))
    buf = torch.zeros(log.numel() + 16, dtype=torch.uint8, device=gpu)
    buf[shift: shift + log.numel()] = log
    _both(jl, engine_options, oracle, buf[shift: shift + log.numel()])


@pytest.mark.parametrize("tail", [1, 3, 6, 7, 20, 1000])
def test_eof_cases(gpu, jl, oracle, engine_options, tail):
    """A log cut `tail` bytes into its last block (EOF truncation, EOF bad length)."""
    log = _log(jl, gpu, [300] * 400)
    cut = (log.numel() >> 15 << 15) + tail if (log.numel() >> 15 << 15) + tail <= log.numel() else log.numel() - 1
    _both(jl, engine_options, oracle, log[:cut].clone())


def test_capacity_error_with_full_count(gpu, jl, engine_options):
    import torch

    engine_options(jl.OPT_LOG_SMALL_MAX, SMALL)
    log = _log(jl, gpu, wl.c5_lengths("dbbench_131", target=1 << 20, seed=SEED))
    _, n_full = jl.log_verify_dev(log)
    ev = torch.zeros(100 * 16, dtype=torch.uint8, device=gpu)
    n = ctypes.c_uint64(0)
    rc = jl.lib().jl_log_verify_dev(log.data_ptr(), log.numel(), 1, ev.data_ptr(), 100, ctypes.byref(n),
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == -5 and n.value == n_full


def test_async_and_alternating_sizes(gpu, jl, oracle, engine_options):
    """Back-to-back asynchronous calls, then synchronous ones of alternating sizes
    (16 MiB: 512 blocks, more than one look-back step; 0.1 MiB; 9 MiB) through
    one workspace: each call's statuses carry its own tag."""
    import torch

    engine_options(jl.OPT_LOG_SMALL_MAX, SMALL)
    logs = [_log(jl, gpu, wl.c5_lengths(w, target=t, seed=SEED + i), seed=SEED + i)
            for i, (w, t) in enumerate([("c1_1056", 16 << 20), ("random_0_200", 100 << 10),
                                        ("dbbench_131", 9 << 20), ("mixed_1b_100k", 16 << 20)])]
    for log in logs:
        log[log.numel() // 2] ^= 0x01
    wants = [_live(oracle.log_events(x.cpu().numpy())) for x in logs]
    evs = [torch.zeros((x.numel() // 7 + 2) * 16, dtype=torch.uint8, device=gpu) for x in logs]
    res = [torch.zeros(3, dtype=torch.int64, device=gpu) for _ in logs]
    for _ in range(2):
        for x, e, r in zip(logs, evs, res):
            jl.log_verify_dev_async(x, events=e, result=r)
        torch.cuda.synchronize()
        for e, r, w in zip(evs, res, wants):
            n = int(r[0])
            assert int(r[2]) == 0
            assert np.array_equal(_live(e[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)), w)
    for i in [0, 1, 2, 1, 3, 0]:
        assert np.array_equal(_live(_dev(jl, logs[i])), wants[i])


def test_host_memory_log(gpu, jl, oracle, engine_options):
    """jl_log_verify from host memory: a 40 MiB log is one 64 MiB pipeline chunk;
    with JL_OPT_LOG_SMALL_MAX at 64 MiB it takes the one-launch path."""
    engine_options(jl.OPT_LOG_SMALL_MAX, SMALL)
    log = _log(jl, gpu, wl.c5_lengths("random_0_200", target=40 << 20, seed=SEED)).cpu().numpy()
    log[12345] ^= 0x02
    got = jl.log_verify(log)
    engine_options(jl.OPT_LOG_SMALL_MAX, CHUNKED)
    assert np.array_equal(got, jl.log_verify(log))
    assert np.array_equal(_live(got), _live(oracle.log_events(log)))
