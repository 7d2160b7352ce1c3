"""The fused log-verify path (jleveldb_amd/csrc/log_stream.hip, JL_LOG_CHECKSUM_FUSED)
against the oracle's LogReader.readPhysicalRecord walk (J/db/LogReader.java:297-383)
and against the engine's two-pass path (JL_LOG_CHECKSUM_TWO_PASS: walk kernel +
batched crc), event for event.

The fused kernel walks each 32 KiB block's headers from the streamed bytes and
masks every record boundary inside a 128-B window, so the cases aim at the
window geometry: headers at every offset of a window (including the ones whose
7 bytes straddle into the next window), several tiny records in one window,
records that end exactly on a window or block edge, byte flips in every field
of a header and in payloads, the EOF cases of a short last block, blocks with
more records than the kernel's per-block slots (fallback path) and logs long
enough to run several rounds per wave with a partial last round.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("log_path")]

FUSED, TWO_PASS = 3, 2


def _live(ev):
    ev = ev[ev["kind"] != 0]
    return [(int(e["offset"]), int(e["length"]), int(e["type"]), int(e["kind"])) for e in ev]


def _check(jl, oracle, log, read_records=False):
    want = _live(oracle.log_events(log))
    assert _live(jl.log_verify(log, FUSED)) == want
    assert _live(jl.log_verify(log, TWO_PASS)) == want
    if read_records:
        assert jl.log_read_records(log, FUSED) == oracle.log_read(log, True)
    return want


def _payloads(rng, sizes):
    return [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in sizes]


def test_every_short_length(gpu, jl, oracle):
    # lengths 0..400 in a row: every header offset in a window, tiny records
    # (several per window), headers straddling windows and blocks
    rng = np.random.default_rng(1)
    log = oracle.log_write(_payloads(rng, list(range(401)) * 2))
    _check(jl, oracle, log, read_records=True)


@pytest.mark.parametrize("shift", range(0, 16))
def test_header_at_every_window_edge(gpu, jl, oracle, shift):
    # first record sized so the next header starts at window offset 112 + shift
    # (straddling for shift >= 10), then C1-shaped records
    rng = np.random.default_rng(100 + shift)
    first = 128 * 3 + 112 + shift - 7
    log = oracle.log_write(_payloads(rng, [first] + [1056] * 70 + [shift, 128 - 7, 121, 0, 1, 2]))
    _check(jl, oracle, log)


def test_records_ending_on_window_and_block_edges(gpu, jl, oracle):
    rng = np.random.default_rng(7)
    sizes = [128 - 7] * 5 + [256 - 7] * 3 + [32768 - 7, 32768 - 14, 0, 32768 * 2, 5, 32768 - 7 * 3]
    _check(jl, oracle, oracle.log_write(_payloads(rng, sizes)), read_records=True)


@pytest.mark.parametrize("seed", range(6))
def test_random_logs_with_flips(gpu, jl, oracle, seed):
    rng = np.random.default_rng(2000 + seed)
    sizes = np.concatenate([rng.integers(0, 300, 200), rng.integers(300, 5000, 60), rng.integers(5000, 90000, 6),
                            np.full(100, 1056)])
    rng.shuffle(sizes)
    log = bytearray(oracle.log_write(_payloads(rng, sizes)))
    _check(jl, oracle, bytes(log))
    for pos in rng.integers(0, len(log), 12):
        log[int(pos)] ^= 1 << int(rng.integers(0, 8))
    want = _check(jl, oracle, bytes(log), read_records=True)
    assert any(k != 1 for _, _, _, k in want)


def test_every_header_field_flipped(gpu, jl, oracle):
    # flips in the crc, length and type bytes of one header, and in its payload's
    # first / last byte: a bad crc drops the rest of the block, a bad length is a
    # bad-length report; every case must match the oracle
    rng = np.random.default_rng(3)
    sizes = [1056] * 40
    base = oracle.log_write(_payloads(rng, sizes))
    h = 5 * 1063  # sixth header
    for off in list(range(7)) + [7, 7 + 1055]:
        for bit in (0, 3, 7):
            log = bytearray(base)
            log[h + off] ^= 1 << bit
            _check(jl, oracle, bytes(log))


@pytest.mark.parametrize("tail", [0, 1, 3, 6, 7, 8, 200, 32767])
def test_short_last_block(gpu, jl, oracle, tail):
    # a log cut inside its last block: EOF_TRUNC / EOF_BAD_LENGTH and the rest
    rng = np.random.default_rng(50 + tail)
    full = oracle.log_write(_payloads(rng, [1000] * 130))
    cut = 2 * 32768 + tail
    assert len(full) > cut
    _check(jl, oracle, full[:cut])
    _check(jl, oracle, full[:cut] + b"\x01\x02\x03")


def test_exact_block_multiples_and_empty(gpu, jl, oracle):
    full = oracle.log_write([bytes(32768 - 7)])
    for log in (b"", full, full * 3, full + full[:3], bytes(32768), bytes(65536)):
        _check(jl, oracle, log)


@pytest.mark.parametrize("n", [250, 256, 257, 300, 4680])
def test_many_records_per_block_fallback(gpu, jl, oracle, n):
    # more events in a block than the fused kernel's 256 slots: the fallback path
    rng = np.random.default_rng(n)
    per = max(0, 32768 // n - 7)
    _check(jl, oracle, oracle.log_write(_payloads(rng, [per] * (3 * n))))


def test_many_rounds_partial_last(gpu, jl, oracle):
    # ~20k blocks (~650 MB): more rounds of 8 blocks than the grid has waves, so
    # waves run one or two rounds, the last one partial, and a short last block;
    # flips in a few blocks
    rng = np.random.default_rng(9)
    sizes = np.concatenate([rng.integers(0, 3000, 300000), np.full(300000, 1056)])
    rng.shuffle(sizes)
    buf = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(sizes)])
    log = bytearray(oracle.log_write([buf[offs[i]:offs[i + 1]] for i in range(sizes.size)]))
    assert len(log) > 16384 * 32768
    for pos in (123, 32768 * 17 + 5000, 32768 * 17000 + 40, len(log) - 100):
        log[pos] ^= 0x10
    _check(jl, oracle, bytes(log))


def test_device_resident_matches(gpu, jl, oracle):
    import torch

    rng = np.random.default_rng(11)
    log = bytearray(oracle.log_write(_payloads(rng, rng.integers(0, 2000, 3000))))
    log[40000] ^= 4
    d = torch.from_numpy(np.frombuffer(bytes(log), np.uint8).copy()).to(gpu)
    for mode in (FUSED, TWO_PASS):
        ev, n = jl.log_verify_dev(d, mode)
        got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
        assert _live(got) == _live(oracle.log_events(bytes(log)))


@pytest.mark.parametrize("case", ["equal_131", "equal_0", "equal_400", "random_0_200", "runs", "stops"])
def test_dense_blocks(gpu, jl, oracle, case):
    """Blocks of more than 64 records (lc_dense: the block staged in LDS, its
    headers walked with 64-lane speculation, one thread per record's crc): runs
    of equal records (the speculation's case: 64 headers per round), random
    lengths (one header per round), runs that change length mid-block, and
    every stop decision inside a dense block (bad length, zero-type skip, a
    failing crc, EOF cases of a short last block), flips included."""
    rng = np.random.default_rng(["equal_131", "equal_0", "equal_400", "random_0_200", "runs", "stops"].index(case))
    if case.startswith("equal"):
        sizes = [int(case.split("_")[1])] * (3 * 32768 // (int(case.split("_")[1]) + 7) + 50)
    elif case == "random_0_200":
        sizes = rng.integers(0, 201, 1500).tolist()
    elif case == "runs":
        sizes = sum(([int(n)] * int(k) for n, k in zip(rng.integers(0, 300, 40), rng.integers(1, 90, 40))), [])
    else:
        sizes = [120] * 1200
    log = bytearray(oracle.log_write(_payloads(rng, sizes)))
    if case == "stops":
        blk = lambda b, o: b * 32768 + o  # noqa: E731
        log[blk(0, 127 * 10 + 4):blk(0, 127 * 10 + 6)] = b"\xff\x7f"  # bad length in block 0
        log[blk(1, 5000)] ^= 0x20  # a payload flip: BAD_CRC, rest of block 1 dropped
        h = 32768 * 2 + 127 * 100  # a header of block 2 (127-B records: the layout does not depend on the seed)
        log[h + 4:h + 7] = b"\0\0\0"  # zero type, zero length: the rest of block 2 skipped
        log = log[: len(log) - 3]  # EOF inside the last record
    else:
        for _ in range(4):
            log[int(rng.integers(0, len(log)))] ^= 1 << int(rng.integers(0, 8))
    log = bytes(log)
    want = _check(jl, oracle, log, read_records=True)
    assert len(want) > 65


@pytest.mark.parametrize("big", [520, 600, 4200, 9000, 31691, 40000])
def test_dense_blocks_with_long_records(gpu, jl, oracle, big):
    """Dense blocks (8 short records in their first 4 KiB) that also hold a long
    record: lc_dense leaves records above kLDLongDw dwords to the rounds (their
    chunks counted into the group's histogram, placed by lc_build, checked by
    crc_gv4 / lc_combine); 31 691 B fills a block after ten 100-B records, 40 000
    fragments across blocks.  Flips in long and short records, clean blocks
    between, events and read records against the oracle."""
    rng = np.random.default_rng(big)
    sizes = ([100] * 10 + [big]) * (6 * 32768 // (10 * 107 + big + 7) + 3) + [100] * 40
    log = bytearray(oracle.log_write(_payloads(rng, sizes)))
    per = 10 * 107 + big + 7
    for k in (1, 4):  # inside a long record, then inside a short one further on
        log[k * per + 10 * 107 + 7 + int(rng.integers(0, big))] ^= 0x10
        log[(k + 1) * per + 3 * 107 + 20] ^= 0x01
    log = bytes(log)
    want = _check(jl, oracle, log, read_records=True)
    assert any(e[3] == 2 for e in want)  # a BAD_CRC seen


@pytest.mark.parametrize("shift", [1, 3, 8, 15])
def test_dense_blocks_unaligned_log(gpu, jl, oracle, shift):
    """lc_dense's byte-staging path: a log that does not start on 16 bytes (a
    device view at byte offset `shift`) stages every block bytewise, not only the
    short last one; DBBench-shaped records (every block dense) with flips, full
    events against the oracle (dropped records included)."""
    import torch

    from jleveldb_amd import workloads

    rng = np.random.default_rng(300 + shift)
    log = bytearray(oracle.log_write(_payloads(rng, [workloads.DBBENCH_PAYLOAD] * (6 * 32768 // 138 + 17))))
    for _ in range(5):
        log[int(rng.integers(0, len(log)))] ^= 1 << int(rng.integers(0, 8))
    host = np.zeros(len(log) + 16, np.uint8)
    host[shift:shift + len(log)] = np.frombuffer(bytes(log), np.uint8)
    d = torch.from_numpy(host).to(gpu)[shift:shift + len(log)]
    assert d.data_ptr() % 16 == shift % 16
    for mode in (0, 1, TWO_PASS):
        ev, n = jl.log_verify_dev(d, mode)
        got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
        assert _live(got) == _live(oracle.log_events(bytes(log), checksum=mode != 0)), mode
