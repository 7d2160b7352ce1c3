"""GPU parity of the HIP engine against the CPU oracle (bit-exact: integer work).

Every test calls the product through the C-ABI (libjlcrc.so) and compares with
oracle/ on the same seeded bytes, plus the committed golden fixtures.  Full-size
cases (BASELINE config C2: 1M x 4 KiB) are compared block-for-block with the
multithreaded oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 16


def to_dev(a, dev):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


# ------------------------------------------------------------- fixed blocks
@pytest.mark.parametrize("n_blocks", [1, 2, 15, 16, 17, 255, 4096, 4097, 70001])
def test_fixed_4k_random(gpu, jl, oracle, n_blocks):
    rng = np.random.default_rng(n_blocks)
    host = rng.integers(0, 256, n_blocks * 4096, dtype=np.uint8)
    d = to_dev(host, gpu)
    got = u32(jl.crc32c_fixed_dev(d, 4096))
    want = oracle.fixed(host, 4096, n_blocks, threads=THREADS)
    assert np.array_equal(got, want)
    raw = u32(jl.crc32c_fixed_dev(d, 4096, flags=0))
    assert np.array_equal(raw, oracle.fixed(host, 4096, n_blocks, flags=0, threads=THREADS))


@pytest.mark.parametrize("n_blocks", [1, 7, 8, 9, 63, 64, 65, 1000, 16385, 65536 + 13])
def test_fixed_4k_ragged(gpu, jl, oracle, n_blocks):
    """The 4 KiB kernel at ragged counts around the round (8 blocks), group (64
    blocks) and grid boundaries, masked and raw."""
    rng = np.random.default_rng(1000 + n_blocks)
    host = rng.integers(0, 256, n_blocks * 4096, dtype=np.uint8)
    d = to_dev(host, gpu)
    for flags in (1, 0):
        got = u32(jl.crc32c_fixed_dev(d, 4096, flags=flags))
        assert np.array_equal(got, oracle.fixed(host, 4096, n_blocks, flags=flags, threads=THREADS)), flags


def test_fixed_4k_v4_out_of_place_views(gpu, jl, oracle):
    """v4 kernel on a sub-view (unaligned-to-group base, block count not a round multiple)."""
    rng = np.random.default_rng(77)
    host = rng.integers(0, 256, 300 * 4096, dtype=np.uint8)
    d = to_dev(host, gpu)
    got = u32(jl.crc32c_fixed_dev(d[5 * 4096:], 4096, 290))
    assert np.array_equal(got, oracle.fixed(host[5 * 4096:], 4096, 290, threads=THREADS))


def test_fixed_4k_dbbench_x(gpu, jl, golden):
    """DBBench.crc32c input (J/benchmark/DBBench.java:775-793): 4096 x 'x'."""
    d = to_dev(np.frombuffer(b"x" * 4096 * 3, dtype=np.uint8), gpu)
    got = u32(jl.crc32c_fixed_dev(d, 4096, flags=0))
    assert list(got) == [golden("golden.json")["derived"]["dbbench_4k_x"]] * 3


@pytest.mark.parametrize("block_bytes", [1, 3, 4, 7, 64, 255, 256, 1000, 1057, 4095, 4097, 8192, 32768, 65536, 100003])
def test_fixed_other_sizes(gpu, jl, oracle, block_bytes):
    n = max(1, min(3000, (8 << 20) // block_bytes))
    rng = np.random.default_rng(block_bytes)
    host = rng.integers(0, 256, n * block_bytes, dtype=np.uint8)
    got = u32(jl.crc32c_fixed_dev(to_dev(host, gpu), block_bytes, n))
    assert np.array_equal(got, oracle.fixed(host, block_bytes, n, threads=THREADS))


def test_fixed_zero_and_ones_kats(gpu, jl, golden):
    kats = {k["name"]: k for k in golden("golden.json")["kats"]}
    for name in ("zeros32", "ones32", "ramp32", "rramp32"):
        data = np.frombuffer(bytes.fromhex(kats[name]["hex"]) * 4, dtype=np.uint8)
        got = u32(jl.crc32c_fixed_dev(to_dev(data, gpu), 32, 4, flags=0))
        assert list(got) == [kats[name]["value"]] * 4, name


# --------------------------------------------------------- variable blocks
def test_batch_every_length_and_alignment(gpu, jl, oracle):
    rng = np.random.default_rng(11)
    lens, offs, pos = [], [], 0
    for n in range(0, 1301):
        for a in range(4):
            pos += a
            offs.append(pos)
            lens.append(n)
            pos += n
    arena = rng.integers(0, 256, pos + 8, dtype=np.uint8)
    off = np.array(offs, np.uint64)
    ln = np.array(lens, np.uint32)
    init = rng.integers(0, 2**32, len(lens), dtype=np.uint64).astype(np.uint32)
    sfx = rng.integers(0, 256, len(lens), dtype=np.uint8)
    d_arena, d_off, d_len = to_dev(arena, gpu), to_dev(off.view(np.int64), gpu), to_dev(ln.view(np.int32), gpu)
    got = u32(jl.crc32c_batch_dev(d_arena, d_off, d_len))
    assert np.array_equal(got, oracle.batch(arena, off, ln, threads=THREADS))
    got = u32(jl.crc32c_batch_dev(d_arena, d_off, d_len, init=to_dev(init.view(np.int32), gpu), flags=0))
    assert np.array_equal(got, oracle.batch(arena, off, ln, init=init, flags=0, threads=THREADS))
    got = u32(jl.crc32c_batch_dev(d_arena, d_off, d_len, suffix=to_dev(sfx, gpu)))
    assert np.array_equal(got, oracle.batch(arena, off, ln, suffix=sfx, threads=THREADS))


@pytest.mark.parametrize("depth,partition", [("32", True), ("48", False), ("16", False)])
def test_stream_depths_and_partition(gpu, jl, oracle, engine_options, depth, partition):
    """Stream-kernel ring depths (JL_OPT_STREAM_DEPTH) and the count split (JL_OPT_STREAM_PARTITION 0)."""
    engine_options(jl.OPT_GENERAL_PATH, jl.PATH_STREAM)
    engine_options(jl.OPT_STREAM_DEPTH, int(depth))
    if not partition:
        engine_options(jl.OPT_STREAM_PARTITION, 0)
    test_batch_every_length_and_alignment(gpu, jl, oracle)
    test_batch_large_and_zipf(gpu, jl, oracle)


def test_batch_large_and_zipf(gpu, jl, oracle):
    rng = np.random.default_rng(12)
    ks = rng.zipf(1.1, 20000)
    ks = ks[ks <= 64][:6000]
    lens = (1024 * (ks - 1) + 1 + rng.integers(0, 1024, ks.size)).astype(np.uint32)
    lens = np.concatenate([lens, np.array([65536, 65535, 200000, 1 << 20, 4096 * 33 + 5], np.uint32)])
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = rng.integers(0, 256, int(lens.sum()) + 8, dtype=np.uint8)
    got = u32(jl.crc32c_batch_dev(to_dev(arena, gpu), to_dev(offs.view(np.int64), gpu), to_dev(lens.view(np.int32), gpu)))
    assert np.array_equal(got, oracle.batch(arena, offs, lens, threads=THREADS))


def test_batch_golden_fixture(gpu, jl, golden):
    arena = np.frombuffer(golden("blocks.bin"), dtype=np.uint8)
    b = golden("blocks.json")
    off = np.array(b["off"], np.uint64)
    ln = np.array(b["len"], np.uint32)
    d = (to_dev(arena, gpu), to_dev(off.view(np.int64), gpu), to_dev(ln.view(np.int32), gpu))
    assert list(u32(jl.crc32c_batch_dev(*d, flags=0))) == b["crc"]
    assert list(u32(jl.crc32c_batch_dev(*d))) == b["masked"]
    init = np.array(b["init"], np.uint32)
    assert list(u32(jl.crc32c_batch_dev(*d, init=to_dev(init.view(np.int32), gpu), flags=0))) == b["extend"]
    sfx = np.zeros(len(ln), np.uint8)
    assert list(u32(jl.crc32c_batch_dev(*d, suffix=to_dev(sfx, gpu), flags=0))) == b["suffix_crc_type0"]
    # host-memory entry point
    assert list(jl.crc32c_batch(arena, off, ln)) == b["masked"]


def test_empty_batches(gpu, jl):
    import torch

    z = torch.zeros(16, dtype=torch.uint8, device=gpu)
    assert jl.crc32c_fixed_dev(z, 4096, 0).numel() == 0
    e64 = torch.zeros(0, dtype=torch.int64, device=gpu)
    e32 = torch.zeros(0, dtype=torch.int32, device=gpu)
    assert jl.crc32c_batch_dev(z, e64, e32).numel() == 0


# ------------------------------------------------------------ table shims
def test_table_trailers_and_verify(gpu, jl, oracle, golden):
    f = np.frombuffer(golden("table.bin"), dtype=np.uint8)
    meta = golden("table.json")
    off = np.array([h[0] for h in meta["handles"]], np.uint64)
    size = np.array([h[1] for h in meta["handles"]], np.uint32)
    d_f, d_off, d_size = to_dev(f, gpu), to_dev(off.view(np.int64), gpu), to_dev(size.view(np.int32), gpu)
    tr = jl.table_trailers_dev(d_f, d_off, d_size).cpu().numpy().reshape(-1, 5)
    assert [bytes(t).hex() for t in tr] == meta["trailers"]
    assert list(jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy()) == [1] * len(off)
    assert list(jl.table_verify(f, off, size)) == [1] * len(off)
    # byte flips (TestCorruption.corrupt XORs 0x80): every flipped byte of block+trailer is detected
    rng = np.random.default_rng(3)
    for i, (o, n) in enumerate(zip(off, size)):
        for pos in {int(o), int(o) + int(n), int(o) + int(n) + 4, int(o) + int(rng.integers(0, n + 5))}:
            bad = f.copy()
            bad[pos] ^= 0x80
            st = jl.table_verify(bad, off, size)
            assert st[i] == 0 and oracle.table_verify(bad, int(o), int(n)) is False
            assert all(st[j] == 1 for j in range(len(off)) if j != i)


def test_table_many_blocks(gpu, jl, oracle):
    rng = np.random.default_rng(5)
    sizes = rng.integers(0, 9000, 5000).astype(np.uint32)
    blocks = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in sizes]
    types = rng.integers(0, 2, len(sizes), dtype=np.uint8)
    parts, offs, pos = [], [], 0
    for b, t in zip(blocks, types):
        offs.append(pos)
        parts.append(b + oracle.table_trailer(b, int(t)))
        pos += len(b) + 5
    f = np.frombuffer(b"".join(parts), dtype=np.uint8)
    off = np.array(offs, np.uint64)
    d_f, d_off, d_size = to_dev(f, gpu), to_dev(off.view(np.int64), gpu), to_dev(sizes.view(np.int32), gpu)
    tr = jl.table_trailers_dev(d_f, d_off, d_size, types=to_dev(types, gpu)).cpu().numpy().reshape(-1, 5)
    want = np.stack([np.frombuffer(p[-5:], np.uint8) for p in parts])
    assert np.array_equal(tr, want)
    st = jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy()
    assert st.all()


# --------------------------------------------------------------- log shims
def _events(ev):
    return [(int(e["offset"]), int(e["length"]), int(e["type"]), int(e["kind"])) for e in ev if e["kind"] != 0]


def _random_log(oracle, rng, n, max_len):
    sizes = rng.integers(0, max_len, n)
    payloads = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    return payloads, oracle.log_write(payloads)


@pytest.mark.usefixtures("log_path")
def test_log_golden(gpu, jl, oracle, golden):
    log = golden("log.bin")
    meta = golden("log.json")
    assert [list(e) for e in _events(jl.log_verify(log))] == meta["events"]
    recs, reps = jl.log_read_records(log)
    assert reps == [] and [r[0] for r in recs] == meta["record_offsets"]
    assert (recs, reps) == oracle.log_read(log)


@pytest.mark.usefixtures("log_path")
@pytest.mark.parametrize("seed", range(6))
def test_log_random_with_corruption(gpu, jl, oracle, seed):
    rng = np.random.default_rng(100 + seed)
    payloads, log = _random_log(oracle, rng, 300, [2000, 40000, 100, 70000, 1200, 5000][seed])
    log = bytearray(log)
    for _ in range(seed * 3):
        log[int(rng.integers(0, len(log)))] ^= 1 << int(rng.integers(0, 8))
    if seed % 2:
        log = log[: len(log) - int(rng.integers(1, 40000))]  # truncated tail (writer died)
    log = bytes(log)
    for checksum in (True, False):
        assert _events(jl.log_verify(log, checksum)) == _events(oracle.log_events(log, checksum))
        assert jl.log_read_records(log, checksum) == oracle.log_read(log, checksum)
    for initial in (1, 32768 - 3, 32768 * 2 + 100, len(log) // 2):
        assert jl.log_read_records(log, True, initial) == oracle.log_read(log, True, initial)


@pytest.mark.usefixtures("log_path")
def test_log_special_records(gpu, jl, oracle):
    """Zero-type zero-length skip, bad length, stray trailer bytes, types 5..255."""
    base = oracle.log_write([b"a" * 100, b"b" * 10, b"c" * 20])
    cases = []
    z = bytearray(base)
    z[107 + 4:107 + 7] = b"\0\0\0"  # record 2 header: length 0, type 0 -> skip rest of block
    cases.append(bytes(z))
    bl = bytearray(base)
    bl[107 + 4] = 0xFF
    bl[107 + 5] = 0x7F  # huge length
    cases.append(bytes(bl))
    cases.append(base + b"\x01\x02\x03")  # stray bytes at EOF
    for t in (0, 5, 6, 7, 200):  # unknown / special types with a valid crc
        payload = b"payload"
        hdr = bytearray(7)
        crc = oracle.mask(oracle.extend(oracle.value(bytes([t])), payload))
        hdr[0:4] = crc.to_bytes(4, "little")
        hdr[4:6] = len(payload).to_bytes(2, "little")
        hdr[6] = t
        cases.append(base + bytes(hdr) + payload + oracle.log_write([b"after"]))
    full = oracle.log_write([bytes(32768 - 7)])  # exactly one full block
    cases.append(full)
    cases.append(full + full[:3])
    cases.append(b"")
    for log in cases:
        for checksum in (True, False):
            assert _events(jl.log_verify(log, checksum)) == _events(oracle.log_events(log, checksum))
            assert jl.log_read_records(log, checksum) == oracle.log_read(log, checksum)


@pytest.mark.usefixtures("log_path")
def test_log_corruption_recovery(gpu, jl, oracle):
    """TestCorruption.testRecovery (T/TestCorruption.java:250-270) through the device path."""
    from test_oracle import _batch_payload

    payloads = [_batch_payload(i) for i in range(100)]
    log = bytearray(oracle.log_write(payloads))
    for pos in (19, 32768 + 1000):
        log[pos] ^= 0x80
    recs, reps = jl.log_read_records(bytes(log))
    assert len(recs) == 36 and [r[1] for r in recs] == payloads[64:]
    assert reps == [(32768, 2, 0), (480, 6, 0), (32281, 2, 0), (967, 6, 0)]


def test_log_headers_dev(gpu, jl, oracle, golden):
    d = golden("golden.json")["derived"]
    cases = [(b"", 1, d["log_hdr_full_empty"]), (b"foo", 1, d["log_hdr_full_foo"]),
             (b"x" * 100, 2, d["log_hdr_first_100x"]), (b"hello world", 4, d["log_hdr_last_hello_world"])]
    arena = np.frombuffer(b"".join(c[0] for c in cases) + b"\0" * 8, np.uint8)
    lens = np.array([len(c[0]) for c in cases], np.uint32)
    offs = np.zeros(len(cases), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    types = np.array([c[1] for c in cases], np.uint8)
    hdr = jl.log_headers_dev(to_dev(arena, gpu), to_dev(offs.view(np.int64), gpu), to_dev(lens.view(np.int32), gpu),
                             to_dev(types, gpu)).cpu().numpy().reshape(-1, 7)
    assert [bytes(h).hex() for h in hdr] == [c[2] for c in cases]


@pytest.mark.usefixtures("log_path")
def test_log_dev_resident(gpu, jl, oracle):
    rng = np.random.default_rng(9)
    payloads, log = _random_log(oracle, rng, 2000, 3000)
    d = to_dev(np.frombuffer(log, np.uint8), gpu)
    ev, n = jl.log_verify_dev(d)
    got = np.frombuffer(ev.cpu().numpy().tobytes()[: n * 16], dtype=jl.LOG_EVENT_DTYPE)
    assert _events(got) == _events(oracle.log_events(log))


@pytest.mark.usefixtures("log_path")
def test_log_dev_async(gpu, jl, oracle):
    """jl_log_verify_dev_async: several logs verified back to back on one stream
    with no host round trip (a corrupted one, a tiny one, an empty one, and one of
    0-30 B records whose blocks are all dense), then checked against the oracle
    from their device result words: complete events for every density, the
    dense blocks counted in result[1]."""
    import torch

    rng = np.random.default_rng(41)
    logs = []
    for n, mx, flips in ((2000, 3000, 5), (300, 70000, 3), (3, 50, 0)):
        _, log = _random_log(oracle, rng, n, mx)
        log = bytearray(log)
        for _ in range(flips):
            log[int(rng.integers(0, len(log)))] ^= 1 << int(rng.integers(0, 8))
        logs.append(bytes(log))
    logs.append(b"")
    dense = bytearray(oracle.log_write([rng.integers(0, 256, int(s), dtype=np.uint8).tobytes()
                                        for s in rng.integers(0, 30, 6000)]))
    dense[40_000] ^= 0x02  # a flip inside a dense block
    logs.append(bytes(dense))
    runs = []
    for log in logs:
        d = to_dev(np.frombuffer(log, np.uint8), gpu) if log else torch.empty(0, dtype=torch.uint8, device=gpu)
        ev = torch.empty((len(log) // 7 + 2) * 16, dtype=torch.uint8, device=gpu)
        runs.append((log, d, *jl.log_verify_dev_async(d, True, events=ev)))
    for log, d, ev, res in runs:
        n, n_dense, capf = (int(x) for x in res.cpu().numpy())
        assert capf == 0
        if jl.get_option(jl.OPT_LOG_SMALL_MAX) == 0:  # the chunked path counts its dense blocks (lc_small: 0)
            assert (n_dense > 0) == (log is logs[-1])
        got = np.frombuffer(ev.cpu().numpy().tobytes()[: n * 16], dtype=jl.LOG_EVENT_DTYPE)
        assert _events(got) == _events(oracle.log_events(log))


# ----------------------------------------------------------------- helpers
def test_fill_random_matches_oracle(gpu, jl, oracle):
    import torch

    for nbytes, first in [(4096 * 3, 0), (1000, 5), (13, 7)]:
        t = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
        jl.fill_random_dev(t, 0x4A4C4442, first)
        assert np.array_equal(t.cpu().numpy(), oracle.fill_splitmix(nbytes, 0x4A4C4442, first))


# ------------------------------------------------------------- full sizes
def test_full_size_c2_block_for_block(gpu, jl, oracle):
    """BASELINE config C2: 1M x 4 KiB random blocks, device-resident; every block vs the oracle."""
    import torch

    n = 1 << 20
    data = torch.empty(n * 4096, dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(data, 0x4A4C4442)
    got = u32(jl.crc32c_fixed_dev(data, 4096))
    host = data.cpu().numpy()
    want = oracle.fixed(host, 4096, n, threads=THREADS)
    assert np.array_equal(got, want)
    # size-independent property: flipping one byte changes exactly that block's crc
    data[123456 * 4096 + 77] ^= 1
    got2 = u32(jl.crc32c_fixed_dev(data, 4096))
    diff = np.nonzero(got2 != got)[0]
    assert list(diff) == [123456]


# ------------------------------------------------- host-memory streaming path
@pytest.mark.parametrize("block_bytes,n_blocks", [(4096, 2 * 16384 + 100), (1000, 70000), (4096, 3), (65536, 1025)])
def test_fixed_host_streaming_pageable(gpu, jl, oracle, block_bytes, n_blocks):
    """jl_crc32c_fixed over pageable host memory: several 64 MiB chunks + a partial one."""
    rng = np.random.default_rng(block_bytes + n_blocks)
    host = rng.integers(0, 256, block_bytes * n_blocks, dtype=np.uint8)
    got = jl.crc32c_fixed(host, block_bytes)
    assert np.array_equal(got, oracle.fixed(host, block_bytes, n_blocks, threads=THREADS))
    raw = jl.crc32c_fixed(host, block_bytes, flags=0)
    assert np.array_equal(raw, oracle.fixed(host, block_bytes, n_blocks, flags=0, threads=THREADS))


def test_fixed_host_streaming_pinned(gpu, jl, oracle):
    import torch

    n = 16384 + 77
    t = torch.empty(n * 4096, dtype=torch.uint8, pin_memory=True)
    rng = np.random.default_rng(5)
    t.numpy()[:] = rng.integers(0, 256, n * 4096, dtype=np.uint8)
    got = jl.crc32c_fixed(t, 4096)
    assert np.array_equal(got, oracle.fixed(t.numpy(), 4096, n, threads=THREADS))


# ------------------------------------------------ batched LogWriter on device
@pytest.mark.parametrize("dest_length", [0, 32768 - 5, 777])
def test_log_emit_dev_matches_logwriter(gpu, jl, oracle, dest_length):
    rng = np.random.default_rng(40 + dest_length)
    lens = rng.choice([0, 1, 6, 7, 100, 1056, 32761, 32762, 40000, 100000], size=80).astype(np.uint32)
    payloads = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in lens]
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    src = np.frombuffer(b"".join(payloads), dtype=np.uint8)
    plan = jl.log_layout(offs, lens, dest_length)
    got = jl.log_emit_dev(to_dev(src, gpu), plan).cpu().numpy().tobytes()
    assert got == oracle.log_write(payloads, dest_length)
    # and the device reader accepts every record of a freshly written log
    if dest_length == 0:
        recs, reps = jl.log_read_records(got)
        assert reps == [] and [r[1] for r in recs] == payloads


@pytest.mark.usefixtures("log_path")
def test_log_many_small_records(gpu, jl, oracle):
    """Blocks with far more than 64 physical records (the walk keeps the first 64
    decisions of a block and re-walks the rest) next to blocks with fewer, with
    bit flips; device-resident and host entry points."""
    rng = np.random.default_rng(31)
    sizes = np.concatenate([rng.integers(0, 40, 4000), rng.integers(500, 3000, 60), rng.integers(0, 9, 3000)])
    payloads = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    log = bytearray(oracle.log_write(payloads))
    for _ in range(6):
        log[int(rng.integers(0, len(log)))] ^= 1 << int(rng.integers(0, 8))
    log = bytes(log)
    want = _events(oracle.log_events(log, True))
    assert _events(jl.log_verify(log, True)) == want
    assert jl.log_read_records(log, True) == oracle.log_read(log, True)
