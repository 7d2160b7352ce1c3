"""Host-memory entry points through the chunked double-buffered pipeline.

jl_log_verify, jl_table_verify, jl_crc32c_batch and jl_crc32c_fixed stream
host input in JL_STREAM_CHUNK_BYTES (64 MiB) chunks; these inputs span several
chunks (with a partial last one) and are checked against the oracle
(`oracle.log_events` restates J/db/LogReader.java:297-383, `oracle.batch`
J/util/Crc32C.java:85-93) for every way host memory reaches the device:
pageable staged through pinned buffers, pageable pinned for the call
(hipHostRegister), and pinned tensors.  Also: offsets that do not ascend (one
window), a block larger than a chunk, corruption on both sides of a chunk
boundary, and several threads calling at once (per-thread workspaces).
"""
import threading

import numpy as np
import pytest

from jleveldb_amd import workloads as wl

pytestmark = pytest.mark.gpu

CH = 64 << 20
SEED = 0x4A4C4442
MODES = ["staged", "registered", "pinned"]


def _as_mode(jl, engine_options, a, mode):
    """The host buffer for `mode` (and the engine options it needs)."""
    import torch

    engine_options(jl.OPT_HOST_REGISTER, 1 if mode == "registered" else 0)
    if mode == "pinned":
        t = torch.empty(a.size, dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = a
        return t
    return a


def _live(ev):
    ev = ev[ev["kind"] != 0]
    return np.stack([ev["offset"], ev["length"].astype(np.uint64), ev["type"].astype(np.uint64),
                     ev["kind"].astype(np.uint64)])


@pytest.fixture(scope="module")
def log_image(gpu, jl):
    """~200 MiB log (3 full chunks + a partial one ending in a short block) of
    mixed 1 B - 100 KiB records written by the product LogWriter, with flips in
    the last block of chunk 0, the first of chunk 1 and one inside chunk 2."""
    import torch

    lens = wl.c5_lengths(True, target=200 << 20, seed=SEED)
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(src, SEED + 9)
    log = jl.log_emit_dev(src, plan).cpu().numpy().copy()
    nb = log.size
    assert nb > 3 * CH and nb % 32768 != 0
    for at in (CH - 32768 + 9_000, CH + 5_000, 2 * CH + 777_777):
        log[at] ^= 0x10
    return log


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("checksum", [0, 1, 3])
def test_log_verify_chunked(jl, oracle, engine_options, log_image, mode, checksum):
    buf = _as_mode(jl, engine_options, log_image, mode)
    got = jl.log_verify(buf, checksum)
    want = oracle.log_events(log_image, checksum=bool(checksum))
    g, w = _live(got), _live(want)
    assert g.shape == w.shape and np.array_equal(g, w)
    if checksum:  # the flips are seen (bad crc or bad length), as the oracle sees them
        assert int(np.isin(w[3], [jl.LOG_BAD_CRC, jl.LOG_BAD_LENGTH]).sum()) >= 1


def test_log_verify_capacity(jl, log_image):
    """A short event array: JL_ERR_CAPACITY with the full count."""
    import ctypes

    ev = np.zeros(1000, dtype=jl.LOG_EVENT_DTYPE)
    n = ctypes.c_uint64(0)
    rc = jl.lib().jl_log_verify(log_image.ctypes.data, log_image.size, 1, ev.ctypes.data, 1000, ctypes.byref(n))
    assert rc == -5 and n.value == jl.log_verify(log_image).size


@pytest.fixture(scope="module")
def arena():
    """~160 MiB arena of C3-shaped blocks plus one 70 MiB block (a chunk of its own)."""
    rng = np.random.default_rng(SEED)
    lens = wl.c3_lengths(9000, SEED)
    lens = np.concatenate([lens[:4000], np.array([70 << 20], np.uint32), lens[4000:]])
    offs = wl.packed_offsets(lens)
    data = rng.integers(0, 256, int(lens.sum(dtype=np.uint64)) + 4096, dtype=np.uint8)
    return data, offs, lens


@pytest.mark.parametrize("mode", MODES)
def test_batch_chunked(jl, oracle, engine_options, arena, mode):
    data, offs, lens = arena
    assert data.size > 2 * CH
    buf = _as_mode(jl, engine_options, data, mode)
    init = (np.arange(offs.size, dtype=np.uint32) * 2654435761).astype(np.uint32)
    sfx = (np.arange(offs.size) % 7).astype(np.uint8)
    assert np.array_equal(jl.crc32c_batch(buf, offs, lens), oracle.batch(data, offs, lens, threads=8))
    assert np.array_equal(jl.crc32c_batch(buf, offs, lens, init=init, suffix=sfx),
                          oracle.batch(data, offs, lens, init=init, suffix=sfx, threads=8))


def test_batch_unordered(jl, oracle, arena):
    data, offs, lens = arena
    perm = np.random.default_rng(3).permutation(offs.size)
    o, ln = offs[perm], lens[perm]
    assert np.array_equal(jl.crc32c_batch(data, o, ln), oracle.batch(data, o, ln, threads=8))


@pytest.mark.parametrize("mode", MODES)
def test_table_verify_chunked(jl, oracle, engine_options, mode):
    """A synthetic ~150 MiB 'table': blocks with valid 5-byte trailers, three of
    them corrupted (one on each side of the 64 MiB chunk boundary)."""
    rng = np.random.default_rng(SEED + 1)
    sizes = rng.integers(1, 1 << 17, 2400).astype(np.uint32)
    offs = wl.packed_offsets(sizes + 5)
    data = rng.integers(0, 256, int(offs[-1]) + int(sizes[-1]) + 5 + 100, dtype=np.uint8)
    crc = oracle.batch(data, offs, sizes + 1, flags=1, threads=8)  # crc of block || type, masked
    for i in range(sizes.size):
        p = int(offs[i]) + int(sizes[i]) + 1
        data[p:p + 4] = np.frombuffer(int(crc[i]).to_bytes(4, "little"), np.uint8)
    k = int(np.searchsorted(offs, CH))  # first block starting past the boundary
    bad = [5, k - 1, k]
    for i in bad:
        data[int(offs[i])] ^= 0x01
    buf = _as_mode(jl, engine_options, data, mode)
    st = jl.table_verify(buf, offs, sizes)
    assert sorted(np.nonzero(st == 0)[0].tolist()) == bad


@pytest.mark.parametrize("mode", MODES)
def test_fixed_chunked(jl, oracle, engine_options, mode):
    data = np.random.default_rng(SEED + 2).integers(0, 256, (2 * CH + (3 << 20)), dtype=np.uint8)
    buf = _as_mode(jl, engine_options, data, mode)
    assert np.array_equal(jl.crc32c_fixed(buf, 4096), oracle.fixed(data, 4096, data.size // 4096, threads=8))


def test_concurrent_callers(jl, oracle, arena, log_image):
    """Four threads at once on the host entry points: each gets its own workspace."""
    data, offs, lens = arena
    want_b = oracle.batch(data, offs, lens, threads=8)
    want_l = _live(oracle.log_events(log_image))
    errs = []

    def work(t):
        try:
            for _ in range(3):
                if t % 2:
                    assert np.array_equal(jl.crc32c_batch(data, offs, lens), want_b)
                else:
                    assert np.array_equal(_live(jl.log_verify(log_image)), want_l)
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(f"thread {t}: {e!r}")

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs


def test_async_then_host_call_share_scratch(gpu, jl, oracle, log_image):
    """A verification left in flight by jl_log_verify_dev_async on torch's default
    (null) stream, then at once a host jl_log_verify of another log (the
    workspace's own stream) and a synchronous device call on a side stream: the
    later calls reuse the thread's scratch only after the async call is done
    (a completion event, not the stream handle, tracks it: NULL is a valid
    stream).  All three results equal the oracle's."""
    import torch

    a = torch.from_numpy(log_image[: 96 << 20].copy()).to(gpu)
    ev = torch.zeros((a.numel() // 7 + 2) * 16, dtype=torch.uint8, device=gpu)
    assert torch.cuda.current_stream().cuda_stream == 0  # the null stream
    _, res = jl.log_verify_dev_async(a, events=ev)
    host = log_image[CH:]
    got_h = jl.log_verify(host)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        ev2, n2 = jl.log_verify_dev(a)
    side.synchronize()
    torch.cuda.synchronize()
    n = int(res.cpu()[0])
    want_a = _live(oracle.log_events(log_image[: 96 << 20]))
    assert np.array_equal(_live(ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)), want_a)
    assert np.array_equal(_live(ev2[: n2 * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)), want_a)
    assert np.array_equal(_live(got_h), _live(oracle.log_events(host)))


def test_async_then_empty_sync_call_then_device_call(gpu, jl, oracle, log_image):
    """An async verification in flight on the null stream, then an EMPTY
    synchronous jl_log_verify_dev on a side stream (it returns before any launch,
    so it never waits for the async call), then a device-path jl_log_verify_dev of
    another log on a third stream: the third call must still wait for the async
    one before it reuses the thread's scratch (empty WAL / MANIFEST files are
    common in a batch of logs).  Both results equal the oracle's."""
    import torch

    a = torch.from_numpy(log_image[: 96 << 20].copy()).to(gpu)
    b = torch.from_numpy(log_image[CH: CH + (80 << 20)].copy()).to(gpu)
    empty = torch.zeros(16, dtype=torch.uint8, device=gpu)
    ev = torch.zeros((a.numel() // 7 + 2) * 16, dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0  # the null stream
    _, res = jl.log_verify_dev_async(a, events=ev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        _, n0 = jl.log_verify_dev(empty[:0])
    assert n0 == 0
    with torch.cuda.stream(s2):
        ev2, n2 = jl.log_verify_dev(b)
    torch.cuda.synchronize()
    n = int(res.cpu()[0])
    assert np.array_equal(_live(ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)),
                          _live(oracle.log_events(log_image[: 96 << 20])))
    assert np.array_equal(_live(ev2[: n2 * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)),
                          _live(oracle.log_events(log_image[CH: CH + (80 << 20)])))


def test_stream_capture_refused(gpu, jl, oracle, log_image):
    """A device entry point called on a stream being captured into a HIP graph
    returns JL_ERR_INVALID before it enqueues anything (the per-call host
    bookkeeping cannot be replayed; jlcrc.h conventions); the thread's engine
    state is unharmed: the next uncaptured call equals the oracle."""
    import torch

    a = torch.from_numpy(log_image[: 8 << 20].copy()).to(gpu)
    ev = torch.zeros((a.numel() // 7 + 2) * 16, dtype=torch.uint8, device=gpu)
    res = torch.zeros(3, dtype=torch.int64, device=gpu)
    off = torch.arange(0, 64, dtype=torch.int64, device=gpu) * 4096
    ln = torch.full((64,), 4096, dtype=torch.int32, device=gpu)
    out = torch.zeros(64, dtype=torch.int32, device=gpu)
    s = torch.cuda.Stream()
    errs = []
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for fn in (lambda: jl.log_verify_dev_async(a, events=ev, result=res, stream=s),
                   lambda: jl.crc32c_batch_dev(a, off, ln, out=out, stream=s)):
            try:
                fn()
            except jl.JLError as e:
                errs.append(str(e))
    assert len(errs) == 2 and all("stream capture" in e for e in errs), errs
    ev2, n2 = jl.log_verify_dev(a)
    torch.cuda.synchronize()
    assert np.array_equal(_live(ev2[: n2 * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)),
                          _live(oracle.log_events(log_image[: 8 << 20])))


def test_null_stream_during_global_capture(gpu, jl):
    """A device entry point called on the NULL (legacy) stream while another
    stream captures in global mode: the NULL stream itself is not capturing.
    With torch's non-blocking capture stream HIP lets the call run (the NULL
    stream does not synchronise with it): the results are right and the other
    stream's capture goes on.  Where HIP reports the implicit capture instead
    (hipErrorStreamCaptureImplicit) the call is refused with its own message,
    nothing is enqueued.  Either way the graph replays what it captured."""
    import ctypes
    import torch

    data = torch.zeros(4 * 4096, dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(data, 11)
    want = jl.crc32c_fixed_dev(data, 4096).clone()
    out = torch.zeros(4, dtype=torch.int32, device=gpu)
    x = torch.arange(16, dtype=torch.float32, device=gpu)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):  # torch's default capture mode: global
        y = x * 2.0
        rc = jl.lib().jl_crc32c_fixed_dev(data.data_ptr(), 4096, 4, jl.FLAG_MASK, out.data_ptr(), ctypes.c_void_p(0))
        msg = jl.lib().jl_last_error().decode()
        y = y + 1.0
    torch.cuda.synchronize()
    if rc == 0:
        assert torch.equal(out, want)
    else:
        assert rc == -1 and "null stream" in msg, (rc, msg)
        assert int(out.abs().sum()) == 0  # nothing ran
    x.copy_(torch.arange(16, dtype=torch.float32, device=gpu) + 1.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, (torch.arange(16, dtype=torch.float32, device=gpu) + 1.0) * 2.0 + 1.0)


@pytest.mark.parametrize("mode", ["staged", "pinned"])
def test_dense_log_host(gpu, jl, oracle, engine_options, mode):
    """~150 MiB DBBench-default log (131-B payloads: every 32 KiB block dense) with
    flips, through the host pipeline: the dense blocks' events equal the oracle's."""
    import torch

    lens = wl.c5_lengths("dbbench_131", target=150 << 20, seed=SEED)
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(src, SEED + 13)
    log = jl.log_emit_dev(src, plan).cpu().numpy().copy()
    for at in (CH - 32768 + 17, CH + 5, 2 * CH + 300_001):
        log[at] ^= 0x04
    buf = _as_mode(jl, engine_options, log, mode)
    g, w = _live(jl.log_verify(buf)), _live(oracle.log_events(log))
    assert g.shape == w.shape and np.array_equal(g, w)
    assert int((w[3] == jl.LOG_BAD_CRC).sum()) + int((w[3] == jl.LOG_BAD_LENGTH).sum()) >= 3


def test_work_counters_between_verifications(gpu, jl, oracle, log_image):
    """The chunked verification's work counters (dense-block list, lc_dense's and
    gv4's dealing, lc_scan's ids) are zeroed by each verification's last kernel
    for the next one (a memset only for a new workspace).  A sequence on one
    thread that grows the workspace, shrinks it, alternates dense and sparse
    logs, walk-only and checksummed calls, and async and sync forms must give
    the oracle's events every time."""
    import torch

    lens = wl.c5_lengths("dbbench_131", target=24 << 20, seed=SEED + 1)
    plan = jl.log_layout(wl.packed_offsets(lens), lens)
    src = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=gpu)
    jl.fill_random_dev(src, SEED + 21)
    dense = jl.log_emit_dev(src, plan)
    dense[4_000_000] ^= 0x20
    dense_h = dense.cpu().numpy()
    sparse_h = log_image[: 40 << 20]
    sparse = torch.from_numpy(sparse_h.copy()).to(gpu)
    small_h = log_image[: 3 << 20]
    small = torch.from_numpy(small_h.copy()).to(gpu)
    want = {}
    for name, h in (("dense", dense_h), ("sparse", sparse_h), ("small", small_h)):
        for cs in (0, 1):
            want[name, cs] = _live(oracle.log_events(h, checksum=bool(cs)))
    logs = {"dense": dense, "sparse": sparse, "small": small}
    seq = [("small", 1, False), ("dense", 1, False), ("dense", 1, True), ("sparse", 1, False), ("small", 0, False),
           ("dense", 0, True), ("dense", 1, False), ("sparse", 1, True), ("small", 1, True), ("dense", 1, True)]
    for name, cs, use_async in seq:
        t = logs[name]
        if use_async:
            ev = torch.zeros((t.numel() // 7 + 2) * 16, dtype=torch.uint8, device=gpu)
            _, res = jl.log_verify_dev_async(t, bool(cs), events=ev)
            torch.cuda.synchronize()
            n = int(res.cpu()[0])
        else:
            ev, n = jl.log_verify_dev(t, bool(cs))
        got = _live(ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE))
        assert got.shape == want[name, cs].shape and np.array_equal(got, want[name, cs]), (name, cs, use_async)
