"""Targeted parity tests for lc_dense's hand-offs that run without a barrier of
their own, each against the oracle's readPhysicalRecord walk
(J/db/LogReader.java:297-383) event for event:

* a block's failure (s_bad) written to first_bad after the NEXT block's first
  barrier: a flip in the LAST record of a multi-pass block (lc_dwalk's offsets,
  then lc_dense's own walk, 4-6 passes of 256 runs), and in the last record of
  two-pass blocks (random 0-200 B records);
* the stash pool refill (thread 0's atomic, one barrier) and the chunk grab
  (s_c[2], written in a stash phase, read after the next block's barriers): a
  flip in EVERY block of a log whose blocks take ~1 000 stash entries each, so
  every refill and every chunk boundary falls on a block that holds a failure;
* a dense block's long record (> 512 B of crc range), checked by the rounds
  (crc_gv4 / lc_combine atomicMin into first_bad after lc_dense's plain store):
  a long-record failure together with a short-record failure before it, after
  it, and each alone.
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


def _last_ok_payload_per_block(w, blocks):
    """Header offset and length of each listed block's last OK record with a payload."""
    ok = w[(w["kind"] == 1) & (w["length"] > 0)]
    blk = ok["offset"] >> 15
    out = []
    for b in blocks:
        sel = ok[blk == b]
        if sel.size:
            out.append((int(sel["offset"][-1]), int(sel["length"][-1])))
    return out


@pytest.mark.parametrize("maxlen", [40, 200])
def test_flip_in_last_record_of_multipass_blocks(gpu, jl, oracle, maxlen):
    rng = np.random.default_rng(SEED + maxlen)
    lens = rng.integers(0, maxlen + 1, (96 << 20) // (maxlen // 2 + 7)).astype(np.uint32)
    log = _log(jl, gpu, lens)
    w = _check(jl, oracle, log)
    nb = log.numel() >> 15
    blocks = [1, 2, nb // 3, nb // 2, nb // 2 + 1, nb - 3]
    for h, n in _last_ok_payload_per_block(w, blocks):
        log[h + 7 + n - 1] ^= 0x04  # the record's last payload byte
    w = _check(jl, oracle, log)
    assert int((w["kind"] == jl.LOG_BAD_CRC).sum()) == len(blocks)


def test_flip_in_every_block(gpu, jl, oracle):
    rng = np.random.default_rng(SEED + 3)
    lens = rng.integers(0, 41, (128 << 20) // 27).astype(np.uint32)
    log = _log(jl, gpu, lens)
    w = _check(jl, oracle, log)
    ok = w[(w["kind"] == 1) & (w["length"] > 0)]
    blk = ok["offset"] >> 15
    nb = log.numel() >> 15
    starts = np.searchsorted(blk, np.arange(nb))
    ends = np.searchsorted(blk, np.arange(nb), side="right")
    flipped = 0
    for b in range(nb):
        if ends[b] > starts[b]:
            r = ok[int(rng.integers(starts[b], ends[b]))]
            log[int(r["offset"]) + 7 + int(rng.integers(0, int(r["length"])))] ^= 0x20
            flipped += 1
    w = _check(jl, oracle, log)
    assert int((w["kind"] == jl.LOG_BAD_CRC).sum()) == flipped


def test_long_and_short_failures_in_one_dense_block(gpu, jl, oracle):
    # 6 x 131 B, one 2 500-B record (deferred to the rounds), 40 x 131 B: dense blocks
    lens = ([131] * 6 + [2500] + [131] * 40) * 80
    log = _log(jl, gpu, lens)
    w = _check(jl, oracle, log)
    ok = w[w["kind"] == 1]
    blk = ok["offset"] >> 15
    longs = ok[ok["length"] == 2500]
    lb = longs["offset"] >> 15
    cases = {}  # block -> (long flip, short before, short after)
    picks = sorted(set(int(b) for b in lb[3:-3]))
    for i, b in enumerate(picks[:8]):
        cases[b] = [(True, True, False), (True, False, True), (True, False, False), (False, False, True),
                    (True, True, True), (False, True, True), (True, True, False), (True, False, True)][i]
    for b, (fl, fb, fa) in cases.items():
        lg = longs[lb == b][0]
        h = int(lg["offset"])
        if fl:
            log[h + 7 + 1234] ^= 0x01
        shorts = ok[(blk == b) & (ok["length"] == 131)]
        before = shorts[shorts["offset"] < h]
        after = shorts[shorts["offset"] > h]
        if fb and before.size:
            log[int(before["offset"][-1]) + 7 + 50] ^= 0x02
        if fa and after.size:
            log[int(after["offset"][0]) + 7 + 60] ^= 0x02
    w = _check(jl, oracle, log)
    assert int((w["kind"] == jl.LOG_BAD_CRC).sum()) >= len(cases)


@pytest.mark.parametrize("maxlen", [40, 200, 800])
def test_inconsistent_dwalk_offsets_recovered(gpu, jl, oracle, maxlen):
    """lc_dense trusts lc_dwalk's header offsets only as the chain its staged
    bytes give (offsets that disagreed made it check garbage
    ranges and write long-record slots past the block's, an aperture fault in
    crc_gv4).  JL_OPT_FAILPOINT perturbs the offsets of every listed block five
    ways (an inner offset, the count past kDWMax, the resume position, the first
    offset, the last offset past the block); every such block must be re-walked
    by lc_dense itself: events equal the oracle's, flips included, no fault."""
    rng = np.random.default_rng(SEED + 7 * maxlen)
    lens = rng.integers(0, maxlen + 1, (48 << 20) // (maxlen // 2 + 7)).astype(np.uint32)
    log = _log(jl, gpu, lens)
    nb = log.numel() >> 15
    for b in (2, 5, nb // 2, nb - 4):  # flips in a few blocks' records
        log[(b << 15) + 3000] ^= 0x10
    prev = jl.set_option(jl.OPT_FAILPOINT, 1)
    try:
        w = _check(jl, oracle, log)
    finally:
        jl.set_option(jl.OPT_FAILPOINT, prev)
    assert int((w["kind"] == jl.LOG_BAD_CRC).sum()) >= 1
    _check(jl, oracle, log)  # and the same log without the failpoint


def _segments(rng, shape):
    """User record lengths for the in-place placement tests (each ~24 MiB of log):
    random 0-200 B lengths (lc_dwalk's blocks), 131-B runs (lc_walk's run blocks),
    both in alternating 2 MiB segments, and runs in which some pairs of records are
    merged into one of the same bytes (2 x 131 + 7): blocks that pass the run checks
    (lc_walk's equal records, lc_dwalk's two headers) but hold one event less than
    predicted, among random blocks (the placement then falls back to lc_build)."""
    def rand(nbytes):
        return rng.integers(0, 201, nbytes // 107).astype(np.uint32)

    def runs(nbytes, merge_every=0):
        n = nbytes // 138
        out = np.full(n, 131, np.uint32)
        if merge_every:
            keep = np.ones(n, bool)
            for i in range(40, n - 1, merge_every):
                out[i] = 2 * 131 + 7
                keep[i + 1] = False
            out = out[keep]
        return out

    seg = 2 << 20
    if shape == "random":
        return rand(24 << 20)
    if shape == "runs":
        return runs(24 << 20)
    if shape == "mixed":
        return np.concatenate([rand(seg) if k % 2 == 0 else runs(seg) for k in range(12)])
    if shape == "mispredicted":
        return np.concatenate([rand(seg) if k % 2 == 0 else runs(seg, 997 if k == 5 else 0) for k in range(12)])
    raise ValueError(shape)


@pytest.mark.parametrize("shape", ["random", "runs", "mixed", "mispredicted"])
def test_inplace_events(gpu, jl, oracle, engine_options, shape):
    """lc_dense writes the events of lc_dwalk's blocks in place, at starts placed by
    the predicted event counts (lc_walk for run blocks, lc_dwalk for the others),
    and lc_build keeps them only where the final count and start agree
    (lc_dense_inplace_kernel, chosen when the workspace's last verification had
    lc_dwalk's blocks).  Each log is verified three times in a row (the first
    call after another log may take either kernel), flips included, and every
    event must equal the oracle's (the device also lists the records a failure
    drops, as kind 0: the live events are compared, as everywhere)."""
    engine_options(jl.OPT_LOG_SMALL_MAX, 0)  # the chunked path at every size
    rng = np.random.default_rng(SEED + len(shape))
    log = _log(jl, gpu, _segments(rng, shape))
    host = log.cpu().numpy().copy()
    for b in rng.choice(host.size // 32768, 24, replace=False):  # a flip in 24 blocks
        host[int(b) * 32768 + int(rng.integers(0, 32768))] ^= 0x10
    import torch

    log = torch.from_numpy(host).to(gpu)
    want = oracle.log_events(host)
    for _ in range(3):
        ev, n = jl.log_verify_dev(log)
        got = ev[: n * 16].cpu().numpy().view(jl.LOG_EVENT_DTYPE)
        g, w = _live(got), _live(want)
        assert g.shape == w.shape and np.array_equal(g, w)
