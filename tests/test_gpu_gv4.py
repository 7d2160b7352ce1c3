"""The general v4 kernel (general_v4.hip; the default general path except for
small offset/length batches; JL_OPT_GENERAL_PATH = JL_PATH_GV4 forces it) against the oracle: the variable-size, fixed-stride, table and log parity
cases of test_gpu_parity.py re-run with it selected, plus cases aimed at its
sorted-round pipeline (every K bucket, partial rounds, empty blocks mixed in,
blocks around the 128-B step grid, a block above the solo threshold)."""
import numpy as np
import pytest

import test_gpu_parity as base
from test_gpu_parity import THREADS, to_dev, u32

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def gv4_kernel(jl, engine_options):
    engine_options(jl.OPT_GENERAL_PATH, jl.PATH_GV4)


def test_gv4_every_length_and_alignment(gpu, jl, oracle):
    base.test_batch_every_length_and_alignment(gpu, jl, oracle)


def test_gv4_large_and_zipf(gpu, jl, oracle):
    base.test_batch_large_and_zipf(gpu, jl, oracle)


def test_gv4_golden_fixture(gpu, jl, golden):
    base.test_batch_golden_fixture(gpu, jl, golden)


@pytest.mark.parametrize("block_bytes", [1, 3, 4, 7, 64, 127, 128, 129, 255, 256, 1000, 1057, 4095, 4097, 65536, 100003])
def test_gv4_fixed_other_sizes(gpu, jl, oracle, block_bytes):
    base.test_fixed_other_sizes(gpu, jl, oracle, block_bytes)


def test_gv4_step_grid_and_partial_rounds(gpu, jl, oracle):
    """Lengths 128k-1..128k+1 for k up to 40, each repeated 1..9 times (partial
    rounds of 8), interleaved with empty blocks, random order and alignment."""
    rng = np.random.default_rng(21)
    lens = []
    for k in range(0, 41):
        for d in (-1, 0, 1):
            if 128 * k + d >= 0:
                lens += [128 * k + d] * int(rng.integers(1, 10))
    lens += [0] * 13
    lens = np.array(lens, np.uint32)
    rng.shuffle(lens)
    gaps = rng.integers(0, 20, lens.size)
    offs = np.zeros(lens.size, np.uint64)
    pos = 0
    for i in range(lens.size):
        pos += int(gaps[i])
        offs[i] = pos
        pos += int(lens[i])
    arena = rng.integers(0, 256, pos + 8, dtype=np.uint8)
    d = (to_dev(arena, gpu), to_dev(offs.view(np.int64), gpu), to_dev(lens.view(np.int32), gpu))
    assert np.array_equal(u32(jl.crc32c_batch_dev(*d)), oracle.batch(arena, offs, lens, threads=THREADS))
    init = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    sfx = rng.integers(0, 256, lens.size, dtype=np.uint8)
    got = u32(jl.crc32c_batch_dev(*d, init=to_dev(init.view(np.int32), gpu), suffix=to_dev(sfx, gpu), flags=0))
    assert np.array_equal(got, oracle.batch(arena, offs, lens, init=init, suffix=sfx, flags=0, threads=THREADS))


def test_gv4_block_at_allocation_edges(gpu, jl, oracle):
    """First block at byte 0 of the allocation and the last ending at its last
    byte (the step-0 chunks and stored-crc chunks must stay inside)."""
    import torch

    rng = np.random.default_rng(22)
    for n in (1, 2, 5, 15, 16, 17, 127, 128, 129, 1000):
        host = rng.integers(0, 256, n, dtype=np.uint8)
        t = torch.from_numpy(host).to(gpu)
        off = torch.zeros(1, dtype=torch.int64, device=gpu)
        ln = torch.full((1,), n, dtype=torch.int32, device=gpu)
        assert u32(jl.crc32c_batch_dev(t, off, ln))[0] == oracle.batch(host, np.zeros(1, np.uint64),
                                                                      np.array([n], np.uint32))[0]


def test_gv4_solo_block(gpu, jl, oracle):
    """A block above the solo threshold (>= 131071 steps = 16 MiB) among small ones."""
    rng = np.random.default_rng(23)
    lens = np.array([5, (1 << 24) + 77, 300, 0, 129], np.uint32)
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = rng.integers(0, 256, int(lens.sum()) + 8, dtype=np.uint8)
    got = u32(jl.crc32c_batch_dev(to_dev(arena, gpu), to_dev(offs.view(np.int64), gpu), to_dev(lens.view(np.int32), gpu)))
    assert np.array_equal(got, oracle.batch(arena, offs, lens, threads=THREADS))


def test_gv4_table(gpu, jl, oracle, golden):
    base.test_table_trailers_and_verify(gpu, jl, oracle, golden)
    base.test_table_many_blocks(gpu, jl, oracle)


def test_gv4_log(gpu, jl, oracle, golden):
    base.test_log_golden(gpu, jl, oracle, golden)
    for seed in (3, 4):
        base.test_log_random_with_corruption(gpu, jl, oracle, seed)
    base.test_log_special_records(gpu, jl, oracle)
    base.test_log_corruption_recovery(gpu, jl, oracle)
    base.test_log_dev_resident(gpu, jl, oracle)


def test_log_through_stream_kernel(gpu, jl, oracle, golden, engine_options):
    """The log verify's batched crc defaults to gv4; the stream kernel stays covered."""
    engine_options(jl.OPT_GENERAL_PATH, jl.PATH_STREAM)
    test_gv4_log(gpu, jl, oracle, golden)


@pytest.mark.parametrize("shift", [1, 16, 100, 127])
@pytest.mark.parametrize("block_bytes", [256, 4096])
def test_gv4_fixed_unaligned_base(gpu, jl, oracle, shift, block_bytes):
    """Fixed stride on a base off the 128-B grid: every block gets front and tail
    pads (the sorted pipeline with implicit offsets, not the implicit rounds)."""
    rng = np.random.default_rng(shift * 7 + block_bytes)
    n = 777
    host = rng.integers(0, 256, n * block_bytes + shift, dtype=np.uint8)
    t = to_dev(host, gpu)[shift:]
    got = u32(jl.crc32c_fixed_dev(t, block_bytes, n))
    assert np.array_equal(got, oracle.fixed(host[shift:], block_bytes, n, threads=THREADS))


@pytest.mark.parametrize("case", ["every_length", "zipf", "table"])
def test_stream_kernel_still_exact(gpu, jl, oracle, golden, engine_options, case):
    """The stream kernel (the default for small offset/length batches) on the
    cases above, forced."""
    engine_options(jl.OPT_GENERAL_PATH, jl.PATH_STREAM)
    if case == "every_length":
        base.test_batch_every_length_and_alignment(gpu, jl, oracle)
    elif case == "zipf":
        base.test_batch_large_and_zipf(gpu, jl, oracle)
    else:
        base.test_table_trailers_and_verify(gpu, jl, oracle, golden)
        base.test_table_many_blocks(gpu, jl, oracle)


def test_gv4_rounds_pipeline_large_bins(gpu, jl, oracle):
    """Blocks of 512 KiB .. 1.5 MiB (steps >= 4096: the global-atomic bins, and
    the scan's second and later 4096-bin tiles) mixed with small ones and
    repeated lengths (partial rounds of one bin), in one batch."""
    rng = np.random.default_rng(24)
    big = [int(x) for x in rng.integers(512 << 10, 1536 << 10, 12)]
    lens = np.array(big + [big[0]] * 9 + [7, 0, 1000, 4096, 129] * 5, np.uint32)
    rng.shuffle(lens)
    offs = np.zeros(lens.size, np.uint64)
    pos = 0
    for i in range(lens.size):
        pos += int(rng.integers(0, 64))
        offs[i] = pos
        pos += int(lens[i])
    arena = rng.integers(0, 256, pos + 8, dtype=np.uint8)
    got = u32(jl.crc32c_batch_dev(to_dev(arena, gpu), to_dev(offs.view(np.int64), gpu), to_dev(lens.view(np.int32), gpu)))
    assert np.array_equal(got, oracle.batch(arena, offs, lens, threads=THREADS))


@pytest.mark.parametrize("part_cap", [None, "8"])
def test_gv4_split_blocks(gpu, jl, oracle, engine_options, part_cap):
    """Blocks above 512 KiB are split into chunks (computed from state 0 on their
    own waves) and folded per block with z^len: lengths around the split
    threshold and the chunk size, an 8 MiB + 77 block, a 40 MiB block (160
    chunks), unaligned starts, with init / suffix / unmasked variants.
    part_cap 8: only the first split blocks get chunk slots, the rest stay whole."""
    if part_cap:
        engine_options(jl.OPT_SPLIT_CAP, int(part_cap))
    rng = np.random.default_rng(25)
    lens = np.array([(512 << 10) + 1, (512 << 10), 600 << 10, (1 << 20) + 3, (768 << 10), (8 << 20) + 77, 40 << 20,
                     5, 4096, 0, (256 << 10) * 3 - 1], np.uint32)
    offs = np.zeros(lens.size, np.uint64)
    pos = 0
    for i in range(lens.size):
        pos += int(rng.integers(0, 200))
        offs[i] = pos
        pos += int(lens[i])
    arena = rng.integers(0, 256, pos + 8, dtype=np.uint8)
    d = (to_dev(arena, gpu), to_dev(offs.view(np.int64), gpu), to_dev(lens.view(np.int32), gpu))
    assert np.array_equal(u32(jl.crc32c_batch_dev(*d)), oracle.batch(arena, offs, lens, threads=THREADS))
    init = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    sfx = rng.integers(0, 256, lens.size, dtype=np.uint8)
    got = u32(jl.crc32c_batch_dev(*d, init=to_dev(init.view(np.int32), gpu), suffix=to_dev(sfx, gpu), flags=0))
    assert np.array_equal(got, oracle.batch(arena, offs, lens, init=init, suffix=sfx, flags=0, threads=THREADS))


@pytest.mark.parametrize("block_bytes", [(1 << 20), (3 << 20) + 5])
def test_gv4_split_fixed_stride(gpu, jl, oracle, block_bytes):
    """Few large fixed-stride blocks (the crc32c_fixed_dev path) go through the split."""
    rng = np.random.default_rng(block_bytes)
    n = 9
    host = rng.integers(0, 256, n * block_bytes, dtype=np.uint8)
    got = u32(jl.crc32c_fixed_dev(to_dev(host, gpu), block_bytes, n))
    assert np.array_equal(got, oracle.fixed(host, block_bytes, n, threads=THREADS))


def test_gv4_concurrent_streams(gpu, jl, oracle):
    """Two streams running rounds pipelines at once (stream-ordered scratch per
    call, no shared workspace on the device path): each gets its own results."""
    import torch

    rng = np.random.default_rng(26)
    batches = []
    for s in range(2):
        lens = rng.integers(0, 20000, 3000).astype(np.uint32)
        offs = np.zeros(lens.size, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)
        arena = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 8, dtype=np.uint8)
        batches.append((arena, offs, lens))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev = [(to_dev(a, gpu), to_dev(o.view(np.int64), gpu), to_dev(ln.view(np.int32), gpu)) for a, o, ln in batches]
    torch.cuda.synchronize()
    outs = [[], []]
    for rep in range(4):
        for s in range(2):
            with torch.cuda.stream(streams[s]):
                outs[s].append(jl.crc32c_batch_dev(*dev[s], stream=streams[s]))
    torch.cuda.synchronize()
    for s in range(2):
        want = oracle.batch(*batches[s], threads=THREADS)
        for o in outs[s]:
            assert np.array_equal(u32(o), want)


def test_gv4_table_verify_batched_rounds(gpu, jl, oracle):
    """A table of 400 000 blocks (~50 000 rounds: past 64 x the grid, so the
    rounds after the heaviest quarter are dealt in batches from the device
    counter, general_v4.hip GPF::seq) through MODE_TABLE_VERIFY: trailers written
    by jl_table_trailers_dev (a sample pinned to the oracle's TableBuilder
    trailer), every block verifies; bytes flipped in 64 blocks (data or trailer)
    fail exactly those."""
    import torch

    rng = np.random.default_rng(77)
    n = 400_000
    sizes = rng.integers(0, 3000, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(sizes.astype(np.uint64) + 5)[:-1]
    total = int(off[-1]) + int(sizes[-1]) + 5
    d_f = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu)
    d_off, d_size = to_dev(off.view(np.int64), gpu), to_dev(sizes.view(np.int32), gpu)
    types = rng.integers(0, 2, n, dtype=np.uint8)
    tr = jl.table_trailers_dev(d_f, d_off, d_size, types=to_dev(types, gpu)).reshape(-1, 5)
    idx = (d_off + d_size.to(torch.int64)).unsqueeze(1) + torch.arange(5, device=gpu).unsqueeze(0)
    d_f[idx.reshape(-1)] = tr.reshape(-1)  # the file now holds each block's trailer
    host = d_f.cpu().numpy()
    for i in rng.integers(0, n, 200):
        o, s = int(off[i]), int(sizes[i])
        assert host[o + s:o + s + 5].tobytes() == oracle.table_trailer(host[o:o + s].tobytes(), int(types[i])), i
    assert jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy().all()
    bad = np.unique(rng.integers(0, n, 64))
    for i in bad:
        o, s = int(off[i]), int(sizes[i])
        d_f[o + int(rng.integers(0, s + 5))] ^= 1 << int(rng.integers(0, 8))
    st = jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy()
    assert set(np.nonzero(st == 0)[0].tolist()) == set(bad.tolist())


def test_gv4_table_verify_zipf_many_flips(gpu, jl):
    """2 000 000 blocks of Zipf(1.3) sizes up to 64 KiB (~5.7 GB: C3's size
    mix), trailers from jl_table_trailers_dev, bits flipped in ~2 000 blocks:
    the failing set is exactly the flipped blocks, three calls in a row (the
    round dealing's batches past the heaviest quarter, at C3's scale)."""
    import torch

    rng = np.random.default_rng(7)
    n = 2_000_000
    sizes = np.minimum(rng.zipf(1.3, n), 65536).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(sizes.astype(np.uint64) + 5)[:-1]
    total = int(off[-1]) + int(sizes[-1]) + 5
    d_f = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu)
    d_off, d_size = to_dev(off.view(np.int64), gpu), to_dev(sizes.view(np.int32), gpu)
    types = rng.integers(0, 2, n, dtype=np.uint8)
    tr = jl.table_trailers_dev(d_f, d_off, d_size, types=to_dev(types, gpu)).reshape(-1, 5)
    idx = (d_off + d_size.to(torch.int64)).unsqueeze(1) + torch.arange(5, device=gpu).unsqueeze(0)
    d_f[idx.reshape(-1)] = tr.reshape(-1)
    del tr, idx
    assert jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy().all()
    bad = np.unique(rng.integers(0, n, 2000))
    for i in bad:
        o, s = int(off[i]), int(sizes[i])
        d_f[o + int(rng.integers(0, s + 5))] ^= 1 << int(rng.integers(0, 8))
    for _ in range(3):
        st = jl.table_verify_dev(d_f, d_off, d_size).cpu().numpy()
        assert np.array_equal(np.nonzero(st == 0)[0], bad)


@pytest.mark.parametrize("n", [140_000, 200_000, 260_000])
def test_gv4_batches_of_one_round(gpu, jl, oracle, n):
    """17 500 - 32 500 rounds: just above 64 x the grid (256 workgroups), so the
    device-counter batches hold ONE round each (general_v4.hip GPF::seq, DB = 1)
    and batch slots are reused every 16 rounds: a slot's next batch waits until
    every round of the one before has read its base.  Every CRC
    against the oracle, five calls in a row."""
    import torch

    rng = np.random.default_rng(n)
    sizes = rng.integers(0, 900, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(sizes.astype(np.uint64) + 3)[:-1]
    total = int(off[-1]) + int(sizes[-1]) + 3
    host = rng.integers(0, 256, total, dtype=np.uint8)
    d_a = torch.from_numpy(host).to(gpu)
    d_off, d_len = to_dev(off.view(np.int64), gpu), to_dev(sizes.view(np.int32), gpu)
    want = oracle.batch(host, off, sizes, threads=THREADS)
    for _ in range(5):
        assert np.array_equal(u32(jl.crc32c_batch_dev(d_a, d_off, d_len)), want)
