"""Device-side descriptor checks of the `_dev` batch and verify entry points:
a handle whose bytes (and, for the table verify, 5-byte trailer) reach past the
caller's base_bytes is never read — it gets result 0 (crc 0 / "block checksum
mismatch") — and every other handle of the batch keeps its exact result.  The
handles of a table come from its (untrusted) index block, TableFormat.java:
66-78 / 207-218, so a corrupt one must not become an out-of-bounds HBM read.
Both kernels that read descriptors are covered: the general v4 rounds
pipeline and the one-launch stream kernel."""
import numpy as np
import pytest

from test_gpu_parity import THREADS, to_dev, u32

pytestmark = pytest.mark.gpu

BAD_OFFS = [2**64 - 1, 2**63, 2**40, None]  # None: just past the end


def _bad_handles(rng, n, size, bad_at, extra):
    off = np.sort(rng.integers(0, size - 70000, n)).astype(np.uint64)
    ln = rng.integers(0, 60000, n).astype(np.uint32)
    for k, i in enumerate(bad_at):
        b = BAD_OFFS[k % len(BAD_OFFS)]
        if b is None:
            off[i] = size - int(ln[i]) - extra + 1  # one byte past the end
        else:
            off[i] = b
    return off, ln


@pytest.mark.parametrize("path", ["auto", "gv4", "stream"])
@pytest.mark.parametrize("n", [100, 5000])
def test_batch_out_of_range_handles(gpu, jl, oracle, engine_options, path, n):
    engine_options(jl.OPT_GENERAL_PATH, {"auto": jl.PATH_AUTO, "gv4": jl.PATH_GV4, "stream": jl.PATH_STREAM}[path])
    rng = np.random.default_rng(n)
    size = 8 << 20
    arena = rng.integers(0, 256, size, dtype=np.uint8)
    bad = sorted(rng.choice(n, 9, replace=False).tolist())
    off, ln = _bad_handles(rng, n, size, bad, 0)
    ln[bad[0]] = 700 << 10  # a would-be split block that is out of range
    off[bad[0]] = size - (700 << 10) + 5
    got = u32(jl.crc32c_batch_dev(to_dev(arena, gpu), to_dev(off.view(np.int64), gpu), to_dev(ln.view(np.int32), gpu)))
    good = np.setdiff1d(np.arange(n), bad)
    want = oracle.batch(arena, off[good], ln[good], threads=THREADS)
    assert np.array_equal(got[good], want)
    assert not got[bad].any()


@pytest.mark.parametrize("path", ["auto", "gv4", "stream"])
@pytest.mark.parametrize("n", [64, 6000])
def test_table_verify_out_of_range_handles(gpu, jl, oracle, engine_options, path, n):
    engine_options(jl.OPT_GENERAL_PATH, {"auto": jl.PATH_AUTO, "gv4": jl.PATH_GV4, "stream": jl.PATH_STREAM}[path])
    rng = np.random.default_rng(7 * n)
    blocks = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in rng.integers(0, 3000, n)]
    parts, off, size = [], [], []
    pos = 0
    for blk in blocks:
        parts.append(blk + oracle.table_trailer(blk))
        off.append(pos)
        size.append(len(blk))
        pos += len(blk) + 5
    file = np.frombuffer(b"".join(parts), np.uint8).copy()
    off = np.array(off, np.uint64)
    size = np.array(size, np.uint32)
    bad = sorted(rng.choice(n, 6, replace=False).tolist())
    for k, i in enumerate(bad):
        b = BAD_OFFS[k % len(BAD_OFFS)]
        off[i] = file.size - int(size[i]) - 5 + 1 if b is None else b  # the trailer one byte short
    st = jl.table_verify_dev(to_dev(file, gpu), to_dev(off.view(np.int64), gpu),
                             to_dev(size.view(np.int32), gpu)).cpu().numpy()
    good = np.setdiff1d(np.arange(n), bad)
    assert st[good].all() and not st[bad].any()
    # a block ending exactly at the file's end is still in range
    last = np.array([off[good[-1]]], np.uint64)
    assert int(last[0]) + int(size[good[-1]]) + 5 <= file.size
