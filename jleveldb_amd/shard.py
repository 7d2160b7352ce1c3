"""Multi-GPU layout of the block-checksum path.

Blocks are independent, so the path shards with NO data-path collective: one
process per GPU, each rank owns a contiguous range of the global set and
checksums it where it lies.  The only collectives are bookkeeping: a barrier
around the timed region, a MAX-reduction of the per-rank wall time (the job
takes as long as its slowest rank), a SUM-reduction of mismatch counts in the
verify modes, and — outside the timed checksum path — an optional gather of the
per-unit results for a caller that wants them all in one place.

Three splits, one per kind of unit:
  * fixed-size blocks (C2/C4): `weak_shard` / `strong_shard` — contiguous block
    ranges;
  * variable-size blocks in one arena (C3, table files): `byte_shard` — block
    ranges cut at the byte prefix sum so every rank gets about equal bytes;
  * logs (C5, WAL / MANIFEST): `log_shard` — ranges of whole 32 KiB log blocks.
    LogReader.readPhysicalRecord decides every physical record inside its own
    block (J/db/LogReader.java:297-383; a bad CRC drops only the rest of that
    block), so the blocks of a shard give exactly the decisions the whole-file
    walk gives them; only the file's last, short block carries the EOF cases, and
    it always falls in the last rank's shard.  Fragmented records (First/Middle/
    Last across blocks) need no exchange: each physical fragment has its own CRC.

Used by bench.py (nccl = RCCL over xGMI) and tests/test_shard.py (gloo, CPU).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

WORDS_PER_BLOCK = 4096 // 8  # fill_random_dev counts 8-byte splitmix64 words
LOG_BLOCK = 32768  # J/db/LogFormat.java:52


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    first_block: int  # global index of the rank's first block
    n_blocks: int

    @property
    def first_word(self) -> int:
        """splitmix64 counter of the shard's first 8-byte word (jl_fill_random_dev's
        first_word): rank r's bytes equal bytes [r*n*4096, ...) of the global set."""
        return self.first_block * WORDS_PER_BLOCK


@dataclass(frozen=True)
class ByteShard:
    """Blocks [first_block, first_block + n_blocks) of an arena whose bytes are
    [byte_lo, byte_hi) (the rank stages only those bytes; its offsets are
    relative to byte_lo)."""

    rank: int
    world: int
    first_block: int
    n_blocks: int
    byte_lo: int
    byte_hi: int


@dataclass(frozen=True)
class LogShard:
    """Log bytes [byte_lo, byte_hi) = 32 KiB log blocks [first_block, ...)."""

    rank: int
    world: int
    first_block: int
    n_blocks: int
    byte_lo: int
    byte_hi: int


def _check(rank: int, world: int) -> None:
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank out of range")


def weak_shard(rank: int, world: int, blocks_per_rank: int) -> Shard:
    """Weak scaling (bench.py): every rank holds `blocks_per_rank` blocks of the
    global set of world * blocks_per_rank (config C4 at 1M per rank)."""
    _check(rank, world)
    return Shard(rank, world, rank * blocks_per_rank, blocks_per_rank)


def strong_shard(rank: int, world: int, total_blocks: int) -> Shard:
    """Strong scaling: a fixed global set of `total_blocks` split into contiguous,
    near-equal ranges (the first total % world ranks get one extra block)."""
    _check(rank, world)
    base, extra = divmod(total_blocks, world)
    first = rank * base + min(rank, extra)
    return Shard(rank, world, first, base + (1 if rank < extra else 0))


def byte_shard(rank: int, world: int, off, length) -> ByteShard:
    """Byte-balanced contiguous split of blocks (off[i], length[i]) laid out in
    ascending order in one arena (config C3: packed back-to-back): rank r takes
    the blocks whose end lies in (r*T/world, (r+1)*T/world], T = the arena's
    end.  Each rank's bytes differ from T/world by at most one block."""
    _check(rank, world)
    off = np.asarray(off, dtype=np.uint64)
    length = np.asarray(length, dtype=np.uint64)
    n = off.size
    if n == 0:
        return ByteShard(rank, world, 0, 0, 0, 0)
    ends = off + length
    if np.any(off[1:] < ends[:-1]):
        raise ValueError("byte_shard: blocks must be in ascending, non-overlapping order")
    total = int(ends[-1])
    cut = [0] + [int(np.searchsorted(ends, total * k // world, side="right")) for k in range(1, world)] + [n]
    cut = np.maximum.accumulate(cut)
    i0, i1 = int(cut[rank]), int(cut[rank + 1])
    if i0 == i1:
        return ByteShard(rank, world, i0, 0, 0, 0)
    return ByteShard(rank, world, i0, i1 - i0, int(off[i0]), int(ends[i1 - 1]))


def log_shard(rank: int, world: int, log_bytes: int) -> LogShard:
    """Split a log of `log_bytes` bytes into contiguous ranges of whole 32 KiB
    log blocks (the first nb % world ranks get one extra block)."""
    _check(rank, world)
    nb = (log_bytes + LOG_BLOCK - 1) // LOG_BLOCK
    sh = strong_shard(rank, world, nb)
    lo = min(log_bytes, sh.first_block * LOG_BLOCK)
    hi = min(log_bytes, (sh.first_block + sh.n_blocks) * LOG_BLOCK)
    return LogShard(rank, world, sh.first_block, sh.n_blocks, lo, hi)


def _pg_world() -> int:
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size()


def _coll_device(device):
    """Where a collective's tensors live: the caller's device under RCCL (nccl),
    the host under gloo (CPU jobs, and bench.py --same-device)."""
    import torch.distributed as dist

    return "cpu" if dist.get_backend() == "gloo" else device


def job_wall_time(local_seconds: float, device=None) -> float:
    """Max over ranks of the timed region (a no-op without a process group)."""
    import torch
    import torch.distributed as dist

    if _pg_world() == 1:
        return float(local_seconds)
    t = torch.tensor([float(local_seconds)], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def per_rank(value: float, device=None) -> list[float]:
    """Every rank's value of one float, in rank order (one all_gather; [value]
    without a process group): bench.py reports the per-rank kernel times beside
    their MAX so a slow rank is visible."""
    import torch
    import torch.distributed as dist

    if _pg_world() == 1:
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64, device=_coll_device(device))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def total_mismatches(local_count: int, device=None) -> int:
    """Verify modes: SUM over ranks of the blocks / records that failed their CRC
    (one all_reduce of one integer; a no-op without a process group)."""
    import torch
    import torch.distributed as dist

    if _pg_world() == 1:
        return int(local_count)
    t = torch.tensor([int(local_count)], dtype=torch.int64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def aggregate_rate(bytes_per_rank: int, world: int, wall_seconds: float, steps: int) -> float:
    """Whole-job throughput in GiB/s: all ranks' bytes over the max-over-ranks time."""
    return world * bytes_per_rank * steps / wall_seconds / float(1 << 30)


def gather_results(local, world: int | None = None):
    """All-gather of each rank's per-unit results (1-D tensors of one dtype, any
    per-rank lengths, e.g. the unequal ranges of strong / byte / log shards), in
    rank order: the ranks first all-gather their lengths, then all-gather the
    results padded to the longest, and every rank trims and concatenates.  Not
    part of the checksum path: callers consume their own shard."""
    import torch
    import torch.distributed as dist

    world = _pg_world() if world is None else world
    if world == 1:
        return local
    home = local.device
    flat = local.reshape(-1).to(_coll_device(home))
    n = torch.tensor([flat.numel()], dtype=torch.int64, device=flat.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    counts = [int(x.item()) for x in ns]
    cap = max(counts)
    if cap == 0:
        return flat[:0].to(home)
    pad = torch.zeros(cap, dtype=flat.dtype, device=flat.device)
    pad[: flat.numel()] = flat
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)]).to(home)
