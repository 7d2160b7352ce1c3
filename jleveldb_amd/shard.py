"""Multi-GPU layout of the block-checksum path.

Blocks are independent, so the path shards with NO data-path collective: one
process per GPU, each rank owns a contiguous range of the global block set and
checksums it where it lies.  The only collectives are bookkeeping: a barrier
around the timed region, a MAX-reduction of the per-rank wall time (the job
takes as long as its slowest rank), and — outside the timed checksum path — an
optional all-gather of the per-block results for a caller that wants them all
on every rank.

Used by bench.py (nccl = RCCL over xGMI) and tests/test_shard.py (gloo, CPU).
"""
from __future__ import annotations

from dataclasses import dataclass

WORDS_PER_BLOCK = 4096 // 8  # fill_random_dev counts 8-byte splitmix64 words


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


def weak_shard(rank: int, world: int, blocks_per_rank: int) -> Shard:
    """Weak scaling (bench.py): every rank holds `blocks_per_rank` blocks of the
    global set of world * blocks_per_rank (config C4 at 1M per rank)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return Shard(rank, world, rank * blocks_per_rank, blocks_per_rank)


def strong_shard(rank: int, world: int, total_blocks: int) -> Shard:
    """Strong scaling: a fixed global set of `total_blocks` split into contiguous,
    near-equal ranges (the first total % world ranks get one extra block)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(total_blocks, world)
    first = rank * base + min(rank, extra)
    return Shard(rank, world, first, base + (1 if rank < extra else 0))


def job_wall_time(local_seconds: float, device=None) -> float:
    """Max over ranks of the timed region (a no-op without a process group)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(local_seconds)
    t = torch.tensor([float(local_seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(bytes_per_rank: int, world: int, wall_seconds: float, steps: int) -> float:
    """Whole-job throughput in GiB/s: all ranks' bytes over the max-over-ranks time."""
    return world * bytes_per_rank * steps / wall_seconds / float(1 << 30)


def gather_results(local, world: int):
    """All-gather of each rank's per-block results (equal shard sizes), in global
    block order.  Not part of the checksum path: callers consume their own shard."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local)
    return torch.cat(parts)
