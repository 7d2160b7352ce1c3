"""bench.py's N-rank path, rehearsed on the one GPU of a test box
(`--same-device`: every rank on GPU 0, gloo collectives): the spawn through
torch.distributed.run from a parent that never initialises HIP, the barriers,
the MAX-over-ranks timing, the padded all-gather of unequal strong shards, and
rank 0's single JSON line with n_gpus = 2 and 8 (the driver's largest N) — plus the gathered results equal to
one launch over the whole set (BASELINE config C4's shape, DBBench.java:775-793
blocks), recorded on the line as parity_gathered_vs_single_launch.  What the
driver's 8-GPU run adds is RCCL instead of gloo and one GPU per rank.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra, gpus=2):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--same-device", "--steps", "2",
           "--warmup", "1", "--settle-ms", "0", "--no-cpu", "--no-secondary", *extra]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_two_ranks_weak():
    r = _bench("--blocks", "4096")
    assert r["n_gpus"] == 2 and r["scaling"] == "weak" and r["steps"] == 2
    assert r["config"]["blocks_per_gpu"] == 4096
    assert r["parity_gathered_vs_single_launch"] is True
    assert r["value"] > 0 and r["result_allgather_ms"] is not None
    assert len(r["rank_kernel_ms"]) == 2 and r["rank_kernel_ms_spread"] >= 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_eight_ranks_weak():
    """The driver's N = 8 launch shape (C4 weak, 1M blocks per GPU there; 4096
    here, 8 ranks sharing GPU 0): 8 processes through torch.distributed.run."""
    r = _bench("--blocks", "4096", gpus=8)
    assert r["n_gpus"] == 8 and r["scaling"] == "weak" and r["config"]["blocks_per_gpu"] == 4096
    assert r["parity_gathered_vs_single_launch"] is True
    assert len(r["rank_kernel_ms"]) == 8 and max(r["rank_kernel_ms"]) > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_eight_ranks_strong():
    """C4 strong over 8 ranks with a total that does not divide (65541 = 8 x 8192
    + 5: ranks 0-4 one block longer)."""
    r = _bench("--strong-total", "65541", gpus=8)
    assert r["n_gpus"] == 8 and r["scaling"] == "strong"
    assert r["config"]["blocks_per_gpu"] == 8193
    assert r["parity_gathered_vs_single_launch"] is True


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_two_ranks_strong_unequal():
    r = _bench("--strong-total", "1001")
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["blocks_per_gpu"] == 501  # rank 0 of 501 + 500
    assert r["parity_gathered_vs_single_launch"] is True


def test_visible_gpus_counts_without_hip(monkeypatch):
    """The parent counts devices from the environment (no HIP initialisation)."""
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3,5")
    assert bench.visible_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0
