"""The r1 chunked kernel (JL_GENERAL=chunk, kept for A/B) against the oracle: the
variable-size, table and log parity cases of test_gpu_parity.py re-run with it
selected (the default is the stream kernel)."""
import pytest

import test_gpu_parity as base

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def chunk_kernel(monkeypatch):
    monkeypatch.setenv("JL_GENERAL", "chunk")


def test_chunk_every_length_and_alignment(gpu, jl, oracle):
    base.test_batch_every_length_and_alignment(gpu, jl, oracle)


def test_chunk_large_and_zipf(gpu, jl, oracle):
    base.test_batch_large_and_zipf(gpu, jl, oracle)


def test_chunk_golden_fixture(gpu, jl, golden):
    base.test_batch_golden_fixture(gpu, jl, golden)


def test_chunk_fixed_other_sizes(gpu, jl, oracle):
    for bb in (1, 3, 7, 255, 256, 1000, 4097, 100003):
        base.test_fixed_other_sizes(gpu, jl, oracle, bb)


def test_chunk_table(gpu, jl, oracle, golden):
    base.test_table_trailers_and_verify(gpu, jl, oracle, golden)
    base.test_table_many_blocks(gpu, jl, oracle)


def test_chunk_log(gpu, jl, oracle, golden):
    base.test_log_golden(gpu, jl, oracle, golden)
    base.test_log_random_with_corruption(gpu, jl, oracle, 3)
    base.test_log_special_records(gpu, jl, oracle)
    for dl in (0, 32768 - 5, 777):
        base.test_log_emit_dev_matches_logwriter(gpu, jl, oracle, dl)
