import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests of the HIP engine")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o

    o.build()
    return o


@pytest.fixture(scope="session")
def jl():
    import jleveldb_amd

    jleveldb_amd.build()
    return jleveldb_amd


@pytest.fixture(scope="session")
def gpu(jl):
    """Initialises the engine on cuda:0 (fails loudly: the product has no CPU path)."""
    import torch

    assert torch.cuda.is_available(), "GPU test collected on a machine without a GPU"
    torch.cuda.set_device(0)
    jl.init(0)
    # the parity tests exercise the device path at every size: small host-memory
    # calls would otherwise take the SSE4.2 host path (JL_OPT_HOST_THRESHOLD,
    # tested on its own in test_gpu_dispatch.py)
    jl.set_option(jl.OPT_HOST_THRESHOLD, 0)
    jl.set_option(jl.OPT_LOG_HOST_THRESHOLD, 0)
    return torch.device("cuda:0")


@pytest.fixture
def engine_options(jl):
    """Sets engine options (jl_set_option) for one test and restores them after it."""
    saved = {}

    def set_(option, value):
        prev = jl.set_option(option, value)
        saved.setdefault(option, prev)

    yield set_
    for option, value in saved.items():
        jl.set_option(option, value)


@pytest.fixture(params=["small", "chunked"])
def log_path(request, jl, engine_options):
    """Runs a log test through both device paths: the one-launch small-log kernel
    (lc_small, every log up to 64 MiB) and the chunked path (walk, dense blocks,
    rounds) forced for every size (JL_OPT_LOG_SMALL_MAX = 0)."""
    engine_options(jl.OPT_LOG_SMALL_MAX, (64 << 20) if request.param == "small" else 0)
    return request.param


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        p = os.path.join(d, name)
        if name.endswith(".json"):
            with open(p) as f:
                return json.load(f)
        with open(p, "rb") as f:
            return f.read()

    return load
