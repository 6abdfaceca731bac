import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


SPAWNING = ("test_multirank_gpu", "test_bench_gpu")


def pytest_collection_modifyitems(config, items):
    """Multi-process GPU tests (ranks, bench.py subprocesses) start their processes before this
    process initialises the GPU: run them first in the session."""
    first = [it for it in items if any(m in it.nodeid for m in SPAWNING)]
    if first:
        rest = [it for it in items if not any(m in it.nodeid for m in SPAWNING)]
        items[:] = first + rest
