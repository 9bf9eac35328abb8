"""Test configuration.

``-m "not gpu"`` (the CPU suite, runs in the build container): the oracle
against the reference's golden vectors, host-side logic, the C-ABI library
loading and exporting every symbol of include/msa.h, and the world_size-2
gloo sharding path.  ``-m gpu`` (MI355X): bit-exact parity of the HIP path,
called through the C-ABI, against the oracle and the golden fixtures.

The oracle (oracle/) is test infrastructure only; it is imported here as the
checker, never as the thing under test.
"""
import faulthandler
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


# a hang leaves every thread's stack on stderr (SIGSEGV / SIGABRT / the timeout below)
faulthandler.enable()

# Every GPU test gets a time limit of its own, below gpurun's 180 s silence window: the thread method
# dumps all stacks and ends the process, so a test stuck inside a GPU call names itself (the whole GPU
# suite runs in ~30 s; the slowest test takes a few seconds).
GPU_TEST_TIMEOUT_S = 120


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through libmsa.so")


def pytest_collection_modifyitems(config, items):
    for item in items:
        if item.get_closest_marker("gpu") is not None and item.get_closest_marker("timeout") is None:
            item.add_marker(pytest.mark.timeout(GPU_TEST_TIMEOUT_S, method="thread"))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def dataset(oracle):
    return oracle.load_dataset()


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU visible")
    return torch.device("cuda", 0)
