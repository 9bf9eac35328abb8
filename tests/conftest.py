"""Test configuration.

``-m "not gpu"`` (the CPU suite, runs in the build container): the oracle
against the reference's golden vectors, host-side logic, the C-ABI library
loading and exporting every symbol of include/msa.h, and the world_size-2
gloo sharding path.  ``-m gpu`` (MI355X): bit-exact parity of the HIP path,
called through the C-ABI, against the oracle and the golden fixtures.

The oracle (oracle/) is test infrastructure only; it is imported here as the
checker, never as the thing under test.
"""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through libmsa.so")


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
