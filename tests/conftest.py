import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
STUBS = os.path.join(ROOT, "tests", "stubs")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-process or long-running")


@pytest.fixture(scope="session")
def native():
    from rocmdash.runtime import native as nat

    return nat.load(build=True)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test without a GPU (run with -m 'not gpu' on CPU)")
    return torch.device("cuda", 0)
