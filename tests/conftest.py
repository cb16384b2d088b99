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


REFERENCE_APP = "/root/reference/app.py"


@pytest.fixture
def st_stub(monkeypatch):
    """The recording Streamlit double, importable as ``streamlit``."""
    monkeypatch.syspath_prepend(STUBS)
    sys.modules.pop("streamlit", None)
    import streamlit

    streamlit.reset()
    yield streamlit
    sys.modules.pop("streamlit", None)


@pytest.fixture
def reference_app(st_stub):
    """The reference app.py imported behind the Streamlit double (behavioural parity
    oracle; skipped where the read-only reference checkout is absent)."""
    import importlib.util

    if not os.path.exists(REFERENCE_APP):
        pytest.skip("reference checkout not present")
    spec = importlib.util.spec_from_file_location("reference_app", REFERENCE_APP)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    st_stub.reset()
    return mod
