import os
import socket
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built extension")
    config.addinivalue_line("markers", "slow: multi-process / long-running CPU test")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture
def port():
    return free_port()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pytorch_distributed_mnist_amd.ops import _ext
    _ext.require()          # GPU tests must run the native path: fail loudly if not built
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _release_native_objects():
    """Between tests: collect the previous test's programs and communicators and release their
    native parts here, outside any hipGraph capture (parallel/comm.py release_retired)."""
    yield
    import sys
    mod = sys.modules.get("pytorch_distributed_mnist_amd.parallel.comm")
    if mod is not None:
        import gc
        gc.collect()
        mod.release_retired()
