import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_runtime():
    """Build the torch-free C++ runtime (g++, seconds) if it is missing or stale."""
    from distributed_llm_inference import _build
    _build.build_runtime()
    yield


@pytest.fixture(autouse=True)
def _restore_kernel_policy():
    """A test may change the process's kernel policy (ops.kernel_policy / set_policy): every
    test starts from, and leaves, the policy it found."""
    from distributed_llm_inference import ops
    saved = ops._POLICY
    yield
    ops._POLICY = saved


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_llm_inference import _build
    _build.build_kernels()
    from distributed_llm_inference import ops
    ops.native()  # raise loudly if the HIP extension cannot be loaded
    return torch.device("cuda:0")
