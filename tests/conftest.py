import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import singa_amd  # noqa: F401
    from singa_amd.ops import native

    native.lib()  # must load: GPU tests never run on a silent fallback
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _gpu_tests_use_the_torch_oracle(request):
    """GPU tests compare the HIP kernels against CPU results: those come from
    the plain PyTorch fp32 expressions (the oracle), not from the native C++
    CppCPU kernels, which have their own parity tests (test_cppcpu_cpu.py)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from singa_amd.ops import cpu as CP

    with CP.torch_oracle():
        yield
