import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "segment-anything-nerf_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import encoders
    encoders.build()
    return encoders.lib()


@pytest.fixture(scope="session")
def hip_lib():
    """The HIP library; built here if missing (hipcc cross-compiles)."""
    import samnerf_amd
    if not os.path.exists(samnerf_amd.LIB_PATH):
        import importlib.util
        spec = importlib.util.spec_from_file_location("samnerf_build", os.path.join(PKG, "build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.build(verbose=False)
    return samnerf_amd.lib()


@pytest.fixture(scope="session")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X (run under gpurun)"
    return torch.device("cuda:0")


@pytest.fixture
def diag(hip_lib):
    """The test runs on the diagnostic build (libsamnerf_hip_diag.so), whose
    kernels take the A/B variant switches from SAMNERF_* environment
    variables; the product library ignores them."""
    from samnerf_amd._lib import diag_library
    with diag_library() as L:
        yield L
