import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the CPU checkers (oracle/) and the product library once per session."""
    import oracle
    oracle.build()
    from bookkeeper_amd.build import build_native, needs_build
    if needs_build():
        build_native()


@pytest.fixture(scope="session")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from bookkeeper_amd import _native
    assert _native.device_count() > 0
    torch.cuda.set_device(0)
    # GPU tests exercise the GPU route of the host-resident batches (the automatic choice on a host
    # with enough cores is the CPU route, which the CPU suite tests); tests of the automatic or CPU
    # route select it explicitly (checksum.host_batch_route)
    from bookkeeper_amd import checksum as ck
    ck.set_host_batch_route(ck.HOST_ROUTE_GPU)
    return torch.device("cuda", 0)
