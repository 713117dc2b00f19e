import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on the GPU box")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def goldens():
    return dict(np.load(os.path.join(GOLDEN, "oracle_small.npz")))


@pytest.fixture(scope="session")
def lenna():
    return np.load(os.path.join(GOLDEN, "lenna_bgr.npz"))["bgr"]


@pytest.fixture(scope="session")
def dev():
    """HIP device helpers for the gpu tests (torch only allocates and copies)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import various_image_processings_amd as vip
    vip.lib()

    class Dev:
        torch_ = torch

        @staticmethod
        def put(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")

        @staticmethod
        def empty(shape, dtype=np.uint8):
            tdt = {np.uint8: torch.uint8, np.float32: torch.float32}[dtype]
            return torch.empty(shape, dtype=tdt, device="cuda")

        @staticmethod
        def get(t):
            torch.cuda.synchronize()
            return t.cpu().numpy()

    return Dev
