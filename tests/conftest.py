import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return load


@pytest.fixture(scope="session")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    torch.cuda.init()
    return torch
