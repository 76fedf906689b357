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
    config.addinivalue_line("markers", "legacy: exercises a superseded FIR kernel (libnsh_hip.so built with "
                            "make LEGACY=1); deselected when the library was built without them")


def _legacy_built():
    try:
        from newsched_amd import nsh

        return nsh.fir_legacy_available()
    except Exception:
        return False


_LEGACY_DROPPED = []


def pytest_collection_modifyitems(config, items):
    """The superseded kernels' parity tests (marker `legacy`) run only against a LEGACY=1 build;
    with the default library they are deselected (reported as such, not as skips)."""
    legacy = [it for it in items if it.get_closest_marker("legacy")]
    if legacy and not _legacy_built():
        keep = [it for it in items if not it.get_closest_marker("legacy")]
        config.hook.pytest_deselected(items=legacy)
        items[:] = keep
        _LEGACY_DROPPED.append(len(legacy))


def pytest_terminal_summary(terminalreporter):
    if _LEGACY_DROPPED:
        terminalreporter.write_line(f"{_LEGACY_DROPPED[0]} legacy-kernel tests deselected: libnsh_hip.so was built "
                                    "without the superseded FIR kernels (make LEGACY=1 to run them)")


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
