import os
os.environ.setdefault("MPLBACKEND", "Agg")   # the Armijo report figures of newton_Algorithm draw off-screen
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device; the parity tests proper")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name if name.endswith(".npz") else name + ".npz"))


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def task2_refs():
    from oracle.acrobot_np import load_task2_refs
    x_ref, u_ref, t_ref = load_task2_refs(os.path.join(GOLDEN, "task2_input_fully_actuated.npz"))
    return x_ref, u_ref, t_ref


def rel_l2(a, b):
    a = np.asarray(a, float); b = np.asarray(b, float)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))
