import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP path")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))


def close(actual, expected, rel, what=""):
    """max|a-e| <= rel * max(1, max|e|) (SURVEY.md §8c tolerance form)."""
    a = np.asarray(actual, dtype=np.float64)
    e = np.asarray(expected, dtype=np.float64)
    assert a.shape == e.shape, f"{what}: shape {a.shape} != {e.shape}"
    scale = max(1.0, float(np.abs(e).max()) if e.size else 1.0)
    err = float(np.abs(a - e).max()) if e.size else 0.0
    assert err <= rel * scale, f"{what}: max|diff|={err:.3e} > {rel:.1e}*{scale:.3e}"
    return err


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    return torch.device("cuda:0")
