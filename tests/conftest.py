"""Shared pytest configuration.

* ``gpu`` marker: tests that need an MI355X (run on the GPU box with -m gpu).
* Puts the repo root (oracle/) and the product package directory
  (copula-msm-and-copula-garch-var_amd/) on sys.path.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "copula-msm-and-copula-garch-var_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_CASES = sorted(f[:-4] for f in os.listdir(GOLDEN)
                      if f.endswith(".npz") and f != "kat_special.npz" and not f.startswith(("optim_", "fullbatch_")))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def golden_kwargs(z):
    """calc_var keyword arguments recorded with a golden case."""
    kw = {}
    if "kw_obj_var" in z:
        kw["obj_var"] = float(z["kw_obj_var"])
    if "kw_first_guess" in z:
        kw["first_guess"] = float(z["kw_first_guess"])
    if "kw_second_guess" in z:
        kw["second_guess"] = tuple(float(v) for v in z["kw_second_guess"])
    return kw


def golden_calls(z):
    n = int(z["n_calls"])
    return [(z[f"call{i:02d}_bounds"], z[f"call{i:02d}_result"]) for i in range(n)]


@pytest.fixture(scope="session")
def gpu_available():
    try:
        from copula_var import _native
        return _native.device_count() > 0
    except Exception:
        return False
