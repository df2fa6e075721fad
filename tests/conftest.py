import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "real-time-disaster-management_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
CFG_DIR = os.path.join(PKG, "rtdm", "cfg")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")


def load_npz(name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def cls_golden():
    return load_npz("cls_golden.npz")


@pytest.fixture(scope="session")
def det_golden():
    return load_npz("det_golden.npz")


@pytest.fixture(scope="session")
def cls_weights():
    z = load_npz("classifier_weights.npz")
    out = {}
    for k, v in z.items():
        m, p = k.split("/", 1)
        out.setdefault(m, {})[p] = v
    return out


def cfg_text(name):
    with open(os.path.join(CFG_DIR, name + ".cfg")) as f:
        return f.read()
