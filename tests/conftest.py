"""Shared test fixtures.  ``-m gpu`` tests need a ROCm GPU and the in-tree libslgpu.so;
everything else runs on CPU (oracle vs golden vectors, host logic, ABI exports, gloo)."""
import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and libslgpu.so")


def load_calibs():
    rig = dict(np.load(os.path.join(GOLDEN, "calib_rig.npz")))
    odd = dict(np.load(os.path.join(GOLDEN, "calib_odd.npz")))
    krays = dict(rig)
    krays["Nc"] = rig["Nc"][:, :5]
    return {"rig": rig, "odd": odd, "rig_krays": krays}


def golden_cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        name = os.path.basename(f)[:-4]
        if name.startswith("calib_"):
            continue
        out.append(name)
    return out


def load_case(name):
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    z["params"] = json.loads(str(z["params"]))
    return z


def decode_kwargs(params):
    return {k: v for k, v in params.items() if k not in ("variant", "calib")}


@pytest.fixture(scope="session")
def calibs():
    return load_calibs()
