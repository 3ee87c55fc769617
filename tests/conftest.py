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
    out = {"rig": rig, "odd": odd, "rig_krays": krays}
    p = os.path.join(GOLDEN, "calib_rig_oc.npz")
    if os.path.exists(p):                         # Oc != 0 (tests/golden/make_golden.py oc_cases)
        oc = dict(np.load(p))
        ock = dict(oc)
        ock["Nc"] = oc["Nc"][:, :5]
        raw = dict(rig)
        raw["Oc"] = oc["Oc"]
        out.update(rig_oc=oc, rig_oc_krays=ock, rig_oc_raw=raw)
    return out


def host_blas_matches_golden() -> bool:
    """True when this host's BLAS rounds ``np.dot(N, Oc)`` exactly as the host that generated
    the Oc != 0 fixtures did (``calib_blas_oc.npz``).  The reference computes its numerator with
    that call (server/processing.py:166,219), so its own Oc != 0 output depends on the host's
    BLAS; on a host that rounds differently the expected cloud is the oracle's (which makes the
    same call) run here, and the golden is within a few ulps."""
    p = os.path.join(GOLDEN, "calib_blas_oc.npz")
    z = dict(np.load(p))
    cal = dict(np.load(os.path.join(GOLDEN, "calib_rig_oc.npz")))
    raw = dict(np.load(os.path.join(GOLDEN, "calib_rig.npz")))
    oc = cal["Oc"].reshape(3, 1)
    got = {f"numer_{k}": np.dot(np.ascontiguousarray(cal[k].T)[:, 0:3], oc).flatten() for k in ("wPlaneCol", "wPlaneRow")}
    got["numer_raw"] = np.dot(np.ascontiguousarray(raw["wPlaneCol"].T)[:, 0:3], oc).flatten()
    return all(np.array_equal(got[k], z[k]) for k in z)


def expected_cloud(z, cal, rm):
    """The reference's cloud for golden case ``z`` at row_mode ``rm`` on THIS host: the fixture,
    except for Oc != 0 on a host whose BLAS rounds np.dot differently (then the oracle here)."""
    if z["params"]["calib"].startswith("rig_oc") and not host_blas_matches_golden():
        from oracle import sl_oracle as O
        P, C = O.reconstruct_processing(z["col"], z["row"], z["mask"], z["texture"], cal, row_mode=rm)
        assert np.allclose(P, z[f"P{rm}"], rtol=1e-12, atol=0) and np.array_equal(C, z[f"C{rm}"])
        return P, C
    return z[f"P{rm}"], z[f"C{rm}"]


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
