"""The drop-in surface's calibration cache (processing._device_calib): a repeated call with the
same calibration must not re-hash the 3 x H*W ray table (VERDICT r2 "next" #6), and an edited
or different calibration must never be served stale tables."""
import time

import numpy as np
import pytest

from structured_light_for_3d_model_replication_amd import processing as PR


def _calib(h, w, seed=0):
    rng = np.random.default_rng(seed)
    return {"cam_K": np.array([[1000.0, 0, w / 2], [0, 1000.0, h / 2], [0, 0, 1]]), "Oc": np.zeros((3, 1)),
            "wPlaneCol": rng.standard_normal((4, 1920)), "wPlaneRow": rng.standard_normal((4, 1080)),
            "Nc": rng.standard_normal((3, h * w))}


def test_cheap_fingerprint_is_fast_and_content_sensitive():
    cal = _calib(4000, 6000)                       # C4: Nc is 576 MB
    PR.calib_fingerprint(cal)
    t = time.perf_counter()
    for _ in range(10):
        fp = PR.calib_fingerprint(cal)
    dt = (time.perf_counter() - t) / 10
    assert dt < 2e-3, dt                           # target < 1 ms; margin for a loaded CI host
    full = PR.calib_fingerprint(cal, full=True)
    assert fp != full
    for k, idx in (("wPlaneCol", (3, 7)), ("Oc", (1, 0)), ("cam_K", (0, 2)), ("Nc", (2, 6000 * 4000 - 1))):
        c2 = dict(cal)
        c2[k] = cal[k].copy()
        c2[k][idx] += 1e-9
        assert PR.calib_fingerprint(c2) != fp, k
        assert PR.calib_fingerprint(c2, full=True) != full, k
    c3 = dict(cal)                                 # an Nc edit outside the sample: full digest only
    c3["Nc"] = cal["Nc"].copy()
    c3["Nc"][0, 12345] += 1.0
    assert PR.calib_fingerprint(c3) == fp and PR.calib_fingerprint(c3, full=True) != full


@pytest.mark.gpu
def test_device_calib_cache_hits_and_misses():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a ROCm device")
    h, w = 4000, 6000
    cal = _calib(h, w)
    PR._CALIBS.clear()
    dc = PR._device_calib(cal, h, w)
    t = time.perf_counter()
    for _ in range(10):
        assert PR._device_calib(cal, h, w) is dc   # same Nc object: cheap digest only
    assert (time.perf_counter() - t) / 10 < 2e-3
    same = {k: np.array(v, copy=True) for k, v in cal.items()}
    assert PR._device_calib(same, h, w) is dc      # equal content, other object: full digest confirms
    edited = dict(same)
    edited["Nc"] = same["Nc"].copy()
    edited["Nc"][1, 777] += 1.0                    # outside the cheap sample
    dc2 = PR._device_calib(edited, h, w)
    assert dc2 is not dc and dc2.rays is not None
    assert float(dc2.rays[1, 777].item()) == edited["Nc"][1, 777]
