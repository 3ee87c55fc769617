"""Generate the golden fixtures in ``tests/golden/`` by running the REFERENCE itself.

Run in the survey container only (needs ``/root/reference``):

    python tests/golden/make_golden.py

For every case below a synthetic capture is rendered (``synth.render_view``), the reference's
own functions are called on it through ``refharness`` (``ProcessingLogic._gray_decode`` with
a file list, ``ProcessingLogic._reconstruct_point_cloud``, and the nested ``gray_decode`` /
``reconstruct_point_cloud`` of ``SLSystem.generate_cloud``), and inputs + outputs are saved as
compressed ``.npz`` data.  The calibration tables come from the reference's own
``SLSystem.calibrate_final`` with the OpenCV solvers stubbed to return the rig's K/R/T
(SURVEY §8(c)); its ``Nc`` is checked bit-identical to ``calibration.pinhole_rays``.
Only data is written (inputs and expected outputs) — no reference source.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE))

import refharness  # noqa: E402
from structured_light_for_3d_model_replication_amd import calibration, synth  # noqa: E402

PL, gray_decode_sl, recon_sl, sl_system = refharness.load()


def ref_calibration(rig: synth.Rig) -> dict:
    """Run ``SLSystem.calibrate_final`` with stubbed solvers; return the saved .mat dict."""
    cv2 = sys.modules["cv2"]
    K1, K2, R, T = rig.K1, rig.K2, rig.R, rig.T
    D = np.zeros((1, 5))
    cv2.calibrateCamera = lambda obj, pts, shape, a, b: (0.0, K1 if pts == "cam" else K2, D, None, None)
    cv2.stereoCalibrate = lambda *a, **k: (0.1, K1, D, K2, D, R, T, None, None)
    cv2.CALIB_FIX_INTRINSIC = 256
    sysobj = sl_system.SLSystem()
    sysobj.load_calib_data = lambda base, poses: ([], "cam", "proj", (rig.cam_w, rig.cam_h), None)
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "calib.mat")
        sysobj.calibrate_final(td, [], out)
        import scipy.io
        data = scipy.io.loadmat(out)
    return {k: data[k] for k in calibration.CALIB_KEYS}


def save(name: str, **arrays):
    np.savez_compressed(HERE / f"{name}.npz", **arrays)
    print(f"  wrote {name}.npz")


def run_processing_case(name, rig, calib, view, params, row_modes=(0, 1, 2), calib_tag="rig"):
    files = refharness.register_frames(f"/mem/{name}", list(view.frames), view.texture)
    kw = dict(params)
    col, row, mask, tex = PL._gray_decode(files, **kw)
    out = dict(frames=view.frames, texture=view.texture, col=col, row=row, mask=mask,
               params=np.array(json.dumps(dict(variant="processing", calib=calib_tag, **kw))))
    for rm in row_modes:
        P, C = PL._reconstruct_point_cloud(col, row, mask, tex, calib, row_mode=rm,
                                           epipolar_tol=2.0)
        out[f"P{rm}"] = np.ascontiguousarray(P)
        out[f"C{rm}"] = np.ascontiguousarray(C)
    save(name, **out)
    return out


def run_sl_case(name, calib, view, calib_tag="rig", expect_error=None):
    folder = f"/mem/{name}"
    files = refharness.register_frames(folder, list(view.frames), view.texture)
    g = dict(sl_system.__dict__)
    fake_glob = types.ModuleType("glob")
    fake_glob.glob = lambda pat: list(files) if pat.endswith("*.png") else []
    g["glob"] = fake_glob
    gd = types.FunctionType(gray_decode_sl.__code__, g, "gray_decode", (1920, 1080))
    out = dict(frames=view.frames, texture=view.texture,
               params=np.array(json.dumps(dict(variant="slsystem", calib=calib_tag))))
    try:
        col, row, mask, tex = gd(folder)
    except Exception as e:  # noqa: BLE001 - record the reference's exception type
        out["error"] = np.array(type(e).__name__)
        save(name, **out)
        return out
    P, C = recon_sl(col, row, mask, tex, calib)
    out.update(col=col, row=row, mask=mask, P0=np.ascontiguousarray(P), C0=np.ascontiguousarray(C))
    save(name, **out)
    return out


OC = np.array([[12.5], [-3.25], [7.0]])       # a nonzero camera origin (VERDICT r2 missing #5)


def calib_with_origin(calib: dict) -> dict:
    """The rig's calibration expressed in a world frame whose camera centre is ``OC``: the same
    stripe planes moved with the camera (d' = d - n.OC), so a consistent capture keeps its
    points in every row_mode.  The reference's ``numer = np.dot(N.T, Oc) + d`` and
    ``P = Oc + r*t`` (server/processing.py:166,180,197,205,214,219,228) then see Oc != 0."""
    out = {k: np.array(v, copy=True) for k, v in calib.items()}
    out["Oc"] = OC.copy()
    for k in ("wPlaneCol", "wPlaneRow"):
        t = out[k]
        t[3, :] = t[3, :] - (t[0, :] * OC[0, 0] + t[1, :] * OC[1, 0] + t[2, :] * OC[2, 0])
    return out


def oc_cases(rig, calib):
    """Oc != 0 through the reference's _reconstruct_point_cloud: Nc-table rays and cam_K rays
    (row_mode 0/1/2), and an Oc that is NOT consistent with the planes (raw)."""
    calib_oc = calib_with_origin(calib)
    save("calib_rig_oc", **{k: np.asarray(v) for k, v in calib_oc.items()})
    # this host's BLAS rounding of np.dot(N, Oc) per plane (position-independent in OpenBLAS's
    # gemv): a GPU box whose BLAS rounds differently reproduces the reference run THERE, not here
    save("calib_blas_oc", **{f"numer_{k}": np.dot(np.ascontiguousarray(calib_oc[k].T)[:, 0:3], OC).flatten()
                             for k in ("wPlaneCol", "wPlaneRow")},
         numer_raw=np.dot(np.ascontiguousarray(calib["wPlaneCol"].T)[:, 0:3], OC).flatten())
    v = synth.render_view(rig, 70.0, seed=41)
    run_processing_case("proc_oc_table", rig, calib_oc, v,
                        dict(n_sets_col=11, n_sets_row=10, thresh_mode="otsu"), calib_tag="rig_oc")
    calib_ock = dict(calib_oc)
    calib_ock["Nc"] = calib_oc["Nc"][:, :5]
    run_processing_case("proc_oc_krays", rig, calib_ock, synth.render_view(rig, 110.0, seed=42),
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="otsu"), calib_tag="rig_oc_krays")
    calib_raw = dict(calib)
    calib_raw["Oc"] = OC.copy()
    run_processing_case("proc_oc_raw", rig, calib_raw, synth.render_view(rig, 150.0, seed=43),
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="otsu"), calib_tag="rig_oc_raw")


def main(only=None):
    rig = synth.default_rig(96, 64, 1920, 1080)
    calib = ref_calibration(rig)
    if only == "oc":
        mine = dict(np.load(HERE / "calib_rig.npz"))
        assert all(np.array_equal(calib[k], mine[k]) for k in calibration.CALIB_KEYS)
        oc_cases(rig, calib)
        return
    mine = rig.tables()
    assert np.array_equal(calib["Nc"], mine["Nc"]), "Nc differs from calibration.pinhole_rays"
    for k in ("wPlaneCol", "wPlaneRow"):
        np.testing.assert_allclose(calib[k], mine[k], rtol=0, atol=1e-9)
    save("calib_rig", **{k: np.asarray(v) for k, v in calib.items()})

    # odd-sized rig for tail handling (W not a multiple of 16, HW not a multiple of 16)
    rig_odd = synth.default_rig(101, 37, 1920, 1080)
    calib_odd = ref_calibration(rig_odd)
    save("calib_odd", **{k: np.asarray(v) for k, v in calib_odd.items()})

    full = synth.render_view(rig, 0.0, seed=11)
    run_processing_case("proc_otsu_full", rig, calib, full,
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="otsu"))
    c2 = synth.render_view(rig, 40.0, seed=12, n_present=44)
    run_processing_case("proc_c2style", rig, calib, c2,
                        dict(n_sets_col=11, n_sets_row=10, thresh_mode="otsu"))
    v3 = synth.render_view(rig, 80.0, seed=13)
    run_processing_case("proc_manual_sets", rig, calib, v3,
                        dict(n_sets_col=7, n_sets_row=5, thresh_mode="manual",
                             shadow_val=40, contrast_val=10))
    v4 = synth.render_view(rig, 120.0, seed=14, n_present=31)
    run_processing_case("proc_missing_odd", rig, calib, v4,
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="otsu"))
    v5 = synth.render_view(rig, 160.0, seed=15, n_present=17)
    run_processing_case("proc_missing_colpart", rig, calib, v5,
                        dict(n_sets_col=9, n_sets_row=11, thresh_mode="manual",
                             shadow_val=25, contrast_val=6))
    # C1-style: 1024-wide projector code (Bc = 10), row frames absent, K-recompute rays
    rig1 = synth.default_rig(96, 64, 1024, 1080)
    v6 = synth.render_view(rig1, 200.0, seed=16, n_present=22)
    calib_k = dict(calib)
    calib_k["Nc"] = calib["Nc"][:, :5]           # wrong size -> rays from cam_K (proc.py:145)
    run_processing_case("proc_c1style_krays", rig1, calib_k, v6,
                        dict(n_cols=1024, n_rows=1080, n_sets_col=10, n_sets_row=11,
                             thresh_mode="otsu"), row_modes=(0,), calib_tag="rig_krays")
    # odd geometry, all modes
    vo = synth.render_view(rig_odd, 250.0, seed=17)
    run_processing_case("proc_odd_geometry", rig_odd, calib_odd, vo,
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="otsu"),
                        calib_tag="odd")
    # degenerate: constant frames -> Otsu returns 0, ties everywhere, empty cloud
    flat = synth.View(frames=np.full((46, 64, 96), 37, np.uint8),
                      texture=np.full((64, 96, 3), 5, np.uint8),
                      proj_col=None, proj_row=None, lit=None)
    run_processing_case("proc_flat_ties", rig, calib, flat,
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="otsu"))
    # manual thresholds given as floats (NEP 50 float32 comparison)
    v7 = synth.render_view(rig, 300.0, seed=18)
    run_processing_case("proc_manual_float", rig, calib, v7,
                        dict(n_sets_col=11, n_sets_row=11, thresh_mode="manual",
                             shadow_val=30.5, contrast_val=7.25))

    # legacy SLSystem.generate_cloud variant (percentile mask, col-only)
    run_sl_case("sl_full", calib, synth.render_view(rig, 20.0, seed=21))
    run_sl_case("sl_missing_even", calib, synth.render_view(rig, 60.0, seed=22, n_present=30))
    run_sl_case("sl_missing_odd", calib, synth.render_view(rig, 60.0, seed=23, n_present=29))
    run_sl_case("sl_odd_geometry", calib_odd, synth.render_view(rig_odd, 10.0, seed=24),
                calib_tag="odd")
    oc_cases(rig, calib)


if __name__ == "__main__":
    # `--only oc`: (re)generate just the Oc != 0 fixtures (round 3), leaving the others untouched
    main(sys.argv[2] if len(sys.argv) > 2 and sys.argv[1] == "--only" else None)
