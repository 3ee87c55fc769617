"""Calibration tables for the reconstruction path (camera rays ``Nc``, origin ``Oc``,
projector stripe planes ``wPlaneCol`` / ``wPlaneRow``).

The tables are *inputs* of the hot path.  The reference produces them once per rig in
``SLSystem.calibrate_final`` (``server/sl_system.py:336-423``) after OpenCV's mono/stereo
calibration and stores them in a MATLAB v5 file that ``process_multi_ply`` loads with
``scipy.io.loadmat`` (``server/processing.py:279-284``).  This module restates the table
geometry for given intrinsics/extrinsics (the OpenCV solvers stay out of scope)
and provides the ``.mat`` round trip in the reference's key/shape convention:

* ``Nc``        (3, H*W) f64, unit camera rays, pixel index ``v*W + u``  (sl_system.py:358-372)
* ``Oc``        (3, 1)   f64, camera centre = 0                        (sl_system.py:355)
* ``wPlaneCol`` (4, PW)  f64, ``[n; d]`` per projector column          (sl_system.py:405-406,417)
* ``wPlaneRow`` (4, PH)  f64, ``[n; d]`` per projector row             (sl_system.py:408-410,418)
* ``cam_K``, ``proj_K``, ``R``, ``T``, ``dc``                           (sl_system.py:413-423)
"""
from __future__ import annotations

import numpy as np

CALIB_KEYS = ("Nc", "Oc", "wPlaneCol", "wPlaneRow", "cam_K")


def pinhole_rays(K: np.ndarray, height: int, width: int) -> np.ndarray:
    """Unit camera rays for every pixel, shape (3, H*W), row-major pixel order.

    Same arithmetic as ``server/sl_system.py:360-372``: ``x=(u-cx)/fx``, ``y=(v-cy)/fy``,
    ``n = sqrt((x*x + y*y) + 1)`` (NumPy reduces the 3-vector left to right) and
    ``(x/n, y/n, 1/n)``.  The GPU kernels recompute exactly these values when the
    calibration's ``Nc`` is bit-identical to this table (see ``engine.CalibTables``).
    """
    fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    u = np.arange(width, dtype=np.float64)
    v = np.arange(height, dtype=np.float64)
    x = (u - cx) / fx                      # (W,)
    y = (v - cy) / fy                      # (H,)
    xx = np.broadcast_to(x[None, :], (height, width))
    yy = np.broadcast_to(y[:, None], (height, width))
    n = np.sqrt((xx * xx + yy * yy) + 1.0)
    out = np.empty((3, height * width), dtype=np.float64)
    out[0] = (xx / n).ravel()
    out[1] = (yy / n).ravel()
    out[2] = (1.0 / n).ravel()
    return out


def stripe_planes(K2: np.ndarray, R: np.ndarray, T: np.ndarray,
                  proj_w: int, proj_h: int) -> tuple[np.ndarray, np.ndarray]:
    """Projector column/row light planes in camera coordinates, each row ``[nx, ny, nz, d]``.

    Geometry of ``server/sl_system.py:379-410``: the plane of projector column ``c`` holds the
    projector centre ``C = -R^T T`` and the back-projected pixels ``(c, 0)`` and ``(c, PH)``;
    a row plane holds ``(0, r)`` and ``(PW, r)``.  ``n = normalize(r1 x r2)``, ``d = -n.C``.
    Returns ``(col_planes (PW,4), row_planes (PH,4))``.
    """
    fxp, fyp, cxp, cyp = float(K2[0, 0]), float(K2[1, 1]), float(K2[0, 2]), float(K2[1, 2])
    Rinv = np.asarray(R, dtype=np.float64).T
    C = -(Rinv @ np.asarray(T, dtype=np.float64).reshape(3, 1)).ravel()

    def planes(a_x, a_y, b_x, b_y):
        p1 = np.stack([a_x, a_y, np.ones_like(a_x)])            # (3, n)
        p2 = np.stack([b_x, b_y, np.ones_like(b_x)])
        r1 = Rinv @ p1
        r2 = Rinv @ p2
        nrm = np.cross(r1.T, r2.T)                                # (n, 3)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        d = -(nrm @ C)
        return np.concatenate([nrm, d[:, None]], axis=1)

    c = np.arange(proj_w, dtype=np.float64)
    cx_n = (c - cxp) / fxp
    col = planes(cx_n, np.full_like(cx_n, (0.0 - cyp) / fyp),
                 cx_n, np.full_like(cx_n, (proj_h - cyp) / fyp))
    r = np.arange(proj_h, dtype=np.float64)
    ry_n = (r - cyp) / fyp
    row = planes(np.full_like(ry_n, (0.0 - cxp) / fxp), ry_n,
                 np.full_like(ry_n, (proj_w - cxp) / fxp), ry_n)
    return col, row


def build_tables(K1, K2, R, T, cam_size, proj_size, dist=None) -> dict:
    """All tables ``calibrate_final`` saves (``server/sl_system.py:413-423``), reference shapes.

    ``cam_size`` = (W, H) of the camera, ``proj_size`` = (PW, PH) of the projector.
    """
    w, h = int(cam_size[0]), int(cam_size[1])
    pw, ph = int(proj_size[0]), int(proj_size[1])
    K1 = np.asarray(K1, dtype=np.float64)
    K2 = np.asarray(K2, dtype=np.float64)
    col, row = stripe_planes(K2, R, T, pw, ph)
    return {
        "Nc": pinhole_rays(K1, h, w),
        "Oc": np.zeros((3, 1)),
        "dc": np.zeros((1, 5)) if dist is None else np.asarray(dist, dtype=np.float64),
        "wPlaneCol": np.ascontiguousarray(col.T),
        "wPlaneRow": np.ascontiguousarray(row.T),
        "cam_K": K1,
        "proj_K": K2,
        "R": np.asarray(R, dtype=np.float64),
        "T": np.asarray(T, dtype=np.float64).reshape(3, 1),
    }


def save_mat(path: str, tables: dict) -> None:
    """Write a reference-format calibration file (``scipy.io.savemat``, MATLAB v5)."""
    import scipy.io
    scipy.io.savemat(path, tables)


def load_mat(path: str) -> dict:
    """Load the five keys the hot path reads (``server/processing.py:279-284``)."""
    import scipy.io
    data = scipy.io.loadmat(path)
    return {k: data[k] for k in CALIB_KEYS}
