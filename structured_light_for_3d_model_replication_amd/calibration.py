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
    projector centre ``C = (-R^T) T`` and the back-projected pixels ``(c, 0)`` and ``(c, PH)``;
    a row plane holds ``(0, r)`` and ``(PW, r)``.  ``n = normalize(r1 x r2)``, ``d = -n.C``.
    Returns ``(col_planes (PW,4), row_planes (PH,4))``.

    Bit-identical with the reference: every plane goes through the same NumPy operations on the
    same shapes as ``get_plane_from_proj_line`` -- a (3,3) @ (3,1) matmul per ray, ``np.cross``
    of 1-D vectors, ``np.linalg.norm`` and ``np.dot`` of 1-D vectors (BLAS ddot) -- because a
    batched form rounds differently in the last bit (matmul / norm / dot take other kernels).
    The ~3000 planes of a rig take ~0.1 s, once per calibration.
    """
    K2 = np.asarray(K2, dtype=np.float64)
    fxp, fyp, cxp, cyp = K2[0, 0], K2[1, 1], K2[0, 2], K2[1, 2]     # NumPy scalars, as the reference
    Rinv = np.asarray(R, dtype=np.float64).T
    C = (-Rinv @ np.asarray(T, dtype=np.float64).reshape(3, 1)).flatten()   # (-R^T) @ T

    def plane(ax, ay, bx, by):
        r1 = Rinv @ np.array([ax, ay, 1]).reshape(3, 1)
        r2 = Rinv @ np.array([bx, by, 1]).reshape(3, 1)
        n = np.cross(r1.flatten(), r2.flatten())
        n /= np.linalg.norm(n)
        return n[0], n[1], n[2], -np.dot(n, C)

    col = np.zeros((int(proj_w), 4))
    row = np.zeros((int(proj_h), 4))
    for c in range(int(proj_w)):            # the column's line from (c, 0) to (c, PH)
        x = (c - cxp) / fxp
        col[c, :] = plane(x, (0 - cyp) / fyp, x, (proj_h - cyp) / fyp)
    for r in range(int(proj_h)):            # the row's line from (0, r) to (PW, r)
        y = (r - cyp) / fyp
        row[r, :] = plane((0 - cxp) / fxp, y, (proj_w - cxp) / fxp, y)
    return col, row


def stripe_planes_fast(K2: np.ndarray, R: np.ndarray, T: np.ndarray,
                       proj_w: int, proj_h: int) -> tuple[np.ndarray, np.ndarray]:
    """:func:`stripe_planes` as whole-array NumPy (opt-in, ~150x faster: 1.3 ms vs 0.19 s for a
    1920x1080 projector).  NOT bit-identical to the reference: batched matmul / einsum round
    differently from the per-plane BLAS gemv / ddot / nrm2 calls of ``get_plane_from_proj_line``
    (``server/sl_system.py:386-410``) -- measured on the default rig: 566 of 1920 column planes
    and 474 of 1080 row planes differ, by at most 4 ulps (6.4e-16 relative).  Which rounding the
    reference itself gets depends on the host's BLAS kernel, so no fixed batched formula can
    match it everywhere: :func:`stripe_planes` (the per-plane loop, once per rig) stays the
    bit-exact path and the default of :func:`build_tables`."""
    K2 = np.asarray(K2, dtype=np.float64)
    fxp, fyp, cxp, cyp = K2[0, 0], K2[1, 1], K2[0, 2], K2[1, 2]
    Rinv = np.asarray(R, dtype=np.float64).T
    C = (-Rinv @ np.asarray(T, dtype=np.float64).reshape(3, 1)).flatten()

    def planes(p1, p2):
        n = np.cross(p1 @ Rinv.T, p2 @ Rinv.T)
        n /= np.sqrt(np.einsum("ij,ij->i", n, n))[:, None]
        return np.column_stack([n, -(n @ C)])

    pw, ph = int(proj_w), int(proj_h)
    x = (np.arange(pw) - cxp) / fxp
    y = (np.arange(ph) - cyp) / fyp
    one_w, one_h = np.ones(pw), np.ones(ph)
    col = planes(np.column_stack([x, np.full(pw, (0 - cyp) / fyp), one_w]),
                 np.column_stack([x, np.full(pw, (ph - cyp) / fyp), one_w]))
    row = planes(np.column_stack([np.full(ph, (0 - cxp) / fxp), y, one_h]),
                 np.column_stack([np.full(ph, (pw - cxp) / fxp), y, one_h]))
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
