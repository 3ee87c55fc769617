"""CPU BASELINE PORT — TEST INFRASTRUCTURE ONLY.

The reference hot path's NumPy *operation sequence*, restated for timing.  Used by
``bench.py``'s ``cpu_baseline`` leg and by ``tools/ref_vs_port.py`` (which times it against the
reference itself); never by the product package, which runs the HIP kernels.  The checker for
parity stays ``oracle/sl_oracle.py``.

Why a second restatement: the oracle computes the same values with cheaper NumPy (``astype``
compares, a 5-pass prefix XOR, ``flatnonzero``, one fused ray formula) and runs ~1.7x faster than
the reference's own code on a C2 view (missing #1), so its rate overstated the CPU
path.  This module performs the reference's operations in the reference's order instead:

* ``ProcessingLogic._gray_decode`` (``server/processing.py:49-124``): every frame "read" as a
  fresh array (``cv2.imread`` returns a new one; frames in memory here, no PNG decode) and cast
  to float32 (``:59-60,98-99``); Otsu on ``white.astype(uint8)`` and on the clipped difference
  (``:66-72``); per bit plane a zeroed int32 plane and a boolean scatter ``bit[p > i] = 1``, then
  ``bitwise_or(left_shift(...))`` (``:100-104``); Gray -> binary by the ``while np.any`` loop of up
  to n XOR passes (``:107-110``); rescale by an int multiply (``:119-122``); the texture "read"
  again (``:124``).
* ``ProcessingLogic._reconstruct_point_cloud`` (``server/processing.py:130-234``): ``flatten`` +
  ``np.where``, the ``Nc[:, idx]`` gather (or ``unravel_index`` + ``np.linalg.norm`` rays), plane
  fancy-index with ``clip``, ``np.sum(N * rays, axis=0)``, ``np.dot(N.T, Oc)``, masked division,
  then the row_mode branch with its full-width temporaries.

Outputs are bit-identical to the reference's (``tests/test_oracle_golden.py`` checks this port
against every golden fixture as well), so it is a port of the reference, timed as such
(``cpu_baseline.kind`` "port").  ``otsu_threshold`` is the oracle's restatement of OpenCV's C
routine, the same stand-in the golden harness gives the reference (``tests/golden/refharness.py``).
"""
from __future__ import annotations

import numpy as np

from .sl_oracle import otsu_threshold


def _read(frame) -> np.ndarray:
    """In-memory stand-in for ``cv2.imread``: a new array per call, as a decode returns."""
    return np.array(frame, copy=True)


def gray_decode(frames, texture, n_cols=1920, n_rows=1080, n_sets_col=11, n_sets_row=11,
                thresh_mode="otsu", shadow_val=40, contrast_val=10):
    """``_gray_decode`` on in-memory frames (capture order) + the BGR texture of frame 0.
    Returns ``(col int32 [H,W], row int32 [H,W], mask bool [H,W], texture uint8 [H,W,3])``."""
    n_files = len(frames)
    if n_files < 4:
        raise ValueError(f"Not enough images (got {n_files}, need at least 4).")
    white = _read(frames[0]).astype(np.float32)
    black = _read(frames[1]).astype(np.float32)
    height, width = white.shape
    if thresh_mode == "otsu":
        t_shadow = otsu_threshold(white.astype(np.uint8))
        shadow_ok = white > t_shadow
        t_contrast = otsu_threshold(np.clip(white - black, 0, 255).astype(np.uint8))
        contrast_ok = (white - black) > t_contrast
    else:
        shadow_ok = white > shadow_val
        contrast_ok = (white - black) > contrast_val
    valid = shadow_ok & contrast_ok

    bits_col = int(np.ceil(np.log2(n_cols)))
    bits_row = int(np.ceil(np.log2(n_rows)))
    use_col = max(1, min(int(n_sets_col), bits_col))
    use_row = max(1, min(int(n_sets_row), bits_row))
    cursor = 2

    def axis_code(n_bits, n_use):
        nonlocal cursor
        code = np.zeros((height, width), dtype=np.int32)
        for b in range(n_bits):
            present = cursor + 1 < n_files
            if present and b < n_use:
                pat = _read(frames[cursor]).astype(np.float32)
                inv = _read(frames[cursor + 1]).astype(np.float32)
                plane = np.zeros((height, width), dtype=np.int32)
                plane[pat > inv] = 1
                code = np.bitwise_or(code, np.left_shift(plane, n_use - 1 - b))
            cursor += 2
        carry = np.right_shift(code, 1)
        while np.any(carry > 0):
            code = np.bitwise_xor(code, carry)
            carry = np.right_shift(carry, 1)
        return code

    col = axis_code(bits_col, use_col) * (1 << (bits_col - use_col))
    row = axis_code(bits_row, use_row) * (1 << (bits_row - use_row))
    return col, row, valid, _read(texture)


def _as_rows(table):
    return table.T if table.shape[0] == 4 else table


def reconstruct(col_map, row_map, mask, texture, calib, row_mode=1, epipolar_tol=2.0):
    """``_reconstruct_point_cloud``: ``(P float64 [N,3], C uint8 [N,3])`` (None for an unknown
    row_mode, as the reference's if-chain falls through)."""
    Nc, Oc = calib["Nc"], calib["Oc"]
    col_tab = _as_rows(calib["wPlaneCol"])
    h, w = col_map.shape
    flat_col = col_map.flatten()
    flat_mask = mask.flatten()
    tex = texture.reshape(-1, 3)
    idx = np.where(flat_mask)[0]
    if Nc.shape[1] == h * w:
        rays = Nc[:, idx]
    else:
        K = calib["cam_K"]
        yy, xx = np.unravel_index(idx, (h, w))
        xn = (xx - K[0, 2]) / K[0, 0]
        yn = (yy - K[1, 2]) / K[1, 1]
        rays = np.stack((xn, yn, np.ones_like(xn)))
        rays /= np.linalg.norm(rays, axis=0)

    def planes_at(table, flat):
        sel = np.clip(flat[idx], 0, table.shape[0] - 1)
        pl = table[sel, :]
        return pl[:, 0:3].T, pl[:, 3]

    def hit(normals, d):
        den = np.sum(normals * rays, axis=0)
        num = np.dot(normals.T, Oc).flatten() + d
        ok = np.abs(den) > 1e-6
        t = np.zeros_like(den)
        t[ok] = -num[ok] / den[ok]
        return ok, t

    def cloud(keep, t):
        P = Oc + rays[:, keep] * t[keep]
        return P, tex[idx[keep]]

    n_col, d_col = planes_at(col_tab, flat_col)
    ok_col, t_col = hit(n_col, d_col)
    if row_mode == 0:
        P, C = cloud(ok_col, t_col)
        return P.T, C
    row_tab = _as_rows(calib["wPlaneRow"])
    n_row, d_row = planes_at(row_tab, row_map.flatten())
    if row_mode == 1:
        P_all = Oc + rays * t_col
        dist = np.abs(np.sum(n_row * P_all, axis=0) + d_row)
        P, C = cloud(ok_col & (dist < epipolar_tol), t_col)
        return P.T, C
    if row_mode == 2:
        P1, C1 = cloud(ok_col, t_col)
        ok_row, t_row = hit(n_row, d_row)
        P2, C2 = cloud(ok_row, t_row)
        return np.hstack((P1, P2)).T, np.vstack((C1, C2))
    return None
