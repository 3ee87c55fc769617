"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A NumPy restatement of the reference's structured-light hot path, used solely as the checker
by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.  Product
code (``structured_light_for_3d_model_replication_amd``) never imports this module; the
product path runs the HIP kernels and fails loudly when they are missing.

Pinning:
* decode / mask / triangulation are checked bit-for-bit against the reference's own
  functions (``ProcessingLogic._gray_decode``, ``ProcessingLogic._reconstruct_point_cloud``,
  and the nested ``gray_decode`` / ``reconstruct_point_cloud`` of ``SLSystem.generate_cloud``)
  run in the survey container on rendered captures -> ``tests/golden/*.npz`` made by
  ``tests/golden/make_golden.py``;
* ``otsu_threshold`` restates OpenCV's C ``getThreshVal_Otsu_8u`` (opencv-python, unpinned in
  ``requirements.txt:2``, absent from the image).  The reference holds no vectors for it, so
  it is pinned by exact-rational known-answer tests (``tests/test_oracle_kat.py``), including
  the cases an implementation with another evaluation order could resolve differently: exact
  sigma ties between two splits (sequential fp64 picks the LATER one there) and single
  non-empty bins at 0 / 255.  opencv-python wheels on x86-64 may dispatch Otsu to IPP's
  ``ippiComputeThreshold_Otsu``; agreement with that path is PARITY UNPINNED;
* the numerator ``np.dot(N.T, Oc) + d`` (``server/processing.py:166,219``) is computed with the
  same ``np.dot`` call, so it carries the host BLAS's gemv rounding exactly as the reference
  does on that host (for Oc != 0 that rounding differs between BLAS kernels; the Oc != 0
  fixtures record this host's, ``tests/golden/calib_blas_oc.npz``);
* the percentile threshold of the legacy variant calls NumPy itself (same library the
  reference calls, ``server/sl_system.py:535``).
"""
from __future__ import annotations

import math

import numpy as np

FLT_EPSILON = float(np.finfo(np.float32).eps)


# ---------------------------------------------------------------------------------------
# Thresholds
# ---------------------------------------------------------------------------------------
def otsu_from_hist(h) -> float:
    """OpenCV ``getThreshVal_Otsu_8u`` on a 256-bin histogram (sequential fp64, strict '>').

    Follows the published OpenCV algorithm that ``cv2.threshold(..., THRESH_OTSU)`` runs for
    ``server/processing.py:67,71``: mu = sum(i*h[i]) * scale; per bin
    ``mu1 *= q1; q1 += p_i; q2 = 1-q1``; skip when ``min(q1,q2) < FLT_EPSILON`` or
    ``max(q1,q2) > 1-FLT_EPSILON``; ``mu1 = (mu1 + i*p_i)/q1``; ``mu2 = (mu - q1*mu1)/q2``;
    ``sigma = q1*q2*(mu1-mu2)*(mu1-mu2)``; keep the first bin with ``sigma > max_sigma``.
    """
    h = [int(x) for x in h]
    total = sum(h)
    scale = 1.0 / float(total)
    mu = 0.0
    for i in range(256):
        mu += i * float(h[i])
    mu *= scale
    mu1 = 0.0
    q1 = 0.0
    max_sigma = 0.0
    max_val = 0.0
    for i in range(256):
        p_i = h[i] * scale
        mu1 *= q1
        q1 += p_i
        q2 = 1.0 - q1
        if min(q1, q2) < FLT_EPSILON or max(q1, q2) > 1.0 - FLT_EPSILON:
            continue
        mu1 = (mu1 + i * p_i) / q1
        mu2 = (mu - q1 * mu1) / q2
        sigma = q1 * q2 * (mu1 - mu2) * (mu1 - mu2)
        if sigma > max_sigma:
            max_sigma = sigma
            max_val = float(i)
    return max_val


def otsu_threshold(img_u8: np.ndarray) -> float:
    """Otsu threshold of a uint8 image (value returned by ``cv2.threshold``)."""
    h = np.bincount(np.asarray(img_u8, dtype=np.uint8).ravel(), minlength=256)
    return otsu_from_hist(h)


def mask_processing(white: np.ndarray, black: np.ndarray, thresh_mode="otsu",
                    shadow_val=40, contrast_val=10) -> np.ndarray:
    """Valid mask of ``server/processing.py:59-78`` (frames as uint8 arrays)."""
    w = white.astype(np.float32)
    b = black.astype(np.float32)
    if thresh_mode == "otsu":
        ts = otsu_threshold(w.astype(np.uint8))
        tc = otsu_threshold(np.clip(w - b, 0, 255).astype(np.uint8))
        return (w > ts) & ((w - b) > tc)
    return (w > shadow_val) & ((w - b) > contrast_val)


def mask_percentile(white: np.ndarray, black: np.ndarray) -> np.ndarray:
    """Valid mask of the legacy variant ``server/sl_system.py:527-543``."""
    w = white.astype(np.float32)
    b = black.astype(np.float32)
    contrast = w - b
    noise_floor = np.percentile(b, 95)
    dynamic_range = np.max(contrast)
    return (w > (noise_floor * 1.5)) & (contrast > (dynamic_range * 0.05))


# ---------------------------------------------------------------------------------------
# Gray-code decode
# ---------------------------------------------------------------------------------------
def _gray_to_binary(g: np.ndarray) -> np.ndarray:
    # prefix XOR == the reference's "mask = g>>1; while any(mask): g ^= mask; mask >>= 1"
    shift = 1
    while shift < 32:
        g = g ^ (g >> shift)
        shift <<= 1
    return g


def decode_processing(frames, n_cols=1920, n_rows=1080, n_sets_col=11, n_sets_row=11,
                      thresh_mode="otsu", shadow_val=40, contrast_val=10):
    """``ProcessingLogic._gray_decode`` on an in-memory frame list (``server/processing.py:28-124``).

    ``frames`` is a sequence of uint8 [H, W] images in capture order (len >= 4).
    Returns (col int32, row int32, mask bool).
    """
    n_files = len(frames)
    if n_files < 4:
        raise ValueError(f"Not enough images (got {n_files}, need at least 4).")
    white, black = np.asarray(frames[0]), np.asarray(frames[1])
    mask = mask_processing(white, black, thresh_mode, shadow_val, contrast_val)
    Bc = int(np.ceil(np.log2(n_cols)))
    Br = int(np.ceil(np.log2(n_rows)))
    nc = max(1, min(int(n_sets_col), Bc))
    nr = max(1, min(int(n_sets_row), Br))
    idx = 2

    def axis(max_bits, n_use):
        nonlocal idx
        g = np.zeros(white.shape, dtype=np.int32)
        for b in range(max_bits):
            if idx + 1 >= n_files:          # missing pair: skipped, pointer still advances
                idx += 2
                continue
            if b < n_use:
                bit = (np.asarray(frames[idx]).astype(np.float32) >
                       np.asarray(frames[idx + 1]).astype(np.float32)).astype(np.int32)
                g |= bit << (n_use - 1 - b)
            idx += 2
        return _gray_to_binary(g)

    col = axis(Bc, nc) * np.int32(1 << (Bc - nc))
    row = axis(Br, nr) * np.int32(1 << (Br - nr))
    return col.astype(np.int32), row.astype(np.int32), mask


def decode_slsystem(frames, n_cols=1920, n_rows=1080):
    """Nested ``gray_decode`` of ``SLSystem.generate_cloud`` (``server/sl_system.py:516-588``):
    percentile mask, all bits, no rescale, ``break`` on the first missing frame (an odd
    trailing frame raises ``IndexError`` like the reference's ``files[current_idx]``)."""
    n_files = len(frames)
    if n_files < 4:
        raise ValueError("Not enough images in folder to decode.")
    white, black = np.asarray(frames[0]), np.asarray(frames[1])
    mask = mask_percentile(white, black)
    idx = 2

    def axis(n):
        nonlocal idx
        g = np.zeros(white.shape, dtype=np.int32)
        for b in range(n):
            if idx >= n_files:
                break
            if idx + 1 >= n_files:
                raise IndexError("list index out of range")
            bit = (np.asarray(frames[idx]).astype(np.float32) >
                   np.asarray(frames[idx + 1]).astype(np.float32)).astype(np.int32)
            idx += 2
            g |= bit << (n - 1 - b)
        return _gray_to_binary(g)

    col = axis(int(np.ceil(np.log2(n_cols))))
    row = axis(int(np.ceil(np.log2(n_rows))))
    return col, row, mask


# ---------------------------------------------------------------------------------------
# Triangulation
# ---------------------------------------------------------------------------------------
def _rays(calib, valid, h, w):
    Nc = np.asarray(calib["Nc"])
    if Nc.shape[1] == h * w:                               # processing.py:143-144
        return Nc[:, valid].astype(np.float64)
    K = np.asarray(calib["cam_K"])                          # processing.py:145-156
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    yv, xv = valid // w, valid % w
    x = (xv - cx) / fx
    y = (yv - cy) / fy
    n = np.sqrt((x * x + y * y) + 1.0)
    return np.stack([x / n, y / n, 1.0 / n])


def _planes(tab):
    tab = np.asarray(tab)
    return tab.T if tab.shape[0] == 4 else tab             # processing.py:134,186


def _intersect(planes, idx_map, valid, rays, Oc):
    p = planes[np.clip(idx_map.ravel()[valid], 0, planes.shape[0] - 1)]
    n0, n1, n2, d = p[:, 0], p[:, 1], p[:, 2], p[:, 3]
    denom = (n0 * rays[0] + n1 * rays[1]) + n2 * rays[2]
    # processing.py:166,219: np.dot(N.T, Oc) -- the host BLAS's gemv rounding (e.g. OpenBLAS
    # 0.3.29 here evaluates fma(n2,o2, fma(n0,o0, n1*o1))), reproduced by making the same call;
    # == d for Oc = 0 (the calib value)
    numer = np.dot(p[:, 0:3], Oc.reshape(3, 1)).flatten() + d
    ok = np.abs(denom) > 1e-6
    t = np.zeros_like(denom)
    t[ok] = -numer[ok] / denom[ok]
    return ok, t, p


def reconstruct_processing(col, row, mask, texture, calib, row_mode=1, epipolar_tol=2.0):
    """``ProcessingLogic._reconstruct_point_cloud`` (``server/processing.py:127-234``).

    Returns ``(P float64 [N,3], C uint8 [N,3] BGR)`` in ascending pixel order (mode 2: the
    column cloud, then the row cloud)."""
    h, w = col.shape
    valid = np.flatnonzero(np.asarray(mask).ravel())
    tex = np.asarray(texture).reshape(-1, 3)
    Oc = np.asarray(calib["Oc"], dtype=np.float64).reshape(3)
    rays = _rays(calib, valid, h, w)
    okc, tcol, _ = _intersect(_planes(calib["wPlaneCol"]), col, valid, rays, Oc)

    def points(keep, t):
        P = Oc[:, None] + rays[:, keep] * t[keep]
        return P.T, tex[valid[keep]]

    if row_mode == 0:
        return points(okc, tcol)
    prow_tab = _planes(calib["wPlaneRow"])
    if row_mode == 1:
        p = prow_tab[np.clip(np.asarray(row).ravel()[valid], 0, prow_tab.shape[0] - 1)]
        Pt = Oc[:, None] + rays * tcol
        dist = np.abs(((p[:, 0] * Pt[0] + p[:, 1] * Pt[1]) + p[:, 2] * Pt[2]) + p[:, 3])
        return points(okc & (dist < epipolar_tol), tcol)
    if row_mode == 2:
        P1, C1 = points(okc, tcol)
        okr, trow, _ = _intersect(prow_tab, row, valid, rays, Oc)
        P2, C2 = points(okr, trow)
        return np.vstack([P1, P2]), np.vstack([C1, C2])
    return None   # the reference falls through and returns None for other modes


def reconstruct_slsystem(col, row, mask, texture, calib):
    """Nested ``reconstruct_point_cloud`` of ``generate_cloud`` (``server/sl_system.py:592-661``):
    column planes only; identical values to ``row_mode=0``."""
    return reconstruct_processing(col, row, mask, texture, calib, row_mode=0)


def ply_bytes(points, colors) -> bytes:
    """ASCII PLY exactly as ``ProcessingLogic._save_ply`` writes it (``processing.py:236-248``)."""
    out = ["ply\nformat ascii 1.0\n", f"element vertex {len(points)}\n",
           "property float x\nproperty float y\nproperty float z\n",
           "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n"]
    for p, c in zip(points, colors):
        out.append(f"{p[0]:.4f} {p[1]:.4f} {p[2]:.4f} {c[2]} {c[1]} {c[0]}\n")
    return "".join(out).encode()


def gray_code_frames(n_cols: int, n_rows: int, proj_value: int = 200):
    """Projector frame sequence of ``server/sl_system.py:44-86,440-459`` (for KATs)."""
    Bc = int(math.ceil(math.log2(n_cols)))
    Br = int(math.ceil(math.log2(n_rows)))
    c = np.arange(n_cols)
    r = np.arange(n_rows)
    gc = c ^ (c >> 1)
    gr = r ^ (r >> 1)
    seq = [np.full((n_rows, n_cols), proj_value, np.uint8), np.zeros((n_rows, n_cols), np.uint8)]
    for b in range(Bc):
        pat = np.broadcast_to(((gc >> (Bc - 1 - b)) & 1)[None, :], (n_rows, n_cols)).astype(np.uint8)
        seq += [(pat * proj_value).astype(np.uint8), ((1 - pat) * proj_value).astype(np.uint8)]
    for b in range(Br):
        pat = np.broadcast_to(((gr >> (Br - 1 - b)) & 1)[:, None], (n_rows, n_cols)).astype(np.uint8)
        seq += [(pat * proj_value).astype(np.uint8), ((1 - pat) * proj_value).astype(np.uint8)]
    return seq
