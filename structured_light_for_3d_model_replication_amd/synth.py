"""Deterministic synthetic structured-light captures (SURVEY §8(d) "Synthetic inputs").

The reference ships no captures, so tests and the benchmark render their own:
a camera/projector rig, a turntable object (a sphere and a capped cylinder, both off the
turntable axis, rotated by the view angle) in front of a back wall, and the Gray-code frame
sequence the reference projects (``server/sl_system.py:440-459``: white, black, then
(pattern, inverse) per column bit MSB-first, then per row bit).  Each camera pixel is traced
into the scene, tested for projector visibility (frustum + shadow by the other object) and
given a lit or dark level with integer noise, so masks, ties (``p == i``) and shadows are all
exercised.  Only NumPy is used; output is a uint8 ``[F, H, W]`` frame stack plus a BGR texture.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import calibration

PROJ_VALUE = 200           # server/config.py:20


def n_bits(n: int) -> int:
    """``int(np.ceil(np.log2(n)))`` (server/processing.py:80-81, sl_system.py:52-54)."""
    return int(np.ceil(np.log2(n)))


def frame_slots(proj_w: int, proj_h: int) -> int:
    """Number of frames a full capture holds: white, black, 2 per column bit, 2 per row bit."""
    return 2 + 2 * n_bits(proj_w) + 2 * n_bits(proj_h)


@dataclass
class Rig:
    cam_w: int
    cam_h: int
    proj_w: int
    proj_h: int
    K1: np.ndarray
    K2: np.ndarray
    R: np.ndarray
    T: np.ndarray
    turntable_center: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, 650.0]))

    def tables(self) -> dict:
        return calibration.build_tables(self.K1, self.K2, self.R, self.T,
                                        (self.cam_w, self.cam_h), (self.proj_w, self.proj_h))


def default_rig(cam_w=1920, cam_h=1080, proj_w=1920, proj_h=1080) -> Rig:
    """Camera at the origin (≈45° horizontal FOV); projector 200 mm to the right, toed in."""
    fc = 0.5 * cam_w / math.tan(math.radians(22.5))
    K1 = np.array([[fc, 0.0, (cam_w - 1) / 2.0 + 3.25],
                   [0.0, fc * 1.0005, (cam_h - 1) / 2.0 - 2.5],
                   [0.0, 0.0, 1.0]])
    fp = 0.5 * proj_w / math.tan(math.radians(20.0))
    K2 = np.array([[fp, 0.0, proj_w / 2.0 + 1.5],
                   [0.0, fp, proj_h / 2.0 - 0.5],
                   [0.0, 0.0, 1.0]])
    C = np.array([200.0, -15.0, 20.0])                 # projector centre, camera coords (mm)
    target = np.array([0.0, 0.0, 680.0])
    z = target - C
    z /= np.linalg.norm(z)
    x = np.cross(np.array([0.0, 1.0, 0.0]), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z])                            # rows = projector axes in camera frame
    T = -(R @ C).reshape(3, 1)                         # X_p = R X_c + T  (cv2.stereoCalibrate)
    return Rig(cam_w, cam_h, proj_w, proj_h, K1, K2, R, T)


@dataclass
class View:
    frames: np.ndarray        # uint8 [F, H, W]
    texture: np.ndarray       # uint8 [H, W, 3] BGR (what cv2.imread(files[0]) returns)
    proj_col: np.ndarray      # int32 [H, W] ground-truth projector column (-1 if unlit)
    proj_row: np.ndarray      # int32 [H, W]
    lit: np.ndarray           # bool  [H, W]


def _scene(view_deg: float, center: np.ndarray):
    th = math.radians(view_deg)
    c, s = math.cos(th), math.sin(th)

    def rot(off):   # rotate an offset in the turntable (xz) plane
        return center + np.array([c * off[0] + s * off[2], off[1], -s * off[0] + c * off[2]])

    sphere = (rot(np.array([55.0, -40.0, 0.0])), 105.0)
    cyl = (rot(np.array([-45.0, 0.0, 20.0])), 62.0, -150.0, 190.0)   # centre, r, y0, y1
    wall_z = 980.0
    return sphere, cyl, wall_z


def _hit_sphere(o, d, c, r):
    """Smallest t > 1e-6 with |o + t d - c| = r (o: (3,) or (N,3); d: (N,3) unit)."""
    oc = o - c
    b = np.sum(d * oc, axis=-1)
    cc = np.sum(oc * oc, axis=-1) - r * r
    disc = b * b - cc
    sq = np.sqrt(np.maximum(disc, 0.0))
    t0, t1 = -b - sq, -b + sq
    t = np.where(t0 > 1e-6, t0, t1)
    return np.where((disc >= 0) & (t > 1e-6), t, np.inf)


def _hit_cyl(o, d, c, r, y0, y1):
    """Vertical (y-axis) capped-off cylinder side surface."""
    ox = o[..., 0] - c[0]
    oz = o[..., 2] - c[2]
    a = d[..., 0] ** 2 + d[..., 2] ** 2
    b = ox * d[..., 0] + oz * d[..., 2]
    cc = ox * ox + oz * oz - r * r
    disc = b * b - a * cc
    sq = np.sqrt(np.maximum(disc, 0.0))
    a_safe = np.where(a > 1e-12, a, 1.0)
    res = np.full(d.shape[:-1], np.inf)
    for t in ((-b - sq) / a_safe, (-b + sq) / a_safe):
        y = (o[..., 1] if np.ndim(o) > 1 else o[1]) + t * d[..., 1]
        ok = (disc >= 0) & (a > 1e-12) & (t > 1e-6) & (y >= y0) & (y <= y1)
        res = np.where(ok & (t < res), t, res)
    return res


def render_view(rig: Rig, view_deg: float = 0.0, seed: int = 0, n_present: int | None = None,
                proj_value: int = PROJ_VALUE, noise: int = 8, ambient: int = 9) -> View:
    """Render one turntable view of the Gray-code capture sequence.

    ``n_present`` truncates the sequence (the reference tolerates missing trailing frames:
    ``server/processing.py:94-96``).  Deterministic in (rig, view_deg, seed).
    """
    rng = np.random.default_rng(seed)
    H, W = rig.cam_h, rig.cam_w
    Bc, Br = n_bits(rig.proj_w), n_bits(rig.proj_h)
    F = 2 + 2 * Bc + 2 * Br
    if n_present is None:
        n_present = F

    # --- camera rays ---------------------------------------------------------------
    K1 = rig.K1
    u = np.arange(W, dtype=np.float64)
    v = np.arange(H, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    d = np.stack([(uu - K1[0, 2]) / K1[0, 0], (vv - K1[1, 2]) / K1[1, 1], np.ones_like(uu)], -1)
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    d = d.reshape(-1, 3)
    o = np.zeros(3)

    sphere, cyl, wall_z = _scene(view_deg, rig.turntable_center)
    ts = _hit_sphere(o, d, *sphere)
    tc = _hit_cyl(o, d, *cyl)
    tw = np.where(d[:, 2] > 1e-9, wall_z / np.maximum(d[:, 2], 1e-9), np.inf)
    t = np.minimum(np.minimum(ts, tc), tw)
    obj = np.select([t == ts, t == tc], [0, 1], 2)            # 0 sphere, 1 cylinder, 2 wall
    X = d * t[:, None]

    nrm = np.empty_like(X)
    nrm[obj == 0] = (X[obj == 0] - sphere[0]) / sphere[1]
    cyl_v = X[obj == 1] - cyl[0]
    cyl_v[:, 1] = 0.0
    nrm[obj == 1] = cyl_v / cyl[1]
    nrm[obj == 2] = np.array([0.0, 0.0, -1.0])

    # --- projector visibility --------------------------------------------------------
    Cp = -(rig.R.T @ rig.T).ravel()
    Xp = X @ rig.R.T + rig.T.ravel()
    zp = Xp[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        up = rig.K2[0, 0] * Xp[:, 0] / zp + rig.K2[0, 2]
        vp = rig.K2[1, 1] * Xp[:, 1] / zp + rig.K2[1, 2]
    in_frustum = (zp > 1.0) & (up >= 0) & (up < rig.proj_w) & (vp >= 0) & (vp < rig.proj_h)
    to_p = Cp - X
    dist_p = np.linalg.norm(to_p, axis=1)
    dp = to_p / dist_p[:, None]
    Xo = X + 1e-3 * dp
    shadow = np.minimum(_hit_sphere(Xo, dp, *sphere), _hit_cyl(Xo, dp, *cyl)) < dist_p - 1e-2
    cos_p = np.abs(np.sum(nrm * dp, axis=1))
    lit = in_frustum & ~shadow & (cos_p > 0.05)

    col = np.where(lit, np.floor(up), -1).astype(np.int64)
    row = np.where(lit, np.floor(vp), -1).astype(np.int64)

    # --- radiometry -----------------------------------------------------------------
    albedo = np.select([obj == 0, obj == 1], [0.92, 0.78], 0.55)
    level = albedo * proj_value * (0.25 + 0.75 * cos_p)           # lit level
    level = np.clip(level, 0, 255 - ambient - noise)
    bleed = 0.015 * level

    gc = (np.maximum(col, 0) ^ (np.maximum(col, 0) >> 1))
    gr = (np.maximum(row, 0) ^ (np.maximum(row, 0) >> 1))

    frames = np.empty((n_present, H * W), dtype=np.uint8)
    # ambient + floor(level) + noise stays <= 255 by the clip above: u8 arithmetic, no float
    # temporaries per frame (24 MP captures render in seconds)
    on_u8 = (ambient + np.floor(level)).astype(np.uint8)
    off_u8 = (ambient + np.floor(bleed)).astype(np.uint8)

    def emit(k, on):
        if k >= n_present:
            return
        np.add(np.where(on, on_u8, off_u8), rng.integers(0, noise, size=H * W, dtype=np.uint8),
               out=frames[k])

    emit(0, lit)
    emit(1, np.zeros(H * W, dtype=bool))
    k = 2
    for b in range(Bc):
        bit = ((gc >> (Bc - 1 - b)) & 1).astype(bool)
        emit(k, lit & bit)
        emit(k + 1, lit & ~bit)
        k += 2
    for b in range(Br):
        bit = ((gr >> (Br - 1 - b)) & 1).astype(bool)
        emit(k, lit & bit)
        emit(k + 1, lit & ~bit)
        k += 2

    white = frames[0].astype(np.float64) if n_present > 0 else np.zeros(H * W)
    tints = np.array([[0.55, 0.8, 1.0], [1.0, 0.75, 0.45], [0.9, 0.9, 0.9]])   # BGR per object
    tint = tints[obj]
    tex = np.clip(np.floor(white[:, None] * tint), 0, 255).astype(np.uint8).reshape(H, W, 3)

    return View(frames=frames.reshape(n_present, H, W), texture=tex,
                proj_col=col.reshape(H, W).astype(np.int32),
                proj_row=row.reshape(H, W).astype(np.int32),
                lit=lit.reshape(H, W))


_RIG = None         # the rig of render_many's forked workers (inherited, never pickled)


def _render_spec(spec):
    deg, seed, n_present = spec
    return render_view(_RIG, view_deg=deg, seed=seed, n_present=n_present)


def render_many(rig: Rig, specs, workers: int = 1) -> list:
    """``render_view`` for each ``(view_deg, seed, n_present)`` spec, on ``workers`` forked
    processes (host only: call it before the process touches a GPU)."""
    global _RIG
    specs = list(specs)
    if workers <= 1 or len(specs) <= 1:
        return [render_view(rig, view_deg=d, seed=s, n_present=n) for d, s, n in specs]
    import multiprocessing as mp
    _RIG = rig
    with mp.get_context("fork").Pool(min(workers, len(specs))) as pool:
        return pool.map(_render_spec, specs, chunksize=1)


def job_view_angle(obj: int, view: int, n_views: int) -> float:
    """Turntable angle of view ``view`` of object ``obj`` in a scan-farm job (objects start at
    staggered angles so no two objects' captures coincide)."""
    return 360.0 * view / n_views + 45.0 * obj


def write_capture(view: View, folder: str, ext: str = "png") -> list[str]:
    """Write the frames in the reference's capture layout ``01.png, 02.png, ...``
    (``server/sl_system.py:444-459``) as 8-bit grayscale files; returns the file list.
    (For grayscale files ``cv2.imread(files[0])`` yields the white frame replicated to BGR.)"""
    import os
    from PIL import Image
    os.makedirs(folder, exist_ok=True)
    paths = []
    for i, fr in enumerate(view.frames):
        p = os.path.join(folder, f"{i + 1:02d}.{ext}")
        Image.fromarray(fr, mode="L").save(p)
        paths.append(p)
    return paths
