"""Capture discovery and frame ingest (host side of the hot path).

* Discovery keeps the reference's orders: ``ProcessingLogic._gray_decode`` globs ``*.bmp``
  first, then ``*.png`` (``server/processing.py:49-54``); ``SLSystem.generate_cloud`` globs
  ``*.png`` first, then ``*.bmp`` (``server/sl_system.py:518-520``); both ``sorted``.
* ``imread_gray`` / ``imread_bgr`` stand in for ``cv2.imread(path, 0)`` / ``cv2.imread(path)``
  (OpenCV is not in the image).  PNGs: 8-bit grayscale files -- what the reference's scanner
  writes -- take the native fast path (identity on the samples); every other PNG (the phone's
  RGBA canvas captures, ``frontend/App.tsx:234-247``; 16-bit, palette, gray + alpha, Adam7,
  gAMA / sRGB / iCCP tagged) goes through ``slg_png_read``, which returns what OpenCV's libpng
  calls return, pinned byte for byte to the system libpng 1.6.37 (``tests/test_png_color.py``).
  BMP and other formats: PIL, with OpenCV's ``BGR2GRAY`` 14-bit weights for colour BMPs --
  restated from OpenCV's published C, parity unpinned (no OpenCV here).  Decoding runs on a
  host thread pool.
"""
from __future__ import annotations

import glob
import os
import threading
from concurrent.futures import ThreadPoolExecutor, wait

import numpy as np


def discover(source, order=("bmp", "png")):
    """File list of a capture folder (or the list itself), in the reference's order."""
    if isinstance(source, (list, tuple)):
        return list(source)
    for ext in order:
        files = sorted(glob.glob(os.path.join(source, f"*.{ext}")))
        if files:
            return files
    return []


def _open(path):
    from PIL import Image
    try:
        im = Image.open(path)
        im.load()
        return im
    except (OSError, ValueError):
        return None


def _to_gray(im, path) -> np.ndarray:
    """PIL image of a non-PNG file -> ``cv2.imread(path, 0)`` (8-bit samples)."""
    if im.mode == "P":
        im = im.convert("RGBA" if "transparency" in im.info else "RGB")
    a = np.asarray(im)
    if a.dtype == np.uint16:
        a = (a >> 8).astype(np.uint8)
    if a.ndim == 2:
        return np.ascontiguousarray(a, dtype=np.uint8)
    if a.shape[2] < 3:                                # gray + alpha
        return np.ascontiguousarray(a[..., 0], dtype=np.uint8)
    rgb = a[..., :3].astype(np.uint32)
    r, g, b = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    # OpenCV icvCvt_BGR2Gray_8u_C3C1R: (b*1868 + g*9617 + r*4899 + 8192) >> 14
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def _is_png(path) -> bool:
    return str(path).lower().endswith(".png")


def _is_png_gray8(path) -> bool:
    if not _is_png(path):
        return False
    import ctypes
    from . import _native as N
    w, h = ctypes.c_int32(), ctypes.c_int32()
    return N.lib().slg_png_gray8_size(os.fsencode(path), ctypes.byref(w), ctypes.byref(h)) == 0


def _png_gray8(path):
    """Native fast path (``slg_png_gray8_*``): an 8-bit grayscale PNG decoded without PIL;
    ``None`` for any other file (decoded the general way below)."""
    if not _is_png(path):
        return None
    import ctypes
    from . import _native as N
    L = N.lib()
    bp = os.fsencode(path)
    w, h = ctypes.c_int32(), ctypes.c_int32()
    if L.slg_png_gray8_size(bp, ctypes.byref(w), ctypes.byref(h)) != 0:
        return None
    out = np.empty((h.value, w.value), dtype=np.uint8)
    if L.slg_png_gray8_decode(bp, out.ctypes.data_as(ctypes.c_void_p), out.size, w, h) != 0:
        return None
    return out


def png_read(path, gray: bool = True, bgr: bool = False):
    """``slg_png_read``: ``(gray [H, W] or None, bgr [H, W, 3] or None)`` as OpenCV's PNG decoder
    returns them, or None for a file cv2.imread cannot read."""
    import ctypes
    from . import _native as N
    L = N.lib()
    bp = os.fsencode(path)
    info = (ctypes.c_int32 * 7)()
    if L.slg_png_info(bp, info) != 0:
        return None
    h, w = info[1], info[0]
    g = np.empty((h, w), dtype=np.uint8) if gray else None
    c = np.empty((h, w, 3), dtype=np.uint8) if bgr else None
    vp = ctypes.c_void_p
    rc = L.slg_png_read(bp, vp(g.ctypes.data) if gray else None, g.size if gray else 0,
                        vp(c.ctypes.data) if bgr else None, c.size if bgr else 0, info)
    return None if rc != 0 else (g, c)


def imread_gray(path) -> np.ndarray:
    """``cv2.imread(path, 0)``; raises like ``None.astype`` would for unreadable files."""
    a = _png_gray8(path)
    if a is not None:
        return a
    if _is_png(path):
        r = png_read(path, gray=True)
        if r is None:
            raise AttributeError("'NoneType' object has no attribute 'astype'")
        return r[0]
    im = _open(path)
    if im is None:
        raise AttributeError("'NoneType' object has no attribute 'astype'")
    return _to_gray(im, path)


def imread_bgr(path) -> np.ndarray:
    """``cv2.imread(path)``: HxWx3 BGR uint8 (grayscale replicated)."""
    a = _png_gray8(path)
    if a is not None:
        return np.repeat(a[..., None], 3, axis=-1)
    if _is_png(path):
        r = png_read(path, gray=False, bgr=True)
        if r is None:
            raise AttributeError("'NoneType' object has no attribute 'reshape'")
        return r[1]
    im = _open(path)
    if im is None:
        raise AttributeError("'NoneType' object has no attribute 'reshape'")
    if im.mode == "P":
        im = im.convert("RGBA" if "transparency" in im.info else "RGB")
    a = np.asarray(im)
    if a.dtype == np.uint16:
        a = (a >> 8).astype(np.uint8)
    if a.ndim == 2:
        return np.repeat(a[..., None], 3, axis=-1).astype(np.uint8)
    if a.shape[2] < 3:
        return np.repeat(a[..., :1], 3, axis=-1).astype(np.uint8)
    return np.ascontiguousarray(a[..., 2::-1][..., :3], dtype=np.uint8)


def cpu_quota():
    """CPUs of CPU time this process may use: the cgroup CFS quota (cgroup v2 ``cpu.max``, or v1
    ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``), rounded up; None when unlimited.  On the GPU
    box the affinity mask lists every host CPU (256) while the lease's quota is 16."""
    import math
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, math.ceil(q / per))
    except (OSError, ValueError):
        return None


def decode_threads() -> int:
    """Host decode threads: ``SLG_DECODE_THREADS``, else the CPUs this process may use -- the
    smaller of its affinity mask and its cgroup CPU quota (at most 64: past that the PLY writers
    and the device group's stream reads want CPUs too)."""
    env = os.environ.get("SLG_DECODE_THREADS")
    if env:
        return max(1, int(env))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 8
    q = cpu_quota()
    if q is not None:
        n = min(n, q)
    return max(1, min(64, n))


_POOLS: dict = {}
_POOLS_LOCK = threading.Lock()


def decode_pool() -> ThreadPoolExecutor:
    """The process's host decode pool (:func:`decode_threads` threads, kept across views): the
    native decoder keeps its per-thread buffers warm in it, and two folders read at once share
    the CPUs instead of each starting a pool of its own."""
    n = decode_threads()
    with _POOLS_LOCK:
        ex = _POOLS.get(n)
        if ex is None:
            ex = _POOLS[n] = ThreadPoolExecutor(max_workers=n, thread_name_prefix="slg-decode")
        return ex


def decode_all(fn, items) -> list:
    """``[fn(x) for x in items]`` on :func:`decode_pool`; every call has finished when this
    returns or raises (the first failure in item order), so the caller may reuse the buffers
    the calls wrote into."""
    futs = [decode_pool().submit(fn, x) for x in items]
    wait(futs)
    return [f.result() for f in futs]


def load_frames(files, indices=None, workers: int = 0, texture: bool = False):
    """Decode the given frames (grayscale) on a thread pool; returns a list of arrays, plus
    ``cv2.imread(files[0])`` (BGR texture, processing.py:124) decoded in the same pool when
    ``texture`` — so the texture's second decode of frame 0 is not a serial tail."""
    idx = range(len(files)) if indices is None else indices
    paths = [files[i] for i in idx]
    workers = workers or decode_threads()
    if len(paths) + texture <= 1:
        imgs = [imread_gray(p) for p in paths]
        return (imgs, imread_bgr(files[0])) if texture else imgs
    # An 8-bit gray PNG frame 0 that is decoded anyway gives the texture by replication (what
    # cv2.imread(f) returns for it) instead of a second decode.
    reuse = texture and files[0] in paths and _is_png_gray8(files[0])
    with ThreadPoolExecutor(max_workers=min(workers, len(paths) + texture)) as ex:
        tex = ex.submit(imread_bgr, files[0]) if texture and not reuse else None  # longest task first
        imgs = list(ex.map(imread_gray, paths))
        if not texture:
            return imgs
        if reuse:
            return imgs, np.repeat(imgs[paths.index(files[0])][..., None], 3, axis=-1)
        return imgs, tex.result()
