"""ASCII PLY output, byte-identical to ``ProcessingLogic._save_ply``
(``server/processing.py:236-248``) and the inline writer of ``SLSystem.generate_cloud``
(``server/sl_system.py:679-699``): ``"%.4f %.4f %.4f R G B"`` per point, BGR swapped to RGB.
"""
from __future__ import annotations

import numpy as np

HEADER = ("ply\nformat ascii 1.0\nelement vertex {n}\n"
          "property float x\nproperty float y\nproperty float z\n"
          "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")


def format_ascii(points, colors) -> str:
    """The file body as a string (Python's correctly rounded ``%.4f``)."""
    P = np.asarray(points, dtype=np.float64).reshape(-1, 3)
    C = np.asarray(colors).reshape(-1, 3)
    rows = zip(P[:, 0].tolist(), P[:, 1].tolist(), P[:, 2].tolist(),
               C[:, 2].tolist(), C[:, 1].tolist(), C[:, 0].tolist())
    return HEADER.format(n=len(P)) + "".join(
        "%.4f %.4f %.4f %d %d %d\n" % r for r in rows)


def write_ascii(filename, points, colors, threads: int = 0) -> None:
    """Write the PLY with the native multithreaded formatter (``slg_ply_write``)."""
    import ctypes
    from . import _native as N
    P = np.ascontiguousarray(np.asarray(points, dtype=np.float64).reshape(-1, 3))
    C = np.ascontiguousarray(np.asarray(colors, dtype=np.uint8).reshape(-1, 3))
    if len(P) != len(C):
        raise ValueError("points and colors differ in length")
    rc = N.lib().slg_ply_write(str(filename).encode(), P.ctypes.data_as(ctypes.c_void_p),
                               C.ctypes.data_as(ctypes.c_void_p), len(P), int(threads))
    if rc < 0:
        N.check(-rc)
