"""ASCII PLY output, byte-identical to ``ProcessingLogic._save_ply``
(``server/processing.py:236-248``) and the inline writer of ``SLSystem.generate_cloud``
(``server/sl_system.py:679-699``): ``"%.4f %.4f %.4f R G B"`` per point, BGR swapped to RGB.
"""
from __future__ import annotations

import numpy as np

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
