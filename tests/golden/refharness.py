"""Import the reference's hot-path functions in the survey container (fixture generation only).

Used by ``make_golden.py`` — never at test time, never on the GPU box (``/root/reference``
does not exist there).  The reference imports ``cv2``/``open3d``/``tkinter``/``flask_cors``,
which the image lacks, so stub modules are installed first:

* ``cv2.imread(path, 0)`` / ``cv2.imread(path)`` return in-memory frames registered with
  :func:`register_frames` (grayscale / BGR texture), so PNG decoding is out of the picture;
* ``cv2.threshold(img, 0, 255, BINARY|OTSU)`` returns ``(oracle.otsu_threshold(img), None)``
  — OpenCV's Otsu is not available here (parity for it is pinned by KATs instead).

Bytecode writing is disabled so nothing is written under ``/root/reference``.
"""
from __future__ import annotations

import sys
import types

REF_SERVER = "/root/reference/server"

_FRAMES: dict[str, object] = {}
_TEXTURES: dict[str, object] = {}


def register_frames(prefix: str, frames, texture):
    """Expose ``frames`` as files ``{prefix}/01.png ...``; returns the sorted path list."""
    paths = []
    for i, fr in enumerate(frames):
        p = f"{prefix}/{i + 1:02d}.png"
        _FRAMES[p] = fr
        paths.append(p)
    _TEXTURES[paths[0]] = texture
    return paths


def _install_stubs():
    sys.dont_write_bytecode = True
    import numpy as np
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
    from oracle import sl_oracle

    cv2 = types.ModuleType("cv2")
    cv2.THRESH_BINARY = 0
    cv2.THRESH_OTSU = 8

    def imread(path, flag=1):
        if flag == 0:
            return np.array(_FRAMES[path], copy=True)
        return np.array(_TEXTURES[path], copy=True)

    def threshold(img, thresh, maxval, typ):
        assert typ == (cv2.THRESH_BINARY | cv2.THRESH_OTSU)
        return sl_oracle.otsu_threshold(img), None

    cv2.imread = imread
    cv2.threshold = threshold
    sys.modules["cv2"] = cv2
    sys.modules.setdefault("open3d", types.ModuleType("open3d"))
    tk = types.ModuleType("tkinter")
    tk.messagebox = types.ModuleType("tkinter.messagebox")
    tk.messagebox.showinfo = lambda *a, **k: None
    tk.messagebox.showerror = lambda *a, **k: None
    sys.modules["tkinter"] = tk
    sys.modules["tkinter.messagebox"] = tk.messagebox
    fc = types.ModuleType("flask_cors")
    fc.CORS = lambda *a, **k: None
    sys.modules["flask_cors"] = fc
    if REF_SERVER not in sys.path:
        sys.path.insert(0, REF_SERVER)


def load():
    """Return (ProcessingLogic, SLSystem-nested gray_decode, SLSystem-nested reconstruct)."""
    _install_stubs()
    import processing   # /root/reference/server/processing.py
    import sl_system    # /root/reference/server/sl_system.py

    code = sl_system.SLSystem.generate_cloud.__code__
    nested = {c.co_name: c for c in code.co_consts if isinstance(c, types.CodeType)}
    gray_decode = types.FunctionType(nested["gray_decode"], sl_system.__dict__, "gray_decode",
                                     (1920, 1080))
    recon = types.FunctionType(nested["reconstruct_point_cloud"], sl_system.__dict__,
                               "reconstruct_point_cloud")
    return processing.ProcessingLogic, gray_decode, recon, sl_system
