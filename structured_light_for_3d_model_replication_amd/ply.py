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


def header(n: int) -> bytes:
    """The header lines of ``_save_ply`` (server/processing.py:239-242)."""
    return (f"ply\nformat ascii 1.0\nelement vertex {n}\nproperty float x\nproperty float y\n"
            f"property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\n"
            f"end_header\n").encode()


class DeviceFormatter:
    """Formats device clouds into PLY bodies on the GPU (``slg_ply_format``) with reusable device
    buffers; one instance per stream."""

    def __init__(self):
        self._text = None
        self._ws = None

    def _buffers(self, n: int, device):
        from . import _native as N
        import torch
        need_t = int(N.lib().slg_ply_format_bound(n))
        need_w = int(N.lib().slg_ply_format_ws_bytes(n))
        if self._text is None or self._text.numel() < need_t or self._text.device != device:
            self._text = torch.empty(max(need_t, 1), dtype=torch.uint8, device=device)
        if self._ws is None or self._ws.numel() < need_w or self._ws.device != device:
            self._ws = torch.empty(need_w, dtype=torch.uint8, device=device)
        return self._text, self._ws

    def body(self, xyz, bgr, stream=None):
        """Body bytes of the PLY of a device cloud (xyz float64 [n, 3], bgr uint8 [n, 3]) as a
        DEVICE uint8 tensor view, or None when a coordinate needs the host formatter (NaN, inf,
        |x| >= 9.2e14).  Synchronises ``stream`` to read the length.  The view aliases this
        formatter's buffer: copy it out before the next call."""
        import ctypes
        import torch
        from . import _native as N
        n = int(xyz.shape[0])
        if xyz.dtype != torch.float64 or bgr.dtype != torch.uint8 or tuple(bgr.shape) != (n, 3):
            raise ValueError("device PLY formatting needs float64 xyz and uint8 bgr of one length")
        if not (xyz.is_cuda and bgr.is_cuda and xyz.device == bgr.device):
            raise ValueError("device PLY formatting needs both arrays on one GPU")
        xyz, bgr = xyz.contiguous(), bgr.contiguous()
        text, ws = self._buffers(n, xyz.device)
        s = torch.cuda.current_stream(xyz.device) if stream is None else stream
        N.check(N.lib().slg_ply_format(ctypes.c_void_p(xyz.data_ptr()), ctypes.c_void_p(bgr.data_ptr()), n,
                                       ctypes.c_void_p(text.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                       ctypes.c_void_p(s.cuda_stream)))
        s.synchronize()
        hdr = ws[:16].cpu().numpy()
        total = int(np.frombuffer(hdr[:8].tobytes(), np.int64)[0])
        bad = int(np.frombuffer(hdr[8:12].tobytes(), np.int32)[0])
        return None if bad else text[:total]


def write_body(filename, n: int, body_host) -> None:
    """Write ``header(n)`` + a formatted body (host bytes-like) as the PLY file."""
    with open(filename, "wb") as f:
        f.write(header(n))
        f.write(memoryview(body_host))
