"""Test infrastructure: ``cv2.imread(path, 0)`` / ``cv2.imread(path)`` of a PNG reproduced by the
system libpng (``/usr/lib/x86_64-linux-gnu/libpng16.so.16``, 1.6.37) driven through ctypes with
the calls OpenCV's PNG decoder makes.  opencv-python is not installed here; its decoder is a
thin layer over libpng whose calls are public (OpenCV ``modules/imgcodecs/src/grfmt_png.cpp``,
``PngDecoder::readHeader`` / ``readData``, 4.x):

* readHeader: ``png_create_read_struct(PNG_LIBPNG_VER_STRING, 0, 0, 0)``, the file as the
  read source, ``png_read_info``, ``png_get_IHDR``;
* readData, for an 8-bit destination of ``channels`` = 1 (IMREAD_GRAYSCALE) or 3 (IMREAD_COLOR):
  ``png_set_strip_16`` when the file is 16-bit; ``png_set_strip_alpha`` (channels < 4);
  ``png_set_palette_to_rgb`` for palette files; ``png_set_expand_gray_1_2_4_to_8`` for gray
  files below 8 bits; then colour file + colour read -> ``png_set_bgr``, gray file + colour
  read -> ``png_set_gray_to_rgb``, colour file + gray read -> ``png_set_rgb_to_gray(png, 1,
  0.299, 0.587)``; ``png_set_interlace_handling``, ``png_read_update_info``,
  ``png_read_image``, ``png_read_end``.

Only well-formed files may be given to it: without setjmp (impossible from ctypes) a libpng
error would abort the process.  Warnings are collected.  This module is the checker the
product's decoder (``frames.imread_gray`` / ``imread_bgr`` -> ``slg_png_read``) is pinned to; it
is never used by the product.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIBPNG = "/usr/lib/x86_64-linux-gnu/libpng16.so.16"
_png = None
_warnings: list[str] = []

_ERR_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_char_p)


@_ERR_FN
def _warn(_p, msg):
    _warnings.append(msg.decode(errors="replace"))


def available() -> bool:
    return os.path.exists(LIBPNG)


def lib():
    global _png
    if _png is None:
        L = ctypes.CDLL(LIBPNG)
        vp, u32p, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int)
        sig = {
            "png_get_libpng_ver": (ctypes.c_char_p, [vp]),
            "png_create_read_struct": (vp, [ctypes.c_char_p, vp, vp, _ERR_FN]),
            "png_create_info_struct": (vp, [vp]),
            "png_destroy_read_struct": (None, [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp)]),
            "png_init_io": (None, [vp, vp]),
            "png_read_info": (None, [vp, vp]),
            "png_get_IHDR": (ctypes.c_uint32, [vp, vp, u32p, u32p, ip, ip, ip, ip, ip]),
            "png_set_strip_16": (None, [vp]),
            "png_set_strip_alpha": (None, [vp]),
            "png_set_palette_to_rgb": (None, [vp]),
            "png_set_expand_gray_1_2_4_to_8": (None, [vp]),
            "png_set_bgr": (None, [vp]),
            "png_set_gray_to_rgb": (None, [vp]),
            "png_set_rgb_to_gray": (None, [vp, ctypes.c_int, ctypes.c_double, ctypes.c_double]),
            "png_set_interlace_handling": (ctypes.c_int, [vp]),
            "png_read_update_info": (None, [vp, vp]),
            "png_get_rowbytes": (ctypes.c_size_t, [vp, vp]),
            "png_get_channels": (ctypes.c_ubyte, [vp, vp]),
            "png_read_image": (None, [vp, ctypes.POINTER(vp)]),
            "png_read_end": (None, [vp, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        libc = ctypes.CDLL(None)
        libc.fopen.restype, libc.fopen.argtypes = ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p]
        libc.fclose.argtypes = [ctypes.c_void_p]
        L._libc = libc
        _png = L
    return _png


def version() -> str:
    return lib().png_get_libpng_ver(None).decode()


def imread(path: str, color: bool):
    """uint8 [H, W] (gray) or [H, W, 3] (BGR) as OpenCV 4.x's PNG decoder returns it; plus the
    libpng warnings raised while reading."""
    L = lib()
    _warnings.clear()
    f = L._libc.fopen(os.fsencode(path), b"rb")
    if not f:
        raise FileNotFoundError(path)
    png = ctypes.c_void_p(L.png_create_read_struct(version().encode(), None, None, _warn))
    info = ctypes.c_void_p(L.png_create_info_struct(png))
    try:
        L.png_init_io(png, f)
        L.png_read_info(png, info)
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        depth, ctype, inter, comp, filt = (ctypes.c_int() for _ in range(5))
        L.png_get_IHDR(png, info, ctypes.byref(w), ctypes.byref(h), ctypes.byref(depth), ctypes.byref(ctype),
                       ctypes.byref(inter), ctypes.byref(comp), ctypes.byref(filt))
        is_color = bool(ctype.value & 2)
        if depth.value == 16:
            L.png_set_strip_16(png)
        L.png_set_strip_alpha(png)                       # channels < 4
        if ctype.value == 3:
            L.png_set_palette_to_rgb(png)
        if not is_color and depth.value < 8:
            L.png_set_expand_gray_1_2_4_to_8(png)
        if is_color and color:
            L.png_set_bgr(png)
        elif not is_color and color:
            L.png_set_gray_to_rgb(png)
        elif is_color and not color:
            L.png_set_rgb_to_gray(png, 1, 0.299, 0.587)
        L.png_set_interlace_handling(png)
        L.png_read_update_info(png, info)
        rb = L.png_get_rowbytes(png, info)
        ch = 3 if color else 1
        if rb != w.value * ch:
            raise RuntimeError(f"unexpected row bytes {rb} for {w.value} x {ch}")
        out = np.zeros((h.value, rb), dtype=np.uint8)
        base = out.ctypes.data
        rows = (ctypes.c_void_p * h.value)(*[base + y * rb for y in range(h.value)])
        L.png_read_image(png, rows)
        L.png_read_end(png, None)
    finally:
        L.png_destroy_read_struct(ctypes.byref(png), ctypes.byref(info), None)
        L._libc.fclose(f)
    img = out.reshape(h.value, w.value, 3) if color else out
    return img, list(_warnings)
