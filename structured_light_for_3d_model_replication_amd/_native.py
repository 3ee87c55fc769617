"""ctypes binding of ``libslgpu.so`` (C ABI in ``include/slgpu.h``).

The library is built in-tree (``build.build_native``) and must be present: there is no CPU
fallback in the product path.  ``torch`` is imported first so that the library's
``libamdhip64.so.7`` dependency resolves to the HIP runtime torch already loaded (one HIP
runtime per process; a second one would not understand torch's streams or pointers).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_NAME = "libslgpu.so"
PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
# A/B builds of the same ABI (tools/build_ab.sh -> ab_libs/, build_ab/; tools/kbench.py, ab.py):
# only libraries inside those in-tree build directories may replace the product library
AB_DIRS = (os.path.join(REPO_DIR, "ab_libs"), os.path.join(REPO_DIR, "build_ab"))
AB_LIB = None
if os.environ.get("SLG_LIB"):
    _p = os.path.realpath(os.environ["SLG_LIB"])
    if not any(os.path.commonpath([_p, os.path.realpath(d)]) == os.path.realpath(d) for d in AB_DIRS):
        raise ImportError(f"SLG_LIB={_p}: A/B libraries must live in {' or '.join(AB_DIRS)}")
    LIB_PATH = AB_LIB = _p

ABI_VERSION = 2          # SLG_ABI_VERSION in include/slgpu.h
SLG_OK = 0
SLG_ERR_INVALID = 1
SLG_ERR_HIP = 2
SLG_ERR_UNSUPPORTED = 3
SLG_ERR_NOT_ENOUGH = 4
SLG_ERR_INDEX = 5

THRESH_OTSU, THRESH_MANUAL, THRESH_PERCENTILE = 0, 1, 2
VARIANT_PROCESSING, VARIANT_SLSYSTEM = 0, 1
RAYS_TABLE, RAYS_PINHOLE = 0, 1
GRAY_PNG, GRAY_BMP = 0, 1

c_i32, c_i64, c_dbl, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p


class Capture(ctypes.Structure):
    _fields_ = [("frames", c_vp), ("frame_stride", c_i64), ("n_frames", c_i32),
                ("height", c_i32), ("width", c_i32), ("reserved", c_i32), ("texture", c_vp)]


class DecodeParams(ctypes.Structure):
    _fields_ = [("proj_cols", c_i32), ("proj_rows", c_i32), ("n_sets_col", c_i32),
                ("n_sets_row", c_i32), ("variant", c_i32), ("thresh_mode", c_i32),
                ("shadow_val", c_dbl), ("contrast_val", c_dbl)]


class Calib(ctypes.Structure):
    _fields_ = [("rays", c_vp), ("ray_mode", c_i32), ("reserved", c_i32),
                ("fx", c_dbl), ("fy", c_dbl), ("cx", c_dbl), ("cy", c_dbl),
                ("oc", c_dbl * 3), ("col_planes", c_vp), ("n_col_planes", c_i32),
                ("reserved2", c_i32), ("row_planes", c_vp), ("n_row_planes", c_i32),
                ("reserved3", c_i32), ("col_planes_num", c_vp), ("row_planes_num", c_vp)]


class TriParams(ctypes.Structure):
    _fields_ = [("row_mode", c_i32), ("xyz_f64", c_i32), ("epipolar_tol", c_dbl)]


class Maps(ctypes.Structure):
    _fields_ = [("col", c_vp), ("row", c_vp), ("mask", c_vp), ("texture", c_vp),
                ("height", c_i32), ("width", c_i32)]


class Cloud(ctypes.Structure):
    _fields_ = [("xyz", c_vp), ("bgr", c_vp), ("count", c_vp), ("capacity", c_i64)]


class PngFrame(ctypes.Structure):
    _fields_ = [("z", c_vp), ("zlen", c_i64), ("raw", c_vp), ("out", c_vp), ("out_pitch", c_i64),
                ("width", c_i32), ("height", c_i32), ("channels", c_i32), ("reserved", c_i32)]


PNG_E_STREAM, PNG_E_SIZE, PNG_E_ADLER, PNG_E_FILTER, PNG_E_UNSUPPORTED = 1, 2, 3, 4, 5


EXPORTS = {
    "slg_version": (c_i32, []),
    "slg_build_id": (ctypes.c_char_p, []),
    "slg_kernel_table": (c_i32, [ctypes.c_char_p, c_i64]),
    "slg_last_kernel": (c_i32, [ctypes.c_char_p, c_i64]),
    "slg_last_error": (ctypes.c_char_p, []),
    "slg_workspace_bytes": (c_i64, [c_i64]),
    "slg_workspace_init": (c_i32, [c_vp, c_i64, c_vp]),
    "slg_workspace_set_arena": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_vp]),
    "slg_decode_stats": (c_i32, [ctypes.POINTER(Capture), ctypes.POINTER(DecodeParams), c_vp, c_vp]),
    "slg_decode_histograms": (c_i32, [ctypes.POINTER(Capture), ctypes.POINTER(DecodeParams), c_vp, c_vp, c_vp]),
    "slg_thresholds_from_histograms": (c_i32, [c_vp, c_i64, ctypes.POINTER(DecodeParams), c_vp, c_i64, c_vp]),
    "slg_decode": (c_i32, [ctypes.POINTER(Capture), ctypes.POINTER(DecodeParams), c_vp,
                           c_vp, c_vp, c_vp, c_vp]),
    "slg_triangulate": (c_i32, [ctypes.POINTER(Maps), ctypes.POINTER(Calib),
                                ctypes.POINTER(TriParams), c_vp, ctypes.POINTER(Cloud), c_vp]),
    "slg_reconstruct": (c_i32, [ctypes.POINTER(Capture), ctypes.POINTER(DecodeParams),
                                ctypes.POINTER(Calib), ctypes.POINTER(TriParams), c_vp,
                                ctypes.POINTER(Cloud), c_vp]),
    "slg_decode_triangulate": (c_i32, [ctypes.POINTER(Capture), ctypes.POINTER(DecodeParams),
                                       ctypes.POINTER(Calib), ctypes.POINTER(TriParams), c_vp,
                                       ctypes.POINTER(Cloud), c_vp]),
    "slg_reconstruct_batch": (c_i32, [ctypes.POINTER(Capture), c_i32, ctypes.POINTER(DecodeParams),
                                      ctypes.POINTER(Calib), ctypes.POINTER(TriParams), c_vp, c_i64,
                                      ctypes.POINTER(Cloud), ctypes.POINTER(c_vp), c_vp]),
    "slg_decode_stats_batch": (c_i32, [ctypes.POINTER(Capture), c_i32, ctypes.POINTER(DecodeParams),
                                       c_vp, c_i64, c_vp]),
    "slg_decode_triangulate_batch": (c_i32, [ctypes.POINTER(Capture), c_i32, ctypes.POINTER(DecodeParams),
                                             ctypes.POINTER(Calib), ctypes.POINTER(TriParams), c_vp,
                                             c_i64, ctypes.POINTER(Cloud), ctypes.POINTER(c_vp), c_vp]),
    "slg_decode_triangulate_batch_next": (c_i32, [ctypes.POINTER(Capture), c_i32, ctypes.POINTER(DecodeParams),
                                                  ctypes.POINTER(Calib), ctypes.POINTER(TriParams), c_vp,
                                                  c_i64, ctypes.POINTER(Cloud), ctypes.POINTER(Capture), c_i32,
                                                  ctypes.POINTER(c_vp), c_vp]),
    "slg_decode_triangulate_batch_carry": (c_i32, [ctypes.POINTER(Capture), c_i32, ctypes.POINTER(DecodeParams),
                                                   ctypes.POINTER(Calib), ctypes.POINTER(TriParams), c_vp,
                                                   c_i64, ctypes.POINTER(Cloud), ctypes.POINTER(Capture), c_i32,
                                                   c_vp, c_i32, ctypes.POINTER(c_vp), c_vp]),
    "slg_decode_stats_partials_batch": (c_i32, [c_i32, c_i32, c_i32, ctypes.POINTER(DecodeParams), c_vp, c_i64,
                                                c_vp]),
    "slg_ply_write": (c_i64, [ctypes.c_char_p, c_vp, c_vp, c_i64, c_i32]),
    "slg_ply_format_bound": (c_i64, [c_i64]),
    "slg_ply_format_ws_bytes": (c_i64, [c_i64]),
    "slg_ply_format": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "slg_png_gray8_size": (c_i32, [ctypes.c_char_p, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)]),
    "slg_png_gray8_decode": (c_i32, [ctypes.c_char_p, c_vp, c_i64, c_i32, c_i32]),
    "slg_png_zstream": (c_i32, [ctypes.c_char_p, c_vp, c_i64, ctypes.POINTER(c_i32)]),
    "slg_png_info": (c_i32, [ctypes.c_char_p, ctypes.POINTER(c_i32)]),
    "slg_png_read": (c_i32, [ctypes.c_char_p, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(c_i32)]),
    "slg_png_raw_bytes": (c_i64, [c_i32, c_i32, c_i32]),
    "slg_png_decode_device": (c_i32, [c_vp, c_i32, c_vp, c_vp]),
    "slg_stream_create_reserving": (c_i32, [c_i32, c_vp]),
    "slg_stream_destroy": (c_i32, [c_vp]),
    "slg_rays_match_pinhole": (c_i32, [c_vp, c_i32, c_i32, c_dbl, c_dbl, c_dbl, c_dbl, c_vp, c_vp]),
    "slg_rgb_to_gray": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "slg_gray_texture": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "slg_gather_unique_id": (c_i32, [c_vp]),
    "slg_gather_init": (c_i32, [ctypes.POINTER(c_vp), c_i32, c_i32, c_vp]),
    "slg_gather_counts": (c_i32, [c_vp, c_vp, c_i32, c_vp, c_vp]),
    "slg_gatherv": (c_i32, [c_vp, c_vp, c_i64, c_vp, ctypes.POINTER(c_i64), c_i32, c_vp]),
    "slg_gather_destroy": (c_i32, [c_vp]),
    "slg_gatherv_plan": (c_i32, [c_i32, c_i32, c_i32, c_i64, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                 ctypes.POINTER(c_i32)]),
}
GATHER_ID_BYTES = 128


class NativeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"slgpu error {code}: {msg}")
        self.code = code
        self.msg = msg


_lib = None


def lib():
    """Load (once) and return the native library; raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (hipcc --offload-arch=gfx950) first")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            if AB_LIB is not None and not hasattr(h, name):
                continue                     # an A/B build from an older tree (tools/ab.py)
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if h.slg_version() != ABI_VERSION:
            raise ImportError("libslgpu ABI version mismatch")
        if AB_LIB is None:
            # provenance: the product library must be the build of the sources beside it
            from . import build as B
            built, want = h.slg_build_id().decode(), B.BUILD_ID_PREFIX.decode() + B.source_digest()
            if built != want:
                raise ImportError(f"{LIB_PATH} was built from other sources ({built}, sources {want}): "
                                  "rebuild it (__graft_entry__.build())")
        _lib = h
    return _lib


def kernel_table() -> dict:
    """``{symbol: present}`` of the fused kernel's instance table (``slg_kernel_table``)."""
    buf = ctypes.create_string_buffer(1 << 16)
    lib().slg_kernel_table(buf, len(buf))
    out = {}
    for line in buf.value.decode().splitlines():
        name, flag = line.split("\t")
        out[name] = flag == "1"
    return out


def last_kernel() -> str:
    """Symbol of the fused kernel instance this thread's last fused launch picked
    (``slg_last_kernel``; "" when none)."""
    buf = ctypes.create_string_buffer(512)
    check(lib().slg_last_kernel(buf, len(buf)))
    return buf.value.decode()


def check(rc: int):
    if rc != SLG_OK:
        msg = lib().slg_last_error().decode(errors="replace")
        if rc == SLG_ERR_NOT_ENOUGH:
            raise ValueError(msg)
        if rc == SLG_ERR_INDEX:
            raise IndexError(msg)
        raise NativeError(rc, msg)


def loaded_hip_runtimes() -> list[str]:
    """Paths of every libamdhip64 mapped into this process (must be exactly one)."""
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                out.add(line.split()[-1])
    return sorted(out)
