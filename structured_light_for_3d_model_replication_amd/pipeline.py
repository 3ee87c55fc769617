"""Batch mode over view folders as a host/GPU pipeline (``process_multi_ply(mode='batch')``,
``server/processing.py:314-334``; the auto-scan layout of ``server/gui.py:1718,1753``).

The reference loops over the view folders one by one: read 40-odd PNGs, decode, triangulate,
write an ASCII PLY.  Here the same work is a pipeline whose stages overlap:

* **read** (thread pool, up to ``depth`` folders ahead): discover the files, decode the frames the
  decode needs straight into a **pinned** host frame stack (native 8-bit gray PNG decoder into the
  stack rows; colour frames into a pinned RGB(A) stack, converted on the device);
* **device decode** (decode stream, issued first): the last folders of a batch of PNG captures
  (:func:`plan_split`, a rate model: the host threads' measured decode rate against one device
  launch's latency) are read as zlib streams only and inflated by ONE GPU launch while the host
  threads decode the others -- the two decoders' rates add;
* **upload** (copy stream): async H2D of a group of up to ``group`` views;
* **reconstruct** (compute stream): device texture (frame 0 replicated, or frame 0's BGR from the
  colour upload), then ONE batched stats launch + ONE fused decode/triangulate launch for the
  group (``BatchReconstructor.run``, ``slg_reconstruct_batch``) -- launched before the previous
  group is collected, so uploads and kernels of consecutive groups overlap;
* **collect**: counts; each view's PLY body formatted on the device (``slg_ply_format``, on a
  stream of its own beside the next group's kernels) and copied into pinned host memory as
  bytes (a cloud with a value the device formatter leaves to the host: its float64 points);
* **write** (``writers`` threads, files in parallel): header + body (byte-identical ASCII PLY;
  ``slg_ply_write`` for host clouds).

Per-folder behaviour is the reference's: folders without images are skipped with its message,
an exception in any stage of one folder is logged as ``❌ Error in <folder>: <msg>`` and the loop
goes on (a failing group launch falls back to one view at a time to find the culprit), and the
progress lines of each folder come out in folder order, each folder's ``✔ Saved`` after its
``-> Saving`` line.  Returns the number of folders that succeeded.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from collections import deque
from concurrent.futures import Future, ThreadPoolExecutor, wait
from dataclasses import dataclass, field


import numpy as np
import torch

from . import _native as N
from . import engine as E
from . import frames as FR
from . import ply as PLY


class PinnedPool:
    """Reusable page-locked host buffers (cudaHostAlloc is slow; a batch reuses a few sizes)."""

    def __init__(self):
        self._free: dict[int, list] = {}
        self._lock = threading.Lock()       # get() on the reader threads, put() on the main one

    def get(self, nbytes: int) -> torch.Tensor:
        with self._lock:
            lst = self._free.get(nbytes)
            if lst:
                return lst.pop()
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)

    def put(self, t: torch.Tensor | None):
        if t is not None:
            with self._lock:
                self._free.setdefault(t.numel(), []).append(t)


@dataclass
class HostView:
    """One view folder read into pinned host memory."""
    folder: str
    n_files: int
    height: int
    width: int
    stride: int
    kind: str                       # "gray": stack holds gray frames; "rgb": RGB(A) frames
    stack: torch.Tensor             # pinned uint8 [F, stride] (gray) or [F, n_px * channels] (rgb)
    channels: int = 1
    weights: int = N.GRAY_PNG       # rgb: libpng (PNG) or OpenCV (BMP) gray weights
    texture: torch.Tensor | None = None   # pinned [n_px, 3] BGR, or None: derived on the device
    pinned: list = field(default_factory=list)   # buffers to return to the pool
    z: tuple | None = None          # kind "png_z": (frame indices, byte offsets, stream lengths)


def _decode_rgb(path) -> np.ndarray:
    """Decoded colour frame as RGB or RGBA bytes [H, W, C] (8-bit), for the device conversion."""
    im = FR._open(path)
    if im is None:
        raise AttributeError("'NoneType' object has no attribute 'astype'")
    a = np.asarray(im)
    if a.dtype == np.uint16:
        a = (a >> 8).astype(np.uint8)
    return a


def device_png_mode() -> str:
    """Which PNG captures the GPU decodes (``slg_png_decode_device``), from SLG_PNG_DEVICE:
    ``"1"`` all of them, ``"0"`` none, unset or ``"auto"`` a share of a batch (the last folders,
    :func:`device_share`) while host threads decode the rest."""
    v = os.environ.get("SLG_PNG_DEVICE", "auto")
    return "all" if v == "1" else "off" if v == "0" else "auto"


def device_png_enabled() -> bool:
    """Whether a lone capture read (:func:`read_view` without ``device_png``) goes to the device
    decoder: only with SLG_PNG_DEVICE=1.  The inflate is one wave per stream, ~225 ms per 1080p
    frame whatever the launch size (profiles/r4n), so one view alone is far faster on
    the host threads."""
    return device_png_mode() == "all"


# ---- the host / device split of the PNG decode: a rate model
# The device inflate is one wave per zlib stream, a serial Huffman chain each, so ONE launch
# takes about its largest stream's time whatever the number of views (~233 ms for
# 1080p gray frames at 10-16 views, tools/png_views_bench.py: 0.99 correlation with the largest
# stream), plus the device group's zlib-stream reads before the launch starts (65-140 ms).  The
# host decodes at (threads / thread-seconds per frame).  The device takes the LAST n_dev folders
# so that the host's own share still lasts at least the device's latency: then the batch ends
# with the host, sooner than host-only; when even the whole batch decodes on the host within
# that latency, n_dev = 0.  The host's rate is measured (RateMeter: every host frame decode is
# timed; the first batch of a process measures its first folder before deciding), the device's
# is updated from every device group's launch, the priors below only seed them.
HOST_S_PER_MB_PRIOR = 2.5e-3    # thread-seconds per MB of raw samples, 8-bit gray PNG on the host
                                # (EPYC 9575F, 16 threads: ~70 C2 views/s, 44 x 2.07 MB each, r6g-r6l)
DEV_S_PER_MB_PRIOR = 0.112      # one inflate launch per MB of its largest frame (233 ms / 2.07 MB, r6e)
DEV_FIXED_S = 0.07              # the device group's zlib-stream reads before its launch (r6l: 65-140 ms)
DEVICE_MAX_VIEWS = 16


class RateMeter:
    """Measured decode rates of this process (thread-safe): host thread-seconds per MB of raw
    samples (each host frame decode timed on its pool thread) and device inflate seconds per MB of
    a launch's largest frame."""

    def __init__(self):
        self._lock = threading.Lock()
        self.host_s = self.host_mb = 0.0
        self.dev_s = self.dev_mb = 0.0

    def add_host(self, seconds: float, mb: float):
        with self._lock:
            self.host_s += seconds
            self.host_mb += mb

    def add_device(self, seconds: float, mb: float):
        with self._lock:
            self.dev_s += seconds
            self.dev_mb += mb

    def host_measured(self) -> bool:
        return self.host_mb >= 8.0                  # a few frames' worth

    def host_s_per_mb(self) -> float:
        return self.host_s / self.host_mb if self.host_measured() else HOST_S_PER_MB_PRIOR

    def dev_s_per_mb(self) -> float:
        return self.dev_s / self.dev_mb if self.dev_mb > 0 else DEV_S_PER_MB_PRIOR


RATES = RateMeter()


@dataclass
class SplitPlan:
    """What :func:`plan_split` decided and why (logged in the pipeline stats)."""
    n_dev: int
    host_s_per_folder: float
    device_s: float
    cap: int
    threads: int


def device_view_cap(frames_per_folder: int, n_cus: int) -> int:
    """Most views one device launch takes at a CU-mask stride measured to keep it at one launch
    latency (:func:`png_reserve_every` != 0): 15 C2 views of 44 streams at stride 8 on 256 CUs
    (at 16 views the streams no longer fit any measured-good stride)."""
    n = DEVICE_MAX_VIEWS
    while n > 0 and png_reserve_every(n * max(1, frames_per_folder), n_cus) == 0:
        n -= 1
    return n


def plan_split(n_folders: int, frames_per_folder: int, frame_mb: float, threads: int, host_s_per_mb: float,
               dev_s_per_mb: float, n_cus: int, dev_fixed_s: float = DEV_FIXED_S) -> SplitPlan:
    """Device share of a batch: the largest n_dev <= the launch cap whose remaining host share
    takes at least the device's latency (0 when the host finishes the whole batch sooner)."""
    threads = max(1, int(threads))
    per_folder = frames_per_folder * frame_mb * host_s_per_mb / threads
    device_s = dev_fixed_s + frame_mb * dev_s_per_mb
    cap = device_view_cap(frames_per_folder, n_cus)
    n_dev = 0
    if per_folder > 0:
        import math
        n_dev = n_folders - math.ceil(device_s / per_folder)
    return SplitPlan(max(0, min(cap, n_dev)), per_folder, device_s, cap, threads)


_DECODE_STREAMS: dict = {}
PNG_WAVES_PER_CU = 3        # png_inflate_kernel: one 64-lane wave per stream, ~50 KB of LDS each


PNG_RESERVE_CHOICES = (3, 4, 8)   # CU-mask strides measured to keep the inflate at one launch latency


def png_reserve_every(n_streams: int | None, n_cus: int) -> int:
    """Every how-many-th CU the device PNG decode leaves to the other launches: the smallest
    stride of ``PNG_RESERVE_CHOICES`` whose complement still holds all ``n_streams`` inflate waves
    at once (``PNG_WAVES_PER_CU`` each), else 0 (a plain stream); 8 when the count is unknown.
    The mask's CU numbering is the runtime's, not a plain CU index: strides 3, 4 and 8 kept a 10-
    to 16-view launch at ~220 ms, while 6, 12 and 16 doubled it (370-390 ms) at counts that fit
    on paper (tools/png_views_bench.py, profiles/r6e).  Leaving CUs out matters: with 16 free CUs
    an 8-view group's fused launches took ~100 ms instead of ~8 (profiles/r5p).
    SLG_PNG_RESERVE_EVERY overrides."""
    env = os.environ.get("SLG_PNG_RESERVE_EVERY")
    if env is not None:
        return int(env)
    if not n_streams:
        return 8
    for k in PNG_RESERVE_CHOICES:
        if (n_cus - n_cus // k) * PNG_WAVES_PER_CU >= n_streams:
            return k
    return 0                                         # more streams than fit: no CU left out


def png_decode_stream(device: int | None = None, n_streams: int | None = None):
    """The device PNG decode's stream, one per GPU and CU mask for the process: every k-th CU
    (:func:`png_reserve_every`) left out of its CU mask (``slg_stream_create_reserving``), so the
    inflate launch -- ~250-400 ms, one wave per stream -- leaves those CUs to the fused launches
    of the host-decoded views (their 72 KB of LDS per workgroup fit on no CU the inflate's 50 KB
    waves hold); a plain stream when the mask cannot be set."""
    dev = torch.cuda.current_device() if device is None else int(device)
    every = png_reserve_every(n_streams, torch.cuda.get_device_properties(dev).multi_processor_count)
    s = _DECODE_STREAMS.get((dev, every))
    if s is None:
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            if every >= 2 and N.lib().slg_stream_create_reserving(every, ctypes.byref(h)) == 0:
                s = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", dev))
            else:
                s = torch.cuda.Stream(device=dev)
        _DECODE_STREAMS[(dev, every)] = s
    return s


def _layout(folder: str, cfg: E.DecodeConfig, order=("bmp", "png")):
    """(frames the decode reads, MB of raw samples per frame, the device decoder takes them) of a
    capture folder, from its file list and first PNG header (no decode)."""
    from .processing import _needed_frames
    files = FR.discover(folder, order)
    if len(files) < 4 or not FR._is_png(files[0]):
        return 0, 0.0, False
    info = (ctypes.c_int32 * 7)()
    if N.lib().slg_png_info(os.fsencode(files[0]), info) != 0:
        return 0, 0.0, False
    ch = {0: 1, 2: 3, 4: 2, 6: 4}.get(info[2], 0)
    need = _needed_frames(len(files), cfg) if cfg.variant == "processing" else list(range(len(files)))
    device_ok = ch > 0 and info[3] == 8 and info[4] == 0 and info[0] * ch <= 24576
    return len(need), info[0] * info[1] * max(ch, 1) / 1e6, device_ok


def device_share(n_folders: int, mode: str | None = None, layout=None, threads: int | None = None) -> int:
    """Folders (the last ones of the batch) whose PNG frames the GPU decodes: all / none when
    forced (SLG_PNG_DEVICE=1 / 0), else :func:`plan_split` on ``layout`` = (frames per folder, MB
    per frame, device-decodable) with the measured rates (SLG_PNG_HOST_AHEAD=k: the last n - k
    folders, for A/B runs)."""
    mode = device_png_mode() if mode is None else mode
    if mode == "off":
        return 0
    if mode == "all":
        return n_folders
    env = os.environ.get("SLG_PNG_HOST_AHEAD")
    if env is not None:
        return max(0, min(DEVICE_MAX_VIEWS, n_folders - int(env)))
    if not layout or not layout[2]:
        return 0
    n_cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return plan_split(n_folders, layout[0], layout[1], threads or FR.decode_threads(), RATES.host_s_per_mb(),
                      RATES.dev_s_per_mb(), n_cus).n_dev


_Z_POOL: list = []
_Z_POOL_LOCK = threading.Lock()


def _z_pool() -> ThreadPoolExecutor:
    """The zlib-stream readers' pool (file read + chunk CRCs: light on CPU, kept off the decode
    pool's queue)."""
    with _Z_POOL_LOCK:
        if not _Z_POOL:
            _Z_POOL.append(ThreadPoolExecutor(max_workers=8, thread_name_prefix="slg-zread"))
        return _Z_POOL[0]


def read_view_z(folder: str, files, need, pool: PinnedPool) -> HostView | None:
    """Host half of the device PNG decode: the used frames' zlib streams (``slg_png_zstream``:
    file read + chunk CRCs, no inflate) packed into one pinned buffer, 256-byte aligned each.
    None when a used frame is not an 8-bit gray / RGB / RGBA PNG of one common size (the view is
    then decoded on the host the general way)."""
    if not all(files[i].lower().endswith(".png") for i in need):
        return None
    L = N.lib()
    caps = [(os.path.getsize(files[i]) + 8 + 255) // 256 * 256 for i in need]
    offs = [0]
    for c in caps:
        offs.append(offs[-1] + c)
    buf = pool.get(offs[-1])
    base = buf.data_ptr()
    infos = [(ctypes.c_int32 * 4)() for _ in need]

    def one(k):
        return L.slg_png_zstream(os.fsencode(files[need[k]]), ctypes.c_void_p(base + offs[k]), caps[k], infos[k])
    try:
        # on a pool of their own: queued behind the host decoders' frames on the shared decode
        # pool, the device group's streams (and so its launch) came later (profiles/r6k)
        futs = [_z_pool().submit(one, k) for k in range(len(need))]
        wait(futs)
        rcs = [f.result() for f in futs]
    except BaseException:
        pool.put(buf)                   # (a file vanished, an executor error): the buffer goes back
        raise
    shapes = {tuple(i[:3]) for i in infos}
    if any(rcs) or len(shapes) != 1 or next(iter(shapes))[2] not in (1, 3, 4):
        pool.put(buf)
        return None
    W, H, C = next(iter(shapes))
    return HostView(folder, len(files), H, W, (H * W + 15) // 16 * 16, "png_z", buf, channels=C, pinned=[buf],
                    z=(list(need), offs[:-1], [int(i[3]) for i in infos]))


def read_view(folder: str, cfg: E.DecodeConfig, pool: PinnedPool, order=("bmp", "png"),
              device_png: bool | None = None) -> HostView:
    """Discover + read one capture into pinned memory (host work only; safe on any thread):
    PNG captures as their zlib streams for the device decoder (``device_png``, default
    :func:`device_png_enabled`), anything else decoded on the host."""
    from .processing import _needed_frames
    files = FR.discover(folder, order)
    if len(files) < 4:
        raise ValueError(f"Not enough images (got {len(files)}, need at least 4).")
    need = _needed_frames(len(files), cfg) if cfg.variant == "processing" else list(range(len(files)))
    if device_png if device_png is not None else device_png_enabled():
        hv = read_view_z(folder, files, need, pool)
        if hv is not None:
            return hv
    L = N.lib()
    w, h = ctypes.c_int32(), ctypes.c_int32()
    gray8 = (files[0].lower().endswith(".png")
             and L.slg_png_gray8_size(os.fsencode(files[0]), ctypes.byref(w), ctypes.byref(h)) == 0)
    workers = min(FR.decode_threads(), len(need))
    if gray8:
        H, W = h.value, w.value
        n_px = H * W
        stride = (n_px + 15) // 16 * 16
        buf = pool.get(len(files) * stride)
        stack = buf.view(len(files), stride)
        base = stack.data_ptr()

        def one(i):
            p = files[i]
            dst = base + i * stride
            t = time.perf_counter()
            if L.slg_png_gray8_decode(os.fsencode(p), ctypes.c_void_p(dst), n_px, W, H) == 0:
                RATES.add_host(time.perf_counter() - t, n_px / 1e6)
                return
            a = FR.imread_gray(p)                   # any other file: the general decoder
            if a.shape != (H, W):
                raise ValueError("all frames must have the same size")
            stack[i, :n_px].numpy()[:] = a.reshape(-1)
        try:
            FR.decode_all(one, need)
        except BaseException:
            pool.put(buf)                 # (every decode has stopped writing into it)
            raise
        return HostView(folder, len(files), H, W, stride, "gray", stack, pinned=[buf])
    if FR._is_png(files[0]):
        return _read_png_general(folder, files, need, pool)
    # colour (or non-PNG) captures: decoded RGB(A) frames, converted to gray on the device
    first = _decode_rgb(files[0])
    if first.ndim == 2:                               # a gray file the fast path does not take
        imgs, tex = FR.load_frames(files, need, texture=True)
        H, W = imgs[0].shape
        n_px = H * W
        stride = (n_px + 15) // 16 * 16
        buf = pool.get(len(files) * stride)
        stack = buf.view(len(files), stride)
        for i, a in zip(need, imgs):
            if a.shape != (H, W):
                raise ValueError("all frames must have the same size")
            stack[i, :n_px].numpy()[:] = a.reshape(-1)
        tbuf = pool.get(n_px * 3)
        tbuf.view(n_px, 3).numpy()[:] = tex.reshape(n_px, 3)
        return HostView(folder, len(files), H, W, stride, "gray", stack, texture=tbuf.view(n_px, 3),
                        pinned=[buf, tbuf])
    H, W, C = first.shape[0], first.shape[1], min(first.shape[2], 4)
    if C < 3:
        raise ValueError(f"unsupported image layout {first.shape}")
    n_px = H * W
    buf = pool.get(len(files) * n_px * C)
    stack = buf.view(len(files), n_px * C)

    def one(i):
        a = first if i == 0 else _decode_rgb(files[i])
        if a.ndim != 3 or a.shape[0] != H or a.shape[1] != W or min(a.shape[2], 4) != C:
            raise ValueError("all frames must have the same size and layout")
        stack[i].numpy()[:] = a[..., :C].reshape(-1)          # pinned host tensor: plain memcpy
    with ThreadPoolExecutor(max_workers=workers) as ex:
        list(ex.map(one, need))
    weights = N.GRAY_BMP if files[0].lower().endswith(".bmp") else N.GRAY_PNG
    return HostView(folder, len(files), H, W, (n_px + 15) // 16 * 16, "rgb", stack, channels=C,
                    weights=weights, pinned=[buf])


def _read_png_general(folder: str, files, need, pool: PinnedPool) -> HostView:
    """Any PNG capture the gray fast path does not take (colour / RGBA phone captures, 16-bit,
    palette, Adam7, gAMA / sRGB / iCCP tagged): every used frame decoded on the host threads
    straight into the pinned gray stack, as cv2.imread(f, 0) returns it, and frame 0's
    cv2.imread(f) into the pinned texture (``slg_png_read``, pinned to libpng with OpenCV's calls).
    A gray file's texture is its frame 0 replicated: GRAY texture mode, no texture buffer."""
    L = N.lib()
    info0 = (ctypes.c_int32 * 7)()
    if L.slg_png_info(os.fsencode(files[0]), info0) != 0:
        raise AttributeError("'NoneType' object has no attribute 'astype'")   # cv2.imread -> None
    W, H, color = info0[0], info0[1], bool(info0[2] & 2)
    n_px = H * W
    stride = (n_px + 15) // 16 * 16
    buf = pool.get(len(files) * stride)
    stack = buf.view(len(files), stride)
    base = stack.data_ptr()
    tbuf = pool.get(n_px * 3) if color else None
    order = list(need) if (0 in need or not color) else [0] + list(need)

    mb = n_px * {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}.get(info0[2], 1) * max(1, info0[3] // 8) / 1e6

    def one(i):
        info = (ctypes.c_int32 * 7)()
        tex = i == 0 and tbuf is not None
        t = time.perf_counter()
        rc = L.slg_png_read(os.fsencode(files[i]), ctypes.c_void_p(base + i * stride), n_px,
                            ctypes.c_void_p(tbuf.data_ptr()) if tex else None, 3 * n_px if tex else 0, info)
        if rc != 0:
            if L.slg_png_info(os.fsencode(files[i]), info) == 0 and (info[0], info[1]) != (W, H):
                raise ValueError("all frames must have the same size")
            raise AttributeError("'NoneType' object has no attribute 'astype'")
        if (info[0], info[1]) != (W, H):
            raise ValueError("all frames must have the same size")
        RATES.add_host(time.perf_counter() - t, mb)
    try:
        FR.decode_all(one, order)
    except BaseException:
        pool.put(buf)
        pool.put(tbuf)
        raise
    return HostView(folder, len(files), H, W, stride, "gray", stack, texture=tbuf.view(n_px, 3) if color else None,
                    pinned=[buf] + ([tbuf] if color else []))


def _gray_mode(hv: HostView) -> bool:
    """Whether a HostView's texture is its frame 0 replicated (gray stack without an explicit
    texture, or a one-channel PNG for the device decoder): the GRAY texture mode."""
    return (hv.kind == "gray" and hv.texture is None) or (hv.kind == "png_z" and hv.channels == 1)


def upload_views(hvs, stream, marks=None) -> list:
    """Async H2D of HostViews on ``stream`` (pinned sources) + the device textures: none for
    gray captures (GRAY mode: the kernels take frame 0), frame 0's BGR for colour ones
    (``slg_rgb_to_gray``).  The PNG captures (kind "png_z") of the list are decoded by ONE
    ``slg_png_decode_device`` launch over all their frames (a view's 44 streams alone leave the
    GPU nearly idle: the decode is one wave per stream).  The host buffers must stay alive until
    ``stream`` reaches here.  Returns the DeviceFrames in order."""
    sp = ctypes.c_void_p(stream.cuda_stream)
    L = N.lib()
    with torch.cuda.stream(stream):
        # allocated on `stream` (its pool in the caching allocator): if a later step raises, the
        # buffers freed here can only be handed out again behind the work already queued on it
        # gray captures whose texture is frame 0 (the 8-bit gray PNGs the reference's scanner
        # writes) run in GRAY texture mode: no texture buffer, the kernels take frame 0's bytes
        devs = [E.DeviceFrames.allocate(hv.n_files, hv.height, hv.width, gray=_gray_mode(hv)) for hv in hvs]
        pngs = [(hv, dev) for hv, dev in zip(hvs, devs) if hv.kind == "png_z"]
        if pngs:
            decode_png_device(pngs, stream, marks)
        for hv, dev in zip(hvs, devs):
            if hv.kind == "gray":
                dev.data[: hv.n_files].copy_(hv.stack, non_blocking=True)
                if hv.texture is not None:
                    dev.texture.copy_(hv.texture, non_blocking=True)
            elif hv.kind == "rgb":
                rgb = torch.empty(hv.stack.shape, dtype=torch.uint8, device=dev.data.device)
                rgb.copy_(hv.stack, non_blocking=True)
                N.check(L.slg_rgb_to_gray(ctypes.c_void_p(rgb.data_ptr()), hv.channels, dev.n_px,
                                          rgb.shape[1], hv.n_files, ctypes.c_void_p(dev.data.data_ptr()),
                                          dev.stride, ctypes.c_void_p(dev.texture.data_ptr()), hv.weights, sp))
                dev._rgb = rgb                          # keep the staging alive with the frames
    return devs


def upload_view(hv: HostView, stream) -> E.DeviceFrames:
    """:func:`upload_views` of one view."""
    return upload_views([hv], stream)[0]


def decode_png_device(pngs, stream, marks=None) -> None:
    """Device half of the PNG decode for [(HostView "png_z", DeviceFrames)]: H2D of the zlib
    streams, inflate + un-filter on the GPU (``slg_png_decode_device``, one launch for every
    frame of every view) straight into the frame stacks (gray) or into RGB(A) staging stacks that
    ``slg_rgb_to_gray`` converts, then the textures.  Enqueued on ``stream`` (current); each
    view's ``dev._png_status`` (device int32 [2 * frames]) says whether the host must redo it."""
    L = N.lib()
    sp = ctypes.c_void_p(stream.cuda_stream)
    device = pngs[0][1].data.device
    n_all = sum(len(hv.z[0]) for hv, _ in pngs)
    descs = (N.PngFrame * n_all)()
    status = torch.zeros(2 * n_all, dtype=torch.int32, device=device)
    keep, k0 = [], 0
    for hv, dev in pngs:
        need, offs, zlens = hv.z
        n, C, n_px = len(need), hv.channels, hv.height * hv.width
        zdev = torch.empty(hv.stack.numel(), dtype=torch.uint8, device=device)
        zdev.copy_(hv.stack, non_blocking=True)
        raw_b = int(L.slg_png_raw_bytes(hv.width, hv.height, C))
        raw = torch.empty(n * raw_b, dtype=torch.uint8, device=device)
        rgb = torch.empty((hv.n_files, n_px * C), dtype=torch.uint8, device=device) if C > 1 else None
        for k, i in enumerate(need):
            out = dev.data[i] if C == 1 else rgb[i]
            descs[k0 + k] = N.PngFrame(z=zdev.data_ptr() + offs[k], zlen=zlens[k], raw=raw.data_ptr() + k * raw_b,
                                       out=out.data_ptr(), out_pitch=hv.width * C, width=hv.width,
                                       height=hv.height, channels=C, reserved=0)
        dev._png_status = status[2 * k0: 2 * (k0 + n)]
        dev._png_keep = (zdev, raw, rgb)                 # alive until the view is collected
        keep.append((hv, dev, rgb))
        k0 += n
    # the descriptors go up from pageable memory (a small staged copy): pinning them here
    # allocated page-locked memory on every call
    dbytes = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(descs), ctypes.sizeof(descs))),
                              dtype=torch.uint8)
    ddev = dbytes.to(device, non_blocking=True)
    if marks is not None:
        marks.append(torch.cuda.Event(enable_timing=True))
        marks[-1].record(stream)
    N.check(L.slg_png_decode_device(ctypes.c_void_p(ddev.data_ptr()), n_all, ctypes.c_void_p(status.data_ptr()), sp))
    if marks is not None:
        marks.append(torch.cuda.Event(enable_timing=True))
        marks[-1].record(stream)
    for hv, dev, rgb in keep:
        if rgb is None:
            pass                                         # gray: GRAY texture mode (frame 0)
        else:
            N.check(L.slg_rgb_to_gray(ctypes.c_void_p(rgb.data_ptr()), hv.channels, dev.n_px, rgb.shape[1],
                                      hv.n_files, ctypes.c_void_p(dev.data.data_ptr()), dev.stride,
                                      ctypes.c_void_p(dev.texture.data_ptr()), N.GRAY_PNG, sp))
        dev._png_desc = (dbytes, ddev)                   # the descriptors, until the launch ran


def png_failed(dev: E.DeviceFrames) -> bool:
    """Whether any frame of a device-decoded capture needs the host decoder (call after sync)."""
    st = getattr(dev, "_png_status", None)
    return st is not None and bool((st.view(-1, 2)[:, 0] != 0).any().item())


@dataclass
class FormattedCloud:
    """A view's PLY body formatted on the device (``slg_ply_format``), in pinned host memory."""
    n_points: int
    body: torch.Tensor              # pinned uint8, the first `length` bytes are the body
    length: int
    pool: PinnedPool
    released: bool = False

    def write(self, filename) -> None:
        try:
            PLY.write_body(filename, self.n_points, self.body[: self.length].numpy())
        finally:
            self.release()

    def release(self) -> None:
        """Return the pinned body to the pool (once; later calls do nothing)."""
        if not self.released:
            self.released = True
            self.pool.put(self.body)


def n_points(result) -> int:
    """Points of a collected view: a FormattedCloud or a host (P, C) pair."""
    return result.n_points if isinstance(result, FormattedCloud) else len(result[0])


@dataclass
class _Group:
    entries: list                   # [(folder, future | None)] in folder order (None: skipped)
    views: list = field(default_factory=list)   # [(index in entries, HostView, DeviceFrames)]
    errors: dict = field(default_factory=dict)  # entry index -> exception
    event: object = None
    batch: object = None
    clouds: list = field(default_factory=list)
    uploaded: object = None         # device-decoded group: the event its uploads + inflate end on
    gpu_events: tuple = None        # (start, end) around its reconstruct launches


class PipelineStats:
    """Busy time per stage of one :meth:`BatchPipeline.run` (seconds; summed over threads for
    the host stages, HIP events for the GPU ones) and the split between the decoders."""

    def __init__(self):
        self._lock = threading.Lock()
        self.read_s = 0.0             # host: file read + decode (or zstream read) into pinned memory
        self.write_s = 0.0            # host: PLY files written
        self.device_decode_ms = 0.0   # GPU: H2D of the zlib streams + inflate + un-filter
        self.device_kernels_ms = 0.0  # GPU: the inflate + un-filter launches alone
        self.device_enqueue_s = 0.0   # host: issuing the device group's uploads and launches
        self.gpu_ms = 0.0             # GPU: reconstruct launches (stats + fused) of every group
        self.folders_host = 0
        self.folders_device = 0
        self.probe_s = 0.0            # host: the first folder decoded before the split was planned
        self.split = None             # the rate model's inputs and decision (plan_split)
        self.wall_s = 0.0
        # SLG_PIPE_TRACE=1: a timeline of (stage, thread, start_s, end_s, what) from the run's
        # start -- host spans from perf_counter, GPU spans from HIP events (tools/e2e_files.py)
        self.trace = [] if os.environ.get("SLG_PIPE_TRACE") else None
        self.t0 = time.perf_counter()
        self.ev0 = None

    def span(self, name: str, t0: float, t1: float, what: str = ""):
        if self.trace is not None:
            with self._lock:
                self.trace.append((name, threading.current_thread().name, round(t0 - self.t0, 5),
                                   round(t1 - self.t0, 5), what))

    def gpu_span(self, name: str, a, b, what: str = ""):
        """A GPU span between two completed timing events (recorded after ``ev0``)."""
        if self.trace is not None and self.ev0 is not None:
            t0 = self.ev0[1] + self.ev0[0].elapsed_time(a) * 1e-3
            self.span(name, t0, t0 + a.elapsed_time(b) * 1e-3, what)

    def add(self, key: str, v: float):
        with self._lock:
            setattr(self, key, getattr(self, key) + v)

    def as_dict(self) -> dict:
        return {"wall_s": round(self.wall_s, 4), "read_busy_s": round(self.read_s, 4),
                "write_busy_s": round(self.write_s, 4), "device_decode_ms": round(self.device_decode_ms, 3),
                "device_kernels_ms": round(self.device_kernels_ms, 3),
                "device_enqueue_ms": round(self.device_enqueue_s * 1e3, 2),
                "gpu_reconstruct_ms": round(self.gpu_ms, 3), "folders_host_decoded": self.folders_host,
                "folders_device_decoded": self.folders_device, "probe_ms": round(self.probe_s * 1e3, 2),
                "split": self.split}


LAST_STATS: PipelineStats | None = None     # the stats of the last BatchPipeline.run (tools/e2e_files.py)


class BatchPipeline:
    """The pipeline of this module's docstring for one decode configuration + calibration.

    PNG decode is split between the host threads and the GPU (:func:`device_share`): the last
    folders of the batch are read as zlib streams and decoded by ONE device launch issued at the
    start, on a stream of its own that leaves CUs free (:func:`png_decode_stream`), while the host
    threads decode the others; the device group is reconstructed when the pipeline reaches it,
    in folder order.  PLY files are written by ``writers`` threads (a C2 view's ASCII PLY is
    ~60 MB; profiles/r5e: one writer thread bounded the round-4 pipeline)."""

    def __init__(self, cfg: E.DecodeConfig, calib: dict, row_mode=1, epipolar_tol=2.0, group: int = 8,
                 depth: int | None = None, log=print, order=("bmp", "png"), device_ply: bool = True,
                 writers: int | None = None, device_views: int | None = None):
        if row_mode not in (0, 1, 2):
            raise ValueError("row_mode must be 0, 1 or 2")
        self.cfg, self.calib, self.row_mode, self.tol = cfg, calib, int(row_mode), float(epipolar_tol)
        self.group = max(1, min(int(group), E.MAX_VIEWS_PER_LAUNCH))
        self._depth = depth                          # None: max(2 group, 16), 24 beside a device group
        self.log, self.order = log, order
        self.writers = max(1, int(writers if writers is not None else os.environ.get("SLG_PLY_WRITERS", 8)))
        self.device_views = device_views          # None: device_share() of the batch
        self.pool = PinnedPool()
        self.copy_stream = torch.cuda.Stream()
        self.compute_stream = torch.cuda.Stream()
        self.format_stream = torch.cuda.Stream()     # PLY bodies of group k beside group k+1's kernels
        self.decode_stream = None                    # the device group's H2D + inflate (sized to it)
        self.formatter = PLY.DeviceFormatter()
        self.device_ply = device_ply
        self.engines: dict = {}
        self.tables: dict = {}
        self._slot = 0
        self._max_views = self.group
        self.stats = PipelineStats()

    def _engine(self, h, w):
        key = (h, w)
        if key in self.engines and self.engines[key][0].max_views < self._max_views:
            del self.engines[key]                    # a later batch's device group is larger: rebuild
        if key not in self.engines:
            n = self._max_views
            # made on the compute stream: the default stream shares a hardware queue with the
            # device-decode stream (tools/queue_probe.py, profiles/r5j), whose inflate launch
            # would hold these uploads ~225 ms
            with torch.cuda.stream(self.compute_stream):
                beng = E.BatchReconstructor(h, w, n, slots=2)
                clouds = [[E.Cloud(h * w, self.row_mode, True) for _ in range(n)] for _ in range(2)]
                self.engines[key] = (beng, clouds)
                self.tables[key] = E.DeviceCalib(self.calib, h, w)
        return self.engines[key], self.tables[key]

    def _read(self, folder, device_png: bool) -> HostView:
        t = time.perf_counter()
        try:
            hv = read_view(folder, self.cfg, self.pool, self.order, device_png=device_png)
        finally:
            t1 = time.perf_counter()
            self.stats.add("read_s", t1 - t)
            self.stats.span("read_z" if device_png else "read", t, t1, os.path.basename(folder))
        self.stats.add("folders_device" if hv.kind == "png_z" else "folders_host", 1)
        return hv

    # ---- stages
    def _upload(self, g: _Group, got, stream, marks=None):
        """g.views += the uploads of ``got`` [(entry index, HostView)] on ``stream``: one upload
        (one PNG decode launch) for all of them, or -- when that raises -- view by view, with the
        device decoder's views read again for the host decoder, so a failure stays with its
        folder."""
        try:
            devs = upload_views([hv for _, hv in got], stream, marks) if got else []
            g.views += [(k, hv, d) for (k, hv), d in zip(got, devs)]
        except Exception:  # noqa: BLE001
            # what the failed attempt queued (H2D from the pinned stacks, decode launches) must
            # finish before those stacks are reused or re-read
            stream.synchronize()
            for k, hv in got:
                try:
                    if hv.kind == "png_z":             # the device decoder's views: the host decodes them
                        hv2 = self._read(hv.folder, device_png=False)
                        for t in hv.pinned:
                            self.pool.put(t)
                        hv = hv2
                    g.views.append((k, hv, upload_view(hv, self.copy_stream)))
                except Exception as e:  # noqa: BLE001
                    g.errors[k] = e
                    for t in hv.pinned:
                        self.pool.put(t)

    @staticmethod
    def _results(g: _Group):
        got = []
        for k, (folder, fut) in enumerate(g.entries):
            if fut is None:
                continue
            try:
                got.append((k, fut.result()))
            except Exception as e:  # noqa: BLE001 - per-folder isolation like the reference
                g.errors[k] = e
        return got

    def _start_device_group(self, g: _Group):
        """Upload + inflate the device group's zlib streams now, on the decode stream."""
        got = self._results(g)
        t = time.perf_counter()
        self.decode_stream = png_decode_stream(n_streams=sum(len(hv.z[0]) for _, hv in got if hv.kind == "png_z"))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(self.decode_stream)
        g.marks = []
        self._upload(g, got, self.decode_stream, g.marks)
        ev1.record(self.decode_stream)
        g.uploaded = (ev0, ev1)
        t1 = time.perf_counter()
        self.stats.add("device_enqueue_s", t1 - t)
        self.stats.span("device_enqueue", t, t1)

    def _launch(self, g: _Group):
        """Upload g's views (copy stream; done already for the device group) and launch their
        reconstruction (compute stream)."""
        t = time.perf_counter()
        if g.uploaded is None:
            got = self._results(g)
            self.stats.span("wait_reads", t, time.perf_counter())
            self._upload(g, got, self.copy_stream)
        if not g.views:
            return
        if g.uploaded is not None:
            self.compute_stream.wait_event(g.uploaded[1])
            self.compute_stream.wait_stream(self.copy_stream)     # (a fallback's per-view uploads)
        else:
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            self.compute_stream.wait_event(ev)
        shapes = {(d.height, d.width) for _, _, d in g.views}
        slot = self._slot
        self._slot ^= 1
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record(self.compute_stream)
        try:
            if len(shapes) != 1:
                raise ValueError("views of different sizes")
            (beng, clouds), dc = self._engine(*shapes.pop())
            outs = clouds[slot][: len(g.views)]
            g.batch = beng.prepare([d for _, _, d in g.views], self.cfg, dc, outs, self.row_mode, self.tol, slot=slot)
            beng.run(g.batch, stream=self.compute_stream)
            g.clouds = outs
        except Exception:  # noqa: BLE001 - the group falls back to one view at a time
            g.batch = None
        g1.record(self.compute_stream)
        g.gpu_events = (g0, g1)
        g.event = torch.cuda.Event()
        g.event.record(self.compute_stream)
        self.stats.span("launch", t, time.perf_counter(), f"{len(g.views)} views")

    def _collect(self, g: _Group, ready=None):
        """Results of g's views as host (P float64 [N,3], C uint8 [N,3]) or exceptions.
        ``ready(k, result)``, when given, is called for each device-formatted view as soon as its
        bytes are in host memory (its write can start while the group's later views copy)."""
        res = {}
        if not g.views:
            return res
        t = time.perf_counter()
        g.event.synchronize()
        t_sync = time.perf_counter()
        self.stats.span("wait_gpu", t, t_sync)
        self.stats.add("gpu_ms", g.gpu_events[0].elapsed_time(g.gpu_events[1]))
        self.stats.gpu_span("gpu_reconstruct", *g.gpu_events, f"{len(g.views)} views")
        if g.uploaded is not None:
            self.stats.add("device_decode_ms", g.uploaded[0].elapsed_time(g.uploaded[1]))
            self.stats.gpu_span("gpu_device_decode", *g.uploaded)
            if len(getattr(g, "marks", ())) == 2:         # the inflate + un-filter launches alone
                ms = g.marks[0].elapsed_time(g.marks[1])
                self.stats.add("device_kernels_ms", ms)
                self.stats.gpu_span("gpu_inflate", *g.marks)
                mb = max((hv.width * hv.height * hv.channels / 1e6 for _, hv, _ in g.views if hv.kind == "png_z"),
                         default=0.0)
                if mb > 0:
                    RATES.add_device(ms / 1e3, mb)          # the launch's latency per MB of its largest frame
        from .processing import reconstruct_view
        with torch.cuda.stream(self.format_stream):
            redo = {k for k, _, dev in g.views if png_failed(dev)}
        for k, hv, dev in g.views:               # a frame the device decoder refused: the host decodes
            if k in redo:                        # the whole view again (general path) and runs it alone
                try:
                    hv2 = self._read(hv.folder, device_png=False)
                    try:
                        dev2 = upload_view(hv2, self.copy_stream)
                        self.copy_stream.synchronize()
                        (_, _), dc = self._engine(dev2.height, dev2.width)
                        res[k] = reconstruct_view(dev2, self.cfg, self.calib, self.row_mode, self.tol, dc=dc)
                    finally:
                        for b in hv2.pinned:
                            self.pool.put(b)
                except Exception as e:  # noqa: BLE001
                    res[k] = e
        if g.batch is not None:
            # the reads and copies go on the format stream, not the default one: a stream that
            # shares its hardware queue with the device-decode stream (4 queues per process)
            # would hold them behind a ~225 ms inflate launch
            with torch.cuda.stream(self.format_stream):
                for (k, hv, _), c in zip(g.views, g.clouds):
                    if k in redo:
                        continue
                    n = int(c.count.item())
                    body = self.formatter.body(c.xyz[:n], c.bgr[:n], self.format_stream) if self.device_ply else None
                    if body is None:                    # host formatting (or a value it must print)
                        res[k] = (c.xyz[:n].cpu().numpy(), c.bgr[:n].cpu().numpy())
                    else:                               # the PLY body leaves HBM as bytes
                        host = self.pool.get((body.numel() + (16 << 20) - 1) // (16 << 20) * (16 << 20))
                        host[: body.numel()].copy_(body)
                        res[k] = FormattedCloud(n, host, body.numel(), self.pool)
                        if ready is not None:
                            ready(k, res[k])
        else:                                       # isolate the failing view(s)
            for k, hv, dev in g.views:
                if k in redo:
                    continue
                try:
                    (_, _), dc = self._engine(dev.height, dev.width)
                    res[k] = reconstruct_view(dev, self.cfg, self.calib, self.row_mode, self.tol, dc=dc)
                except Exception as e:  # noqa: BLE001
                    res[k] = e
        for _, hv, _ in g.views:                    # uploads are complete: recycle the host buffers
            for b in hv.pinned:
                self.pool.put(b)
        self.stats.span("format_d2h", t_sync, time.perf_counter(), f"{len(g.views)} views")
        return res

    def run(self, subfolders, write) -> int:
        """Process ``subfolders`` in order; ``write(folder, (P, C)) -> output name``."""
        global LAST_STATS
        from .processing import has_images
        t_run = time.perf_counter()
        self.stats = LAST_STATS = PipelineStats()
        if self.stats.trace is not None:             # the GPU spans' time base
            self.stats.ev0 = (torch.cuda.Event(enable_timing=True), 0.0)
            torch.cuda.synchronize()
            self.stats.ev0[0].record(self.compute_stream)
            self.stats.ev0 = (self.stats.ev0[0], time.perf_counter())
        entries = [(f, has_images(f)) for f in subfolders]
        success = 0
        order = [f for f, ok in entries if ok]
        mode = device_png_mode()
        pre = {}                                    # folder -> its read, done before the split
        if self.device_views is not None:
            n_dev = max(0, min(int(self.device_views), len(order)))
        elif mode == "auto" and len(order) > 1 and "SLG_PNG_HOST_AHEAD" not in os.environ:
            layout = _layout(order[0], self.cfg, self.order)
            if layout[2] and not RATES.host_measured():
                # no host rate measured in this process yet: the first folder (read first anyway)
                # is decoded now and timed, then the split is planned on that rate
                t = time.perf_counter()
                fut = Future()
                try:
                    fut.set_result(self._read(order[0], False))
                except Exception as e:  # noqa: BLE001 - the folder's error is reported in order
                    fut.set_exception(e)
                pre[order[0]] = fut
                self.stats.add("probe_s", time.perf_counter() - t)
            n_dev = device_share(len(order) - len(pre), mode, layout)
            self.stats.split = {"n_dev": n_dev, "folders": len(order), "frames_per_folder": layout[0],
                                "mb_per_frame": round(layout[1], 3), "device_ok": layout[2],
                                "threads": FR.decode_threads(), "host_s_per_mb": round(RATES.host_s_per_mb(), 6),
                                "dev_s_per_mb": round(RATES.dev_s_per_mb(), 4)}
        else:
            n_dev = device_share(len(order), mode)
        if mode == "all" and self.device_views is None:
            n_dev = 0                               # every group is read for the device decoder
        if n_dev:
            self._max_views = max(self.group, n_dev)
        # read-ahead: the host keeps decoding while the device group's inflate holds most CUs
        self.depth = self._depth or int(os.environ.get("SLG_PIPE_DEPTH", 0)) or (
            max(2 * self.group, 24) if n_dev else max(2 * self.group, 16))
        dev_first = len(order) - n_dev              # the device group: the last n_dev image folders
        cut = len(entries)
        if n_dev:
            cut = next(i for i, (f, ok) in enumerate(entries) if ok and f == order[dev_first])

        def timed_write(folder, result):
            t = time.perf_counter()
            try:
                return write(folder, result)
            finally:
                t1 = time.perf_counter()
                self.stats.add("write_s", t1 - t)
                self.stats.span("write", t, t1, os.path.basename(folder))

        # the device group's zlib-stream reads (file read + CRCs, no inflate) on a pool of their
        # own, so they do not queue behind the host decoders' folders (or these behind them)
        zpool = ThreadPoolExecutor(max_workers=4) if n_dev else None
        try:
            success = self._run_groups(entries, order, mode, n_dev, cut, zpool, timed_write, pre)
        finally:
            if zpool is not None:
                zpool.shutdown()
        self.stats.wall_s = time.perf_counter() - t_run
        return success

    def _run_groups(self, entries, order, mode, n_dev, cut, zpool, timed_write, pre=None) -> int:
        """The group loop of :meth:`run` (reads, device group, launches, collects, writes);
        ``pre``: folder -> the future of a read already done."""
        success = 0
        dev_first = len(order) - n_dev
        with ThreadPoolExecutor(max_workers=2) as reader, ThreadPoolExecutor(max_workers=self.writers) as writer:
            futs = dict(pre or {})
            all_dev = mode == "all"
            dev_group = None
            if n_dev:                                # the device group's zlib streams first: its
                ents = entries[cut:]                 # launch starts while the host decodes the rest
                dev_group = _Group([(f, zpool.submit(self._read, f, True) if ok else None) for f, ok in ents])
            host_order = order[:dev_first]
            nxt = 0

            def prefetch(upto):
                nonlocal nxt
                while nxt < len(host_order) and nxt < upto:
                    if host_order[nxt] not in futs:
                        futs[host_order[nxt]] = reader.submit(self._read, host_order[nxt], all_dev)
                    nxt += 1

            # host groups: consecutive entries holding up to `group` folders with images
            groups, cur, n_img = [], [], 0
            for f, ok in entries[:cut]:
                cur.append((f, ok))
                n_img += ok
                if n_img == self.group:
                    groups.append(cur)
                    cur, n_img = [], 0
            if cur:
                groups.append(cur)
            if dev_group is not None:
                # the inflate launch is enqueued as soon as the device group's streams are read;
                # the host decoders start meanwhile (the whole read-ahead: two reader threads at
                # most, so the z reads keep CPUs; holding them back measured slower, r6l)
                prefetch(self.depth)
                self._start_device_group(dev_group)
            prefetch(self.depth)
            done_imgs = 0
            prev = None
            todo = list(groups)                    # host groups as entry lists (made when reached)
            if dev_group is not None:
                todo.append(dev_group)
            # groups whose PLYs are being written: their log lines go out in folder order once
            # their writes are done; the loop blocks on the oldest only past `max_writing` views
            # (blocking on every group serialised its writes with the next group's collect:
            # ~10 ms per C2 view, profiles/r5n)
            writing: deque = deque()
            max_writing = max(3 * self.writers, 2 * self.group)

            def flush(block_until: int):
                nonlocal success
                t = time.perf_counter()
                while writing and (sum(len(o) for _, o in writing) > block_until
                                   or all(wf is None or wf.done() for _, wf, _ in writing[0][1].values())):
                    success += self._log_group(*writing.popleft())
                if time.perf_counter() - t > 1e-4:
                    self.stats.span("report_wait", t, time.perf_counter())

            for gi, item in enumerate(todo + [None]):
                g = None
                if isinstance(item, _Group):
                    g = item
                elif item is not None:
                    g = _Group([(f, futs.pop(f) if ok else None) for f, ok in item])
                if g is not None:
                    self._launch(g)
                if prev is not None:
                    early = {}                     # entry index -> its write, started early

                    def ready(k, r, g=prev, early=early):
                        early[k] = writer.submit(timed_write, g.entries[k][0], r)
                    res = self._collect(prev, ready)
                    done_imgs += sum(1 for _, fut in prev.entries if fut is not None)
                    prefetch(done_imgs + self.depth)
                    writing.append((prev, self._submit_writes(prev, res, timed_write, writer, early)))
                    flush(max_writing)
                prev = g
            flush(-1)
        return success

    @staticmethod
    def _submit_writes(g: _Group, res, write, writer, early=None) -> dict:
        """Start the group's PLY writes (writer threads) not started yet (``early``: entry index
        -> a write already started by :meth:`_collect`): entry index -> (result, write future or
        None, error)."""
        early = early or {}
        outcome = {}
        for k, (folder, fut) in enumerate(g.entries):
            if fut is None:
                continue
            err = g.errors.get(k)
            r = res.get(k) if err is None else None
            if err is None and isinstance(r, Exception):
                err = r
            if err is not None:
                wf = None
            else:
                wf = early[k] if k in early else writer.submit(write, folder, r)
            outcome[k] = (r, wf, err)
        return outcome

    def _log_group(self, g: _Group, outcome: dict) -> int:
        """The group's log lines (after its writes) in exactly the reference's order per folder:
        Decoding, then Reconstructing / Saving / ✔ Saved, or the ❌ Error line.  Returns the
        folders that succeeded."""
        log, ok, cfg = self.log, 0, self.cfg
        for k, (folder, fut) in enumerate(g.entries):
            name = os.path.basename(folder)
            if fut is None:
                log(f"  Skipping {name} (No images found).")
                continue
            log(f"  -> Decoding folder '{name}'  [col-sets={cfg.n_sets_col}  row-sets={cfg.n_sets_row}]...")
            r, wf, err = outcome[k]
            if err is None:
                log("  -> Reconstructing 3D points...")
                log(f"  -> Saving {n_points(r)} points...")
                try:
                    out = wf.result()
                    ok += 1
                    log(f"  ✔ Saved: {out}\n")
                    continue
                except Exception as e:  # noqa: BLE001
                    err = e
                finally:                # a write stage that never called r.write() (or failed
                    if isinstance(r, FormattedCloud):   # before it) still returns the buffer
                        r.release()
            log(f"  ❌ Error in {name}: {err}\n")
        return ok
