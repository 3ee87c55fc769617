"""Drop-in for the hot path of ``server/processing.py`` (class ``ProcessingLogic``).

Same names, signatures, return types and error behaviour as the reference
(``server/processing.py:27-334``); the arithmetic runs in the HIP kernels of ``libslgpu.so``.
Only the reconstruction path is provided — the Open3D post-processing methods of the
reference class (``remove_background`` ... ``mesh_360``, processing.py:336-860) are out of
scope.
"""
from __future__ import annotations

import collections
import glob
import os

import numpy as np
import torch

from . import engine as E
from . import frames as FR
from . import ply as PLY

_ENGINES: dict = {}
_CALIBS: "collections.OrderedDict" = collections.OrderedDict()
_CALIBS_MAX = 4


def _engine(h, w):
    key = (h, w, torch.cuda.current_device())
    if key not in _ENGINES:
        _ENGINES[key] = E.Reconstructor(h, w)
    return _ENGINES[key]


def _hasher():
    try:
        import xxhash
        return xxhash.xxh3_64()
    except ImportError:                     # pragma: no cover - xxhash ships with the image
        import hashlib
        return hashlib.blake2b(digest_size=16)


_NC_SAMPLE = 1 << 16                        # Nc elements hashed by the cheap fingerprint


def _logical_sample(a: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """``a.reshape(-1)[idx]`` (C order) without copying ``a``: a flat view when ``a`` is
    C-contiguous, its transpose's flat view when it is a Fortran-ordered 2-D table."""
    if a.flags.c_contiguous:
        return a.reshape(-1)[idx]
    if a.ndim == 2 and a.flags.f_contiguous:
        r, c = np.divmod(idx, a.shape[1])
        return a.T.reshape(-1)[c * a.shape[0] + r]
    return a[np.unravel_index(idx, a.shape)]


def calib_fingerprint(calib, full: bool = False) -> str:
    """Digest of the calibration arrays the path reads (xxh3 over shapes, dtypes and bytes).

    ``cam_K``, ``Oc`` and the plane tables (<= 131 KB) are always hashed whole.  ``Nc`` (3 x H*W
    float64: 50 MB at 1080p, 576 MB at 24 MP) is hashed whole only with ``full=True``; the cheap
    form hashes its shape, dtype and a strided sample of 65536 elements (first and last
    included, taken by logical index so a Fortran-ordered table -- what ``scipy.io.loadmat``
    returns -- is neither copied nor hashed differently from its C-ordered twin), which costs
    well under a millisecond at any size.  The full form hashes a Fortran-ordered table through
    its C-contiguous transpose (no copy either) and tags the order in the digest."""
    h = _hasher()
    for k in ("cam_K", "Oc", "wPlaneCol", "wPlaneRow", "Nc"):
        a = calib.get(k) if hasattr(calib, "get") else None
        if a is None:
            h.update(f"{k}:none;".encode())
            continue
        a = np.asarray(a)
        h.update(f"{k}:{a.shape}:{a.dtype.str};".encode())
        if k == "Nc" and a.size > _NC_SAMPLE:
            if not full:
                a = _logical_sample(a, np.linspace(0, a.size - 1, _NC_SAMPLE).astype(np.int64))
            elif a.ndim == 2 and not a.flags.c_contiguous and a.flags.f_contiguous:
                h.update(b"F;")
                a = a.T                                # C-contiguous view of the same bytes
        h.update(memoryview(np.ascontiguousarray(a)).cast("B"))
    return h.hexdigest()


def _ref(obj):
    import weakref
    try:
        return weakref.ref(obj)
    except TypeError:
        return None


def _device_calib(calib, h, w):
    """Device tables of ``calib`` for one geometry on the current GPU: a small LRU keyed on
    (device, geometry, cheap content digest), so it neither pins callers' dicts nor grows
    without bound, and an edited calibration is uploaded afresh.

    A hit with the very ``Nc`` object of the cached entry costs only the cheap digest.  A hit
    with another ``Nc`` object (e.g. the same ``.mat`` loaded again) is confirmed by the full
    digest of its ``Nc`` against the one taken when the entry was made; a mismatch replaces the
    entry.  (An in-place edit of ``Nc`` entries outside the sample, on the same object, is not
    seen: edit a copy.)"""
    key = (torch.cuda.current_device(), h, w, calib_fingerprint(calib))
    nc = calib.get("Nc") if hasattr(calib, "get") else None
    ent = _CALIBS.get(key)
    if ent is not None:
        dc, ref, full = ent
        if nc is not None and ref is not None and ref() is nc:
            _CALIBS.move_to_end(key)
            return dc
        if calib_fingerprint(calib, full=True) == full:
            _CALIBS[key] = (dc, _ref(nc), full)
            _CALIBS.move_to_end(key)
            return dc
    dc = E.DeviceCalib(calib, h, w)
    _CALIBS[key] = (dc, _ref(nc), calib_fingerprint(calib, full=True))
    _CALIBS.move_to_end(key)
    while len(_CALIBS) > _CALIBS_MAX:
        _CALIBS.popitem(last=False)
    return dc


def _needed_frames(n_files, cfg: E.DecodeConfig):
    """Frame indices the reference reads (processing.py:59-60,88-105)."""
    Bc, Br = E.n_bits(cfg.n_cols), E.n_bits(cfg.n_rows)
    need = [0, 1]
    nc = max(1, min(int(cfg.n_sets_col), Bc))
    nr = max(1, min(int(cfg.n_sets_row), Br))
    idx = 2
    for max_bits, n_use in ((Bc, nc), (Br, nr)):
        for b in range(max_bits):
            if idx + 1 < n_files and b < n_use:
                need += [idx, idx + 1]
            idx += 2
    return need


def read_capture(source, cfg: E.DecodeConfig, order=("bmp", "png")):
    """Discover and decode (host thread pool) one capture: ``(frame stack, texture)``; frames
    the decode does not read stay ``None``.  Host work only (safe on a prefetch thread)."""
    files = FR.discover(source, order)
    if len(files) < 4:
        raise ValueError(f"Not enough images (got {len(files)}, need at least 4).")
    need = _needed_frames(len(files), cfg) if cfg.variant == "processing" else list(range(len(files)))
    imgs, texture = FR.load_frames(files, need, texture=True)
    stack = [None] * len(files)
    for i, im in zip(need, imgs):
        stack[i] = im
    return stack, texture


def has_images(folder: str) -> bool:
    """Batch mode's folder filter (processing.py:320-321)."""
    return bool(glob.glob(os.path.join(folder, "*.bmp")) or glob.glob(os.path.join(folder, "*.png")))


def run_view_folders(subfolders, log, reconstruct, read=None, write=None) -> int:
    """The per-folder loop of batch mode (processing.py:314-334) as a three-stage pipeline.

    ``read(folder) -> host`` (frame read + PNG decode) runs one folder ahead on a prefetch
    thread; ``reconstruct(folder, get_host) -> result`` (H2D, kernels, D2H) on the calling
    thread, where ``get_host()`` waits for that folder's read (so the stage can log its
    progress line first, as the reference does before reading);
    ``write(folder, result) -> out_name`` (ASCII PLY) on a writer thread while the next folder is
    reconstructed.  At most one folder is in each stage.  Per-folder isolation as in the
    reference: an exception in any stage is logged as ``❌ Error in <folder>`` at that folder's
    turn and the loop goes on; folders without images are skipped.  Log order differs from the
    serial loop only in that a folder's ``✔ Saved`` line comes after the next folder's first
    progress lines.  Returns the number of folders that succeeded."""
    from concurrent.futures import ThreadPoolExecutor
    with_imgs = [f for f in subfolders if has_images(f)]
    success = 0
    with ThreadPoolExecutor(max_workers=1) as pre, ThreadPoolExecutor(max_workers=1) as wr:
        pending = {}
        writing = []

        def prefetch(i):
            if read is not None and i < len(with_imgs) and with_imgs[i] not in pending:
                pending[with_imgs[i]] = pre.submit(read, with_imgs[i])

        def drain():
            nonlocal success
            while writing:
                folder, fut = writing.pop()
                try:
                    name = fut.result()
                    success += 1
                    log(f"  ✔ Saved: {name}\n")
                except Exception as e:  # noqa: BLE001 - per-folder isolation like the reference
                    log(f"  ❌ Error in {os.path.basename(folder)}: {e}\n")

        prefetch(0)
        k = 0
        for folder in subfolders:
            if not (k < len(with_imgs) and with_imgs[k] == folder):
                log(f"  Skipping {os.path.basename(folder)} (No images found).")
                continue
            k += 1
            prefetch(k)                                  # the next folder with images
            try:
                fut = pending.pop(folder) if read is not None else None
                result = reconstruct(folder, fut.result if fut is not None else (lambda: None))
            except Exception as e:  # noqa: BLE001
                drain()
                log(f"  ❌ Error in {os.path.basename(folder)}: {e}\n")
                continue
            drain()
            if write is None:
                success += 1
            else:
                writing.append((folder, wr.submit(write, folder, result)))
        drain()
    return success


def load_capture(source, cfg: E.DecodeConfig, order=("bmp", "png"), host=None):
    """Discover, decode and upload one capture: ``(DeviceFrames, texture)``.  ``host``: the
    result of :func:`read_capture` when it was already done (e.g. prefetched)."""
    stack, texture = host if host is not None else read_capture(source, cfg, order)
    return E.DeviceFrames(stack, E.GRAY if _is_frame0(texture, stack) else texture), texture


def _is_frame0(texture, stack) -> bool:
    """Whether the BGR texture is frame 0 replicated (an 8-bit gray capture): the device copy
    then runs in GRAY texture mode and the texture is never uploaded."""
    t = np.asarray(texture)
    f0 = stack[0]
    if f0 is None or t.ndim != 3 or t.shape[2] != 3:
        return False
    f0 = np.asarray(f0)
    return t.shape[:2] == f0.shape and all(np.array_equal(t[..., c], f0) for c in range(3))


class ProcessingLogic:
    """Reconstruction half of the reference's ``ProcessingLogic`` (processing.py:12-334)."""

    # --- Multi PLY Processing Functions ---
    @staticmethod
    def _gray_decode(source, n_cols=1920, n_rows=1080,
                     n_sets_col=11, n_sets_row=11,
                     thresh_mode='otsu', shadow_val=40, contrast_val=10):
        """Decode Gray-code images (server/processing.py:28-124).

        ``source``: folder path or sorted file list, as in the reference; additionally a
        ``DeviceFrames`` or a uint8 ``[F, H, W]`` array/tensor already in memory.
        Returns ``(col int32[H,W], row int32[H,W], mask bool[H,W], texture uint8[H,W,3])``.
        """
        cfg = E.DecodeConfig(n_cols, n_rows, n_sets_col, n_sets_row, thresh_mode, shadow_val,
                             contrast_val, "processing")
        if isinstance(source, E.DeviceFrames):
            dev = source
            texture = source.texture_bgr().reshape(dev.height, dev.width, 3).cpu().numpy()
        elif isinstance(source, (np.ndarray, torch.Tensor)) and source.ndim == 3:
            dev = E.DeviceFrames(source)
            texture = dev.texture.reshape(dev.height, dev.width, 3).cpu().numpy()
        else:
            dev, texture = load_capture(source, cfg)
        eng = _engine(dev.height, dev.width)
        col, row, mask = eng.decode(dev, cfg)
        shape = (dev.height, dev.width)
        return (col.reshape(shape).cpu().numpy(), row.reshape(shape).cpu().numpy(),
                mask.reshape(shape).cpu().numpy().astype(bool), texture)

    @staticmethod
    def _reconstruct_point_cloud(col_map, row_map, mask, texture, calib,
                                 row_mode=1, epipolar_tol=2.0):
        """Ray-plane triangulation (server/processing.py:127-234).

        Returns ``(P float64[N,3], C uint8[N,3] BGR)``; ``None`` for a ``row_mode`` other than
        0/1/2 (the reference falls through its if-chain).
        """
        if row_mode not in (0, 1, 2):
            return None
        h, w = np.asarray(col_map).shape
        eng = _engine(h, w)
        dev = eng.device

        def up(a, dt):
            t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a, dtype=dt))
            return t.reshape(-1).to(device=dev, dtype=torch.int32 if dt == np.int32 else torch.uint8)

        col = up(col_map, np.int32)
        row = up(row_map, np.int32) if row_mode != 0 else None
        m = up(np.asarray(mask).astype(np.uint8) if not isinstance(mask, torch.Tensor) else mask, np.uint8)
        tex = up(np.asarray(texture).reshape(-1, 3) if not isinstance(texture, torch.Tensor) else texture, np.uint8)
        dc = _device_calib(calib, h, w)
        out = eng.triangulate(col, row, m, tex, dc, row_mode, epipolar_tol, xyz_f64=True)
        P, C = out.result()
        return P.cpu().numpy(), C.cpu().numpy()

    @staticmethod
    def _save_ply(points, colors, filename):
        """ASCII PLY, byte-identical to server/processing.py:236-248."""
        PLY.write_ascii(filename, points, colors)

    @staticmethod
    def process_multi_ply(calib_path, target_path, mode, log_callback=None,
                          n_sets_col=11, n_sets_row=11,
                          row_mode=1, epipolar_tol=2.0,
                          thresh_mode='otsu', shadow_val=40, contrast_val=10,
                          file_list=None, out_path_override=None):
        """Process structured-light images -> .ply point cloud (server/processing.py:251-334).

        Each view runs the fused decode+triangulate kernel (maps never leave the chip)."""
        def log(msg):
            if log_callback: log_callback(msg)
            else: print(msg)

        log("Loading Calibration Data...")
        import scipy.io
        data = scipy.io.loadmat(calib_path)
        calib_data = {
            "Nc": data["Nc"], "Oc": data["Oc"],
            "wPlaneCol": data["wPlaneCol"], "wPlaneRow": data["wPlaneRow"],
            "cam_K": data["cam_K"]
        }
        cfg = E.DecodeConfig(1920, 1080, n_sets_col, n_sets_row, thresh_mode, shadow_val,
                             contrast_val, "processing")

        def _process_source(source, out_path, label, host=None):
            log(f"  -> Decoding {label}  "
                f"[col-sets={n_sets_col}  row-sets={n_sets_row}]...")
            dev, _ = load_capture(source, cfg, host=None if host is None else host.result())
            log("  -> Reconstructing 3D points...")
            points, colors = reconstruct_view(dev, cfg, calib_data, row_mode, epipolar_tol)
            log(f"  -> Saving {len(points)} points...")
            ProcessingLogic._save_ply(points, colors, out_path)
            log(f"  ✔ Saved: {os.path.basename(out_path)}\n")

        if mode == "files":
            if not file_list:
                raise ValueError("mode='files' requires a non-empty file_list.")
            if not out_path_override:
                raise ValueError("mode='files' requires out_path_override.")
            _process_source(file_list, out_path_override,
                            f"{len(file_list)} selected files")

        elif mode == "single":
            ply_name = os.path.basename(target_path) + ".ply"
            out_path = os.path.join(target_path, ply_name)
            _process_source(target_path, out_path,
                            f"folder '{os.path.basename(target_path)}'")

        else:  # batch
            subfolders = [f.path for f in os.scandir(target_path) if f.is_dir()]
            log(f"Found {len(subfolders)} subfolders to process.")

            # A host/GPU pipeline (pipeline.BatchPipeline): frames decoded ahead into pinned
            # memory, groups of views uploaded asynchronously and reconstructed by one batched
            # launch, PLYs written on a writer thread; per-folder errors and log lines as in
            # the reference.
            from .pipeline import BatchPipeline
            success_count = BatchPipeline(cfg, calib_data, row_mode, epipolar_tol, group=batch_views(),
                                          log=log).run(subfolders, batch_write_stage())
            log(f"=== Batch Complete: {success_count}/{len(subfolders)} succeeded ===")


def batch_views() -> int:
    """Views per batched launch in batch mode: ``SLG_BATCH_VIEWS`` (1..16), default 1.  The file
    path is bound by the host PNG decode (~70 C2 views/s on 16 CPUs), not by the GPU, and a
    group waits for all its reads before its launch: over 36 C2 folders, groups of 1 / 4 / 8
    measured 0.0135-0.0149 / 0.0138-0.0144 / 0.0143-0.0163 s/view with the device taking its
    share of the PNGs, 0.0157 / 0.0161-0.0166 host-only (profiles/r5t/e2e.json).  Groups pay
    off for in-memory sources (BatchReconstructor, bench.py)."""
    try:
        return max(1, min(16, int(os.environ.get("SLG_BATCH_VIEWS", "1"))))
    except ValueError:
        return 1


def batch_reconstruct_stage(cfg, calib, row_mode, epipolar_tol, log):
    """``reconstruct`` stage of :func:`run_view_folders`: upload + fused kernels -> host cloud,
    with the reference's progress lines (processing.py:264-272).  The device tables are made
    once per geometry for the whole batch."""
    tables = {}

    def stage(folder, get_host):
        log(f"  -> Decoding folder '{os.path.basename(folder)}'  "
            f"[col-sets={cfg.n_sets_col}  row-sets={cfg.n_sets_row}]...")
        dev, _ = load_capture(folder, cfg, host=get_host())
        log("  -> Reconstructing 3D points...")
        geom = (dev.height, dev.width, torch.cuda.current_device())
        if geom not in tables:
            tables[geom] = E.DeviceCalib(calib, dev.height, dev.width)
        points, colors = reconstruct_view(dev, cfg, calib, row_mode, epipolar_tol, dc=tables[geom])
        log(f"  -> Saving {len(points)} points...")
        return points, colors
    return stage


def batch_write_stage():
    """``write`` stage of :func:`run_view_folders`: ``<folder>/<folder name>.ply``."""
    from .pipeline import FormattedCloud

    def stage(folder, result):
        name = os.path.basename(folder) + ".ply"
        if isinstance(result, FormattedCloud):          # body formatted on the device
            result.write(os.path.join(folder, name))
        else:
            ProcessingLogic._save_ply(result[0], result[1], os.path.join(folder, name))
        return name
    return stage


def reconstruct_view(dev: E.DeviceFrames, cfg: E.DecodeConfig, calib: dict, row_mode=1,
                     epipolar_tol=2.0, xyz_f64=True, dc: E.DeviceCalib | None = None):
    """Fused decode + triangulate of one in-HBM capture -> host ``(P, C)`` like the reference
    pair ``_gray_decode`` + ``_reconstruct_point_cloud``.  ``dc``: device tables of ``calib``
    already made for this geometry (else looked up in the module cache)."""
    if row_mode not in (0, 1, 2):
        return None
    eng = _engine(dev.height, dev.width)
    dc = dc if dc is not None else _device_calib(calib, dev.height, dev.width)
    out = eng.reconstruct(dev, cfg, dc, row_mode, epipolar_tol, xyz_f64=xyz_f64)
    P, C = out.result()
    return P.cpu().numpy(), C.cpu().numpy()
