"""One view split over ranks by bands of rows ("single huge view (C4)").

A 24 MP capture (BASELINE configs[3]) is one view: view sharding gives one GPU all of it.  Split
by rows instead, every pixel's decode and triangulation stay independent
(``server/processing.py:80-234`` is per pixel once the mask thresholds are known), and the only
quantity that spans the bands is the mask thresholds: Otsu of the whole view's white histogram
and of its ``clip(white - black)`` histogram (``server/processing.py:59-72``), or the percentile
rule's black histogram and ``max(white - black)`` (``server/sl_system.py:534-540``).  So the split
has exactly one exchange step, 2 KB per rank:

1. each rank counts its band's histograms (``slg_decode_histograms``);
2. one all-reduce (RCCL over xGMI: SUM of the 512 bins, MAX of the max code);
3. each rank sets the view's thresholds from the totals (``slg_thresholds_from_histograms``: the
   same Otsu tail on the same histograms, so the unsplit view's thresholds bit for bit) and runs
   the fused decode + triangulate launch over its band (``slg_decode_triangulate``);
4. the band clouds are the view's points of those rows in pixel order, so the view's cloud is
   their concatenation in rank order (row_mode 2: every band's column cloud, then every band's row
   cloud -- ``np.vstack((P_col, P_row))`` of ``server/processing.py:209-234``), gathered to one
   rank by :func:`distributed.gather_clouds`.

Manual thresholds need no exchange.  Rays: with ``cam_K`` pinhole rays a band uses
``cy - r0`` (``y = (v - cy) / fy`` of ``server/processing.py:145-156`` then has the same operands,
since ``cy - r0`` is exact: checked), a ray table is sliced to the band's pixels.
"""
from __future__ import annotations

import copy
from fractions import Fraction

import torch
import torch.distributed as dist

from . import engine as E
from .distributed import gather_clouds, shard_range

N_HIST = 513                      # [0..511] histograms, [512] max(white - black) + 256


def band_rows(height: int, rank: int, world: int) -> tuple[int, int]:
    """Rows ``[r0, r1)`` of ``rank``'s band: contiguous, sizes differ by at most one."""
    if world > height:
        raise ValueError(f"{world} bands need at least {world} rows (got {height})")
    return shard_range(height, rank, world)


def band_frames(frames: E.DeviceFrames, r0: int, r1: int) -> E.DeviceFrames:
    """A capture's rows ``[r0, r1)`` (every frame and the texture) as a capture of its own, in
    buffers of its own (device-to-device copies; a rank holding only its band loads just these)."""
    W = frames.width
    if not 0 <= r0 < r1 <= frames.height:
        raise ValueError(f"band [{r0}, {r1}) outside 0..{frames.height}")
    b = E.DeviceFrames.allocate(frames.n_frames, r1 - r0, W, device=frames.data.device, gray=frames.texture is None)
    F = frames.n_frames
    b.data[:F, : b.n_px].copy_(frames.data[:F, r0 * W: r1 * W])
    if frames.texture is not None:
        b.texture.copy_(frames.texture[r0 * W: r1 * W])
    return b


def band_calib(calib: E.DeviceCalib, r0: int, r1: int) -> E.DeviceCalib:
    """The calibration of rows ``[r0, r1)``: the plane tables are shared; pinhole rays take
    ``cy - r0`` (exact, or ValueError), a ray table its band of pixels."""
    b = copy.copy(calib)
    b.height = r1 - r0
    if calib.rays is not None:
        W = calib.width
        b.rays = calib.rays[:, r0 * W: r1 * W].contiguous()
    else:
        cy = calib.cy - r0
        if Fraction(cy) != Fraction(calib.cy) - r0:
            raise ValueError(f"cy - {r0} is not exact in float64: pass a ray table (DeviceCalib keep_table)")
        b.cy = cy
    return b


def allreduce_histograms(hist: torch.Tensor, group=None) -> torch.Tensor:
    """The exchange step, in place: SUM of the bins ``[0..511]``, MAX of ``[512]`` over the
    ranks of ``group`` (identity without a process group)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = hist
        if hist.is_cuda and dist.get_backend(group) != "nccl":
            t = hist.cpu()                           # (gloo rehearsal: host tensors)
        dist.all_reduce(t[:512], op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(t[512:], op=dist.ReduceOp.MAX, group=group)
        if t is not hist:
            hist.copy_(t)
    return hist


class BandReconstructor:
    """One rank's band of a view (rows ``[r0, r1)`` of ``height``): histograms, exchange,
    thresholds, the fused launch.  Stream-ordered on the current stream; the exchange is the one
    collective."""

    def __init__(self, height: int, width: int, r0: int, r1: int, device=None):
        if not 0 <= r0 < r1 <= height:
            raise ValueError(f"band [{r0}, {r1}) outside 0..{height}")
        self.height, self.width, self.r0, self.r1 = int(height), int(width), int(r0), int(r1)
        self.n_px_view = self.height * self.width
        self.engine = E.Reconstructor(r1 - r0, width, device=device)
        self.hist = torch.zeros(N_HIST, dtype=torch.int32, device=self.engine.device)

    def run(self, frames: E.DeviceFrames, cfg: E.DecodeConfig, calib: E.DeviceCalib, row_mode: int = 1,
            epipolar_tol: float = 2.0, xyz_f64: bool = True, out: E.Cloud | None = None, exchange=None,
            sync: bool = True):
        """The band's cloud (a :class:`engine.Cloud`) and, for row_mode 2, its column-cloud size
        (else None).  ``frames`` / ``calib``: the band's (:func:`band_frames`, :func:`band_calib`).
        ``exchange(hist)``: the all-reduce (default :func:`allreduce_histograms` over the default
        process group).  ``sync=False``: only enqueue (no column-cloud size)."""
        eng = self.engine
        out = out or E.Cloud(eng.n_px, row_mode, xyz_f64, eng.device)
        if cfg.thresh_mode == "manual" and cfg.variant != "slsystem":
            eng.stats(frames, cfg)                   # the same thresholds on every rank
        else:
            eng.histograms(frames, cfg, out=self.hist)
            (exchange or allreduce_histograms)(self.hist)
            eng.thresholds_from_histograms(self.hist, self.n_px_view, cfg)
        eng.decode_triangulate(frames, cfg, calib, out, row_mode, epipolar_tol)
        if not sync:
            return out, None
        out.result()
        return out, (eng.column_points() if row_mode == 2 else None)


def assemble(parts, column_points, row_mode: int):
    """The view's cloud from its bands' clouds in rank order: ``parts`` = [(xyz, bgr), ...],
    ``column_points`` = each band's column-cloud size (row_mode 2; else ignored)."""
    if row_mode != 2:
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
    cols = [(x[:c], b[:c]) for (x, b), c in zip(parts, column_points)]
    rows = [(x[c:], b[c:]) for (x, b), c in zip(parts, column_points)]
    return (torch.cat([p[0] for p in cols] + [p[0] for p in rows]),
            torch.cat([p[1] for p in cols] + [p[1] for p in rows]))


def gather_banded(xyz: torch.Tensor, bgr: torch.Tensor, column_points: int | None, row_mode: int, dst: int = 0):
    """The whole view's cloud on ``dst`` (None elsewhere): the band clouds by
    :func:`distributed.gather_clouds` (exact sizes) and, for row_mode 2, each band's column-cloud
    size by one all-gather, then :func:`assemble`."""
    parts = gather_clouds(xyz, bgr, dst)
    cols = None
    if row_mode == 2:
        c = torch.tensor([int(column_points)], dtype=torch.int64, device=xyz.device)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            allc = [torch.zeros_like(c) for _ in range(dist.get_world_size())]
            dist.all_gather(allc, c)
        else:
            allc = [c]
        cols = [int(x.item()) for x in allc]
    if parts is None:
        return None
    return assemble(parts, cols, row_mode)
