"""HBM-resident scan jobs: many views of one geometry, staged in HBM, reconstructed as one job.

The reference's scan-farm flow is an auto-scan per object (``server/gui.py:1700-1787``: one
capture folder per turntable angle) followed by ``process_multi_ply(mode='batch')`` over the
folders (``server/processing.py:314-334``, a serial loop).  BASELINE.json's C5 workload is that
flow at farm scale: 8 objects x 72 views at 4K, 220 GB of frames -- which fits the 288 GB of one
MI355X's HBM.  :class:`ResidentJob` runs such a job with every view already resident:

* views in groups of ``batch`` per fused decode/triangulate launch, on the two-stream carried
  pipeline (``BatchReconstructor.run_pipelined(mode="fused2")``: each launch carries the Otsu
  histograms of the group four ahead and finishes the thresholds of the group two ahead, so no
  stats kernel runs after the first four groups);
* every view's cloud written to its own region of ONE packed output arena (:func:`packed_clouds`):
  view j starts at the sum of the capacity hints of views < j.  The arena ends with ``H*W``
  points of slack, so from any view's start there are at least ``H*W`` points to the arena's end
  -- the C ABI's capacity contract (``slg_cloud.capacity >= H*W``) holds for every view and no
  store can leave the allocation.  A view whose count exceeds its hint has written into its
  successors' regions: :meth:`ResidentJob.overflowed` names such views, and
  :meth:`ResidentJob.damaged` adds the views whose region an overflow reached (re-run all of
  them into clouds of their own).  With exact hints (a previous pass over the same frames, or per-view valid-pixel
  counts) 576 4K clouds take 41 GB instead of the 72 GB of worst-case slots.
"""
from __future__ import annotations

import torch

from . import engine as E


def packed_clouds(n_px: int, hints, xyz_f64: bool = False, device=None):
    """Clouds over one arena: view j's region starts at ``sum(hints[:j])``; ``H*W`` points of
    slack at the end.  Returns ``(clouds, offsets, arena_xyz, arena_bgr, counts)``; ``counts`` is
    the one int64 device tensor every cloud's ``count`` is a slice of."""
    device = device or E.default_device()
    hints = [int(h) for h in hints]
    if any(h < 0 for h in hints):
        raise ValueError("capacity hints must be >= 0")
    offsets = [0]
    for h in hints:
        offsets.append(offsets[-1] + h)
    total = offsets[-1] + n_px
    xyz = torch.empty((total, 3), device=device, dtype=torch.float64 if xyz_f64 else torch.float32)
    bgr = torch.empty((total, 3), device=device, dtype=torch.uint8)
    counts = torch.zeros(len(hints), device=device, dtype=torch.int64)
    clouds = []
    for j in range(len(hints)):
        c = E.Cloud.__new__(E.Cloud)
        c.xyz, c.bgr, c.count = xyz[offsets[j]:], bgr[offsets[j]:], counts[j:j + 1]
        c.capacity = total - offsets[j]          # >= n_px: the contract holds for every view
        c.xyz_f64, c.stream = xyz_f64, None
        clouds.append(c)
    return clouds, offsets, xyz, bgr, counts


def stage_copies(sources, plan, device=None):
    """Resident job views: ``plan[j]`` = index of the source ``DeviceFrames`` whose frames and
    texture view j holds, each view in HBM buffers of its own (device-to-device copies)."""
    out = []
    for j, s in enumerate(plan):
        src = sources[s]
        d = E.DeviceFrames.allocate(src.n_frames, src.height, src.width, device=device or src.data.device,
                                    gray=src.texture is None)
        d.data.copy_(src.data)
        if src.texture is not None:
            d.texture.copy_(src.texture)
        out.append(d)
    return out


class ResidentJob:
    """One job over HBM-resident views of one geometry (see the module docstring)."""

    def __init__(self, views, cfg: E.DecodeConfig, calib: E.DeviceCalib, batch: int = 4, row_mode: int = 1,
                 epipolar_tol: float = 2.0, xyz_f64: bool = False, capacity_hints=None, device=None):
        if not views:
            raise ValueError("a job needs at least one view")
        if cfg.thresh_mode != "otsu" or cfg.variant != "processing":
            raise ValueError("resident jobs run the Otsu pipeline of the processing variant")
        if row_mode not in (0, 1):
            raise ValueError("resident jobs pack row_mode 0/1 clouds (row_mode 2 needs 2*H*W slack)")
        self.views = list(views)
        h, w = self.views[0].height, self.views[0].width
        self.height, self.width, self.n_px = h, w, h * w
        self.device = device or self.views[0].data.device
        self.batch = max(1, min(int(batch), E.MAX_VIEWS_PER_LAUNCH))
        hints = capacity_hints if capacity_hints is not None else [self.n_px] * len(self.views)
        if len(hints) != len(self.views):
            raise ValueError("one capacity hint per view")
        self.hints = [int(x) for x in hints]
        self.clouds, self.offsets, self.xyz, self.bgr, self.counts = packed_clouds(
            self.n_px, self.hints, xyz_f64, self.device)
        self.engine = E.BatchReconstructor(h, w, self.batch, device=self.device, slots=4)
        groups = [list(range(g, min(g + self.batch, len(self.views)))) for g in range(0, len(self.views), self.batch)]
        self.groups = groups
        self.batches = [self.engine.prepare([self.views[k] for k in g], cfg, calib, [self.clouds[k] for k in g],
                                            row_mode, epipolar_tol, slot=i % 4) for i, g in enumerate(groups)]

    def run(self, s0, s1):
        """Enqueue the whole job (first four groups' stats passes, then one fused launch per group
        on the two streams); afterwards ``s0`` has joined ``s1``.  No host sync."""
        s1.wait_stream(s0)
        self.engine.run_pipelined(self.batches, s0, s1, mode="fused2")
        s0.wait_stream(s1)

    def host_counts(self):
        return self.counts.tolist()

    def overflowed(self, counts=None):
        """Views whose cloud ran past their capacity hint (into the next view's region)."""
        counts = self.host_counts() if counts is None else counts
        return [j for j, (n, h) in enumerate(zip(counts, self.hints)) if n > h]

    def damaged(self, counts=None):
        """Views whose cloud cannot be trusted: the overflowed ones and every later view whose
        region starts before an overflowed view's last point (its points may be overwritten)."""
        counts = self.host_counts() if counts is None else counts
        bad = set()
        for j in self.overflowed(counts):
            bad.add(j)
            end = self.offsets[j] + counts[j]
            bad.update(k for k in range(j + 1, len(self.hints)) if self.offsets[k] < end)
        return sorted(bad)

    def cloud(self, j, counts=None):
        """``(xyz, bgr)`` of view j (device slices of the arena)."""
        n = (self.host_counts() if counts is None else counts)[j]
        return self.xyz[self.offsets[j]: self.offsets[j] + n], self.bgr[self.offsets[j]: self.offsets[j] + n]
