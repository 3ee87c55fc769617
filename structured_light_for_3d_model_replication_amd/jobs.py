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
* every view's cloud written to its own region of ONE packed output arena.

**Sizing (default: on the device, inside the job).**  The job's workspace slices are bound to the
arena (``slg_workspace_set_arena``): whichever kernel finishes a view's Otsu thresholds -- the
first groups' stats passes or the fused launches' finishing workgroups, two launches before the
view is decoded -- also reserves the view's region with one ``atomicAdd`` on a device cursor,
``min(#white >= smin, #(white - black) >= cmin)`` points (x 2 for row_mode 2), read off the
histograms the thresholds come from: an upper bound of the view's points, so no view can write
past its region, by construction.  No sizing pass, no host sync before the launches.  A view
the arena has no room left for stores nothing and reports offset -1; :meth:`ResidentJob.recover`
re-runs it into a cloud of its own.  The arena's layout follows reservation order (each view's
cloud is still contiguous and bit-identical to the single-view path).  By default the arena is
sized to the HBM left free (capped at the worst case, H*W points per view).

Caller hints (a list of ints) or ``None`` (H*W per view) keep the host-packed layout: view j at
the sum of the earlier hints, ``H*W`` points of slack at the end; a view whose count exceeds its
hint has written into its successors' regions (:meth:`ResidentJob.overflowed`,
:meth:`ResidentJob.damaged`).

**Isolation.**  :meth:`ResidentJob.recover` re-runs refused / damaged views into clouds of their
own, and :meth:`ResidentJob.cloud` refuses a damaged view that was not recovered -- the reference
isolates each folder in the same spirit (``server/processing.py:323-330``: one folder's failure
is logged and the loop goes on with the next).
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as N
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


def device_capacity_hints(views, cfg: E.DecodeConfig, engine: E.BatchReconstructor | None = None,
                          stream=None) -> list[int]:
    """Per-view upper bounds of the row_mode 0/1 point count, computed on the device
    (``BatchReconstructor.valid_bounds``: one batched stats pass over white / black, the bound
    read off the Otsu histograms).  One host sync at the end."""
    if not views:
        return []
    h, w = views[0].height, views[0].width
    eng = engine or E.BatchReconstructor(h, w, min(E.MAX_VIEWS_PER_LAUNCH, len(views)),
                                         device=views[0].data.device, slots=1)
    return [int(x) for x in eng.valid_bounds(views, cfg, stream=stream).tolist()]


class DamagedViewError(RuntimeError):
    """A resident job's view whose cloud another view's overflow may have overwritten."""


class ResidentJob:
    """One job over HBM-resident views of one geometry (see the module docstring).

    ``capacity_hints``: ``"device"`` (default: the device-reserved arena of ``arena_points``
    points, default the free HBM's worth capped at H*W per view), a list of ints (one per view,
    host-packed, taken as given), or ``None`` (H*W per view: the worst case, host-packed)."""

    def __init__(self, views, cfg: E.DecodeConfig, calib: E.DeviceCalib, batch: int = 4, row_mode: int = 1,
                 epipolar_tol: float = 2.0, xyz_f64: bool = False, capacity_hints="device", device=None,
                 arena_points: int | None = None):
        if not views:
            raise ValueError("a job needs at least one view")
        if cfg.thresh_mode != "otsu" or cfg.variant != "processing":
            raise ValueError("resident jobs run the Otsu pipeline of the processing variant")
        if row_mode not in (0, 1, 2):
            raise ValueError("row_mode must be 0, 1 or 2")
        self.views = list(views)
        h, w = self.views[0].height, self.views[0].width
        self.height, self.width, self.n_px = h, w, h * w
        self.device = device or self.views[0].data.device
        self.batch = max(1, min(int(batch), E.MAX_VIEWS_PER_LAUNCH))
        self.cfg, self.calib, self.row_mode, self.tol, self.xyz_f64 = cfg, calib, row_mode, epipolar_tol, xyz_f64
        self.mult = 2 if row_mode == 2 else 1
        self.engine = E.BatchReconstructor(h, w, self.batch, device=self.device, slots=4)
        self.device_arena = isinstance(capacity_hints, str)
        if self.device_arena:
            if capacity_hints != "device":
                raise ValueError("capacity_hints: 'device', a list of ints, or None")
            self.hints_source = "device_reserved"
            self.hints = None
            worst = len(self.views) * self.n_px * self.mult
            if arena_points is None:
                free, _ = torch.cuda.mem_get_info(self.device)
                per_point = 3 * (8 if xyz_f64 else 4) + 3
                arena_points = min(worst, int(0.92 * free) // per_point)
            arena_points = max(int(arena_points), self.n_px * self.mult)
            self.xyz = torch.empty((arena_points, 3), device=self.device,
                                   dtype=torch.float64 if xyz_f64 else torch.float32)
            self.bgr = torch.empty((arena_points, 3), device=self.device, dtype=torch.uint8)
            self.counts = torch.zeros((len(self.views), 2), device=self.device, dtype=torch.int64)
            self.cursor = torch.zeros(1, device=self.device, dtype=torch.int64)
            self.offsets = None
            self.clouds = []
            for j in range(len(self.views)):
                c = E.Cloud.__new__(E.Cloud)
                c.xyz, c.bgr, c.count = self.xyz, self.bgr, self.counts[j]
                c.capacity, c.xyz_f64, c.stream = arena_points, xyz_f64, None
                self.clouds.append(c)
            eng = self.engine
            N.check(N.lib().slg_workspace_set_arena(eng._ws(0), eng.ws_stride, eng.max_views * eng.slots,
                                                    ctypes.c_void_p(self.cursor.data_ptr()), arena_points,
                                                    self.mult, E._stream()))
        else:
            if capacity_hints is None:
                hints, self.hints_source = [self.n_px * self.mult] * len(self.views), "worst_case"
            else:
                hints, self.hints_source = capacity_hints, "caller"
            if len(hints) != len(self.views):
                raise ValueError("one capacity hint per view")
            self.hints = [int(x) for x in hints]
            self.clouds, self.offsets, self.xyz, self.bgr, self.counts = packed_clouds(
                self.n_px * self.mult, self.hints, xyz_f64, self.device)
        groups = [list(range(g, min(g + self.batch, len(self.views)))) for g in range(0, len(self.views), self.batch)]
        self.groups = groups
        self.batches = [self.engine.prepare([self.views[k] for k in g], cfg, calib, [self.clouds[k] for k in g],
                                            row_mode, epipolar_tol, slot=i % 4) for i, g in enumerate(groups)]
        self._recovered: dict = {}            # view -> (xyz, bgr) of its own, or the exception of its re-run
        self._rec = None
        torch.cuda.current_stream(self.device).synchronize()     # (bound before any pool stream runs)

    @property
    def arena_points(self) -> int:
        """Points the arena holds."""
        return int(self.xyz.shape[0])

    def run(self, s0, s1):
        """Enqueue the whole job (first four groups' stats passes, then one fused launch per group
        on the two streams); afterwards ``s0`` has joined ``s1``.  No host sync.  Forgets any
        earlier :meth:`recover`."""
        self._recovered.clear()
        s0.wait_stream(torch.cuda.current_stream(self.device))   # the staged views, tables, arena
        if self.device_arena:
            with torch.cuda.stream(s0):
                self.cursor.zero_()                              # every job reserves afresh
        s1.wait_stream(s0)
        self.engine.run_pipelined(self.batches, s0, s1, mode="fused2")
        s0.wait_stream(s1)

    def host_counts(self):
        """Points of every view (one host sync)."""
        c = self.counts.tolist()
        return [int(x[0]) for x in c] if self.device_arena else c

    def host_offsets(self):
        """First point index of every view in the arena (-1: refused for lack of room)."""
        if self.device_arena:
            return [int(x[1]) for x in self.counts.tolist()]
        return list(self.offsets[:-1]) if len(self.offsets) > len(self.views) else list(self.offsets)

    def overflowed(self, counts=None):
        """Views whose cloud ran past their capacity hint (into the next view's region); with the
        device-reserved arena: the views refused for lack of room (nothing can run past)."""
        if self.device_arena:
            return [j for j, o in enumerate(self.host_offsets()) if o < 0]
        counts = self.host_counts() if counts is None else counts
        return [j for j, (n, h) in enumerate(zip(counts, self.hints)) if n > h]

    def damaged(self, counts=None):
        """Views whose cloud cannot be trusted: the overflowed (refused) ones and, host-packed,
        every later view whose region starts before an overflowed view's last point."""
        if self.device_arena:
            return self.overflowed()
        counts = self.host_counts() if counts is None else counts
        bad = set()
        for j in self.overflowed(counts):
            bad.add(j)
            end = self.offsets[j] + counts[j]
            bad.update(k for k in range(j + 1, len(self.hints)) if self.offsets[k] < end)
        return sorted(bad)

    def recover(self, counts=None, stream=None) -> list[int]:
        """Re-run every damaged view (:meth:`damaged`) alone into a cloud of its own (worst-case
        capacity), stream-ordered after the job.  A view whose re-run raises keeps the exception,
        which :meth:`cloud` raises for it.  Returns the views re-run."""
        counts = self.host_counts() if counts is None else counts
        bad = [j for j in self.damaged(counts) if j not in self._recovered]
        if bad and self._rec is None:
            self._rec = E.Reconstructor(self.height, self.width, device=self.device)
        for j in bad:
            try:
                c = self._rec.reconstruct(self.views[j], self.cfg, self.calib, self.row_mode, self.tol,
                                          xyz_f64=self.xyz_f64, stream=stream)
                self._recovered[j] = c.result()
            except Exception as e:  # noqa: BLE001 - per-view isolation
                self._recovered[j] = e
        return bad

    def cloud(self, j, counts=None):
        """``(xyz, bgr)`` of view j: its recovered cloud after :meth:`recover`, else the arena
        slices.  Raises :class:`DamagedViewError` for a damaged view that was not recovered (its
        points may belong to another view, or were never stored), and the re-run's exception for
        one whose re-run failed."""
        r = self._recovered.get(j)
        if isinstance(r, Exception):
            raise r
        if r is not None:
            return r
        counts = self.host_counts() if counts is None else counts
        if j in self.damaged(counts):
            raise DamagedViewError(f"view {j}: its cloud did not fit the arena or was overwritten by an earlier "
                                   "view's overflow; call recover() first")
        n = counts[j]
        o = self.host_offsets()[j] if self.device_arena else self.offsets[j]
        return self.xyz[o: o + n], self.bgr[o: o + n]
