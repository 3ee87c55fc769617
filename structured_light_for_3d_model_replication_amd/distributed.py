"""View-sharded multi-GPU processing.

Turntable views are independent (``process_multi_ply(mode='batch')`` loops over view folders,
``server/processing.py:314-334``; the auto-scan writes one folder per angle,
``server/gui.py:1718,1753``).  One process per GPU (torchrun) takes a contiguous block of
views, ``[r*V/G, (r+1)*V/G)``, and runs the whole hot path locally: no collective touches the
data path.  Two optional collectives exist for the end of a job:

* ``batch_summary`` — all-reduce of per-rank success counts so rank 0 can log the reference's
  ``=== Batch Complete: s/n succeeded ===`` line for the whole job;
* ``RcclCloudGather`` — the final cloud gather of the north star: exact-size gatherv of the
  per-view clouds to rank 0 through the C ABI over RCCL/xGMI (``slg_gather_*``), for a
  consumer that wants every point on one rank (e.g. the 360° merge that follows the path);
  ``gather_clouds`` is the same protocol over torch.distributed (gloo or RCCL).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of items for ``rank``; sizes differ by at most one."""
    q, r = divmod(n_items, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard(items, rank: int | None = None, world: int | None = None):
    if rank is None or world is None:
        rank, world = env_rank_world()
    lo, hi = shard_range(len(items), rank, world)
    return list(items)[lo:hi]


def view_folders(target_path: str):
    """Batch-mode view folders in a deterministic order (the reference iterates
    ``os.scandir`` order, which is unspecified; sharding needs an order every rank agrees on)."""
    return sorted(f.path for f in os.scandir(target_path) if f.is_dir())


def batch_summary(success: int, total: int, device=None) -> tuple[int, int]:
    """Job-wide (success, folders) over all ranks (identity without a process group)."""
    if not (dist.is_available() and dist.is_initialized()):
        return success, total
    t = torch.tensor([success, total], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t[0]), int(t[1])


PER_RANK_KEYS = ("views", "points", "kernel_ms", "d2h_ms", "step_ms")


def per_rank_table(row: dict, device=None) -> list[dict]:
    """Every rank's timing row on every rank (one all_gather of a float64 vector; identity
    without a process group): ``row`` holds :data:`PER_RANK_KEYS` (numbers), the result is the
    rows in rank order with ``rank`` added.  A bench line reports them beside its max-over-ranks
    headline, so a slow rank (its kernels, or its PCIe copies) is visible."""
    vec = torch.tensor([float(row[k]) for k in PER_RANK_KEYS], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        parts = [torch.empty_like(vec) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, vec)
    else:
        parts = [vec]
    out = []
    for r, v in enumerate(parts):
        d = {"rank": r}
        for k, x in zip(PER_RANK_KEYS, v.tolist()):
            d[k] = int(x) if k in ("views", "points") else round(x, 4)
        out.append(d)
    return out


def gather_clouds(xyz: torch.Tensor, bgr: torch.Tensor, dst: int = 0):
    """Exact-size gatherv of variable-size clouds to ``dst`` over torch.distributed (gloo or
    RCCL): the counts go by one all_gather, then every rank sends exactly its own points
    (point-to-point, grouped; no padding to the largest rank).  Returns ``[(xyz_r, bgr_r), ...]``
    on ``dst`` (rank order), ``None`` elsewhere.  ``xyz`` [n,3] float, ``bgr`` [n,3] uint8, on the
    device the process group's backend expects (CUDA for RCCL, CPU for gloo).  The C-ABI RCCL
    path for GPU clouds is :class:`RcclCloudGather`."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [(xyz, bgr)]
    world, rank = dist.get_world_size(), dist.get_rank()
    n = torch.tensor([xyz.shape[0]], dtype=torch.int64, device=xyz.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    nccl = dist.get_backend() == "nccl"
    ops, reqs = [], []

    def p2p(fn, t, peer):
        if nccl:
            ops.append(dist.P2POp(fn, t, peer))
        else:
            reqs.append(fn(t, peer))

    out = None
    if rank == dst:
        out = []
        for r in range(world):
            if r == dst:
                out.append((xyz, bgr))
                continue
            bx = torch.empty((counts[r], 3), dtype=xyz.dtype, device=xyz.device)
            bb = torch.empty((counts[r], 3), dtype=torch.uint8, device=xyz.device)
            if counts[r]:
                p2p(dist.irecv, bx, r)
                p2p(dist.irecv, bb, r)
            out.append((bx, bb))
    elif counts[rank]:
        p2p(dist.isend, xyz.contiguous(), dst)
        p2p(dist.isend, bgr.contiguous(), dst)
    if ops:
        reqs += dist.batch_isend_irecv(ops)
    for q in reqs:
        q.wait()
    return out


BAD_SLOT = -1       # width slot of a rank whose gather arguments are invalid


def local_gather_row(clouds, n_per_rank: int, xyz_dtype=None) -> list[int]:
    """This rank's row of the count table: ``n_per_rank`` view counts (-1 = padding slot), then
    the XYZ element width (0 = no views).  Invalid arguments (more views than ``n_per_rank``,
    mixed XYZ widths, a dtype other than ``xyz_dtype``) put ``BAD_SLOT`` in the width slot
    instead of raising here: the counts all-gather is a collective, so a rank that raised before
    it would leave its peers blocked in it.  :func:`gather_plan` raises on every rank."""
    row = [-1] * (n_per_rank + 1)
    widths = {x.element_size() for x, _ in clouds}
    if (len(clouds) > n_per_rank or len(widths) > 1
            or (xyz_dtype is not None and any(x.dtype != xyz_dtype for x, _ in clouds))):
        row[n_per_rank] = BAD_SLOT
        return row
    for k, (x, _) in enumerate(clouds):
        row[k] = int(x.shape[0])
    row[n_per_rank] = widths.pop() if widths else 0
    return row


def gather_plan(table, n_per_rank: int, xyz_dtype=None):
    """The root's view of a gather from the all-gathered count table (host logic of
    :meth:`RcclCloudGather.gather`, testable without RCCL).  ``table[r]`` is rank r's
    ``n_per_rank`` view counts (-1 = padding slot) followed by its XYZ element width in bytes (0
    when it holds no views, ``BAD_SLOT`` when the rank's own arguments are invalid).  Returns
    ``(xyz dtype, counts)`` with ``counts[r]`` the real views' point counts of rank r; raises
    ``ValueError`` -- on every rank alike, since every rank holds the same table -- when a rank
    flagged its arguments or ranks disagree on the width."""
    bad = [r for r, row in enumerate(table) if int(row[n_per_rank]) == BAD_SLOT]
    if bad:
        raise ValueError(f"rank(s) {bad} passed more views than n_per_rank or clouds of mixed "
                         f"XYZ dtypes (or not of xyz_dtype)")
    seen = {int(row[n_per_rank]) for row in table} - {0}
    if xyz_dtype is not None:
        seen.add(torch.empty(0, dtype=xyz_dtype).element_size())
    if len(seen) > 1:
        raise ValueError(f"ranks hold XYZ clouds of different widths {sorted(seen)} bytes")
    if xyz_dtype is None:
        xyz_dtype = {4: torch.float32, 8: torch.float64}[seen.pop()] if seen else torch.float32
    return xyz_dtype, [[int(c) for c in row[:n_per_rank] if c >= 0] for row in table]


class RcclCloudGather:
    """The final cloud gather through the C ABI (``slg_gather_*`` over the process's RCCL):
    one communicator per job (its 128-byte id travels by a torch.distributed broadcast), then
    per gather one all-gather of the per-view counts and one grouped exact-size gatherv of XYZ
    and of BGR to the root.  Every rank calls :meth:`gather` with its block of views."""

    def __init__(self, device=None):
        import ctypes
        from . import _native as N
        self.N, self.ct = N, ctypes
        pg = dist.is_available() and dist.is_initialized()
        self.rank, self.world = (dist.get_rank(), dist.get_world_size()) if pg else (0, 1)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        uid = torch.zeros(N.GATHER_ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            N.check(N.lib().slg_gather_unique_id(ctypes.c_void_p(uid.data_ptr())))
        if not pg:
            pass
        elif dist.get_backend() == "nccl":
            d = uid.to(self.device)
            dist.broadcast(d, 0)
            uid = d.cpu()
        else:
            dist.broadcast(uid, 0)
        self._uid = uid
        self.comm = ctypes.c_void_p()
        N.check(N.lib().slg_gather_init(ctypes.byref(self.comm), self.world, self.rank,
                                        ctypes.c_void_p(uid.data_ptr())))

    def close(self):
        if self.comm:
            self.N.check(self.N.lib().slg_gather_destroy(self.comm))
            self.comm = self.ct.c_void_p()

    def gather(self, clouds, n_per_rank: int, root: int = 0, stream=None, xyz_dtype=None):
        """``clouds``: this rank's ``[(xyz [n,3], bgr [n,3] uint8), ...]`` (device tensors, at most
        ``n_per_rank`` views; a rank may hold none).  Returns on ``root`` the list over every
        rank's real views, rank-major (padding slots of ranks with fewer views are dropped), of
        ``(xyz, bgr)`` slices of one gathered device buffer; ``None`` elsewhere.

        The XYZ dtype is agreed across ranks, not guessed from a possibly empty list: every rank
        sends its element width with its counts (0 when it holds no views), ``xyz_dtype``
        (optional) fixes it, and ranks holding clouds of different widths raise ``ValueError``
        on every rank before any byte moves.  So do invalid arguments on any one rank (more
        views than ``n_per_rank``, mixed widths): they travel as a flag in the count table, and
        every rank raises after the counts all-gather instead of one rank raising before it."""
        N, ct = self.N, self.ct
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        sp = ct.c_void_p(s.cuda_stream)
        slots = n_per_rank + 1                    # per rank: view counts (-1 = padding), XYZ width
        with torch.cuda.stream(s):
            cnt = torch.tensor(local_gather_row(clouds, n_per_rank, xyz_dtype), dtype=torch.int64).to(self.device)
            allc = torch.empty(self.world * slots, dtype=torch.int64, device=self.device)
            N.check(N.lib().slg_gather_counts(self.comm, ct.c_void_p(cnt.data_ptr()), slots,
                                              ct.c_void_p(allc.data_ptr()), sp))
            table = allc.cpu().view(self.world, slots).tolist()   # sizes the root's buffers (host sync)
            dt, counts = gather_plan(table, n_per_rank, xyz_dtype)
            esz = 3 * torch.empty(0, dtype=dt).element_size()
            xs = torch.cat([x.reshape(-1, 3) for x, _ in clouds]) if clouds else torch.empty((0, 3), dtype=dt, device=self.device)
            bs = torch.cat([b.reshape(-1, 3) for _, b in clouds]) if clouds else torch.empty((0, 3), dtype=torch.uint8, device=self.device)
            per_rank = [sum(c) for c in counts]
            total = sum(per_rank)
            rx = torch.empty((total, 3), dtype=dt, device=self.device) if self.rank == root else None
            rb = torch.empty((total, 3), dtype=torch.uint8, device=self.device) if self.rank == root else None
            for send, recv, w in ((xs, rx, esz), (bs, rb, 3)):
                rbytes = (ct.c_int64 * self.world)(*[c * w for c in per_rank])
                N.check(N.lib().slg_gatherv(self.comm, ct.c_void_p(send.data_ptr()), send.shape[0] * w,
                                            ct.c_void_p(recv.data_ptr() if recv is not None else 0),
                                            rbytes, root, sp))
        self.last_buffers = (rx, rb)                      # root: the gathered job, contiguous
        if self.rank != root:
            return None
        out, off = [], 0
        for c in (c for row in counts for c in row):
            out.append((rx[off:off + c], rb[off:off + c]))
            off += c
        return out


def process_batch_sharded(calib_path, target_path, log_callback=None, process_source=None, **kw):
    """``process_multi_ply(mode='batch')`` with the view folders sharded over the ranks of the
    current process group (each rank on its own GPU).  Per-folder errors are caught and logged
    as in the reference (processing.py:323-330); rank 0 logs the job-wide summary.

    ``process_source(folder, out_path)`` defaults to the single-view drop-in path."""
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)

    def log(msg):
        if log_callback:
            log_callback(msg)
        else:
            print(msg)

    from . import processing as PR
    folders = view_folders(target_path)
    mine = shard(folders, rank, world)
    if process_source is None:
        # the single-process batch pipeline (pinned reads ahead, batched launches, writer
        # thread) on this rank's block of folders
        import scipy.io
        from . import engine as E
        data = scipy.io.loadmat(calib_path)
        calib = {k: data[k] for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow", "cam_K")}
        cfg_kw = {k: kw[k] for k in ("n_sets_col", "n_sets_row", "thresh_mode", "shadow_val",
                                     "contrast_val") if k in kw}
        cfg = E.DecodeConfig(1920, 1080, **cfg_kw)
        from .pipeline import BatchPipeline
        ok = BatchPipeline(cfg, calib, kw.get("row_mode", 1), kw.get("epipolar_tol", 2.0),
                           group=kw.get("batch_views", PR.batch_views()), log=log).run(mine, PR.batch_write_stage())
    else:
        def one(folder, _host):
            name = os.path.basename(folder) + ".ply"
            process_source(folder, os.path.join(folder, name))
            log(f"  ✔ Saved: {name}")
        ok = PR.run_view_folders(mine, log, one)
    dev = torch.device("cuda", torch.cuda.current_device()) if (
        dist.is_initialized() and dist.get_backend() == "nccl") else None
    total_ok, _ = batch_summary(ok, len(mine), dev)
    if rank == 0:
        log(f"=== Batch Complete: {total_ok}/{len(folders)} succeeded ===")
    return ok
