"""View-sharded multi-GPU processing.

Turntable views are independent (``process_multi_ply(mode='batch')`` loops over view folders,
``server/processing.py:314-334``; the auto-scan writes one folder per angle,
``server/gui.py:1718,1753``).  One process per GPU (torchrun) takes a contiguous block of
views, ``[r*V/G, (r+1)*V/G)``, and runs the whole hot path locally: no collective touches the
data path.  Two optional collectives exist for the end of a job:

* ``batch_summary`` — all-reduce of per-rank success counts so rank 0 can log the reference's
  ``=== Batch Complete: s/n succeeded ===`` line for the whole job;
* ``gather_clouds`` — gatherv of the per-view clouds to rank 0 (counts first, then padded
  XYZ/BGR buffers) over RCCL/xGMI (backend ``nccl``) or gloo, for a consumer that wants
  every point on one rank (e.g. the 360° merge that follows the path).
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


def gather_clouds(xyz: torch.Tensor, bgr: torch.Tensor, dst: int = 0):
    """Gatherv of variable-size clouds to ``dst``: returns ``[(xyz_r, bgr_r), ...]`` on ``dst``
    (rank order), ``None`` elsewhere.  ``xyz`` [n,3] float, ``bgr`` [n,3] uint8, same device
    as the process group's backend expects (CUDA for RCCL, CPU for gloo)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [(xyz, bgr)]
    world, rank = dist.get_world_size(), dist.get_rank()
    n = torch.tensor([xyz.shape[0]], dtype=torch.int64, device=xyz.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    px = torch.zeros((cap, 3), dtype=xyz.dtype, device=xyz.device)
    pb = torch.zeros((cap, 3), dtype=torch.uint8, device=xyz.device)
    px[: xyz.shape[0]] = xyz
    pb[: xyz.shape[0]] = bgr
    gx = [torch.empty_like(px) for _ in range(world)] if rank == dst else None
    gb = [torch.empty_like(pb) for _ in range(world)] if rank == dst else None
    dist.gather(px, gx, dst=dst)
    dist.gather(pb, gb, dst=dst)
    if rank != dst:
        return None
    return [(x[:c], b[:c]) for c, x, b in zip(counts, gx, gb)]


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
        # the single-process batch pipeline (prefetch read, GPU, writer thread) on this
        # rank's block of folders
        import scipy.io
        from . import engine as E
        data = scipy.io.loadmat(calib_path)
        calib = {k: data[k] for k in ("Nc", "Oc", "wPlaneCol", "wPlaneRow", "cam_K")}
        cfg_kw = {k: kw[k] for k in ("n_sets_col", "n_sets_row", "thresh_mode", "shadow_val",
                                     "contrast_val") if k in kw}
        cfg = E.DecodeConfig(1920, 1080, **cfg_kw)
        ok = PR.run_view_folders(
            mine, log, PR.batch_reconstruct_stage(cfg, calib, kw.get("row_mode", 1),
                                                  kw.get("epipolar_tol", 2.0), log),
            read=lambda f: PR.read_capture(f, cfg), write=PR.batch_write_stage())
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
