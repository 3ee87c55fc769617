"""``bench.py --config c3``: the 36-view 360-degree turntable scan (BASELINE.json configs[2]) as ONE
job per step, views sharded across the ranks (strong scaling).

Per step every rank runs the whole path on its contiguous block of the scan's views, resident
in HBM (``distributed.shard_range``): per group of <= 12 views one batched stats launch and one
fused decode/triangulate launch (``BatchReconstructor.run``), then every rank copies its own
clouds to its own pinned host memory (the node's host memory holds the whole scan when the step
ends: the "host point-cloud gather" of the config).  That is what the product does -- the sharded
batch (``distributed.process_batch_sharded``, ``cli_batch.py``) writes each rank's PLYs from its
own host copies, with no collective -- so it is the headline ``value``.  Beside it
(``gather_to_rank0``): the north star's RCCL variant, the clouds gathered to rank 0 through the
C ABI (``slg_gather_counts`` + ``slg_gatherv``, exact sizes) and copied to host there, for a
consumer that wants the whole scan in one process; it funnels the scan through rank 0's PCIe
link, so it does not scale with N.  Reference CPU path: ``server/processing.py:314-334`` (a
serial loop over view folders).
"""
from __future__ import annotations

import json
import os
import sys
import time

import bench
from bench import log


def main(args, wl):
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    from structured_light_for_3d_model_replication_amd import synth, distributed as D

    V = args.views
    lo, hi = D.shard_range(V, rank, world)
    n_per_rank = (V + world - 1) // world
    (W, H), (PW, PH), (NC, NR) = wl["cam"], wl["proj"], wl["nsets"]
    rig = synth.default_rig(W, H, PW, PH)
    cal = rig.tables()
    t = time.perf_counter()
    views = {i: synth.render_view(rig, view_deg=360.0 * i / V, seed=i, n_present=wl["n_present"]) for i in range(lo, hi)}
    log(f"[rank {rank}] rendered views {lo}..{hi - 1} in {time.perf_counter() - t:.1f}s")
    cpu = bench.rank0_cpu_baseline(args, rank, [views[i] for i in range(lo, hi)], cal, wl)
    if args.cpu_baseline_only:
        return bench.cpu_baseline_only(args, rank, world, cpu)

    # the one-GPU rehearsal knobs of bench.py (never set by the driver): every rank on one
    # device, gloo instead of RCCL -- the gather then goes through host memory (two RCCL ranks
    # cannot share a GPU)
    if os.environ.get("SLG_BENCH_DEVICE"):
        local = int(os.environ["SLG_BENCH_DEVICE"])
    backend = os.environ.get("SLG_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from structured_light_for_3d_model_replication_amd import engine as E

    cfg = E.DecodeConfig(PW, PH, NC, NR, "otsu")
    row_mode, tol, f64 = 1, 2.0, args.xyz == "f64"
    mine = list(range(lo, hi))
    dframes = [E.DeviceFrames(list(views[i].frames), views[i].texture, device=dev) for i in mine]
    dcal = E.DeviceCalib(cal, H, W, device=dev)
    B = max(1, min(args.batch, E.MAX_VIEWS_PER_LAUNCH))
    groups = [list(range(g, min(g + B, len(mine)))) for g in range(0, len(mine), B)]
    beng = E.BatchReconstructor(H, W, B, device=dev, slots=max(1, len(groups)))
    clouds = [E.Cloud(H * W, row_mode, f64, device=dev) for _ in mine]
    preps = [beng.prepare([dframes[k] for k in g], cfg, dcal, [clouds[k] for k in g], row_mode, tol, slot=j)
             for j, g in enumerate(groups)]
    s = torch.cuda.Stream(device=dev)
    gather = D.RcclCloudGather(device=dev) if backend == "nccl" else None
    sizes = [D.shard_range(V, r, world) for r in range(world)]

    def host_gather(parts):
        """Rehearsal gather (gloo): per view slot, host copies through gather_clouds."""
        by_rank = [[] for _ in range(world)]
        for k in range(n_per_rank):
            x, b = parts[k] if k < len(parts) else (clouds[0].xyz[:0], clouds[0].bgr[:0])
            res = D.gather_clouds(x.cpu(), b.cpu(), dst=0)
            if res is not None:
                for r, (rx_, rb_) in enumerate(res):
                    if k < sizes[r][1] - sizes[r][0]:
                        by_rank[r].append((rx_, rb_))
        return [c for r in by_rank for c in r] if rank == 0 else None
    host_x = host_b = None
    own_x = own_b = None
    own_counts = []
    d2h_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    d2h_ms = [0.0]                     # this rank's D2H copy time over the timed steps

    def reconstruct():
        for pb in preps:
            beng.run(pb, stream=s)
        s.synchronize()               # per-view slices need the counts on the host
        return [int(c.count.item()) for c in clouds]

    def d2h_step():
        """The product's step: reconstruct this rank's views, copy its own clouds to its own
        pinned host memory (no collective)."""
        nonlocal own_x, own_b, own_counts
        counts = reconstruct()
        if own_x is None or own_x.shape[0] < sum(counts):
            own_x = torch.empty((max(1, sum(counts)), 3), dtype=clouds[0].xyz.dtype, pin_memory=True)
            own_b = torch.empty((max(1, sum(counts)), 3), dtype=torch.uint8, pin_memory=True)
        off = 0
        with torch.cuda.stream(s):
            d2h_ev[0].record(s)
            for c, n in zip(clouds, counts):
                own_x[off:off + n].copy_(c.xyz[:n], non_blocking=True)
                own_b[off:off + n].copy_(c.bgr[:n], non_blocking=True)
                off += n
            d2h_ev[1].record(s)
        own_counts = counts

    def gather_step():
        """The RCCL variant: reconstruct, gather every rank's clouds to rank 0, D2H there."""
        nonlocal host_x, host_b
        counts = reconstruct()
        parts = [(c.xyz[:n], c.bgr[:n]) for c, n in zip(clouds, counts)]
        if gather is None:
            return host_gather(parts)
        got = gather.gather(parts, n_per_rank, root=0, stream=s)
        if rank == 0:
            rx, rb = gather.last_buffers
            if host_x is None or host_x.shape[0] < rx.shape[0]:
                host_x = torch.empty((max(1, rx.shape[0]), 3), dtype=rx.dtype, pin_memory=True)
                host_b = torch.empty((max(1, rx.shape[0]), 3), dtype=torch.uint8, pin_memory=True)
            with torch.cuda.stream(s):
                host_x[: rx.shape[0]].copy_(rx, non_blocking=True)
                host_b[: rb.shape[0]].copy_(rb, non_blocking=True)
        return got

    def timed(fn, k, local=None):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
            if fn is d2h_step:             # (the step's own sync on its counts orders the events)
                d2h_ev[1].synchronize()
                d2h_ms[0] += d2h_ev[0].elapsed_time(d2h_ev[1])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        mine_s = time.perf_counter() - t0
        if local is not None:
            local.append(mine_s)
        dt = torch.tensor([mine_s], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    K, Wm = args.steps, args.warmup
    for _ in range(max(1, Wm)):
        d2h_step()
        gather_step()
    torch.cuda.synchronize()
    # reconstruct-only kernel time of this rank: HIP events around each fused launch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in preps]
    for a, b in ev:                                  # materialise the HIP events
        a.record(s)
        b.record(s)
    for (a, b), pb in zip(ev, preps):
        beng.run(pb, events=[a.cuda_event, b.cuda_event], stream=s)
    torch.cuda.synchronize()
    kern_ms = sum(a.elapsed_time(b) for a, b in ev)

    local_dt = []
    d2h_ms[0] = 0.0
    dt = timed(d2h_step, K, local_dt)
    dt_gather = timed(gather_step, K)
    got = gather_step()
    d2h_step()
    torch.cuda.synchronize()
    counts_local = list(own_counts)
    # per-rank rows beside the max-over-ranks headline: kernels, D2H, the rank's own step time
    per_rank = D.per_rank_table({"views": len(mine), "points": sum(counts_local), "kernel_ms": kern_ms,
                                 "d2h_ms": d2h_ms[0] / K, "step_ms": local_dt[0] / K * 1e3}, device=dev)
    pts_local = torch.tensor([float(sum(counts_local))], dtype=torch.float64, device=dev)
    kern = torch.tensor([kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(pts_local)
        dist.all_reduce(kern, op=dist.ReduceOp.MAX)
    all_pts = float(pts_local.item())

    verify = None
    if rank == 0 and not args.no_verify:
        gathered = [g[0].shape[0] for g in got]
        view_ok = None
        from oracle import sl_oracle as O
        vw = views[lo]
        oc, orow, om = O.decode_processing(list(vw.frames), n_cols=PW, n_rows=PH, n_sets_col=NC, n_sets_row=NR)
        Po, Co = O.reconstruct_processing(oc, orow, om, vw.texture, cal, row_mode=1)
        n0 = counts_local[0]
        hx = own_x[:n0].double().numpy()             # rank 0's host copy of its first view
        if n0 == len(Po):
            rel = float(np.max(np.abs(hx - Po) / np.maximum(np.abs(Po), 1e-3)))
            view_ok = bool(np.array_equal(own_b[:n0].numpy(), Co) and rel <= (0.0 if f64 else 1e-4)
                           and torch.equal(got[0][0].cpu(), own_x[:n0]))
        verify = {"gathered_views": len(gathered), "gathered_points": int(sum(gathered)),
                  "gathered_equals_all_ranks": bool(sum(gathered) == int(all_pts)),
                  "rank0_counts_match": gathered[: len(counts_local)] == counts_local,
                  "oracle_view0_ok": view_ok}
        verify["ok"] = bool(verify["gathered_equals_all_ranks"] and verify["rank0_counts_match"] and view_ok)
        if not verify["ok"]:
            log(f"VERIFY FAILED: {verify}")
    if rank == 0:
        frame_b = (2 + 2 * (NC + NR)) * H * W
        out_b = 30 if f64 else 18
        bytes_rank0 = len(mine) * frame_b + out_b * sum(counts_local)
        kern_s = float(kern.item()) / 1e3
        achieved = bytes_rank0 / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else None
        out = {
            "metric": bench.METRIC,
            "value": None if verify is not None and not verify["ok"] else round(all_pts / (dt / K) / 1e6, 2),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(dt / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{wl['text']}, Otsu, row_mode 1 tol 2.0, XYZ {args.xyz} + BGR out",
                       "step": "the whole 36-view job: reconstruct (sharded) + every rank's clouds copied to its own "
                               "pinned host memory (what process_batch_sharded / cli_batch do; no collective)",
                       "views": V, "views_rank0": len(mine), "points_per_job": int(all_pts),
                       "reconstruct_kernel_ms_max_rank": round(kern_s * 1e3, 4),
                       "gather_to_rank0": {"ms_per_step": round(dt_gather / K * 1e3, 4),
                                           "value": round(all_pts / (dt_gather / K) / 1e6, 2),
                                           "what": ("RCCL gatherv (C ABI) of every rank's clouds to rank 0, then D2H "
                                                    "there" if gather is not None else
                                                    f"{backend} host gather (rehearsal)")},
                       "batch_views": B,
                       "per_rank": per_rank,
                       "per_rank_what": "each rank's views, points, reconstruct kernel ms (HIP events), D2H ms per "
                                        "step (HIP events around its copies) and own step ms; the headline is the "
                                        "max over ranks",
                       "parallelism": f"view-sharded x{world}, per-rank D2H"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                         "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / bench.HBM_PEAK_GBS, 4) if achieved else None, "traffic": None,
                         "kernel": "stats + main3_kernel launches of rank 0's views (HIP events)"},
            "cpu_baseline": cpu,
            "verify": verify,
        }
        print(json.dumps(out), file=getattr(args, "result_out", None) or sys.stdout, flush=True)
    if gather is not None:
        gather.close()
    if world > 1:
        dist.destroy_process_group()
    if verify is not None and not verify["ok"]:
        sys.exit(1)
