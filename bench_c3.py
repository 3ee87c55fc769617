"""``bench.py --config c3``: the 36-view 360-degree turntable scan (BASELINE.json configs[2]) as ONE
job per step, views sharded across the ranks (strong scaling).

Per step every rank runs the whole path on its contiguous block of the scan's views, resident
in HBM (``distributed.shard_range``): per group of <= 12 views one batched stats launch and one
fused decode/triangulate launch (``BatchReconstructor.run``), then the final point-cloud gather
to rank 0 through the C ABI over RCCL (``slg_gather_counts`` + ``slg_gatherv``, exact sizes),
then rank 0 copies the job's cloud to pinned host memory (the "host point-cloud gather" of the
config).  The alternative the survey asks to report -- every rank copying its own clouds to
host memory, no collective -- is timed separately (``alt_per_rank_d2h``).  Reference CPU path:
``server/processing.py:314-334`` (a serial loop over view folders).
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
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = bench.cpu_baseline([views[i] for i in range(lo, hi)], cal, args.cpu_seconds, wl)

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

    def step():
        """One whole-job step: reconstruct this rank's views, gather to rank 0, D2H there."""
        nonlocal host_x, host_b
        for pb in preps:
            beng.run(pb, stream=s)
        s.synchronize()               # per-view slices need the counts on the host
        parts = []
        for c in clouds:
            n = int(c.count.item())
            parts.append((c.xyz[:n], c.bgr[:n]))
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

    def alt_step():
        """The alternative: every rank copies its own clouds to its own pinned host memory."""
        nonlocal own_x, own_b
        for pb in preps:
            beng.run(pb, stream=s)
        s.synchronize()
        counts = [int(c.count.item()) for c in clouds]
        if own_x is None or own_x.shape[0] < sum(counts):
            own_x = torch.empty((max(1, sum(counts)), 3), dtype=clouds[0].xyz.dtype, pin_memory=True)
            own_b = torch.empty((max(1, sum(counts)), 3), dtype=torch.uint8, pin_memory=True)
        off = 0
        with torch.cuda.stream(s):
            for c, n in zip(clouds, counts):
                own_x[off:off + n].copy_(c.xyz[:n], non_blocking=True)
                own_b[off:off + n].copy_(c.bgr[:n], non_blocking=True)
                off += n

    def timed(fn, k):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    K, Wm = args.steps, args.warmup
    for _ in range(max(1, Wm)):
        got = step()
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

    dt = timed(step, K)
    dt_alt = timed(alt_step, K)
    got = step()
    torch.cuda.synchronize()
    counts_local = [int(c.count.item()) for c in clouds]
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
        gx = got[0][0].double().cpu().numpy()
        if len(gx) == len(Po):
            rel = float(np.max(np.abs(gx - Po) / np.maximum(np.abs(Po), 1e-3)))
            view_ok = bool(np.array_equal(got[0][1].cpu().numpy(), Co) and rel <= (0.0 if f64 else 1e-4))
        verify = {"gathered_views": len(gathered), "gathered_points": int(sum(gathered)),
                  "gathered_equals_all_ranks": bool(sum(gathered) == int(all_pts)),
                  "rank0_counts_match": gathered[: len(counts_local)] == counts_local,
                  "oracle_view0_ok": view_ok}
        if not (verify["gathered_equals_all_ranks"] and verify["rank0_counts_match"] and view_ok):
            log(f"VERIFY FAILED: {verify}")
    if rank == 0:
        frame_b = (2 + 2 * (NC + NR)) * H * W
        out_b = 30 if f64 else 18
        bytes_rank0 = len(mine) * frame_b + out_b * sum(counts_local)
        kern_s = float(kern.item()) / 1e3
        achieved = bytes_rank0 / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else None
        out = {
            "metric": bench.METRIC,
            "value": round(all_pts / (dt / K) / 1e6, 2),
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
                       "step": "the whole 36-view job: reconstruct (sharded) + RCCL gatherv to rank 0 + D2H to "
                               "pinned host memory on rank 0",
                       "views": V, "views_rank0": len(mine), "points_per_job": int(all_pts),
                       "reconstruct_kernel_ms_max_rank": round(kern_s * 1e3, 4),
                       "alt_per_rank_d2h": {"ms_per_step": round(dt_alt / K * 1e3, 4),
                                            "value": round(all_pts / (dt_alt / K) / 1e6, 2),
                                            "what": "each rank copies its own clouds to its own pinned host "
                                                    "memory, no collective"},
                       "batch_views": B,
                       "parallelism": f"view-sharded x{world} + " + ("RCCL gatherv (C ABI)" if gather is not None
                                                                    else f"{backend} host gather (rehearsal)")},
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
