"""``bench.py --config c5job``: BASELINE.json configs[4] -- a scan-farm batch of 8 objects x 72
views at 3840x2160 (projector 1920x1080, 11 + 11 Gray bits + inverses + white/black, 46 frames),
every view resident in HBM, reconstructed as ONE job per step (strong scaling).

Reference flow: per object an auto-scan writes one capture folder per turntable angle
(``server/gui.py:1700-1787``), then ``process_multi_ply(mode='batch')`` reconstructs the folders
in a serial loop (``server/processing.py:314-334``).  Here the job's 576 views are sharded over
the ranks in contiguous blocks (``distributed.shard_range``: all 576 on one GPU -- 220 GB of
frames + 14 GB of textures + the clouds fit its 288 GB -- or 72 per rank, one object each, on
8), staged in HBM, and one step is :class:`jobs.ResidentJob` over the rank's block: fused
launches of ``--batch`` views on the two-stream carried-Otsu pipeline, every cloud written to its
own region of one packed arena.  The job sizes itself inside its own launches: the kernel that
finishes a view's Otsu thresholds also reserves the view's arena region with one atomicAdd on a
device cursor (min(#white >= smin, #(white - black) >= cmin) points, an upper bound of its count:
jobs.ResidentJob's device-reserved arena) -- no sizing pass, no host sync, nothing to add to the
step time.

Views of one object come from ``--distinct`` rendered captures per object (synth.render_view,
seed 1000*object + k, staggered turntable angles), each job view an HBM copy of its own: the
kernel streams every view's 381.5 MB from HBM, as it would distinct captures.  The timed region
is the whole job, its four priming stats passes and every reservation included.  Verification
(outside the timing): no view is refused by the arena, the reserved regions are disjoint, every view's cloud equals
its source's single-view cloud bit for bit, and one source's cloud equals the oracle's; a failed
verification makes ``value`` null and the exit status non-zero.
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
    from structured_light_for_3d_model_replication_amd import distributed as D, synth

    n_obj, per_obj = args.objects, args.views_per_object
    distinct = max(1, min(args.distinct, per_obj))
    V = n_obj * per_obj
    lo, hi = D.shard_range(V, rank, world)
    (W, H), (PW, PH), (NC, NR) = wl["cam"], wl["proj"], wl["nsets"]

    def source_of(j):                                    # job view -> (object, distinct capture)
        o, a = divmod(j, per_obj)
        return o, a * distinct // per_obj

    keys = sorted({source_of(j) for j in range(lo, hi)})
    rig = synth.default_rig(W, H, PW, PH)
    cal = rig.tables()
    t = time.perf_counter()
    quota = bench.cpu_quota() or os.cpu_count() or 1
    specs = [(synth.job_view_angle(o, k * per_obj // distinct, per_obj), 1000 * o + k, wl["n_present"]) for o, k in keys]
    rendered = synth.render_many(rig, specs, workers=min(8, quota, len(specs)))
    src = dict(zip(keys, rendered))
    log(f"[rank {rank}] rendered {len(keys)} captures for job views {lo}..{hi - 1} in {time.perf_counter() - t:.1f}s")
    cpu = bench.rank0_cpu_baseline(args, rank, rendered[: max(1, min(4, len(rendered)))], cal, wl)
    if args.cpu_baseline_only:
        return bench.cpu_baseline_only(args, rank, world, cpu)

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
    from structured_light_for_3d_model_replication_amd import engine as E, jobs as J

    cfg = E.DecodeConfig(PW, PH, NC, NR, "otsu")
    row_mode, tol = 1, 2.0
    dcal = E.DeviceCalib(cal, H, W, device=dev)
    sources = [E.DeviceFrames(list(src[k].frames), src[k].texture, device=dev) for k in keys]
    del rendered, src
    # each capture once through the single-view path: the clouds the job must reproduce
    # (verification only; the job sizes itself)
    rec = E.Reconstructor(H, W, device=dev)
    first = []
    for s in sources:
        c = rec.reconstruct(s, cfg, dcal, row_mode, tol, xyz_f64=False)
        x, b = c.result()
        first.append((x.clone(), b.clone()))
    src_counts = [int(x.shape[0]) for x, _ in first]
    seg = [bench.mask_first_segments(s, cfg, H, W, dev) for s in sources]
    plan = [keys.index(source_of(j)) for j in range(lo, hi)]
    exact = [src_counts[p] for p in plan]

    n_views = hi - lo
    F = sources[0].n_frames
    per_view = F * sources[0].stride + 3 * H * W
    # (a pre-check only: the reservations, an upper bound of the counts, are made by the job)
    need = n_views * per_view + int(1.15 * sum(exact)) * 15 + 4 * args.batch * 4 * (1 << 26)
    free, total = torch.cuda.mem_get_info(dev)
    log(f"[rank {rank}] staging {n_views} views: {n_views * per_view / 1e9:.1f} GB of frames + textures, "
        f"~{sum(exact) * 15 / 1e9:.1f} GB of clouds; HBM free {free / 1e9:.1f} of {total / 1e9:.1f} GB")
    if need > free:
        raise SystemExit(f"c5job: needs ~{need / 1e9:.1f} GB of HBM on rank {rank}, {free / 1e9:.1f} GB free "
                         f"(use more ranks or fewer --objects/--views-per-object)")
    t = time.perf_counter()
    views = []
    for j0 in range(0, n_views, 36):
        views += J.stage_copies(sources, plan[j0:j0 + 36], device=dev)
        torch.cuda.synchronize()
        log(f"[rank {rank}] staged {len(views)}/{n_views} views ({time.perf_counter() - t:.1f}s)")
    B = max(1, min(args.batch, E.MAX_VIEWS_PER_LAUNCH))
    # the job reserves each view's arena region itself, inside its launches (device cursor)
    job = J.ResidentJob(views, cfg, dcal, batch=B, row_mode=row_mode, epipolar_tol=tol, xyz_f64=False,
                        device=dev)
    log(f"[rank {rank}] device-reserved arena of {job.arena_points * 15 / 1e9:.2f} GB "
        f"(exact counts take {sum(exact) * 15 / 1e9:.2f} GB)")
    s0, s1 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    K, Wm = args.steps, args.warmup
    for _ in range(max(1, Wm)):
        job.run(s0, s1)
    torch.cuda.synchronize()
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(s0)
    for _ in range(K):
        job.run(s0, s1)
    ev[1].record(s0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = ev[0].elapsed_time(ev[1])

    counts = job.host_counts()
    offs = job.host_offsets()
    reserved = int(job.cursor.item())                     # points the last job reserved
    verify = None
    if not args.no_verify:
        over = job.overflowed(counts)
        spans = sorted((o, o + n) for o, n in zip(offs, counts) if o >= 0)
        disjoint = all(a[1] <= b[0] for a, b in zip(spans, spans[1:])) and (not spans or spans[-1][1] <= job.arena_points)
        same = all(torch.equal(job.cloud(j, counts)[0], first[plan[j]][0]) and
                   torch.equal(job.cloud(j, counts)[1], first[plan[j]][1]) for j in range(n_views))
        verify = {"views": n_views, "counts_equal_single_view_path": counts == exact, "refused": over,
                  "regions_disjoint": bool(disjoint), "damaged": job.damaged(counts),
                  "clouds_equal_single_view_path_bitwise": bool(same)}
        if rank == 0:
            from oracle import sl_oracle as O
            k0 = keys[0]
            o_, k_ = k0
            vw = synth.render_view(rig, view_deg=synth.job_view_angle(o_, k_ * per_obj // distinct, per_obj),
                                   seed=1000 * o_ + k_, n_present=wl["n_present"])
            oc, orow, om = O.decode_processing(list(vw.frames), n_cols=PW, n_rows=PH, n_sets_col=NC, n_sets_row=NR)
            Po, Co = O.reconstruct_processing(oc, orow, om, vw.texture, cal, row_mode=1)
            gx = first[0][0].double().cpu().numpy()
            rel = float(np.max(np.abs(gx - Po) / np.maximum(np.abs(Po), 1e-3))) if len(gx) == len(Po) else None
            verify.update(oracle_source=str(k0), oracle_count_equal=bool(len(Po) == len(gx)),
                          oracle_colours_equal=bool(len(Po) == len(gx) and np.array_equal(first[0][1].cpu().numpy(), Co)),
                          oracle_xyz_max_rel=rel)
            verify["oracle_ok"] = bool(verify["oracle_colours_equal"] and rel is not None and rel <= 1e-4)
        ok = (verify["counts_equal_single_view_path"] and not over and disjoint and same
              and verify.get("oracle_ok", True))
        verify["ok"] = bool(ok)
        if not ok:
            log(f"[rank {rank}] VERIFY FAILED: {verify}")
    ok_t = torch.tensor([0.0 if (verify is not None and not verify["ok"]) else 1.0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
    all_ok = bool(ok_t.item() == 1.0)

    frame_b = (2 + 2 * (NC + NR)) * H * W
    pts_local = float(sum(counts))
    dense_local = n_views * frame_b + 18.0 * pts_local
    mf_local = sum(2 * H * W + 64 * seg[p] for p in plan) + 18.0 * pts_local
    stats = torch.tensor([pts_local, dense_local, mf_local, float(n_views)], dtype=torch.float64, device=dev)
    tk = torch.tensor([dt, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats)
        dist.all_reduce(tk, op=dist.ReduceOp.MAX)
    all_pts, dense, mf, all_views = (float(x) for x in stats.tolist())
    dt_max, kern_max = (float(x) for x in tk.tolist())
    if rank == 0:
        job_s = kern_max / 1e3 / K                     # HIP events on s0 around the K jobs / K
        achieved = dense / job_s / 1e9 / world         # per GPU: each rank streams its own block
        mf_ach = mf / job_s / 1e9 / world
        value = round(all_pts / (dt_max / K) / 1e6, 2)
        out = {
            "metric": bench.METRIC,
            "value": value if all_ok else None,
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(dt_max / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{wl['text']}, Otsu, row_mode 1 tol 2.0, XYZ f32 + BGR out",
                       "step": f"the whole job: {int(all_views)} HBM-resident views ({n_obj} objects x {per_obj} "
                               f"views), fused launches of {B} views on the two-stream carried-Otsu pipeline, "
                               "every cloud kept in HBM (packed arena)",
                       "views": int(all_views), "views_rank0": n_views, "objects": n_obj,
                       "views_per_object": per_obj, "distinct_captures_per_object": distinct,
                       "points_per_job": int(all_pts), "points_per_view": int(all_pts / max(1.0, all_views)),
                       "us_per_view": round(dt_max / K / max(1.0, all_views / world) * 1e6, 3),
                       "job_ms_events": round(job_s * 1e3, 4), "batch_views": B,
                       "capacity": {
                           "source": "device-reserved arena (jobs.ResidentJob, slg_workspace_set_arena): the kernel "
                                     "that finishes a view's Otsu thresholds reserves min(#white >= smin, "
                                     "#(white-black) >= cmin) points with one atomicAdd -- inside the timed job, "
                                     "no sizing pass",
                           "arena_gb_rank0": round(job.arena_points * 15 / 1e9, 2),
                           "reserved_gb_rank0": round(reserved * 15 / 1e9, 2),
                           "exact_counts_gb_rank0": round(sum(exact) * 15 / 1e9, 2),
                           "reserved_over_count": round(reserved / max(1, sum(exact)), 4)},
                       "hbm_resident_gb_rank0": round(n_views * per_view / 1e9, 1),
                       "parallelism": f"view-sharded x{world} (contiguous blocks of the job), no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / bench.HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": f"main3_kernel (fused decode+triangulate+compaction, {B} views per launch) + 4 "
                                   "priming stats passes per job",
                         "kernel_avg_us": round(job_s * 1e6 / max(1, len(job.batches)), 2),
                         "kernel_time": "HIP events on the job's first stream around the K jobs (both streams "
                                        "joined) / K / launches per job",
                         "alg_bytes": "SURVEY 8(d): (2 + 2(nc+nr)) B per pixel + 18 B per point, per GPU",
                         "mask_first": {"achieved": round(mf_ach, 1), "frac": round(mf_ach / bench.HBM_PEAK_GBS, 4)}},
            "cpu_baseline": cpu,
            "verify": verify,
        }
        print(json.dumps(out), file=getattr(args, "result_out", None) or sys.stdout, flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not all_ok:
        raise SystemExit(3)                               # a wrong job is not a measurement
