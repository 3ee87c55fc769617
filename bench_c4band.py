"""``bench.py --config c4band``: BASELINE.json configs[3] -- ONE 24 MP (6000x4000) capture,
projector 3840x2160, 12 + 12 Gray bits + inverses + white/black (50 frames) -- split over the
ranks by bands of rows (strong scaling; SURVEY §8(e) "single huge view", ``bands.py``).

Every rank holds its band of the view in HBM (rows ``bands.band_rows``, 1.2 GB / N of frames).
One step is the whole view: on every rank the band's histograms (``slg_decode_histograms``),
the one exchange step (RCCL all-reduce of 513 int32: the bins summed, the max code maxed), the
view's thresholds (``slg_thresholds_from_histograms``) and the fused decode + triangulate launch
over the band; the step ends when every rank's band is done (barrier + max over ranks).  At N = 1
the one band is the whole view through the same calls.  Reference path:
``server/processing.py:28-234`` on one capture (``_gray_decode`` + ``_reconstruct_point_cloud``).

Verification (outside the timing): the bands' clouds gathered to rank 0 and reassembled
(``bands.gather_banded``) equal the unsplit view's cloud from the single-view fused path, bit for
bit (``--no-verify`` skips it).
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
    from structured_light_for_3d_model_replication_amd import synth

    (W, H), (PW, PH), (NC, NR) = wl["cam"], wl["proj"], wl["nsets"]
    rig = synth.default_rig(W, H, PW, PH)
    cal = rig.tables()
    t = time.perf_counter()
    view = synth.render_view(rig, view_deg=30.0, seed=4, n_present=wl["n_present"])
    log(f"[rank {rank}] rendered the view in {time.perf_counter() - t:.1f}s")
    cpu = bench.rank0_cpu_baseline(args, rank, [view], cal, wl)
    if args.cpu_baseline_only:
        return bench.cpu_baseline_only(args, rank, world, cpu)

    if os.environ.get("SLG_BENCH_DEVICE"):           # one-GPU rehearsal (bench.py): never the driver's
        local = int(os.environ["SLG_BENCH_DEVICE"])
    backend = os.environ.get("SLG_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from structured_light_for_3d_model_replication_amd import bands as B, engine as E

    r0, r1 = B.band_rows(H, rank, world)
    cfg = E.DecodeConfig(PW, PH, NC, NR, "otsu")
    row_mode, tol, f64 = 1, 2.0, args.xyz == "f64"
    band = E.DeviceFrames([np.ascontiguousarray(np.asarray(f)[r0:r1]) for f in view.frames],
                          np.ascontiguousarray(view.texture[r0:r1]), device=dev)
    dcal = E.DeviceCalib(cal, H, W, device=dev)
    bcal = B.band_calib(dcal, r0, r1)
    rec = B.BandReconstructor(H, W, r0, r1, device=dev)
    out = E.Cloud(band.n_px, row_mode, f64, device=dev)

    def step():
        rec.run(band, cfg, bcal, row_mode, tol, f64, out=out, sync=False)

    def timed(k):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    K, Wm = args.steps, args.warmup
    timed(max(1, Wm))
    # this rank's step on the GPU alone: HIP events around the band's three launches (+ exchange)
    s = torch.cuda.current_stream(dev)
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.record(s)
    for _ in range(K):
        step()
    eb.record(s)
    torch.cuda.synchronize()
    band_ms = ea.elapsed_time(eb) / K
    dt_local = timed(K)
    dt = torch.tensor([dt_local], dtype=torch.float64, device=dev)
    n_band = int(out.count.item())
    pts = torch.tensor([float(n_band)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        dist.all_reduce(pts)
    dt, all_pts = float(dt.item()), float(pts.item())

    verify = None
    if not args.no_verify:
        xyz, bgr = out.xyz[:n_band], out.bgr[:n_band]
        if backend != "nccl" and world > 1:
            xyz, bgr = xyz.cpu(), bgr.cpu()
        got = B.gather_banded(xyz, bgr, None, row_mode, dst=0)
        if rank == 0:
            whole = E.DeviceFrames(list(view.frames), view.texture, device=dev)
            one = E.Reconstructor(H, W, device=dev)
            wx, wb = one.reconstruct(whole, cfg, dcal, row_mode, tol, xyz_f64=f64).result()
            same = bool(got[0].shape == wx.shape and torch.equal(got[0].to(dev), wx) and torch.equal(got[1].to(dev), wb))
            verify = {"bands": world, "points": int(got[0].shape[0]), "equals_unsplit_view_bitwise": same}
            if not same:
                log(f"VERIFY FAILED: {verify}")
    if rank == 0:
        frame_b = bench.frames_used(wl) * W * (r1 - r0)
        out_b = 30 if f64 else 18
        band_bytes = frame_b + out_b * n_band
        achieved = band_bytes / (band_ms / 1e3) / 1e9
        res = {
            "metric": bench.METRIC,
            "value": None if verify is not None and not verify["equals_unsplit_view_bitwise"] else round(all_pts / (dt / K) / 1e6, 2),
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
                       "step": "the whole view: on every rank its band's histograms, the RCCL all-reduce of the "
                               "histograms, the view's thresholds and the fused launch over the band",
                       "bands": world, "rows_rank0": r1 - r0, "points_per_view": int(all_pts),
                       "rank0_band_ms": round(band_ms, 4),
                       "parallelism": f"row bands x{world}, one all-reduce per view"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / bench.HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "rank 0's band: stats_kernel (histograms only) + hist_thresholds_kernel + "
                                   "main3_kernel, HIP events around the step",
                         "alg_bytes_per_launch": band_bytes,
                         "alg_bytes": f"SURVEY 8(d): (2 + 2(nc+nr)) B per pixel of the band + {out_b} B per point"},
            "cpu_baseline": cpu,
            "verify": verify,
        }
        print(json.dumps(res), file=getattr(args, "result_out", None) or sys.stdout, flush=True)
        if verify is not None and not verify["equals_unsplit_view_bitwise"]:
            sys.exit(1)
    if world > 1:
        dist.destroy_process_group()
