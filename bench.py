#!/usr/bin/env python
"""Benchmark: decoded+triangulated Mpoints/s of the structured-light hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): one 1920x1080 view per step, 11 column + 10 row
Gray-code bits with inverses + white/black (44 frames), Otsu mask, row_mode 1 (epipolar
filter, tol 2.0), fp32 XYZ + BGR out.  Every step does the full path for its view, inputs
resident in HBM: the stats pass (histograms -> Otsu thresholds) and the fused
decode/triangulate/compaction pass.  Steps rotate over a pool of distinct rendered turntable
views (12 x 95 MB frame stacks > 256 MiB Infinity Cache) so frames stream from HBM.  Views are
issued in batches (C3/C5 style): one fused main3 launch per batch of up to 16 views.  Default
--pipeline fused: batch k's fused launch also computes batch k+2's Otsu histograms (per-tile
partials) and a small kernel on a side stream turns them into thresholds beside batch k+1's
launch; the first two batches of a run get a regular stats pass (BatchReconstructor.
run_pipelined).  --pipeline overlap: a separate stats pass of batch k+1 on a side stream;
--pipeline serial: stats + fused launch per batch on one stream (slg_reconstruct_batch).  One process per GPU (torchrun); each rank renders its own
views (weak scaling, no data-path collective); value = all ranks' points / max-over-ranks time.

Prints ONE JSON line on stdout (rank 0).  Diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded+triangulated Mpoints/sec (1 GPU & 8-GPU node); % of HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 measured copy)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Workloads (BASELINE.json configs / SURVEY §8(d)).  c2 is the metric's configuration and the
# default; c4 / c5 are the larger single-view geometries, run on request (--config).
CONFIGS = {
    "c2": dict(cam=(1920, 1080), proj=(1920, 1080), nsets=(11, 10), n_present=44, views=12, copies=3, batch=12,
               text="C2: 1920x1080 view, 11 col + 10 row Gray bits + inverses + white/black (44 frames)"),
    "c4": dict(cam=(6000, 4000), proj=(3840, 2160), nsets=(12, 12), n_present=None, views=2, copies=2, batch=2,
               text="C4: 6000x4000 view, projector 3840x2160, 12 col + 12 row Gray bits + inverses + "
                    "white/black (50 frames)"),
    "c5": dict(cam=(3840, 2160), proj=(1920, 1080), nsets=(11, 11), n_present=None, views=4, copies=2, batch=4,
               text="C5: 3840x2160 view, projector 1920x1080, 11 col + 11 row Gray bits + inverses + "
                    "white/black (46 frames)"),
}


def cpu_baseline(views, cal, seconds, wl):
    """Oracle (NumPy port of the reference path) on this host, one thread, frames in memory."""
    import numpy as np
    from oracle import sl_oracle as O
    (PW, PH), (nc, nr) = wl["proj"], wl["nsets"]
    done, pts, t0 = 0, 0, time.perf_counter()
    while True:
        v = views[done % len(views)]
        col, row, mask = O.decode_processing(list(v.frames), n_cols=PW, n_rows=PH, n_sets_col=nc, n_sets_row=nr)
        P, _ = O.reconstruct_processing(col, row, mask, v.texture, cal, row_mode=1)
        pts += len(P)
        done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(pts / dt / 1e6, 4), "unit": "Mpoints/s", "cores": 1, "kind": "port",
            "sample": f"{done} {wl['text'].split(':')[0]} views ({wl['cam'][0]}x{wl['cam'][1]}, "
                      f"{nc}+{nr} bits, Otsu, row_mode 1), frames in "
                      f"memory, oracle/sl_oracle.py NumPy restatement, 1 thread, {dt:.1f} s"}


def load_traffic_per_view():
    """HBM bytes per view of the fused kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_main_kernel.json, written by tools/summarize_profile.py), if any."""
    p = os.path.join(ROOT, "profiles", "pmc_main_kernel.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_view")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1200)
    ap.add_argument("--warmup", type=int, default=24)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="workload (default c2, the metric's configuration)")
    ap.add_argument("--views", type=int, default=None, help="distinct rendered views")
    ap.add_argument("--copies", type=int, default=None, help="device copies of each view in the pool")
    ap.add_argument("--batch", type=int, default=None, help="views per fused launch (<= 16)")
    ap.add_argument("--xyz", choices=["f32", "f64"], default="f32")
    ap.add_argument("--pipeline", choices=["serial", "overlap", "fused"], default="fused",
                    help="serial: stats + fused launch per batch on one stream; overlap: the next "
                         "batch's stats on a side stream during this batch's fused launch; fused: "
                         "batch k's fused launch computes batch k+2's histograms")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    wl = CONFIGS[args.config]
    for k in ("views", "copies", "batch"):
        if getattr(args, k) is None:
            setattr(args, k, wl[k])

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from structured_light_for_3d_model_replication_amd import engine as E, synth, _native

    (W, H), (PW, PH), (NC, NR) = wl["cam"], wl["proj"], wl["nsets"]
    rig = synth.default_rig(W, H, PW, PH)
    cal = rig.tables()
    t = time.perf_counter()
    views = [synth.render_view(rig, view_deg=(rank * args.views + i) * 360.0 / (world * args.views),
                               seed=1000 * rank + i, n_present=wl["n_present"]) for i in range(args.views)]
    log(f"[rank {rank}] rendered {len(views)} views in {time.perf_counter() - t:.1f}s")

    cfg = E.DecodeConfig(PW, PH, NC, NR, "otsu")
    row_mode, tol, f64 = 1, 2.0, args.xyz == "f64"
    # Device pool: every rendered view uploaded `copies` times (distinct HBM buffers), so a batch
    # never shares frames with the batch before or after next -- e.g. the histograms a fused
    # launch computes for batch k+2 are cold HBM reads, as in a real turntable stream.
    dframes = [E.DeviceFrames(list(v.frames), v.texture, device=dev) for _ in range(args.copies) for v in views]
    P = len(dframes)
    dcal = E.DeviceCalib(cal, H, W, device=dev)
    B = max(1, min(args.batch, E.MAX_VIEWS_PER_LAUNCH))
    s_main = torch.cuda.Stream(device=dev)
    s_stats = torch.cuda.Stream(device=dev)
    beng = E.BatchReconstructor(H, W, B, device=dev, slots=2)
    clouds = [[E.Cloud(H * W, row_mode, f64, device=dev) for _ in range(B)] for _ in range(2)]
    preps = {}

    def prep(start, n, slot):
        """Batch of n consecutive pool views from `start` on workspace/cloud slot `slot`."""
        key = (start, n, slot)
        if key not in preps:
            fr = [dframes[(start + k) % P] for k in range(n)]
            preps[key] = beng.prepare(fr, cfg, dcal, clouds[slot][:n], row_mode, tol, slot=slot)
        return preps[key]

    # points per view: one sanity pass over the pool in batches of B (same launch shape as timed)
    pts = []
    for v0 in range(0, P, B):
        n = min(B, P - v0)
        beng.run(prep(v0, n, 0), stream=s_main)
        s_main.synchronize()
        pts += [int(clouds[0][k].count.item()) for k in range(n)]

    def batches_for(first, count):
        """Steps [first, first+count) as batches of <= B views on alternating slots."""
        out, j = [], 0
        while j < count:
            n = min(B, count - j)
            out.append(prep((first + j) % P, n, len(out) % 2))
            j += n
        return out

    K, Wm = args.steps, args.warmup
    warm = batches_for(0, Wm)
    timed = batches_for(Wm, K)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in timed]
    for a, b in ev:                                  # materialise the HIP events
        a.record(s_main)
        b.record(s_main)
    torch.cuda.synchronize()
    out_b = 30 if f64 else 18            # 3 B texture read + 12|24 B XYZ + 3 B BGR per point
    frame_b = (2 + 2 * (NC + NR)) * H * W
    total_pts, bytes_alg = 0, 0.0
    for v in range(Wm, Wm + K):
        total_pts += pts[v % P]
        bytes_alg += frame_b + out_b * pts[v % P]

    def run_all(batches, events=None):
        if args.pipeline in ("overlap", "fused"):
            beng.run_pipelined(batches, s_main, s_stats, events=events, mode=args.pipeline)
        else:
            for k, pb in enumerate(batches):
                beng.run(pb, events=None if events is None else events[k], stream=s_main)

    if warm:
        run_all(warm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_all(timed, events=[(a.cuda_event, b.cuda_event) for a, b in ev])
    t_enq = time.perf_counter() - t0              # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev)
    n_launch = len(ev)
    helper_runs = sum(int(np.frombuffer(beng.header(s, k)[3084:3088].cpu().numpy().tobytes(), np.uint32)[0] & 2 != 0)
                      for s in range(2) for k in range(B))

    stats = torch.tensor([dt, float(total_pts), kern_ms, bytes_alg], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = stats[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        sums = stats[1:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        dt_max = float(tmax.item())
        all_pts, kern_sum, bytes_sum = (float(x) for x in sums.tolist())
    else:
        dt_max, all_pts, kern_sum, bytes_sum = dt, float(total_pts), kern_ms, bytes_alg

    if rank == 0:
        launches = n_launch * world
        kern_avg_s = kern_sum / launches / 1e3
        achieved = bytes_sum / launches / kern_avg_s / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # committed PMC bytes are per C2 view: other workloads report none
                "traffic": (round(load_traffic_per_view() * K / n_launch)
                            if load_traffic_per_view() and args.config == "c2" else None),
                "kernel": "main3_kernel<1,0,1,1> (fused decode+triangulate+compaction, "
                          f"{B} views per launch)",
                "kernel_avg_us": round(kern_avg_s * 1e6, 2),
                "alg_bytes_per_launch": round(bytes_sum / launches)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(views, cal, args.cpu_seconds, wl)
        out = {
            "metric": METRIC,
            "value": round(all_pts / dt_max / 1e6, 2),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(dt_max / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{wl['text']}, Otsu, row_mode 1 tol 2.0, XYZ {args.xyz} + BGR out",
                       "views_per_rank": len(views), "device_pool": P, "points_per_view": int(np.mean(pts)),
                       "batch_views": B,
                       "launches": n_launch,
                       "stats_pipeline": args.pipeline,
                       "lookback_helper_runs": helper_runs,
                       "host_enqueue_ms_per_step": round(t_enq / K * 1e3, 4),
                       "decode": "u8 compares, int32 codes; triangulation f64",
                       "parallelism": f"view-sharded x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
