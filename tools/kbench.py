#!/usr/bin/env python
"""Per-kernel microbenchmark (one process, interleaved variants, HIP events on the launch
stream).  Usage on the GPU box:  python tools/kbench.py [--iters 50] [--size 1920x1080]

Reports, per variant, the median / min device time of:
  stats      slg_decode_stats (histograms + Otsu / percentile)
  main_rm{0,1,2}  slg_decode_triangulate (fused decode + triangulate + compaction)
  decode     slg_decode (maps out)
  tri_rm1    slg_triangulate (from maps)
with frames rotated over a pool of views so they stream from HBM.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--views", type=int, default=12)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    from structured_light_for_3d_model_replication_amd import engine as E, synth

    W, H = (int(x) for x in args.size.split("x"))
    rig = synth.default_rig(W, H, 1920, 1080)
    cal = rig.tables()
    views = [synth.render_view(rig, 360.0 * i / args.views, seed=i, n_present=44) for i in range(args.views)]
    dfr = [E.DeviceFrames(list(v.frames), v.texture) for v in views]
    dcal = E.DeviceCalib(cal, H, W)
    eng = E.Reconstructor(H, W)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    s = torch.cuda.current_stream()
    clouds = {rm: E.Cloud(H * W, rm, False) for rm in (0, 1, 2)}
    maps = [eng.decode(d, cfg) for d in dfr]
    n_px = H * W

    def timeit(fn, pre=None):
        ts = []
        for i in range(args.iters):
            v = i % len(dfr)
            if pre:
                pre(v)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn(v)
            b.record(s)
            ts.append((a, b))
        torch.cuda.synchronize()
        us = [x.elapsed_time(y) * 1e3 for x, y in ts][3:]
        return {"median_us": round(statistics.median(us), 2), "min_us": round(min(us), 2)}

    res = {}
    want = set(args.only.split(",")) if args.only else None

    def run(name, fn, pre=None, alg_bytes=None):
        if want and name not in want:
            return
        r = timeit(fn, pre)
        if alg_bytes:
            r["alg_GBps_at_median"] = round(alg_bytes / (r["median_us"] * 1e-6) / 1e9, 1)
        res[name] = r
        print(name, r, file=sys.stderr, flush=True)

    run("stats", lambda v: eng.stats(dfr[v], cfg))
    pts = {}
    for rm in (0, 1, 2):
        def f(v, rm=rm):
            eng.decode_triangulate(dfr[v], cfg, dcal, clouds[rm], rm)
        eng.stats(dfr[0], cfg)
        f(0)
        pts[rm] = int(clouds[rm].count.item())
        frame_b = (2 + 2 * 11 + (2 * 10 if rm else 0)) * n_px
        run(f"main_rm{rm}", f, pre=lambda v: eng.stats(dfr[v], cfg), alg_bytes=frame_b + 18 * pts[rm])
    # batched fused launches: all pool views in ONE main3 launch (stats done beforehand)
    frame_b1 = (2 + 2 * 11 + 2 * 10) * n_px
    for nb in sorted({min(6, len(dfr)), len(dfr)}):
        beng = E.BatchReconstructor(H, W, nb)
        bclouds = [E.Cloud(H * W, 1, False) for _ in range(nb)]
        pb = beng.prepare(dfr[:nb], cfg, dcal, bclouds, 1)
        beng.stats(pb)
        torch.cuda.synchronize()
        run(f"stats_batch{nb}", lambda v: beng.stats(pb))
        os.environ["SLG_DBG"] = "16"                 # Otsu replaced by a constant
        run(f"stats_batch{nb}_no_otsu", lambda v: beng.stats(pb))
        os.environ.pop("SLG_DBG")
        tags = [("", None)]
        if nb == len(dfr):
            tags += [(f"_dbg{d}", str(d)) for d in (1, 2, 4, 7)]
            tags += [(f"_nap{c}", str(c << 8)) for c in (1, 2, 4, 16, 64)]
        for tag, dbg in tags:
            if dbg:
                os.environ["SLG_DBG"] = dbg
            name = f"main3_batch{nb}{tag}"
            run(name, lambda v: beng.main(pb), pre=lambda v: beng.stats(pb),   # stats re-arm the look-back
                alg_bytes=nb * (frame_b1 + 18 * pts[1]))
            os.environ.pop("SLG_DBG", None)
            if name in res:
                res[name]["per_view_us"] = round(res[name]["median_us"] / nb, 2)
                print(name, "per view", res[name]["per_view_us"], file=sys.stderr, flush=True)
        if nb == len(dfr):                           # the same launch carrying a batch's histograms
            name = f"main3_batch{nb}_next"
            dfr2 = [E.DeviceFrames(list(v.frames), v.texture) for v in views]   # distinct buffers: cold
            pbn = beng.prepare(dfr2, cfg, dcal, bclouds, 1)
            run(name, lambda v: beng.main_next(pb, pbn), pre=lambda v: beng.stats(pb),
                alg_bytes=nb * (frame_b1 + 18 * pts[1]))
            run(f"stats_partials{nb}", lambda v: beng.stats_partials(pb))
            if name in res:
                res[name]["per_view_us"] = round(res[name]["median_us"] / nb, 2)
                print(name, "per view", res[name]["per_view_us"], file=sys.stderr, flush=True)
    # phase timing of the fused kernel (SLG_DBG bit 6: per-workgroup s_memrealtime stamps)
    if not want or "phases" in want:
        nb = len(dfr)
        beng = E.BatchReconstructor(H, W, nb)
        bclouds = [E.Cloud(H * W, 1, False) for _ in range(nb)]
        pb = beng.prepare(dfr, cfg, dcal, bclouds, 1)

        def prof():
            h = [np.frombuffer(beng.header(0, v)[3136:3136 + 64].cpu().numpy().tobytes(), np.uint64).astype(np.float64)
                 for v in range(nb)]
            out = h[0].copy()                        # phases sum into view 0; look-back counts per view
            out[5:] = sum(x[5:] for x in h)
            return out
        os.environ["SLG_DBG"] = "64"
        p0 = prof()
        for _ in range(6):
            beng.stats(pb)
            beng.main(pb)
        torch.cuda.synchronize()
        d = prof() - p0
        os.environ.pop("SLG_DBG")
        wgs = max(d[4], 1.0)
        ph = {k: round(d[i] / wgs * 0.01, 3) for i, k in enumerate(["A_decode", "B_tri", "C_lookback", "D_stores"])}
        ph["workgroups"] = int(d[4])
        ph["polls_per_tile"] = round(d[5] / wgs, 3)
        ph["windows_per_tile"] = round(d[6] / wgs, 3)
        ph["sleep_units_per_tile"] = round(d[7] / wgs, 2)
        res["phase_us_per_workgroup"] = ph
        print("phase us per workgroup", ph, file=sys.stderr, flush=True)
    # pipelined: stats of batch k+1 on a side stream during batch k's fused launch
    nb = len(dfr)
    beng = E.BatchReconstructor(H, W, nb, slots=2)
    bclouds = [[E.Cloud(H * W, 1, False) for _ in range(nb)] for _ in range(2)]
    pbs = [beng.prepare(dfr, cfg, dcal, bclouds[k], 1, slot=k) for k in range(2)]
    s2 = torch.cuda.Stream()
    for mode in ("overlap", "fused"):
        for rep in range(2):
            seq = [pbs[k % 2] for k in range(16)]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record(s)
            s2.wait_stream(s)
            beng.run_pipelined(seq, s, s2, mode=mode)
            s.wait_stream(s2)
            b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / (16 * nb)
        res[f"pipelined_{mode}_per_view_us"] = round(us, 2)
        print(f"pipelined {mode} per view", round(us, 2), file=sys.stderr, flush=True)
    for rep in range(2):                             # stats + fused launch on one stream
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(s)
        for k in range(16):
            beng.run(pbs[k % 2], stream=s)
        b.record(s)
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / (16 * nb)
    res["serial_per_view_us"] = round(us, 2)
    print("serial per view", round(us, 2), file=sys.stderr, flush=True)
    run("decode", lambda v: eng.decode(dfr[v], cfg), alg_bytes=(44 + 9) * n_px)
    run("tri_rm1", lambda v: eng.triangulate(maps[v][0], maps[v][1], maps[v][2], dfr[v].texture, dcal, 1,
                                             xyz_f64=False, out=clouds[1]),
        alg_bytes=9 * n_px + 18 * pts[1])
    os.environ["SLG_DBG"] = "16"
    run("stats_no_otsu", lambda v: eng.stats(dfr[v], cfg))
    for dbg in (8, 15, 1, 2, 4, 3, 7):
        os.environ["SLG_DBG"] = str(dbg)
        run(f"tri_rm1_dbg{dbg}", lambda v: eng.triangulate(maps[v][0], maps[v][1], maps[v][2], dfr[v].texture,
                                                          dcal, 1, xyz_f64=False, out=clouds[1]))
        run(f"main_rm1_dbg{dbg}", lambda v: eng.decode_triangulate(dfr[v], cfg, dcal, clouds[1], 1),
            pre=lambda v: eng.stats(dfr[v], cfg))
    os.environ.pop("SLG_DBG", None)
    res["points"] = pts
    res["error_flags"] = eng.error_flags()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
