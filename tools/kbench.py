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
    ap.add_argument("--only", default="")   # names, comma- or plus-separated
    ap.add_argument("--thresh", default="otsu", choices=("otsu", "percentile"))
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
    cfg = E.DecodeConfig(1920, 1080, 11, 10, args.thresh)
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
    want = set(args.only.replace("+", ",").split(",")) if args.only else None   # "+" too: tools/gpu.sh turns commas into spaces

    def run(name, fn, pre=None, alg_bytes=None):
        if want and name not in want:
            return
        r = timeit(fn, pre)
        if alg_bytes:
            r["alg_GBps_at_median"] = round(alg_bytes / (r["median_us"] * 1e-6) / 1e9, 1)
        res[name] = r
        print(name, r, file=sys.stderr, flush=True)

    run("stats", lambda v: eng.stats(dfr[v], cfg))
    # one view's whole drop-in call (_gray_decode + _reconstruct_point_cloud fused): stats + main
    # in one event pair, f32 and the drop-in's f64
    for tag, x64 in (("", False), ("_f64", True)):
        solo_out = E.Cloud(H * W, 1, x64)
        run(f"solo_rm1{tag}", lambda v, o=solo_out: eng.reconstruct(dfr[v], cfg, dcal, 1, 2.0, out=o))
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
        tags = [("", None)]
        if nb == len(dfr):
            dl = os.environ.get("KBENCH_DBG", "1,2,4,3,5,6,7,8,128,11,131")
            tags += [(f"_dbg{d}", str(d)) for d in (int(x) for x in dl.split(",") if x)]
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
    # phase timing of the fused kernel (SLG_DBG bit 6: one 32-byte record per workgroup in view
    # 0's partials region: A, B, C, D in 100 MHz ticks, polls, sleep units, items, view)
    if not want or "phases" in want:
        nb = len(dfr)
        beng = E.BatchReconstructor(H, W, nb)
        bclouds = [E.Cloud(H * W, 1, False) for _ in range(nb)]
        pb = beng.prepare(dfr, cfg, dcal, bclouds, 1)
        al = lambda x: (x + 255) // 256 * 256
        tpx = int(os.environ.get("SLG_TILE_PX", "4096"))     # main3 tile (kTilePx)
        n_tiles = (n_px + tpx - 1) // tpx
        parts_off = 65536 + al(2 * n_tiles * 8) + al(n_px * 24) + al(n_px * 3)
        n_wg = n_tiles * nb
        extras = [int(x) for x in os.environ.get("KBENCH_PHASE_EXTRA", "0,1,2").split(",") if x]
        for extra in extras:                         # + ablations: no wait / trivial tri / ...
            os.environ["SLG_DBG"] = str(64 | extra)
            recs, us = [], 0.0
            for _ in range(4):
                beng.stats(pb)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                beng.main(pb)
                b.record(s)
                torch.cuda.synchronize()
                us += a.elapsed_time(b) * 1e3
                raw = beng.workspace[parts_off: parts_off + n_wg * 32].cpu().numpy()
                recs.append(np.frombuffer(raw.tobytes(), np.uint32).reshape(n_wg, 8).astype(np.float64))
            os.environ.pop("SLG_DBG")
            r = np.concatenate(recs)
            ph = {k: round(float(r[:, i].mean()) * 0.01, 3) for i, k in enumerate(["A_decode", "B_tri", "C_lookback", "D_stores"])}
            ph["lifetime"] = round(float(r[:, :4].sum(1).mean()) * 0.01, 2)
            ph["polls_per_tile"] = round(float(r[:, 4].mean()), 2)
            ph["sleep_units_per_tile"] = round(float(r[:, 5].mean()), 1)
            ph["items_per_tile"] = round(float(r[:, 6].mean()), 1)
            ph["C_p50_p90_p99"] = [round(float(np.percentile(r[:, 2], q)) * 0.01, 2) for q in (50, 90, 99)]
            # look-back wait vs this tile's items and its predecessor's (same view): content skew
            rr = recs[-1]
            tile_of = np.arange(n_wg) // nb
            pred = np.where(tile_of > 0, np.arange(n_wg) - nb, -1)
            mine, theirs = rr[:, 6], np.where(pred >= 0, rr[np.maximum(pred, 0), 6], 0)
            for lbl, sel in (("C_when_pred_heavier", theirs > mine + 256), ("C_when_pred_lighter", theirs + 256 < mine),
                             ("C_when_similar", np.abs(theirs - mine) <= 256)):
                ph[lbl] = round(float(rr[sel, 2].mean()) * 0.01, 2) if sel.any() else None
            # phase occupancy over time (last run): mean / p10 / p90 of workgroups in A and B+C+D
            t0 = rr[:, 7] - rr[:, 7].min()
            ends = np.cumsum(rr[:, :4], axis=1)
            grid = np.arange(0, float((t0 + ends[:, 3]).max()), 10.0)   # 0.1 us steps
            inA = np.zeros_like(grid)
            inR = np.zeros_like(grid)
            for st, e in zip(t0, ends):
                a0, a1 = np.searchsorted(grid, [st, st + e[0]])
                inA[a0:a1] += 1
                r0_, r1_ = np.searchsorted(grid, [st + e[0], st + e[3]])
                inR[r0_:r1_] += 1
            mid = slice(len(grid) // 10, len(grid) * 9 // 10)
            ph["in_A_mean_p10_p90"] = [round(float(inA[mid].mean()), 1), round(float(np.percentile(inA[mid], 10)), 1),
                                       round(float(np.percentile(inA[mid], 90)), 1)]
            ph["in_BCD_mean"] = round(float(inR[mid].mean()), 1)
            if extra == 0:
                np.save(os.path.join(ROOT, "gpurun_out", "phase_occupancy.npy"), np.stack([grid, inA, inR]))
            ph["kernel_us_per_view"] = round(us / 4 / nb, 2)
            ph["lifetime_sum_over_kernel_x1024"] = round(float(r[:, :4].sum()) * 0.01 / (us * 1024), 3)
            res[f"phases_dbg{extra}"] = ph
            print(f"phases (dbg {extra})", ph, file=sys.stderr, flush=True)
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
    for dbg in (1, 2, 4, 3, 7):        # profiling instance (row_mode 1, f32, frames, pinhole)
        os.environ["SLG_DBG"] = str(dbg)
        run(f"main_rm1_dbg{dbg}", lambda v: eng.decode_triangulate(dfr[v], cfg, dcal, clouds[1], 1),
            pre=lambda v: eng.stats(dfr[v], cfg))
    os.environ.pop("SLG_DBG", None)
    res["points"] = pts
    res["error_flags"] = eng.error_flags()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
