#!/usr/bin/env python
"""Phase timeline of a one-view fused launch (main3 SOLO) from a build with -DSLG_SOLO_PROF=1:
per workgroup, s_memrealtime (100 MHz) at start, stats done, frame loads issued, thresholds seen,
phase A done, exit; the finisher's Otsu start and flag.  Prints one JSON line of percentiles
(microseconds from the launch's first workgroup start).

    SLG_LIB=ab_libs/solo_prof.so python tools/solo_prof.py [--reps 8]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["start", "stats_done", "loads_issued", "thresholds_seen", "phaseA_done", "exit"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--xyz", default="f32")
    ap.add_argument("--stats", action="store_true",
                    help="time the one-view stats launch instead (stats_kernel's stamps: start, "
                         "counted, atomics done, ticket; the last arriver's sums read, Otsu done, end)")
    args = ap.parse_args()
    os.environ["SLG_SOLO"] = "0" if args.stats else "1"   # the one-view fused launch is opt-in
    import numpy as np
    import torch
    from structured_light_for_3d_model_replication_amd import _native as N, engine as E, synth

    W, H = 1920, 1080
    rig = synth.default_rig(W, H, 1920, 1080)
    views = [synth.render_view(rig, 30.0 * i, seed=i, n_present=44) for i in range(4)]
    dfr = [E.DeviceFrames(list(v.frames), v.texture) for v in views]
    dcal = E.DeviceCalib(rig.tables(), H, W)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    eng = E.Reconstructor(H, W)
    out = E.Cloud(H * W, 1, args.xyz == "f64")
    lib = N.lib()
    rd = lib.slg_solo_prof_read
    rd.restype, rd.argtypes = ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int64]
    n_wg = (H * W + 4095) // 4096 if not args.stats else (H * W + 8191) // 8192   # stats: 8192 px per workgroup
    buf = np.zeros(1024 * 8, np.uint64)
    s = torch.cuda.current_stream()
    rows, kus = [], []
    for r in range(args.reps + 2):
        buf[:] = 0
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        if args.stats:
            eng.stats(dfr[r % len(dfr)], cfg)
        else:
            eng.reconstruct(dfr[r % len(dfr)], cfg, dcal, 1, 2.0, out=out)
        b.record(s)
        torch.cuda.synchronize()
        if rd(buf.ctypes.data, buf.size) != 0:
            raise RuntimeError("slg_solo_prof_read failed (library built without SLG_SOLO_PROF?)")
        if r < 2:
            continue
        kus.append(a.elapsed_time(b) * 1e3)
        rec = buf.reshape(1024, 8)[:n_wg].astype(np.float64)
        t0 = rec[:, 0].min()
        rel = (rec - t0) * 0.01                         # us
        fin = np.nonzero(rec[:, 6])[0]
        rows.append((rel, fin))
    res = {"kernel_event_us_median": round(float(np.median(kus)), 2), "n_wg": n_wg, "error_flags": eng.error_flags()}
    allrel = np.concatenate([r for r, _ in rows])
    if args.stats:
        names = ["start", "counted", "atomics_done", "ticket"]
        for i, nm in enumerate(names):
            res[nm] = [round(float(np.percentile(allrel[:, i], q)), 2) for q in (0, 10, 50, 90, 100)]
        last = []
        for r, _ in rows:
            k = int(np.argmax(r[:, 4]))                 # the last arriver (the only one with [4..6])
            last.append([round(float(r[k, i]), 2) for i in range(7)])
        res["last_arriver_stamps"] = last[:4]
        res["last_arriver_what"] = "start, counted, atomics done, ticket, sums read, Otsu done, end (us)"
        print(json.dumps(res), flush=True)
        return
    for i, nm in enumerate(NAMES):
        res[nm] = [round(float(np.percentile(allrel[:, i], q)), 2) for q in (0, 10, 50, 90, 100)]
    for i, nm in enumerate(NAMES[1:], start=1):
        res["dur_" + nm] = [round(float(np.percentile(allrel[:, i] - allrel[:, i - 1], q)), 2) for q in (10, 50, 90, 100)]
    fins = [(r[f[0], 6], r[f[0], 7], r[f[0], 1]) for r, f in rows if len(f)]
    res["finisher_otsu_start_flag_statsdone"] = [[round(float(x), 2) for x in t] for t in fins[:4]]
    res["last_exit"] = round(float(np.median([r[:, 5].max() for r, _ in rows])), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
