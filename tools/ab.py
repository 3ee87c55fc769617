#!/usr/bin/env python
"""A/B of libslgpu.so builds on the benchmark's exact shape (C2, 16 views per fused launch,
two-stream carried-histogram pipeline "fused2", a pool of 48 HBM views; --batch / --pipeline
give round 2-3's 12-view one-stream shape), one subprocess per variant, rounds interleaved.
The time is the step period: one HIP event pair around the timed launches, both streams joined
(median_us = us per launch = per step).

    python tools/ab.py --libs build_ab/base.so,build_ab/w5b6.so [--rounds 3] [--launches 200] [--xyz f64]

Each worker loads the same cached rendered views (rendered once into /tmp), runs warmup + timed
launches with HIP events on the launch stream, and checks every view's point count and the
clouds' bitwise checksum against the first variant's (so a faster-but-wrong build shows up).
Prints one JSON summary line (median over rounds of each variant's median launch time).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CACHE = "/tmp/slg_ab_views.npz"


def worker(a):
    import numpy as np
    sys.path.insert(0, ROOT)
    import torch
    from structured_light_for_3d_model_replication_amd import engine as E, synth
    W, H = 1920, 1080
    rig = synth.default_rig(W, H, 1920, 1080)
    if os.path.exists(CACHE):
        z = np.load(CACHE)
        frames, tex = z["frames"], z["tex"]
    else:
        vs = [synth.render_view(rig, 30.0 * i, seed=i, n_present=44) for i in range(12)]
        frames = np.stack([v.frames for v in vs])
        tex = np.stack([v.texture for v in vs])
        np.savez(CACHE + ".tmp.npz", frames=frames, tex=tex)
        os.replace(CACHE + ".tmp.npz", CACHE)
    cal = rig.tables()
    dev = torch.device("cuda", 0)
    B, NSL = a.batch, (4 if a.pipeline == "fused2" else 2)
    pool = [E.DeviceFrames(list(frames[i]), tex[i], device=dev) for _ in range(4) for i in range(12)]
    P = len(pool)
    dcal = E.DeviceCalib(cal, H, W, device=dev, tables=a.tables != "none", keep_table=a.tables == "rays")
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    beng = E.BatchReconstructor(H, W, B, device=dev, slots=NSL)
    clouds = [[E.Cloud(H * W, 1, a.xyz == "f64", device=dev) for _ in range(B)] for _ in range(NSL)]
    preps = {}

    def prep(b):
        key = ((b * B) % P, b % NSL)
        if key not in preps:
            preps[key] = beng.prepare([pool[(b * B + k) % P] for k in range(B)], cfg, dcal, clouds[b % NSL], 1, 2.0,
                                      slot=b % NSL)
        return preps[key]

    n = a.warmup + a.launches + NSL
    batches = [prep(b) for b in range(n)]
    s0, s1 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    beng.run_pipelined(batches, s0, s1, mode=a.pipeline, start=0, stop=a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(s0)
    s1.wait_event(e0)
    beng.run_pipelined(batches, s0, s1, mode=a.pipeline, start=a.warmup, stop=a.warmup + a.launches)
    s0.wait_stream(s1)
    e1.record(s0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.launches * 1e6
    step_us = e0.elapsed_time(e1) * 1e3 / a.launches
    us = [step_us]
    last = a.warmup + a.launches - 1
    cl = clouds[last % NSL]
    counts = [int(c.count.item()) for c in cl]
    chk = float(sum(c.xyz[: int(c.count.item())].double().sum().item() for c in cl))
    # and the bits: a wrapping int64 sum of the XYZ words and the colours
    bits = sum(int(c.xyz[: int(c.count.item())].reshape(-1).view(torch.int32).to(torch.int64).sum().item())
               + int(c.bgr[: int(c.count.item())].to(torch.int64).sum().item()) for c in cl)
    chk = f"{chk!r}/{bits}"
    err = int(np.frombuffer(beng.header(0, 0)[3084:3088].cpu().numpy().tobytes(), np.uint32)[0])
    print(json.dumps({"lib": os.environ.get("SLG_LIB", "default"), "median_us": round(statistics.median(us), 2),
                      "p10_us": round(us[len(us) // 10], 2), "p90_us": round(us[9 * len(us) // 10], 2),
                      "wall_us_per_launch": round(wall, 2), "counts": counts, "checksum": chk, "err": err}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--batch", type=int, default=16, help="views per fused launch (bench: 16)")
    ap.add_argument("--pipeline", default="fused2", help="fused2 (bench: two streams) | fused (one stream)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--xyz", default="f32", help="f32 | f64 (the drop-in's float64 clouds)")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--tables", default="num", help="worker: num | none (DeviceCalib numerator tables) | rays (also the Nc ray table)")
    ap.add_argument("--variants", default="", help="comma list of lib[:tables] (overrides --libs)")
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    if a.worker:
        return worker(a)
    libs = [x for x in (a.variants or a.libs).split(",") if x] or [""]
    res = {lib: [] for lib in libs}
    ref = None
    for r in range(a.rounds):
        for lib in libs:
            env = dict(os.environ)
            spec, _, envs = lib.partition("@")          # lib[:tables][@NAME=VAL+NAME=VAL]
            for kv in filter(None, envs.split("+")):
                k, _, v = kv.partition("=")
                env[k] = v
            path, _, opt = spec.partition(":")
            if path:
                env["SLG_LIB"] = path
            cmd = [sys.executable, __file__, "--worker", "--launches", str(a.launches), "--warmup", str(a.warmup),
                   "--batch", str(a.batch), "--pipeline", a.pipeline, "--xyz", a.xyz]
            if opt:
                cmd += ["--tables", opt]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
            if p.returncode != 0:
                print(f"[ab] {lib} round {r} FAILED rc={p.returncode}\n{p.stderr[-3000:]}", file=sys.stderr, flush=True)
                sys.exit(1)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
            d = json.loads(line)
            if ref is None:
                ref = (d["counts"], d["checksum"])
            d["same_as_first"] = (d["counts"], d["checksum"]) == ref
            res[lib].append(d)
            print(f"[ab] round {r} {lib or 'default'}: median {d['median_us']} us  wall {d['wall_us_per_launch']} us  "
                  f"same={d['same_as_first']} err={d['err']}", file=sys.stderr, flush=True)
    summ = {lib or "default": {"median_us": statistics.median(x["median_us"] for x in v),
                               "wall_us": statistics.median(x["wall_us_per_launch"] for x in v),
                               "all_same": all(x["same_as_first"] for x in v), "errs": [x["err"] for x in v]}
            for lib, v in res.items()}
    print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
