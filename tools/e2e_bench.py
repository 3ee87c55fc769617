#!/usr/bin/env python
"""Host-buffer (PCIe-inclusive) throughput of the C2 path -- reported in DESIGN.md, never the
bench metric.  A turntable stream whose frames arrive in host memory: per view, the frame stack
(+ BGR texture) is copied from pinned host memory into one of two HBM slots on a copy stream,
reconstructed (stats + fused kernel, slg_reconstruct) on the compute stream, and -- with
``--d2h`` -- the cloud (XYZ f32 + BGR, sized from a sanity pass) copied back to pinned host
memory.  Copies of view k+1 overlap the kernels of view k.

Prints one JSON line: Mpoints/s and GB/s of H2D, next to the device-resident figure.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--d2h", action="store_true", help="also copy each cloud back to host")
    args = ap.parse_args()

    import numpy as np
    import torch
    from structured_light_for_3d_model_replication_amd import engine as E, synth

    dev = torch.device("cuda", 0)
    W, H, PW, PH = 1920, 1080, 1920, 1080
    rig = synth.default_rig(W, H, PW, PH)
    cal = rig.tables()
    views = [synth.render_view(rig, 90.0 * i, seed=i, n_present=44) for i in range(args.views)]
    F = views[0].frames.shape[0]
    slots = [E.DeviceFrames(list(views[0].frames), views[0].texture, device=dev) for _ in range(2)]
    stride = slots[0].stride
    host = []
    for v in views:                                   # pinned host stacks in the HBM layout
        fr = torch.zeros((slots[0].data.shape[0], stride), dtype=torch.uint8).pin_memory()
        fr[:F, : H * W].copy_(torch.from_numpy(v.frames.reshape(F, -1)))
        tx = torch.from_numpy(np.ascontiguousarray(v.texture).reshape(H * W, 3)).pin_memory()
        host.append((fr, tx))
    cfg = E.DecodeConfig(PW, PH, 11, 10, "otsu")
    dcal = E.DeviceCalib(cal, H, W, device=dev)
    engs = [E.Reconstructor(H, W, device=dev) for _ in range(2)]
    outs = [E.Cloud(H * W, 1, False, device=dev) for _ in range(2)]
    counts = []
    for v in range(args.views):                       # sanity pass: points per view
        slots[0].data.copy_(host[v][0]); slots[0].texture.copy_(host[v][1])
        engs[0].reconstruct(slots[0], cfg, dcal, 1, 2.0, out=outs[0])
        counts.append(int(outs[0].count.item()))
    cap = max(counts)
    hx = [torch.empty((cap, 3), dtype=torch.float32).pin_memory() for _ in range(2)]
    hb = [torch.empty((cap, 3), dtype=torch.uint8).pin_memory() for _ in range(2)]

    s_copy, s_comp, s_back = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_done = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]
    for e in ev_done + ev_out:
        e.record(s_comp)

    def step(k):
        s, v = k % 2, k % args.views
        with torch.cuda.stream(s_copy):
            s_copy.wait_event(ev_done[s])             # slot s free: view k-2's kernels are done
            slots[s].data.copy_(host[v][0], non_blocking=True)
            slots[s].texture.copy_(host[v][1], non_blocking=True)
            ev_in[s].record(s_copy)
        s_comp.wait_event(ev_in[s])
        if args.d2h:
            s_comp.wait_event(ev_out[s])              # cloud slot s read back
        engs[s].reconstruct(slots[s], cfg, dcal, 1, 2.0, out=outs[s], stream=s_comp)
        ev_done[s].record(s_comp)
        if args.d2h:
            n = counts[v]
            with torch.cuda.stream(s_back):
                s_back.wait_event(ev_done[s])
                hx[s][:n].copy_(outs[s].xyz[:n], non_blocking=True)
                hb[s][:n].copy_(outs[s].bgr[:n], non_blocking=True)
                ev_out[s].record(s_back)
        return counts[v]

    for k in range(8):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pts = sum(step(k) for k in range(args.steps))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    h2d = (F * stride + H * W * 3) * args.steps
    print(json.dumps({"what": "C2 host-buffer stream (PCIe-inclusive)", "d2h": args.d2h,
                      "views": args.steps, "ms_per_view": round(dt / args.steps * 1e3, 4),
                      "Mpoints_per_s": round(pts / dt / 1e6, 1),
                      "h2d_GB_per_s": round(h2d / dt / 1e9, 2),
                      "h2d_MB_per_view": round(h2d / args.steps / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
