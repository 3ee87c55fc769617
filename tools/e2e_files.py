#!/usr/bin/env python
"""End-to-end file path of the drop-in: ``process_multi_ply(mode='batch')`` over C2 view folders
of 8-bit PNG captures, the reference GUI's live path (``server/gui.py:1360-1376`` ->
``server/processing.py:314-334``; the C3 folder layout of ``server/gui.py:1718,1753``).
Reported in DESIGN.md, never the bench metric.

Prints one JSON line: seconds per view for the whole batch under each decoder split

* ``host``   -- every folder's PNGs decoded on host threads (``SLG_PNG_DEVICE=0``);
* ``auto``   -- the product default: the last folders' zlib streams inflated by one GPU launch
  while the host threads decode the rest (``pipeline.device_share``);
* ``device`` -- every folder on the GPU decoder (``SLG_PNG_DEVICE=1``),

at the given views-per-launch groups (``SLG_BATCH_VIEWS``), each run's per-stage busy times
(``pipeline.LAST_STATS``: host read/decode and PLY write busy seconds summed over threads, GPU
device-decode and reconstruct milliseconds from HIP events), and whether every run wrote the same
PLY bytes.  ``--parts`` adds the serial cost of the stages measured view by view.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=36)
    ap.add_argument("--geom", default="c2", help="c2 (1920x1080, 11+10 bits, 44 frames) | c5 (3840x2160, "
                                                 "projector 1920x1080, 11+11 bits, 46 frames)")
    ap.add_argument("--runs", default="host:1,host:4,host:8,auto:4,auto:8,device:16",
                    help="comma list of decoder:group[:NAME=VAL+NAME=VAL] (decoder host | auto | device; "
                         "extra environment for that run, e.g. auto:8:SLG_PNG_RESERVE_EVERY=0)")
    ap.add_argument("--reps", type=int, default=1, help="repetitions of the whole list (interleaved)")
    ap.add_argument("--parts", action="store_true", help="also the serial per-stage costs")
    ap.add_argument("--out", default="", help="also write the JSON here")
    ap.add_argument("--trace", default="", help="write each run's pipeline timeline (SLG_PIPE_TRACE) here")
    args = ap.parse_args()

    from structured_light_for_3d_model_replication_amd import calibration, synth
    from structured_light_for_3d_model_replication_amd import pipeline as PL
    from structured_light_for_3d_model_replication_amd import processing as PR

    W, H, nf, kw = ((3840, 2160, 46, dict(n_sets_col=11, n_sets_row=11)) if args.geom == "c5"
                    else (1920, 1080, 44, dict(n_sets_col=11, n_sets_row=10)))
    rig = synth.default_rig(W, H, 1920, 1080)
    with tempfile.TemporaryDirectory() as tmp:
        calib = os.path.join(tmp, "calib.mat")
        calibration.save_mat(calib, rig.tables())
        root = os.path.join(tmp, "scan")
        t = time.perf_counter()

        def make(i):
            v = synth.render_view(rig, 360.0 * i / args.views, seed=i, n_present=nf)
            synth.write_capture(v, os.path.join(root, f"obj_{i:02d}_scan"))
        with ThreadPoolExecutor(8) as ex:
            list(ex.map(make, range(args.views)))
        print(f"[e2e] wrote {args.views} captures in {time.perf_counter() - t:.1f}s", file=sys.stderr, flush=True)
        folders = [f.path for f in os.scandir(root) if f.is_dir()]     # the order batch mode uses
        PR.ProcessingLogic.process_multi_ply(calib, folders[0], "single", log_callback=lambda m: None, **kw)  # warm-up
        runs = [(r.split(":") + [""])[:3] for r in args.runs.split(",") if r]
        res, plys, traces = {}, {}, {}
        if args.trace:
            os.environ["SLG_PIPE_TRACE"] = "1"
        env = {"host": "0", "auto": "auto", "device": "1"}
        for rep in range(args.reps):
            for dec, g, extra in runs:
                os.environ["SLG_PNG_DEVICE"] = env[dec]
                os.environ["SLG_BATCH_VIEWS"] = g
                saved = {}
                for kv in filter(None, extra.split("+")):
                    k, _, v = kv.partition("=")
                    saved[k] = os.environ.get(k)
                    os.environ[k] = v
                t0 = time.perf_counter()
                PR.ProcessingLogic.process_multi_ply(calib, root, "batch", log_callback=lambda m: None, **kw)
                dt = time.perf_counter() - t0
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
                key = f"{dec}_group{g}" + (f"_{extra}" if extra else "")
                st = PL.LAST_STATS.as_dict()
                res.setdefault(key, []).append({"s_per_view": round(dt / args.views, 4), **st})
                if PL.LAST_STATS.trace is not None:
                    traces[f"{key}_rep{rep}"] = sorted(PL.LAST_STATS.trace, key=lambda e: e[2])
                print(f"[e2e] rep {rep} {key}: {dt / args.views:.4f} s/view {st}", file=sys.stderr, flush=True)
                plys[key] = [open(os.path.join(f, os.path.basename(f) + ".ply"), "rb").read() for f in folders]
        first = next(iter(plys.values()))
        out = {"what": f"process_multi_ply batch over {args.geom.upper()} PNG folders (end to end), s/view per "
                       "decoder split", "geom": args.geom, "views": args.views, "runs": res,
               "best": min(((k, min(x["s_per_view"] for x in v)) for k, v in res.items()), key=lambda kv: kv[1]),
               "ply_bytes_equal_all_runs": all(p == first for p in plys.values()),
               "ply_mb_per_view": round(sum(len(b) for b in first) / len(first) / 1e6, 2),
               "decode_threads": PR.FR.decode_threads(), "host_cpus": os.cpu_count(),
               "cpu_quota": _quota()}

        if args.parts:                                 # the stages one view at a time, serially
            import torch
            cfg = PR.E.DecodeConfig(1920, 1080, kw["n_sets_col"], kw["n_sets_row"], "otsu")
            cal = calibration.load_mat(calib)
            pool = PL.PinnedPool()
            s = torch.cuda.Stream()
            parts = {}
            for dec in ("device", "host"):
                t_read = t_rec = t_ply = 0.0
                for f in folders[:16]:
                    t = time.perf_counter()
                    hv = PL.read_view(f, cfg, pool, device_png=dec == "device")
                    t_read += time.perf_counter() - t
                    t = time.perf_counter()
                    dev = PL.upload_view(hv, s)
                    s.synchronize()
                    P, C = PR.reconstruct_view(dev, cfg, cal, 1, 2.0)
                    t_rec += time.perf_counter() - t
                    for b in hv.pinned:
                        pool.put(b)
                    t = time.perf_counter()
                    PR.ProcessingLogic._save_ply(P, C, os.path.join(tmp, "x.ply"))
                    t_ply += time.perf_counter() - t
                n = len(folders[:16])
                parts[dec] = {"read_pinned": round(t_read / n, 4), "h2d_decode_kernels_d2h": round(t_rec / n, 4),
                              "ply_write": round(t_ply / n, 4)}
            out["s_per_view_parts_serial"] = parts
        if args.trace:
            with open(args.trace, "w") as f:
                json.dump(traces, f)
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")


def _quota():
    from structured_light_for_3d_model_replication_amd import frames as FR
    return FR.cpu_quota()


if __name__ == "__main__":
    main()
