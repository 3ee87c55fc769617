#!/usr/bin/env python
"""Device PNG inflate time per view and per group over the e2e scan (tools/e2e_files.py's 36
rendered C2 folders): each view's 44 streams alone, and groups of the last k views in one launch
(what BatchPipeline's device share sends).  Tells whether a launch's time is its slowest stream
(then the device share should be picked by stream size) or grows with the stream count.

    python tools/png_views_bench.py [--views 36] [--groups 10,14]
Prints one JSON line.
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
    ap.add_argument("--groups", default="10,14")
    ap.add_argument("--every", default="", help="also time each group with these CU masks "
                    "(SLG_PNG_RESERVE_EVERY values; 0 = a plain stream)")
    ap.add_argument("--no-alone", action="store_true")
    args = ap.parse_args()
    import torch
    from structured_light_for_3d_model_replication_amd import engine as E, synth
    from structured_light_for_3d_model_replication_amd import pipeline as PL

    rig = synth.default_rig(1920, 1080, 1920, 1080)
    cfg = E.DecodeConfig(1920, 1080, 11, 10, "otsu")
    with tempfile.TemporaryDirectory() as tmp:
        def make(i):
            v = synth.render_view(rig, 360.0 * i / args.views, seed=i, n_present=44)
            f = os.path.join(tmp, f"obj_{i:02d}_scan")
            synth.write_capture(v, f)
            return f
        with ThreadPoolExecutor(8) as ex:
            folders = list(ex.map(make, range(args.views)))
        pool = PL.PinnedPool()
        hvs = [PL.read_view(f, cfg, pool, device_png=True) for f in folders]
        zb = [int(sum(hv.z[2])) for hv in hvs]
        zmax = [int(max(hv.z[2])) for hv in hvs]

        def launch(sel, n_streams):
            s = PL.png_decode_stream(n_streams=n_streams)
            best = None
            for _ in range(2):
                torch.cuda.synchronize()
                marks = []
                PL.upload_views([hvs[k] for k in sel], s, marks)
                s.synchronize()
                ms = marks[0].elapsed_time(marks[1])
                best = ms if best is None else min(best, ms)
            return round(best, 1)
        alone = [] if args.no_alone else [launch([k], len(hvs[k].z[0])) for k in range(len(hvs))]
        out = {"what": "device inflate + un-filter ms per launch (HIP events around slg_png_decode_device)",
               "views": args.views, "alone_ms": alone, "z_bytes_per_view": zb, "z_max_stream_bytes": zmax}
        for g in (int(x) for x in args.groups.split(",") if x):
            sel = list(range(len(hvs) - g, len(hvs)))
            out[f"last_{g}_ms"] = launch(sel, sum(len(hvs[k].z[0]) for k in sel))
            light = sorted(range(len(hvs)), key=lambda k: zmax[k])[:g]
            out[f"lightest_{g}_ms"] = launch(light, sum(len(hvs[k].z[0]) for k in light))
            n = sum(len(hvs[k].z[0]) for k in sel)
            out[f"last_{g}_reserve_every_auto"] = PL.png_reserve_every(n, torch.cuda.get_device_properties(0).multi_processor_count)
            for e in (x for x in args.every.split(",") if x):
                os.environ["SLG_PNG_RESERVE_EVERY"] = e
                out[f"last_{g}_every{e}_ms"] = launch(sel, n)
                del os.environ["SLG_PNG_RESERVE_EVERY"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
