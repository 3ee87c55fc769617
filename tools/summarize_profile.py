#!/usr/bin/env python
"""Copy a gpu_profile.sh run (gpurun_out/<tag>) into profiles/<tag>/ and summarise it.

  python tools/summarize_profile.py r1b [--kernel main3_kernel] [--tiles-per-view 507]

Writes profiles/<tag>/{bench.json, kernel_stats.csv, kernel_by_grid.json, pmc_summary.json} and
refreshes profiles/pmc_main_kernel.json, which bench.py reads for `roofline.traffic`.

The fused kernel runs one launch per batch of views, so launches of different sizes appear in
one trace (the bench's sanity pass, a ragged last batch).  Durations and bytes are therefore
grouped by grid size, and the HBM bytes are normalised per VIEW (grid threads / 256 lanes /
tiles per view).  HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads, so it is doubled.
"""
from __future__ import annotations

import argparse
import collections
import csv
import gzip
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LANES = 512                      # main3 workgroup (kTileBlock)


def rows_of(path, kernel):
    if not os.path.exists(path) and os.path.exists(path + ".gz"):    # (tools/gpu.sh gzips big traces)
        with gzip.open(path + ".gz", "rt") as f:
            return [r for r in csv.DictReader(f) if kernel in r["Kernel_Name"]]
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [r for r in csv.DictReader(f) if kernel in r["Kernel_Name"]]


TILES_PER_VIEW = {"c1": 225, "c2": 507, "c4": 5860, "c5": 2025}   # ceil(H*W / 4096): 1280x720, 1920x1080, 6000x4000, 3840x2160


def pmc_file(config: str, xyz: str = "f32") -> str:
    """bench.py's name for the config's committed PMC summary (pmc_main_kernel[_<config>][_f64].json)."""
    key = config if xyz == "f32" else ("f64" if config == "c2" else f"{config}_f64")
    return "pmc_main_kernel.json" if key == "c2" else f"pmc_main_kernel_{key}.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="main3_kernel")
    ap.add_argument("--config", default="c2", choices=tuple(TILES_PER_VIEW),
                    help="bench config profiled: sets --tiles-per-view and which profiles/pmc_main_kernel*.json "
                         "is refreshed (c2: pmc_main_kernel.json, else pmc_main_kernel_<config>.json)")
    ap.add_argument("--tiles-per-view", type=int, default=0, help="default: ceil(H*W / 4096) of --config")
    ap.add_argument("--xyz", choices=["f32", "f64"], default="f32", help="the profiled bench's --xyz (f64: *_f64.json)")
    ap.add_argument("--timed-last", type=int, default=0,
                    help="also report the mean over the last N launches of the most frequent grid (the "
                         "bench's timed steps: the trace run's --steps; settle/warmup launches excluded)")
    ap.add_argument("--no-refresh", action="store_true",
                    help="leave profiles/pmc_main_kernel*.json (bench.py's traffic figures) untouched")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    for s, d in (("bench.json", "bench.json"), ("trace/trace_kernel_stats.csv", "kernel_stats.csv"),
                 ("bench_trace.json", "bench_trace.json")):
        if os.path.exists(os.path.join(src, s)):
            shutil.copy(os.path.join(src, s), os.path.join(dst, d))
    grid_threads_per_view = LANES * (a.tiles_per_view or TILES_PER_VIEW[a.config])

    # kernel trace: duration per launch grouped by grid size
    by_grid = collections.defaultdict(list)
    timed = collections.defaultdict(list)           # grid -> [(start, duration us)] in launch order
    for r in rows_of(os.path.join(src, "trace", "trace_kernel_trace.csv"), a.kernel):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        by_grid[int(r["Grid_Size_X"])].append(d)
        timed[int(r["Grid_Size_X"])].append((int(r["Start_Timestamp"]), d, int(r["End_Timestamp"])))
    # a pipelined launch also carries its finishing workgroups (fewer than one view's tiles)
    vof = lambda g: max(1, g // grid_threads_per_view)
    trace = {str(g): {"views": vof(g), "launches": len(d),
                      "avg_us": round(statistics.mean(d), 2),
                      "avg_us_per_view": round(statistics.mean(d) / vof(g), 2)}
             for g, d in sorted(by_grid.items())}
    res = {"kernel": a.kernel, "by_grid_threads": trace}
    if a.timed_last and timed:
        g = max(timed, key=lambda k: len(timed[k]))
        rows = sorted(timed[g])[-a.timed_last:]
        last = [d for _, d, _ in rows]
        # launches on two streams (--pipeline fused2) overlap: a launch's own duration then
        # exceeds the step; the span of the timed launches per launch is the step period
        span = (max(e for _, _, e in rows) - rows[0][0]) / 1e3 / len(rows)
        res["timed_steps"] = {"grid_threads": g, "views": vof(g), "launches": len(last),
                              "avg_us": round(statistics.mean(last), 2),
                              "median_us": round(statistics.median(last), 2),
                              "span_us_per_launch": round(span, 2),
                              "what": f"the last {a.timed_last} launches of the most frequent grid, in start order "
                                      "(the bench's timed steps; settle, cold-start and warmup launches excluded)"}
    with open(os.path.join(dst, "kernel_by_grid.json"), "w") as f:
        json.dump(res, f, indent=1)

    # PMC: HBM bytes per view
    out = {"source": f"gpurun_out/{a.tag}", "kernel": a.kernel,
           "units": "bytes; reads 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B (calibrated on known "
                    "byte counts, profiles/r4c; = FETCH_SIZE KiB x 1024 x 2 when all reads are 128-B requests), "
                    "WRITE_SIZE KiB x 1024"}
    per = {}
    for pmc, key, scale in (("fetch", "FETCH_SIZE", 2048), ("write", "WRITE_SIZE", 1024)):
        rows = rows_of(os.path.join(src, pmc, f"{pmc}_counter_collection.csv"), a.kernel)
        rows = [r for r in rows if r["Counter_Name"] == key]
        if rows:
            views = sum(vof(int(r["Grid_Size"])) for r in rows)
            per[key] = sum(float(r["Counter_Value"]) * scale for r in rows) / views
            out[key.lower() + "_bytes_per_view"] = round(per[key])
            out[key.lower() + "_launches"] = len(rows)
    rr = rows_of(os.path.join(src, "rdreq", "rdreq_counter_collection.csv"), a.kernel)
    if rr:                                   # the request-size reading of the reads (validated)
        byc = collections.defaultdict(float)
        views = sum(vof(int(r["Grid_Size"])) for r in rr if r["Counter_Name"] == "TCC_EA0_RDREQ_sum")
        for r in rr:
            byc[r["Counter_Name"]] += float(r["Counter_Value"])
        rd = (32 * byc["TCC_EA0_RDREQ_32B_sum"] + 64 * byc["TCC_EA0_RDREQ_64B_sum"]
              + 128 * byc["TCC_EA0_RDREQ_128B_sum"]) / max(1, views)
        out["rdreq_bytes_per_view"] = round(rd)
        out["rdreq_128B_share"] = round(byc["TCC_EA0_RDREQ_128B_sum"] / max(1.0, byc["TCC_EA0_RDREQ_sum"]), 4)
        per["FETCH_SIZE"] = rd                       # the validated formula replaces FETCH_SIZE x 2
    if per:
        out["hbm_bytes_per_view"] = round(sum(per.values()))
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    if per and not a.no_refresh:
        with open(os.path.join(ROOT, "profiles", pmc_file(a.config, a.xyz)), "w") as f:
            json.dump({"tag": a.tag, "config": a.config, "xyz": a.xyz, "kernel": a.kernel, "hbm_bytes_per_view": out["hbm_bytes_per_view"],
                       "fetch_bytes_per_view": round(per["FETCH_SIZE"]) if "FETCH_SIZE" in per else None,
                       "write_bytes_per_view": out.get("write_size_bytes_per_view"),
                       "formula": out["units"]}, f, indent=1)
    print(json.dumps({"trace": res, "pmc": out}, indent=1))


if __name__ == "__main__":
    main()
