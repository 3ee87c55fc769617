#!/usr/bin/env python
"""Copy a gpu_profile.sh run (gpurun_out/<tag>) into profiles/<tag>/ and summarise it.

  python tools/summarize_profile.py r1a [--kernel main2_kernel]

Writes profiles/<tag>/{bench.json, kernel_stats.csv, pmc_summary.json} and refreshes
profiles/pmc_main_kernel.json (HBM bytes per launch of the dominant kernel, read by bench.py as
`roofline.traffic`).  HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads, so it is doubled.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="main2_kernel")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    for s, d in (("bench.json", "bench.json"), ("trace/trace_kernel_stats.csv", "kernel_stats.csv"),
                 ("bench_trace.json", "bench_trace.json")):
        if os.path.exists(os.path.join(src, s)):
            shutil.copy(os.path.join(src, s), os.path.join(dst, d))
    out = {"source": f"gpurun_out/{a.tag}", "kernel": a.kernel,
           "units": "bytes per launch; FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read correction), "
                    "WRITE_SIZE KiB x 1024"}
    fetch = per_kernel(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    kern = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        kern[name] = {"launches": max(len(f), len(w)),
                      "fetch_bytes": round(statistics.mean(f) * 1024 * 2) if f else None,
                      "write_bytes": round(statistics.mean(w) * 1024) if w else None}
    out["kernels"] = kern
    main_k = [n for n in kern if a.kernel in n]
    if main_k:
        k = kern[main_k[0]]
        out["hbm_bytes_per_launch"] = (k["fetch_bytes"] or 0) + (k["write_bytes"] or 0)
        out["main_kernel_name"] = main_k[0]
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    if main_k:
        with open(os.path.join(ROOT, "profiles", "pmc_main_kernel.json"), "w") as f:
            json.dump({"tag": a.tag, "kernel": main_k[0],
                       "hbm_bytes_per_launch": out["hbm_bytes_per_launch"],
                       "fetch_bytes": kern[main_k[0]]["fetch_bytes"],
                       "write_bytes": kern[main_k[0]]["write_bytes"]}, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
