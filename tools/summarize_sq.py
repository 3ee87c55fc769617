#!/usr/bin/env python
"""Summarise tools/pmc_main.sh's SQ counter passes (gpurun_out/<tag>/p1..p3) for the fused kernel:
per launch of the bench's 16-view grid, where the waves' cycles go (MI355X_MICROARCH.md: SQ
WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY = issue stalls, the rest issuing;
WAVE_CYCLES and the WAIT / ACTIVE counters in quad-cycles) and the instruction mix per view.

    python tools/summarize_sq.py <tag> [--kernel main3_kernel] [--out profiles/<tag>/sq_summary.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import gzip
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    for p in (path, path + ".gz"):
        if os.path.exists(p):
            op = gzip.open if p.endswith(".gz") else open
            with op(p, "rt") as f:
                return list(csv.DictReader(f))
    return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="main3_kernel")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    by = collections.defaultdict(lambda: collections.defaultdict(float))   # grid -> counter -> sum
    n = collections.defaultdict(lambda: collections.defaultdict(set))      # grid -> counter -> dispatches
    for p in ("p1", "p2", "p3"):
        for r in rows(os.path.join(src, p, f"{p}_counter_collection.csv")):
            if a.kernel not in r["Kernel_Name"]:
                continue
            g = int(r["Grid_Size"])
            by[g][r["Counter_Name"]] += float(r["Counter_Value"])
            n[g][r["Counter_Name"]].add((p, r["Dispatch_Id"]))
    if not by:
        raise SystemExit(f"no {a.kernel} rows under {src}")
    g = max(by, key=lambda k: max(len(d) for d in n[k].values()))   # the bench's launch grid
    per = {c: by[g][c] / len(n[g][c]) for c in by[g]}               # per launch
    views = 16
    out = {"source": f"gpurun_out/{a.tag}", "kernel": a.kernel, "grid_threads": g, "views_per_launch": views,
           "launches": max(len(d) for d in n[g].values()), "per_launch": {k: round(v) for k, v in sorted(per.items())}}
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:
        out["wave_cycle_shares"] = {k: round(per[k] / wc, 4) for k in
                                    ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
                                     "SQ_ACTIVE_INST_LDS") if k in per}
        out["wave_cycle_shares_what"] = ("fractions of SQ_WAVE_CYCLES: WAIT_ANY = waves parked on s_waitcnt / "
                                         "barriers, WAIT_INST_ANY = issue stalls, ACTIVE_INST_* = issuing")
    out["per_view"] = {k: round(per[k] / views) for k in per if k.startswith("SQ_INSTS")}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
