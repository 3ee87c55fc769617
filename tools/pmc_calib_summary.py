#!/usr/bin/env python
"""Summarise a tools/pmc_calib.sh run (gpurun_out/<tag>) into profiles/<tag>/pmc_calibration.json.

Also refreshes profiles/pmc_main_kernel.json (bench.py's `roofline.traffic`) from the C2 instance.

For each fetch_probe variant: the bytes it requests (known on the host) against what each
counter formula reports per dispatch -- FETCH_SIZE (KiB) as reported and x2 (the guide's gfx950
correction for wide streaming reads), the request-size counters 32*RDREQ_32B + 64*RDREQ_64B +
128*RDREQ_128B, RDREQ x 64 and x 128, WRITE_SIZE and 64*WRREQ_64B (+32 for the rest).  The same
formulas over bench.py's fused launches, per C2 view (launch grid / 512 lanes / 507 tiles)."""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = {1: ["FETCH_SIZE"], 2: ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum",
                                  "TCC_EA0_RDREQ_sum"],
          3: ["TCC_BUBBLE_sum"], 4: ["WRITE_SIZE"], 5: ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"]}


def load(src, prefix, name_filter):
    """{kernel: {counter: [value per dispatch, ...]}, "_grid": {kernel: [grid]}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    grids = collections.defaultdict(list)
    for n in PASSES:
        for f in glob.glob(os.path.join(src, f"{prefix}_p{n}", "*counter_collection.csv")):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"]
                    if not name_filter(k):
                        continue
                    out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    if n == 1:
                        grids[k].append(int(r["Grid_Size"]))
    return out, grids


def formulas(c):
    """Bytes per dispatch under each reading of the counters (medians over dispatches)."""
    m = {k: statistics.median(v) for k, v in c.items() if v}
    res = {}
    if "FETCH_SIZE" in m:
        res["FETCH_SIZE"] = m["FETCH_SIZE"] * 1024
        res["FETCH_SIZE_x2"] = m["FETCH_SIZE"] * 2048
    if "TCC_EA0_RDREQ_sum" in m:
        r32, r64, r128 = (m.get(f"TCC_EA0_RDREQ_{s}_sum", 0.0) for s in ("32B", "64B", "128B"))
        res["rdreq_by_size"] = 32 * r32 + 64 * r64 + 128 * r128
        res["rdreq_x64"] = 64 * m["TCC_EA0_RDREQ_sum"]
        res["rdreq_x128"] = 128 * m["TCC_EA0_RDREQ_sum"]
        res["rdreq_mix"] = {"n32": r32, "n64": r64, "n128": r128, "total": m["TCC_EA0_RDREQ_sum"]}
    if "TCC_BUBBLE_sum" in m:
        res["bubble_x128"] = 128 * m["TCC_BUBBLE_sum"]
    if "WRITE_SIZE" in m:
        res["WRITE_SIZE"] = m["WRITE_SIZE"] * 1024
    if "TCC_EA0_WRREQ_sum" in m:
        w64 = m.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        res["wrreq_by_size"] = 64 * w64 + 32 * (m["TCC_EA0_WRREQ_sum"] - w64)
        res["wrreq_mix"] = {"n64": w64, "total": m["TCC_EA0_WRREQ_sum"]}
    return res


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    probe = json.load(open(os.path.join(src, "probe.json")))
    pc, _ = load(src, "probe", lambda k: "rd_kernel" in k or "st_kernel" in k)
    out = {"source": f"gpurun_out/{tag} (tools/pmc_calib.sh)", "probe_setup": {k: v for k, v in probe.items() if k != "variants"},
           "probe": {}, "bench": {}}
    for k, counters in pc.items():
        key = next((v for v in probe["variants"] if k.startswith("void " + v + "(")), None)
        if key is None:
            continue
        known = probe["variants"][key]
        f = formulas(counters)
        ratios = {name: round(val / known["requested"], 4) for name, val in f.items() if isinstance(val, float)}
        out["probe"][known["what"]] = {"kernel": key, "known": known, "measured_bytes": f,
                                       "measured_over_requested": ratios}
    bc, grids = load(src, "bench", lambda k: "main3_kernel" in k)
    lanes_per_view = 512 * 507
    for k, counters in bc.items():
        g = statistics.median(grids[k]) if grids[k] else 0
        views = max(1, int(g // lanes_per_view))
        f = formulas(counters)
        per = {n: (round(v / views) if isinstance(v, float) else {a: round(b / views) for a, b in v.items()})
               for n, v in f.items()}
        out["bench"][k[:90]] = {"views_per_launch": views, "dispatches": len(counters.get("FETCH_SIZE", [])),
                                "bytes_per_view": per}
        if "rdreq_by_size" in per and "WRITE_SIZE" in per and "186>" in k:   # the C2 plan instance
            with open(os.path.join(ROOT, "profiles", "pmc_main_kernel.json"), "w") as fh:
                json.dump({"tag": tag, "kernel": k[:90], "hbm_bytes_per_view": per["rdreq_by_size"] + per["WRITE_SIZE"],
                           "fetch_bytes_per_view": per["rdreq_by_size"], "write_bytes_per_view": per["WRITE_SIZE"],
                           "formula": "reads 128*RDREQ_128B + 64*RDREQ_64B + 32*RDREQ_32B (= FETCH_SIZE x 2: all "
                                      "main3 reads are 128-B requests), writes WRITE_SIZE; both calibrated on known "
                                      "byte counts (tools/fetch_probe.hip, probe section of pmc_calibration.json)"},
                          fh, indent=1)
    with open(os.path.join(dst, "pmc_calibration.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
