#!/usr/bin/env python
"""Mean SQ counters per fused 12-view main3 launch from a tools/pmc_main.sh run.

  python tools/summarize_sq.py r2p_sq profiles/r2p_prof/sq_counters.json
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (pass, dispatch) -> counter
    grids = collections.Counter()
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", tag, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "main3_kernel" not in r["Kernel_Name"]:
                continue
            key = (os.path.basename(f), r["Dispatch_Id"], int(r["Grid_Size"]))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            grids[int(r["Grid_Size"])] += 1
    grid = max(grids, key=lambda g: (g >= 12 * 507 * 512, grids[g]))   # the 12-view launches
    res = collections.defaultdict(list)
    for (p, d, g), cs in per.items():
        if g == grid:
            for k, v in cs.items():
                res[k].append(v)
    summ = {k: statistics.mean(v) for k, v in sorted(res.items())}
    summ["_note"] = (f"per fused launch of 12 C2 views (grid {grid} threads, bench.py pipeline), mean over "
                     f"launches; rocprofv3 --pmc, one pass per counter group (tools/pmc_main.sh)")
    json.dump(summ, open(out, "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
