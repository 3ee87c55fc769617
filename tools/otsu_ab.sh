#!/bin/bash
# Otsu tail A/B: tools/otsu_probe.hip builds (ab_libs/otsu_<name>) on the histograms
# tools/otsu_probe.py wrote to ab_libs/otsu_hists.bin, 2 rounds interleaved; every threshold is
# checked against the host loop (non-zero exit on a mismatch).  bash tools/otsu_ab.sh <tag> <name>...
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
for r in 1 2; do
  for n in "$@"; do
    timeout -k 10 120 ./ab_libs/otsu_$n ab_libs/otsu_hists.bin > "$O/otsu_${n}_$r.log" 2>&1 || { tail -5 "$O/otsu_${n}_$r.log"; exit 1; }
    python - "$O/otsu_${n}_$r.log" "$n" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if '"us"' in l]
c2 = rows[:6]
print(sys.argv[2], "C2 hists us", [r["us"] for r in c2], "clocks", [r["clocks"] for r in c2],
      "all", round(sum(r["us"] for r in rows) / len(rows), 3))
PY
  done
done
