#!/bin/bash
# One-view latency + bench-shape A/B of library builds (tools/build_ab.sh -> ab_libs/<name>.so):
#   bash tools/lib_ab.sh <tag> <name> <name> [...]
# tools/kbench.py --views 1 per library, 2 rounds interleaved, then tools/ab.py over the same
# libraries (3 rounds).  Run from the repo root on the GPU box; logs to gpurun_out/<tag>/.
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
for r in 1 2; do
  for n in "$@"; do
    SLG_LIB=ab_libs/$n.so timeout -k 10 300 python tools/kbench.py --views 1 --iters 200 \
      --only stats+solo_rm1+solo_rm1_f64+main_rm1+phases > "$O/kb_${n}_$r.log" 2>&1 || exit 1
    echo "$n $r $(tail -1 "$O/kb_${n}_$r.log" | cut -c1-300)"
  done
done
libs=$(printf "ab_libs/%s.so," "$@")
timeout -k 10 600 python tools/ab.py --libs "${libs%,}" --rounds 3 > "$O/ab_bench.log" 2>&1 || exit 2
tail -1 "$O/ab_bench.log"
