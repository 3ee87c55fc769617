#!/bin/bash
# One-view latency A/B of look-back poll widths (ab_libs/poll{8,16,32}.so, tools/build_ab.sh
# -DSLG_POLL_WORDS=N): tools/kbench.py --views 1 per library, rounds interleaved, then the
# bench-shape A/B (tools/ab.py).  Run from the repo root on the GPU box; logs to gpurun_out/$1/.
# The 16- and 32-word polls measured slower (profiles/r7x, DESIGN.md §4 "One-view calls") and the
# SLG_POLL_WORDS knob was not committed: the tree polls 8 words.
set -o pipefail
O=gpurun_out/$1
mkdir -p "$O"
for r in 1 2; do
  for w in 8 16 32; do
    SLG_LIB=ab_libs/poll$w.so timeout -k 10 300 python tools/kbench.py --views 1 --iters 200 \
      --only stats+solo_rm1+solo_rm1_f64+main_rm1+phases > "$O/kb_poll${w}_$r.log" 2>&1 || exit 1
    tail -1 "$O/kb_poll${w}_$r.log" | cut -c1-400
  done
done
timeout -k 10 600 python tools/ab.py --libs ab_libs/poll8.so,ab_libs/poll16.so,ab_libs/poll32.so --rounds 3 \
  > "$O/ab_bench.log" 2>&1 || exit 2
tail -2 "$O/ab_bench.log"
