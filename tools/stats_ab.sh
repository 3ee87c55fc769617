#!/bin/bash
# Stats-kernel A/B on the GPU box (profiles/r7d, r7g): the GPU suite with the candidate library,
# then tools/kbench.py's one-view / batched-stats timings of every ab_libs/<name>.so given,
# interleaved twice (build them with tools/build_ab.sh first).
#   bash tools/stats_ab.sh <tag> <candidate> <lib> [<lib> ...]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O; shift
CAND=$1; shift
SLG_LIB=ab_libs/$CAND.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$CAND.log 2>&1 || { tail -30 $O/pytest_$CAND.log; exit 1; }
tail -1 $O/pytest_$CAND.log
for i in 1 2; do for L in "$@"; do
  SLG_LIB=ab_libs/$L.so timeout -k 10 300 python tools/kbench.py --iters 60 --only stats,solo_rm1,solo_rm1_f64,stats_batch6,stats_batch12 > $O/kb_${L}_$i.log 2>&1 || { tail -20 $O/kb_${L}_$i.log; exit 2; }
  echo "$L $i"; grep -E "^(stats|solo)" $O/kb_${L}_$i.log | cut -c1-80
done; done
