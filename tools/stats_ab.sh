#!/bin/bash
# Round 6's stats-kernel A/B (profiles/r7d): the GPU suite with the LDS-free counting library, then
# tools/kbench.py's stats / one-view / batched-stats timings of ab_libs/{base,dpp,dpp_c1,dpp_c4}.so
# interleaved twice (build them with tools/build_ab.sh first).  The logs' "*_no_otsu" rows come from
# an ablation switch the kernels no longer have: they time the same launch as the row above them.
set -o pipefail
O=gpurun_out/r7d; mkdir -p $O
SLG_LIB=ab_libs/dpp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dpp.log 2>&1 || { tail -30 $O/pytest_dpp.log; exit 1; }
tail -1 $O/pytest_dpp.log
for i in 1 2; do for L in base dpp dpp_c1 dpp_c4; do
  SLG_LIB=ab_libs/$L.so timeout -k 10 300 python tools/kbench.py --iters 60 --only stats,stats_no_otsu,solo_rm1,solo_rm1_f64,stats_batch6,stats_batch12,stats_batch6_no_otsu,stats_batch12_no_otsu > $O/kb_${L}_$i.log 2>&1 || { tail -20 $O/kb_${L}_$i.log; exit 2; }
  echo "$L $i"; grep -E "^(stats|solo)" $O/kb_${L}_$i.log | cut -c1-80
done; done
