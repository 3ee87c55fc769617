#!/bin/bash
# r3aq: one-view Otsu stats_kernel ablations (SLG_STATS_ABL 0 full, 1 no MFMA, 2 no global merge, 4 no mu1 run, 12 no Otsu chains)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3aq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 4 12 qp0; do
  L=abl$v; [ $v = qp0 ] && L=qp0; SLG_LIB=$R/ab_libs/$L.so timeout -k 10 240 rocprofv3 --kernel-trace -d $O/abl$v -o run -- python3 $R/tools/kbench.py --only stats,stats_no_otsu --iters 60 > $O/kb_$v.log 2>&1 || { echo PROF_FAIL; tail -20 $O/kb_$v.log; exit 2; }
done
echo done
