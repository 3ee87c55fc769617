#!/bin/bash
# r3ar: one-view Otsu stats grid at 2 vs 1 MFMA chunks per wave (q_prev carried in the mu1 run),
# and the one-view kernels (stats, main_rm0/1/2, decode) under a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ar
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 2 1; do
  SLG_LIB=$R/ab_libs/ch$v.so timeout -k 10 240 rocprofv3 --kernel-trace -d $O/ch$v -o run -- python3 $R/tools/kbench.py --only stats,stats_no_otsu,main_rm0,main_rm1,main_rm2,decode --iters 60 > $O/kb_$v.log 2>&1 || { echo PROF_FAIL; tail -20 $O/kb_$v.log; exit 2; }
  echo "== ch$v"; python3 $R/tools/kstats_db.py $O/ch$v stats_kernel main3 decode_maps; grep -E "^(stats|main_rm|decode)" $O/kb_$v.log
done
