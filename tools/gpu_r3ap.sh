#!/bin/bash
# r3ap: branch-free Otsu mu1 run + one-view stats grid 256 -- GPU suite, stats kernel trace
# (stats / stats_no_otsu), bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ap
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for t in otsu percentile; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/$t -o run -- python3 $R/tools/kbench.py --only stats,stats_no_otsu --iters 60 --thresh $t > $O/kb_$t.log 2>&1 || { echo PROF_FAIL; tail -20 $O/kb_$t.log; exit 2; }
  echo "== $t"; python3 $R/tools/kstats_db.py $O/$t stats_kernel; grep "^stats" $O/kb_$t.log
done
cd $R && timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 2; }
cut -c1-400 $O/bench.json
