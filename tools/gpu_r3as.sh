#!/bin/bash
# r3as: speculative 4-op mu1 run (Markstein-checked), edge lanes peeled -- GPU suite, one-view stats trace, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3as}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/otsu -o run -- python3 $R/tools/kbench.py --only stats,stats_no_otsu,main_rm1 --iters 60 > $O/kb.log 2>&1 || { echo PROF_FAIL; tail -20 $O/kb.log; exit 2; }
python3 $R/tools/kstats_db.py $O/otsu stats_kernel parts_kernel; grep -E "^(stats|main_rm)" $O/kb.log
cd $R && timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 2; }
cut -c1-300 $O/bench.json
