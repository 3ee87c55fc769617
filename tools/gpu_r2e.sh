#!/bin/bash
# round 2, step e: GPU suite with the table ABI + A/B tables on/off and look-back window
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r2e}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python tools/ab.py --rounds 3 --launches 200 --variants build_ab/g2.so:num,build_ab/g2.so:none > $O/ab.json 2> $O/ab.err || { echo AB_FAIL; tail -30 $O/ab.err; exit 3; }
grep "\[ab\]" $O/ab.err; cat $O/ab.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { echo BENCH_FAIL; tail -20 $O/bench20.err; exit 2; }; cat $O/bench20.json
