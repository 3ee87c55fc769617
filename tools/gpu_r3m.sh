#!/bin/bash
# round 3: GPU suite (16-view fused2 shape added), default bench (16 views per launch), then an
# interleaved A/B of kernel experiments (fixed C2 plan, t division without scaling, 2-round groups)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 3; }
cat $O/bench_default.json
timeout -k 10 700 python tools/ab.py --variants ab_libs/base.so,ab_libs/plan.so,ab_libs/tdiv.so,ab_libs/g2.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
echo ALL_OK
