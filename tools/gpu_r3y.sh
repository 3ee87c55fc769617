#!/bin/bash
# round 3: carried histograms by per-wave LDS atomics -- GPU suite, A/B against the i8-MFMA
# counting, default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 500 python tools/ab.py --variants ab_libs/base.so,ab_libs/hlds.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['config']['us_per_view'],d['roofline']['frac'],d['verify']['oracle_ok'],d['verify']['pipelined_equals_plain_bitwise'])"
