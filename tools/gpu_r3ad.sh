#!/bin/bash
# round 3 final state: GPU suite, smoke(), default bench (with CPU baseline) and at --steps 20
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ad
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 3; }
cat $O/bench_default.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_steps20.json 2> $O/bench_steps20.err || { echo BENCH20_FAIL; exit 4; }
python -c "import json;d=json.load(open('$O/bench_steps20.json'));print('steps20',d['value'],d['config']['us_per_view'],d['roofline']['frac'])"
echo ALL_OK
