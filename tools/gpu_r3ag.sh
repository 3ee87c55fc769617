#!/bin/bash
# round 3: max-ilp scheduler build -- GPU suite, default bench, C4 / C5
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ag
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print('c2',d['value'],d['config']['us_per_view'],d['roofline']['frac'],d['verify']['oracle_ok'])"
for c in c4 c5; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo BENCH_FAIL $c; tail -20 $O/bench_$c.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['config']['us_per_view'],d['roofline']['frac'],d['verify']['oracle_ok'])"
done
echo ALL_OK
