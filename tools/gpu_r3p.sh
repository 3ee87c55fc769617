#!/bin/bash
# round 3: GPU suite on the current build, phase records (profiling instance), the other
# BASELINE geometries (C4, C5, C3 job)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
KBENCH_DBG=2,4 KBENCH_PHASE_EXTRA=0,2 timeout -k 10 400 python tools/kbench.py --only main3_batch12,main3_batch12_dbg2,main3_batch12_dbg4,phases > $O/kbench.json 2> $O/kbench.err || { echo KB_FAIL; tail -20 $O/kbench.err; exit 2; }
grep -E "per view|phases" $O/kbench.err
for c in c4 c5 c3; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo BENCH_FAIL $c; tail -20 $O/bench_$c.err; exit 3; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));r=d.get('roofline') or {};print('$c',d['value'],d['unit'],d['config'].get('us_per_view'),r.get('frac'),(d.get('verify') or {}).get('oracle_ok'))"
done
echo ALL_OK
