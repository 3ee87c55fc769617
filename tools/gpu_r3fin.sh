#!/bin/bash
# round 3 closing call: GPU suite + smoke on the final tree, default bench, then the profiling recipe
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3fin
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 3; }
cat $O/bench_default.json
bash $R/tools/gpu_profile.sh r3fin_prof || { echo PROF_FAIL; exit 4; }
echo ALL_OK
