#!/bin/bash
# round 2 (session 3) end state: GPU suite, bench + rocprofv3 trace + HBM PMC + SQ counters
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 2; }
STEPS=300 timeout -k 10 800 bash tools/gpu_profile.sh r2x_prof || { echo PROF_FAIL; exit 3; }
timeout -k 10 500 bash tools/pmc_main.sh r2x_sq || { echo SQ_FAIL; exit 4; }
echo ALL_OK
