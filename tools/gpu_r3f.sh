#!/bin/bash
# round 3 state: GPU suite, default bench (fused2 + CPU baseline), rocprofv3 trace + HBM PMC + SQ counters
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 2; }
cat $O/bench_default.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_steps20.json 2> $O/bench_steps20.err || { echo BENCH20_FAIL; exit 3; }
STEPS=300 timeout -k 10 800 bash tools/gpu_profile.sh r3f_prof || { echo PROF_FAIL; exit 4; }
timeout -k 10 500 bash tools/pmc_main.sh r3f_sq || { echo SQ_FAIL; exit 5; }
echo ALL_OK
