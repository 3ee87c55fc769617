#!/bin/bash
# round 2: C3 bench + full profile of the current fused kernel (trace, HBM PMC, SQ counters)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2i
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err || { echo C3_FAIL; tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
STEPS=300 timeout -k 10 700 bash tools/gpu_profile.sh r2i_prof || { echo PROF_FAIL; exit 2; }
timeout -k 10 500 bash tools/pmc_main.sh r2i_sq || { echo SQ_FAIL; exit 3; }
cat $R/gpurun_out/r2i_prof/bench.json
