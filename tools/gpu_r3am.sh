#!/bin/bash
# round 3 end (mask first, plan instances, max-ilp): rocprofv3 trace + HBM PMC of the C4 and C5 configurations on the final build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
STEPS=60 TRACE_STEPS=40 PMC_STEPS=8 BENCH_ARGS="--config c4" timeout -k 10 700 bash tools/gpu_profile.sh r3am_c4 || { echo C4_FAIL; exit 1; }
STEPS=100 TRACE_STEPS=60 PMC_STEPS=12 BENCH_ARGS="--config c5" timeout -k 10 700 bash tools/gpu_profile.sh r3am_c5 || { echo C5_FAIL; exit 2; }
echo ALL_OK
