#!/bin/bash
# round 3 final build (max-ilp scheduler): rocprofv3 kernel trace + stats, HBM PMC passes, SQ counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
STEPS=300 timeout -k 10 800 bash tools/gpu_profile.sh r3ai_prof || { echo PROF_FAIL; exit 4; }
timeout -k 10 500 bash tools/pmc_main.sh r3ai_sq || { echo SQ_FAIL; exit 5; }
echo ALL_OK
