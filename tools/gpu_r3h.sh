#!/bin/bash
# round 3: mask-first build -- phase records + ablations, rocprofv3 trace + HBM PMC, SQ counters
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3h
mkdir -p $O
cd $R
KBENCH_DBG=1,2,4,3,128 KBENCH_PHASE_EXTRA=0,1,2 timeout -k 10 400 python tools/kbench.py --only main3_batch12,main3_batch12_dbg1,main3_batch12_dbg2,main3_batch12_dbg4,main3_batch12_dbg3,main3_batch12_dbg128,main3_batch12_next,phases > $O/kbench.json 2> $O/kbench.err || { echo KB_FAIL; tail -20 $O/kbench.err; exit 1; }
grep -E "per view|phases" $O/kbench.err
STEPS=300 timeout -k 10 800 bash tools/gpu_profile.sh r3h_prof || { echo PROF_FAIL; exit 4; }
timeout -k 10 500 bash tools/pmc_main.sh r3h_sq || { echo SQ_FAIL; exit 5; }
echo ALL_OK
