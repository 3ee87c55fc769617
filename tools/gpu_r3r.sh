#!/bin/bash
# round 3: ablations of the plan-specialised profiling instance (12-view launch, no carry):
# 1 no look-back wait, 2 trivial triangulation, 4 no D at all, 8 no BGR stores, 128 no XYZ stores
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3r
mkdir -p $O
cd $R
KBENCH_DBG=1,2,4,8,128 timeout -k 10 400 python tools/kbench.py --only main3_batch12,main3_batch12_dbg1,main3_batch12_dbg2,main3_batch12_dbg4,main3_batch12_dbg8,main3_batch12_dbg128,main3_batch12_next > $O/kbench.json 2> $O/kbench.err || { echo KB_FAIL; tail -20 $O/kbench.err; exit 1; }
grep -E "per view" $O/kbench.err
