#!/bin/bash
# round 3 A/B: LLVM AMDGPU scheduler strategies (max-ilp, max-memory-clause, iterative-minreg)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ae
mkdir -p $O
cd $R
timeout -k 10 900 python tools/ab.py --variants ab_libs/base.so,ab_libs/milp.so,ab_libs/mclause.so,ab_libs/minreg.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
