#!/bin/bash
# round 3 A/B: carried histograms by per-wave LDS atomics counted in phase C (wave 0 before its
# look-back) against the i8-MFMA counting
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3z
mkdir -p $O
cd $R
timeout -k 10 500 python tools/ab.py --variants ab_libs/base.so,ab_libs/hldsc.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
