#!/bin/bash
# round 3 A/B: phase A (streaming) at wave priority 1 / 3, the rest at 0
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3u
mkdir -p $O
cd $R
timeout -k 10 600 python tools/ab.py --variants ab_libs/base.so,ab_libs/prio1.so,ab_libs/prio3.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
