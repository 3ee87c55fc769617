#!/bin/bash
# round 3 A/B under max-ilp: phase-B groups of 2, look-back window 1x64, item pad 1 per 32
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3aj
mkdir -p $O
cd $R
timeout -k 10 900 python tools/ab.py --variants ab_libs/base.so,ab_libs/g2.so,ab_libs/lk1.so,ab_libs/ipad5.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
