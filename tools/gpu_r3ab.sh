#!/bin/bash
# round 3 A/B: tiles with 5 item rounds triangulated as one group of 5 (else 4 + 1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ab
mkdir -p $O
cd $R
timeout -k 10 500 python tools/ab.py --variants ab_libs/base.so,ab_libs/g5.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
