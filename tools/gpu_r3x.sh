#!/bin/bash
# round 3 A/B: texture behind the first pattern batch, carried white/black behind this tile's
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3x
mkdir -p $O
cd $R
timeout -k 10 600 python tools/ab.py --variants ab_libs/base.so,ab_libs/ldo.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
