#!/bin/bash
# round 3 A/B: pinhole rays recomputed (base) vs the Nc ray table gathered (rayt:rays), texture
# in two loads (tex2)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3q
mkdir -p $O
cd $R
timeout -k 10 600 python tools/ab.py --variants ab_libs/base.so,ab_libs/rayt.so:rays,ab_libs/tex2.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
cat $O/ab.log
