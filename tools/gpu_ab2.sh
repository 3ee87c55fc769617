#!/bin/bash
# interleaved A/B of two library builds (no test suite):  bash tools/gpu_ab2.sh <tag> <libA> <libB> [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 500 python tools/ab.py --variants $2,$3 --rounds ${4:-4} > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
cat $O/ab.log
