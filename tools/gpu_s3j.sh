#!/bin/bash
# session 3: per-byte bit-plane decode + scalar-base frame loads -- GPU suite, then A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3j
mkdir -p $O
cd $R
true
true
timeout -k 10 450 python tools/ab.py --libs tools/bin/ab_bl.so,tools/bin/ab_gb.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
