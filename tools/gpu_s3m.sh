#!/bin/bash
# session 3: per-byte bit-plane decode + scalar-base frame loads -- GPU suite, then A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 450 python tools/ab.py --libs tools/bin/ab_head.so,tools/bin/ab_so.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
