#!/bin/bash
# round 3: multi-item main3 workgroups (next item's frames issued before the look-back):
# GPU suite on the in-tree build, then an interleaved A/B against the round-2 kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 900 python tools/ab.py --variants ab_libs/base.so,ab_libs/pf8.so,ab_libs/pf6.so,ab_libs/pf8.so@SLG_TPW=1 --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
