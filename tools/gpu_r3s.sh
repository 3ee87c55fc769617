#!/bin/bash
# round 3: BGR staged in LDS and written as dwords -- GPU suite, A/B against byte stores
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3s
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 500 python tools/ab.py --variants ab_libs/base.so,ab_libs/stage.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
