#!/bin/bash
# round 3: PLY bodies formatted on the device -- GPU suite (device formatter test, file
# pipeline PLY bytes vs the oracle), then the end-to-end file path
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ac
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 500 python tools/e2e_files.py > $O/e2e_files.json 2> $O/e2e_files.err || { echo E2E_FILES_FAIL; tail -20 $O/e2e_files.err; exit 2; }
cat $O/e2e_files.json
