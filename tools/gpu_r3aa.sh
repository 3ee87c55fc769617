#!/bin/bash
# round 3: end-to-end drop-in paths on the current build -- file batch (PNG folders -> PLYs) and
# host-buffer frames (PCIe-inclusive)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3aa
mkdir -p $O
cd $R
timeout -k 10 500 python tools/e2e_files.py > $O/e2e_files.json 2> $O/e2e_files.err || { echo E2E_FILES_FAIL; tail -20 $O/e2e_files.err; exit 1; }
cat $O/e2e_files.json
timeout -k 10 300 python tools/e2e_bench.py > $O/e2e_bench.json 2> $O/e2e_bench.err || { echo E2E_BENCH_FAIL; tail -20 $O/e2e_bench.err; exit 2; }
cat $O/e2e_bench.json
