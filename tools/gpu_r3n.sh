#!/bin/bash
# round 3: decode-plan specialised main3 instances -- GPU suite, default bench, A/B against the
# previous build, then the mask-first occupancy / compute-tail probe
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 3; }
cat $O/bench_default.json
timeout -k 10 500 python tools/ab.py --variants ab_libs/prev.so,ab_libs/plan.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
python tools/mf_probe.py /tmp/mf_mask.bin && MF_PROBE_ONLY=t timeout -k 10 200 tools/bin/mf_probe /tmp/mf_mask.bin > $O/mf_probe_tail.log 2>&1 || { echo PROBE_FAIL; tail $O/mf_probe_tail.log; exit 4; }
cat $O/mf_probe_tail.log
echo ALL_OK
