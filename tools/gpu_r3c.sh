#!/bin/bash
# round 3: new GPU tests (Otsu ties, calib cache, gather) + views-per-launch A/B (12 vs 16)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "otsu_edge or oc_" tests/test_calib_cache.py tests/test_gather.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_new.log; exit 1; }
tail -2 $O/pytest_new.log
for i in 1 2; do
  for b in 12 16; do
    timeout -k 10 300 python bench.py --batch $b --steps 60 --no-cpu-baseline --no-verify > $O/bench_b${b}_$i.json 2> $O/bench_b${b}_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_b${b}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$O/bench_b${b}_$i.json'));print($b,d['value'],d['config']['us_per_view'],d['roofline']['kernel_avg_us'])"
  done
done
