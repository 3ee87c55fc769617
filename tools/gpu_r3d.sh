#!/bin/bash
# round 3: two-stream overlapped pipeline (fused2) vs fused; texture-late A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3d
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "two_stream" -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_fused2.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_fused2.log; exit 1; }
tail -1 $O/pytest_fused2.log
for i in 1 2; do
  for m in fused fused2; do
    timeout -k 10 300 python bench.py --pipeline $m --steps 60 --no-cpu-baseline > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_${m}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$O/bench_${m}_$i.json'));print('$m',d['value'],d['config']['us_per_view'],d['roofline']['kernel_avg_us'],d['verify']['oracle_ok'],d['verify']['pipelined_equals_plain_bitwise'])"
  done
done
timeout -k 10 600 python tools/ab.py --variants ab_libs/base.so,ab_libs/texlate.so --rounds 4 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 3; }
tail -1 $O/ab.log
