#!/bin/bash
# round 3: fused vs fused2 (two streams) after making the cross-stream wait fused2-only; texture-late build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3e
mkdir -p $O
cd $R
for i in 1 2; do
  for m in fused fused2; do
    timeout -k 10 300 python bench.py --pipeline $m --steps 60 --no-cpu-baseline > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_${m}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$O/bench_${m}_$i.json'));print('$m',d['value'],d['config']['us_per_view'],d['roofline']['kernel_avg_us'],d['config']['host_enqueue_ms_per_step'],d['verify']['oracle_ok'],d['verify']['pipelined_equals_plain_bitwise'])"
  done
done
