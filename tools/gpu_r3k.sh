#!/bin/bash
# round 3: 16 vs 12 views per fused launch with a pool whose carried batch never aliases the decoded one
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3k
mkdir -p $O
cd $R
for i in 1 2; do
  for cfg in "12 3" "16 4" "16 3"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --batch $1 --copies $2 --steps 100 --no-cpu-baseline > $O/bench_b$1_c$2_$i.json 2> $O/bench_b$1_c$2_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_b$1_c$2_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$O/bench_b$1_c$2_$i.json'));print('batch $1 copies $2',d['value'],d['config']['us_per_view'],d['roofline']['kernel_avg_us'],d['verify']['oracle_ok'],d['verify']['pipelined_equals_plain_bitwise'])"
  done
done
