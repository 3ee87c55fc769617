#!/bin/bash
# round 3: views per fused launch (fused2 pipeline), interleaved repeats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3j
mkdir -p $O
cd $R
for i in 1 2; do
  for b in 12 16 8; do
    timeout -k 10 300 python bench.py --batch $b --steps 100 --no-cpu-baseline --no-verify > $O/bench_b${b}_$i.json 2> $O/bench_b${b}_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_b${b}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$O/bench_b${b}_$i.json'));print('batch $b',d['value'],d['config']['us_per_view'],d['roofline']['kernel_avg_us'])"
  done
done
