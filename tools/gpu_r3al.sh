#!/bin/bash
# round 3: clock settling before the timed steps -- the driver-style --steps 20 run after 60 ms
# (default) vs 300 ms of untimed settle launches, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3al
mkdir -p $O
cd $R
for i in 1 2 3; do
  for st in 60 300; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --settle-ms $st --no-cpu-baseline --no-verify > $O/b_${st}_$i.json 2> $O/b_${st}_$i.err || { echo BENCH_FAIL; tail -5 $O/b_${st}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${st}_$i.json'));print('settle $st',d['value'],d['config']['us_per_view'])"
  done
done
