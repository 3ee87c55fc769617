#!/bin/bash
# round 3 final build: long steady-state run (3000 steps: look-back helper never runs, verify
# green), 2-rank self-spawn rehearsal (gloo, one GPU), c3 job
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ak
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 3000 --no-cpu-baseline > $O/bench_3000.json 2> $O/bench_3000.err || { echo BENCH_FAIL; tail -20 $O/bench_3000.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_3000.json'));print('3000 steps',d['value'],d['config']['us_per_view'],d['config']['lookback_helper_runs'],d['verify']['oracle_ok'],d['verify']['pipelined_equals_plain_bitwise'])"
SLG_BENCH_DEVICE=0 SLG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2r.json 2> $O/bench_2r.err || { echo BENCH2_FAIL; tail -20 $O/bench_2r.err; exit 2; }
python -c "import json;d=json.load(open('$O/bench_2r.json'));print('2 ranks',d['n_gpus'],d['value'],d['verify']['oracle_ok'])"
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err || { echo C3_FAIL; tail -20 $O/bench_c3.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3',d['value'],d['ms_per_step'])"
echo ALL_OK
