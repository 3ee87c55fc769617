#!/bin/bash
# round 3: the driver's round-end steps on the current build -- smoke(), 2-rank self-spawn
# rehearsals on one GPU (gloo) for the default and c3 configs, the default bench at --steps 20
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3t
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
SLG_BENCH_DEVICE=0 SLG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2r.json 2> $O/bench_2r.err || { echo BENCH2_FAIL; tail -20 $O/bench_2r.err; exit 3; }
cat $O/bench_2r.json
SLG_BENCH_DEVICE=0 SLG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c3 --steps 5 --warmup 2 > $O/bench_2r_c3.json 2> $O/bench_2r_c3.err || { echo BENCH2C3_FAIL; tail -20 $O/bench_2r_c3.err; exit 4; }
cat $O/bench_2r_c3.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || { echo BENCH20_FAIL; tail -20 $O/bench_steps20.err; exit 5; }
cat $O/bench_steps20.json
echo ALL_OK
