#!/bin/bash
# round 3: plan-specialised build -- pipeline x batch matrix on one box, rocprofv3 trace + HBM PMC,
# SQ counters, phase records
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3o
mkdir -p $O
cd $R
for i in 1 2; do
  for cfg in "fused2 16" "fused 16" "fused2 12" "fused 12"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --pipeline $1 --batch $2 --steps 100 --no-cpu-baseline --no-verify > $O/bench_$1_$2_$i.json 2> $O/bench_$1_$2_$i.err || { echo BENCH_FAIL; tail -20 $O/bench_$1_$2_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$O/bench_$1_$2_$i.json'));print('$1 $2',d['value'],d['config']['us_per_view'],d['roofline']['kernel_avg_us'])"
  done
done
STEPS=300 timeout -k 10 800 bash tools/gpu_profile.sh r3o_prof || { echo PROF_FAIL; exit 4; }
timeout -k 10 500 bash tools/pmc_main.sh r3o_sq || { echo SQ_FAIL; exit 5; }
KBENCH_DBG=2,4 KBENCH_PHASE_EXTRA=0,2 timeout -k 10 400 python tools/kbench.py --only main3_batch12,main3_batch12_dbg2,main3_batch12_dbg4,phases > $O/kbench.json 2> $O/kbench.err || { echo KB_FAIL; tail -20 $O/kbench.err; exit 1; }
grep -E "per view|phases" $O/kbench.err
echo ALL_OK
