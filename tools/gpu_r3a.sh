#!/bin/bash
# round 3 first call: host probe, GPU suite, default bench, 2-rank self-spawn rehearsals
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
{ echo "nproc $(nproc)"; python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>&1; cat /proc/self/cgroup; rocm-smi --showuse 2>&1 | head -20; } > $O/host_probe.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 2; }
cat $O/bench_default.json
SLG_BENCH_DEVICE=0 SLG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2r.json 2> $O/bench_2r.err || { echo BENCH2_FAIL; tail -20 $O/bench_2r.err; exit 3; }
cat $O/bench_2r.json
SLG_BENCH_DEVICE=0 SLG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c3 --steps 5 --warmup 2 > $O/bench_2r_c3.json 2> $O/bench_2r_c3.err || { echo BENCH2C3_FAIL; tail -20 $O/bench_2r_c3.err; exit 4; }
cat $O/bench_2r_c3.json
echo ALL_OK
