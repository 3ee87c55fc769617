#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   bench -> rocprofv3 kernel trace + stats -> separate PMC passes (FETCH_SIZE, WRITE_SIZE,
#   the read request-size counters).
# Every step has its own time limit and the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof}
STEPS=${STEPS:-300}
BA=${BENCH_ARGS:-}          # e.g. BENCH_ARGS="--config c4" (word-split on purpose)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "[prof] bench" && timeout -k 10 300 python "$R/bench.py" $BA --steps "$STEPS" --warmup 10 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
echo "[prof] kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python "$R/bench.py" $BA --steps ${TRACE_STEPS:-200} --warmup 10 --no-cpu-baseline --no-verify > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit 2
echo "[prof] pmc fetch" && timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python "$R/bench.py" $BA --steps ${PMC_STEPS:-24} --warmup 6 --no-verify --no-cpu-baseline > /dev/null 2> "$OUT/fetch.err" || exit 3
echo "[prof] pmc write" && timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python "$R/bench.py" $BA --steps ${PMC_STEPS:-24} --warmup 6 --no-verify --no-cpu-baseline > /dev/null 2> "$OUT/write.err" || exit 4
# the gfx950 read request sizes: reads = 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B
# (calibrated on known byte counts, tools/fetch_probe.hip; = FETCH_SIZE x 2 when all are 128 B)
echo "[prof] pmc rdreq" && timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d "$OUT/rdreq" -o rdreq --output-format csv -- python "$R/bench.py" $BA --steps ${PMC_STEPS:-24} --warmup 6 --no-verify --no-cpu-baseline > /dev/null 2> "$OUT/rdreq.err" || exit 5
echo "[prof] done"
