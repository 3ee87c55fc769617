#!/bin/bash
# Interleaved A/B of library builds on any bench.py configuration (tools/ab.py covers the C2
# shape only): each round runs bench.py once per library (SLG_LIB, in-tree A/B builds), and the
# summary line gives each library's ms_per_step per round.
#   bash tools/ab_bench.sh <tag> <rounds> "<bench.py args>" ab_libs/a.so ab_libs/b.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    SLG_LIB=$lib timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > "$O/abb_${n}_$r.json" 2> "$O/abb_${n}_$r.err" \
      || { echo "[ab_bench] $lib round $r FAILED"; tail -20 "$O/abb_${n}_$r.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['frac'], (d.get('verify') or {}).get('pipelined_equals_plain_bitwise'))" "$O/abb_${n}_$r.json" "$n" "$r"
  done
done
echo "[ab_bench] ALL_OK"
