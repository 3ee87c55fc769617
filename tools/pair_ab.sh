#!/bin/bash
# Paired 16-byte frame / texture loads against the product library (round 6): the GPU suite with
# the candidate, then interleaved A/B at the bench's C2 shape (f32 and f64) and at C1.
#   bash tools/pair_ab.sh <tag> <candidate.so> <lib> [<lib> ...]      (ab_libs/ paths)
set -o pipefail
TAG=$1; CAND=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
SLG_LIB=$CAND timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cand.log 2>&1 \
  || { tail -30 $O/pytest_cand.log; exit 1; }
tail -1 $O/pytest_cand.log
LIBS=$(IFS=,; echo "$*")
bash tools/gpu.sh $TAG ab=$LIBS,4 || exit 2
bash tools/ab_bench.sh $TAG 2 "--config c1 --steps 100" "$@" || exit 3
AB_ARGS="--xyz f64" bash tools/gpu.sh ${TAG}_f64 ab=$LIBS,3 || exit 4
