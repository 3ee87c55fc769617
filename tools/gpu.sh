#!/bin/bash
# The one GPU-box recipe (run through gpurun from the repo root).  Replaces round 3's 65 one-off
# tools/gpu_r*.sh scripts.
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Everything lands in gpurun_out/<tag>/.  Steps run in order, each under its own time limit;
# the script stops at the first failure (non-zero exit = the failing step's number).
#
# steps:
#   tests            pytest -m gpu (whole GPU suite, one process)       -> pytest_gpu.log
#   tests=<expr>     the same, -k <expr>                                -> pytest_gpu_<n>.log
#   smoke            __graft_entry__.smoke()                            -> smoke.log
#   bench            python bench.py (driver defaults)                  -> bench.json / .err
#   bench=<name>=<args>   python bench.py <args> (commas -> spaces)     -> bench_<name>.json / .err
#                    e.g. bench=c4=--config,c4   bench=2r=--gpus,2 (with SLG_BENCH_* exported)
#   prof             kernel trace + FETCH/WRITE PMC passes (tools/gpu_profile.sh) -> <tag>/prof/
#   prof=<name>=<args>   the same for bench.py <args> (commas -> spaces)  -> <tag>/prof_<name>/
#   sq               SQ counter passes (tools/pmc_main.sh)              -> <tag>/sq/
#   ab=<libA>,<libB>[,...][,rounds]  interleaved A/B of library builds (tools/ab.py; AB_ARGS) -> ab_<n>.log
#   py=<script>=<args>   python <script> <args> (commas -> spaces)      -> py_<n>.log
#   kt=<script>=<args>   the same under rocprofv3 --kernel-trace --stats  -> kt_<n>/ (+ kt_<n>.log)
#   mem              device memory as torch sees it                     -> mem.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%=*}
  rest=${step#*=}
  [ "$rest" = "$step" ] && rest=""
  echo "[gpu.sh] step $n: $step"
  case $kind in
    tests)
      log=$O/pytest_gpu.log; k=()
      if [ -n "$rest" ]; then log=$O/pytest_gpu_$n.log; k=(-k "$rest"); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" > "$log" 2>&1 \
        || { echo "[gpu.sh] TESTS FAILED"; tail -40 "$log"; exit $n; }
      tail -1 "$log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$O/smoke.log" 2>&1 \
        || { echo "[gpu.sh] SMOKE FAILED"; tail -20 "$O/smoke.log"; exit $n; }
      tail -1 "$O/smoke.log" ;;
    bench)
      name=${rest%%=*}; args=${rest#*=}
      if [ -z "$rest" ]; then name=default; args=""; fi
      [ "$args" = "$rest" ] && args=""
      timeout -k 10 900 python bench.py ${args//,/ } > "$O/bench_$name.json" 2> "$O/bench_$name.err" \
        || { echo "[gpu.sh] BENCH $name FAILED"; tail -20 "$O/bench_$name.err"; exit $n; }
      cat "$O/bench_$name.json" ;;
    prof)
      if [ -n "$rest" ]; then
        pname=${rest%%=*}; pargs=${rest#*=}
        PMC_TIMEOUT=300 BENCH_ARGS="${pargs//,/ }" bash "$R/tools/gpu_profile.sh" "$TAG/prof_$pname" || { echo "[gpu.sh] PROF $pname FAILED"; exit $n; }
        pdir=$O/prof_$pname
      else
        bash "$R/tools/gpu_profile.sh" "$TAG/prof" || { echo "[gpu.sh] PROF FAILED"; exit $n; }
        pdir=$O/prof
      fi
      # the raw traces run to tens of MB; gpurun copies back at most 64 MiB per call
      find "$pdir" -name "*.csv" -size +512k -exec gzip -f {} \; ;;
    sq)
      bash "$R/tools/pmc_main.sh" "$TAG/sq" || { echo "[gpu.sh] SQ FAILED"; exit $n; }
      find "$O/sq" -name "*.csv" -size +512k -exec gzip -f {} \; ;;
    ab)
      libs=${rest%,[0-9]*}; rounds=${rest##*,}
      [ "$libs" = "$rest" ] && rounds=4
      # AB_ARGS: extra tools/ab.py arguments for every ab step (e.g. "--xyz f64")
      timeout -k 10 900 python tools/ab.py --libs "$libs" --rounds "$rounds" $AB_ARGS > "$O/ab_$n.log" 2>&1 \
        || { echo "[gpu.sh] AB FAILED"; tail -20 "$O/ab_$n.log"; exit $n; }
      tail -3 "$O/ab_$n.log" ;;
    py)
      script=${rest%%=*}; args=${rest#*=}
      [ "$args" = "$rest" ] && args=""
      timeout -k 10 600 python "$script" ${args//,/ } > "$O/py_$n.log" 2>&1 \
        || { echo "[gpu.sh] PY $script FAILED"; tail -30 "$O/py_$n.log"; exit $n; }
      tail -5 "$O/py_$n.log" ;;
    kt)
      script=${rest%%=*}; args=${rest#*=}
      [ "$args" = "$rest" ] && args=""
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/kt_$n" -o kt \
        --output-format csv -- python "$R/$script" ${args//,/ } > "$O/kt_$n.log" 2>&1) \
        || { echo "[gpu.sh] KT $script FAILED"; tail -30 "$O/kt_$n.log"; exit $n; }
      head -12 "$O/kt_$n/kt_kernel_stats.csv" 2>/dev/null || find "$O/kt_$n" -name "*kernel_stats.csv" -exec head -12 {} \; ;;
    mem)
      timeout -k 10 120 python -c "import torch; f,t=torch.cuda.mem_get_info(0); print('free',f,'total',t,torch.cuda.get_device_name(0))" > "$O/mem.log" 2>&1 \
        || { echo "[gpu.sh] MEM FAILED"; cat "$O/mem.log"; exit $n; }
      cat "$O/mem.log" ;;
    *)
      echo "[gpu.sh] unknown step $step"; exit 99 ;;
  esac
done
echo "[gpu.sh] ALL_OK"
