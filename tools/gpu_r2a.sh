set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { echo BENCH_FAIL; tail -20 $O/bench20.err; exit 2; }
cat $O/bench20.json
timeout -k 10 300 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > $O/bench400.json 2> $O/bench400.err || { echo BENCH400_FAIL; tail -20 $O/bench400.err; exit 3; }
cat $O/bench400.json
