#!/bin/bash
# session 3: GPU suite on the scalar look-back build, then bench at 12 and 16 views per launch
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench12.json 2> $O/bench12.err || { echo B12_FAIL; tail -20 $O/bench12.err; exit 2; }
timeout -k 10 240 python bench.py --no-cpu-baseline --batch 16 --views 16 > $O/bench16.json 2> $O/bench16.err || { echo B16_FAIL; tail -20 $O/bench16.err; exit 3; }
python - <<'PY'
import json
for n in ("bench12", "bench16"):
    d = json.load(open(f"gpurun_out/s3a/{n}.json"))
    print(n, d["value"], d["config"]["us_per_view"], d["roofline"]["frac"], d["roofline"]["kernel_avg_us"], d["verify"]["oracle_ok"])
PY
