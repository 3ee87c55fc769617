#!/bin/bash
# end of session 3: smoke(), C4 / C5 / C3 bench configs on the final build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2t
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for c in c4 c5 c3; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo BENCH_FAIL $c; tail -20 $O/bench_$c.err; exit 2; }
done
python - <<'PY'
import json
for c in ("c4", "c5", "c3"):
    d = json.load(open(f"gpurun_out/r2t/bench_{c}.json"))
    print(c, d["value"], d["unit"], d.get("roofline", {}).get("frac"), d["config"].get("us_per_view"), (d.get("verify") or {}).get("oracle_ok"))
PY
