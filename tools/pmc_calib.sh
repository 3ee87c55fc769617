#!/bin/bash
# HBM byte-counter calibration on the GPU box: tools/fetch_probe.hip's known
# byte counts against FETCH_SIZE / WRITE_SIZE and the gfx950 request-size counters, then the same
# request-size passes over bench.py's fused launches.  One rocprofv3 run per counter pass.
#   bash tools/pmc_calib.sh <tag>          (repo root; results in gpurun_out/<tag>/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmc_calib}
mkdir -p "$O"
cd "$R"
echo "[calib] build probe" && timeout -k 10 300 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/fetch_probe.hip -o "$O/fetch_probe" > "$O/build.log" 2>&1 || { cat "$O/build.log"; exit 1; }
echo "[calib] mask" && timeout -k 10 300 python tools/fetch_probe.py "$O/mask.bin" > "$O/mask.log" 2>&1 || { cat "$O/mask.log"; exit 2; }
cat "$O/mask.log"
echo "[calib] probe" && timeout -k 10 120 "$O/fetch_probe" "$O/mask.bin" > "$O/probe.json" 2> "$O/probe.err" || { cat "$O/probe.err"; exit 3; }
cat "$O/probe.json"
cd /tmp && export TMPDIR=/tmp
PASSES=("FETCH_SIZE" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
        "TCC_BUBBLE_sum" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum")
n=0
for P in "${PASSES[@]}"; do
  n=$((n + 1))
  echo "[calib] probe pass $n: $P"
  timeout -s KILL 90 rocprofv3 --pmc $P -d "$O/probe_p$n" -o p$n --output-format csv -- "$O/fetch_probe" "$O/mask.bin" > /dev/null 2> "$O/probe_p$n.err" || { tail -5 "$O/probe_p$n.err"; exit $((10 + n)); }
done
n=0
for P in "${PASSES[@]}"; do
  n=$((n + 1))
  echo "[calib] bench pass $n: $P"
  timeout -s KILL 150 rocprofv3 --pmc $P -d "$O/bench_p$n" -o p$n --output-format csv -- python "$R/bench.py" --steps 24 --warmup 6 --no-verify --no-cpu-baseline > /dev/null 2> "$O/bench_p$n.err" || { tail -5 "$O/bench_p$n.err"; exit $((20 + n)); }
done
echo "[calib] done"
