#!/bin/bash
# Request-size probe on the GPU box: tools/reqsize_probe.hip's cache-policy variants of main3's
# mask-gated loads, timed, then one rocprofv3 pass of the gfx950 request-size counters.
#   bash tools/reqsize_probe.sh <tag>      (repo root; results in gpurun_out/<tag>/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-reqsize}
mkdir -p "$O"
cd "$R"
echo "[req] build" && timeout -k 10 300 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/reqsize_probe.hip -o "$O/reqsize_probe" > "$O/build.log" 2>&1 || { cat "$O/build.log"; exit 1; }
echo "[req] mask" && timeout -k 10 300 python tools/fetch_probe.py "$O/mask.bin" > "$O/mask.log" 2>&1 || { cat "$O/mask.log"; exit 2; }
echo "[req] run" && timeout -k 10 120 "$O/reqsize_probe" "$O/mask.bin" > "$O/probe.json" 2> "$O/probe.err" || { cat "$O/probe.err"; exit 3; }
cat "$O/probe.json"
cd /tmp && export TMPDIR=/tmp
echo "[req] pmc" && timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d "$O/pmc" -o pmc --output-format csv -- "$O/reqsize_probe" "$O/mask.bin" > /dev/null 2> "$O/pmc.err" || { tail -5 "$O/pmc.err"; exit 4; }
echo "[req] done"
