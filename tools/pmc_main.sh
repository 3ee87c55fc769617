#!/bin/bash
# SQ counter passes over the production fused launches (bench.py's C2 pipeline), one rocprofv3
# run per pass (each pass within the per-block counter limits).
# Usage (GPU box, repo root): bash tools/pmc_main.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  echo "[pmc] pass $n"
  timeout -s KILL 150 rocprofv3 --pmc $P -d "$OUT/p$n" -o p$n --output-format csv -- python "$R/bench.py" --steps 24 --warmup 4 --settle-ms 0 --no-verify --no-cpu-baseline > /dev/null 2> "$OUT/p$n.err" || exit $n
done
echo "[pmc] done"
