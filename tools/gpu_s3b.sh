#!/bin/bash
# session 3: scalar look-back window A/B (8 / 16 / 32 predecessors per poll) + phase records
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3b
mkdir -p $O
cd $R
timeout -k 10 500 python tools/ab.py --libs tools/bin/ab_base.so,tools/bin/slb1.so,tools/bin/slb2.so,tools/bin/slb4.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 1; }
tail -1 $O/ab.log
for v in ab_base slb1 slb4; do
  SLG_LIB=tools/bin/$v.so KBENCH_PHASE_EXTRA=0 timeout -k 10 200 python tools/kbench.py --only phases > $O/kbp_$v.json 2> $O/kbp_$v.log || { echo KB_FAIL $v; tail -20 $O/kbp_$v.log; exit 2; }
  grep "phases (dbg" $O/kbp_$v.log
done
