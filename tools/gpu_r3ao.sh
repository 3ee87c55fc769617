#!/bin/bash
# r3ao: one-view stats_kernel grid (SLG_STATS_BLOCKS_SOLO 64/128/256/512), otsu and percentile,
# kernel durations from rocprofv3 kernel traces of kbench "stats"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for t in otsu percentile; do
  for v in 64 128 256 512; do
    SLG_LIB=$R/ab_libs/solo$v.so timeout -k 10 240 rocprofv3 --kernel-trace -d $O/${t}_$v -o run -- python3 $R/tools/kbench.py --only stats --iters 60 --thresh $t > $O/kb_${t}_$v.log 2>&1 || { echo PROF_FAIL $t $v; tail -20 $O/kb_${t}_$v.log; exit 2; }
    echo "== $t $v"; python3 $R/tools/kstats_db.py $O/${t}_$v stats_kernel decode_maps
  done
done
