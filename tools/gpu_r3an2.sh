#!/bin/bash
# r3an2: kernel trace of kbench "decode" (stats + decode_maps) for the old and the plan-specialised build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3an2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then L=$R/ab_libs/old.so; else L=$R/structured_light_for_3d_model_replication_amd/libslgpu.so; fi
  SLG_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 $R/tools/kbench.py --only decode --iters 60 > $O/kb_$v.log 2>&1 || { echo PROF_FAIL $v; tail -20 $O/kb_$v.log; exit 2; }
done
for v in old new; do echo "== $v"; f=$(find $O/$v -name '*kernel_stats.csv' | head -1); grep -E "decode_maps|stats_kernel|otsu" $f | cut -c1-200; done
