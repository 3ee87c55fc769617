#!/bin/bash
# r3an: plan-specialised decode_maps_kernel -- decode-maps parity, then kbench "decode" A/B (old vs new)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3an
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "decode" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 2; }
tail -3 $O/tests.log
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=ab_libs/old.so; else L=structured_light_for_3d_model_replication_amd/libslgpu.so; fi
    SLG_LIB=$L timeout -k 10 200 python tools/kbench.py --only decode --iters 60 > $O/kb_${v}_$r.log 2>&1 || { echo KB_FAIL $v; tail -20 $O/kb_${v}_$r.log; exit 2; }
    echo "== $v $r"; grep -i decode $O/kb_${v}_$r.log
  done
done
