#!/bin/bash
# round 3 A/B: scheduler options on top of max-ilp (AMDGPU RP trackers, no mem-op clustering, relaxed occupancy)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ah
mkdir -p $O
cd $R
timeout -k 10 900 python tools/ab.py --variants ab_libs/base.so,ab_libs/trk.so,ab_libs/nocl.so,ab_libs/relax.so --rounds 3 > $O/ab.log 2>&1 || { echo AB_FAIL; tail -20 $O/ab.log; exit 2; }
tail -1 $O/ab.log
