#!/bin/bash
# A/B library builds of the product sources with extra -D flags, into ab_libs/<name>.so
# (tools/ab.py, tools/ab_bench.sh, kbench via SLG_LIB).   bash tools/build_ab.sh <name> [-DFLAG=V ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
C=$R/structured_light_for_3d_model_replication_amd/csrc
mkdir -p "$R/ab_libs"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
  -fPIC -shared "$@" -o "$R/ab_libs/$name.so.tmp" "$C/slgpu.hip" "$C/png_device.hip" "$C/png_gray.cpp" "$C/gather.cpp" -lz -ldl
mv "$R/ab_libs/$name.so.tmp" "$R/ab_libs/$name.so"
echo "built ab_libs/$name.so $*"
