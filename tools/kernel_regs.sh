#!/bin/bash
# VGPR / SGPR / scratch of the device kernels in csrc/slgpu.hip as built with the product flags
# (plus any extra -D flags given):   bash tools/kernel_regs.sh [-DFLAG=V ...] [| grep main3]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
  --cuda-device-only "$@" -c "$R/structured_light_for_3d_model_replication_amd/csrc/slgpu.hip" -o "$T/k.co" 2>/dev/null
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/k.co" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.o"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/k.o" | grep -E "^ +\.name:|\.vgpr_count:|\.sgpr_count:|\.private_segment_fixed_size:" \
  | paste - - - - | awk '{print $2, "scratch="$4, "sgpr="$6, "vgpr="$8}'
rm -rf "$T"
