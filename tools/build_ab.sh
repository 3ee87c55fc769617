#!/bin/bash
# Build A/B variants of libslgpu.so into build_ab/<name>.so (CPU side, hipcc cross-compiles).
# Usage: bash tools/build_ab.sh name1:"-DFLAG=1 -DX=2" name2:"..."   (run from the repo root)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/structured_light_for_3d_model_replication_amd/csrc
mkdir -p "$R/build_ab"
pids=()
for spec in "$@"; do
  name=${spec%%:*}
  flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp -fPIC -shared $flags \
    -o "$R/build_ab/$name.so" "$P/slgpu.hip" "$P/png_device.hip" "$P/png_gray.cpp" "$P/gather.cpp" -lz -ldl > "$R/build_ab/$name.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
ls -la "$R/build_ab"/*.so
exit $rc
